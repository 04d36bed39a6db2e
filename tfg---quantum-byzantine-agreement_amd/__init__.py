"""MI355X-native engine for the data-parallel core of tfg.py's quantum
Byzantine agreement (Carl0sGV/TFG---Quantum-Byzantine-Agreement).

Submodules:
  comm      in-process MPI world / mpi4py adapter (protocol transport)
  resource  the reference's circuits as gate lists (qsimov API subset)
  engine    torch front end of libqba.so (HIP kernels for gfx950)
  protocol  tfg.py-compatible protocol host (exact set-order semantics)
  countmode protocol decisions from device count histograms (large sizeL)
  tfg       CLI: python -m <pkg>.tfg <sizeL> <nDishonest> [--parties N]
"""
import importlib as _importlib

__all__ = ["comm", "resource", "engine", "protocol", "countmode", "tfg"]
__version__ = "0.1.0"


def __getattr__(name):
    if name in __all__:
        return _importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
