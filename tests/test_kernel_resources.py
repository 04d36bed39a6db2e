"""Static resource guards on the shipped gfx950 code objects (no GPU needed).

The hot kernels' speed rests on properties the compiler decides and a source
change can silently lose (profiles/r5/slab_event/):
  * no scratch: a kernel with a private segment is dispatched ~0.6 us later
    after the previous kernel, and a spill inside the main loop makes every
    step wait for all outstanding row stores;
  * at most 64 VGPRs for the kernels compiled for 8 waves per SIMD (the
    list kernels' 2 workgroups of 1024 threads per CU; the batched kernel).
Read from the kernel descriptors inside libqba.so (tests/kd_util.py).
"""
from pathlib import Path

import pytest

from kd_util import kernel_descriptors

LIB = Path(__file__).resolve().parent.parent / "tfg---quantum-byzantine-agreement_amd" / "_build" / "libqba.so"

# mangled-name prefixes: qba_k_lists<11, 1, CLOSED, 2, 1, 1> (the headline's
# synchronous kernel), qba_k_lists_pbdef<11, 2, 1> (bench.py's deferred step),
# qba_k_lists_def<11, CLOSED, 2, 1> (configs[1]), qba_k_batched<7, CLOSED, 2, 1>
# (configs[3])
HOT = {
    "_Z11qba_k_listsILi11ELi1ELi2ELi2ELi1ELi1EE": 64,
    "_Z17qba_k_lists_pbdefILi11ELi2ELi1EE": 64,
    "_Z15qba_k_lists_defILi11ELi2ELi2ELi1EE": None,
    "_Z13qba_k_batchedILi7ELi2ELi2ELi1EE": 64,
}


@pytest.fixture(scope="module")
def kds():
    if not LIB.exists():
        pytest.skip("libqba.so not built")
    return kernel_descriptors(LIB)


def _find(kds, prefix):
    hits = [v for k, v in kds.items() if k.startswith(prefix)]
    assert len(hits) == 1, (prefix, len(hits))
    return hits[0]


@pytest.mark.parametrize("prefix", sorted(HOT))
def test_hot_kernels_use_no_scratch(kds, prefix):
    assert _find(kds, prefix)["scratch"] == 0


@pytest.mark.parametrize("prefix", sorted(p for p, v in HOT.items() if v))
def test_eight_wave_kernels_fit_64_vgprs(kds, prefix):
    assert _find(kds, prefix)["vgprs"] <= HOT[prefix]


def test_descriptor_reader_sees_every_list_kernel(kds):
    # one closed-form fused kernel per n = 1..11 at least: the reader walks
    # every per-n code object of the library
    for n in range(1, 12):
        assert any(k.startswith(f"_Z11qba_k_listsILi{n}ELi1ELi2E") for k in kds), n
