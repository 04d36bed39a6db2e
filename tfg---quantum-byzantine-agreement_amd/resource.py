"""Resource-state preparation: the reference's circuits as gate lists.

tfg.py builds its two circuits through qsimov's ``QGate``/``QCircuit``
(tfg.py:15-65).  :class:`Gate` and :class:`Circuit` record the same
``add_operation`` calls (the qsimov-API subset the reference uses), and
:func:`notQCorrelated` / :func:`qCorrelated` / :func:`genQCorrCircuit` /
:func:`genNQCorrCircuit` produce the same operation lists.  The gate lists are
then executed by the engine's fp64 statevector kernels
(:meth:`Engine.prepare`), never by a CPU simulator.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from ._lib import GATE_H, GATE_X


def n_qubits(n_parties: int) -> int:
    """ceil(log2(nParties+1)), computed exactly (tfg.py:317)."""
    if n_parties < 1:
        raise ValueError("at least one party is required")
    return int(n_parties).bit_length()


class Gate:
    """Recorder for the qsimov ``QGate`` calls of tfg.py:17-21, 27-39."""

    def __init__(self, size: int, ancilla: int = 0, name: str = ""):
        self.size, self.ancilla, self.name = size, ancilla, name
        self.ops: List[tuple] = []
        self.perm: Optional[np.ndarray] = None

    def add_operation(self, gate, targets=None, controls=None, outputs=None):
        if isinstance(gate, Gate):  # a composite gate added to a circuit
            self.ops.extend(gate.ops)
            if gate.perm is not None:
                self.perm = gate.perm
            return
        if gate == "MEASURE":
            self.ops.append(("MEASURE", int(targets), int(outputs)))
            return
        if gate not in ("H", "X"):
            raise ValueError(f"gate {gate!r} is outside the reference's gate set")
        ctl = -1 if controls is None else int(controls)
        self.ops.append((gate, int(targets), ctl))

    def triples(self) -> np.ndarray:
        """(m, 3) int32 {kind, target, control} for libqba (MEASUREs dropped)."""
        rows = [(GATE_H if g == "H" else GATE_X, t, c) for g, t, c in self.ops if g != "MEASURE"]
        return np.asarray(rows, dtype=np.int32).reshape(-1, 3)


class Circuit(Gate):
    """Recorder for qsimov ``QCircuit`` (tfg.py:46, 59)."""

    def __init__(self, size: int, csize: int = 0, name: str = ""):
        super().__init__(size, 0, name)
        self.csize = csize


def notQCorrelated(nParties: int, nQubits: int) -> Gate:
    """Groups 1..n in |+>, group 0 a CNOT copy of group 1 (tfg.py:15-22)."""
    total = (nParties + 1) * nQubits
    gate = Gate(total, 0, "not Q-Correlated")
    for q in range(nQubits, total):
        gate.add_operation("H", targets=q)
    for j in range(nQubits):
        gate.add_operation("X", targets=j, controls=nQubits + j)
    return gate


def qCorrelated(nParties: int, nQubits: int, rng=None, perm: Optional[Sequence[int]] = None) -> Gate:
    """GHZ-type resource with a random relabelling pi of 1..n (tfg.py:25-40).

    ``rng`` plays np.random's role in tfg.py:30-31 (one ``shuffle`` of
    arange(1, n+1)); ``perm`` fixes pi instead.  The drawn pi is kept on
    ``gate.perm`` (perm[g-1] = pi(g)).
    """
    total = (nParties + 1) * nQubits
    gate = Gate(total, 0, "Q-Correlated")
    for q in range(nQubits):
        gate.add_operation("H", targets=q)
    if perm is None:
        values = np.arange(1, nParties + 1)
        (rng if rng is not None else np.random).shuffle(values)
    else:
        values = np.asarray(perm, dtype=np.int64)
    gate.perm = np.asarray(values, dtype=np.int64).copy()
    for g, val in enumerate(values, start=1):
        for j, bit in enumerate(format(int(val), f"0{nQubits}b")):  # MSB first
            if bit == "1":
                gate.add_operation("X", targets=g * nQubits + j)
    for q in range(nQubits, total):
        gate.add_operation("X", targets=q, controls=q % nQubits)
    return gate


def _measured(gate: Gate, name: str) -> Circuit:
    circ = Circuit(gate.size, gate.size, name)
    circ.add_operation(gate)
    for q in range(gate.size):
        circ.add_operation("MEASURE", targets=q, outputs=q)
    return circ


def genQCorrCircuit(nParties: int, nQubits: int, rng=None, perm=None) -> Circuit:
    """qCorrelated + MEASURE on every qubit (tfg.py:43-52)."""
    return _measured(qCorrelated(nParties, nQubits, rng, perm), "Q-Correlated Circuit")


def genNQCorrCircuit(nParties: int, nQubits: int) -> Circuit:
    """notQCorrelated + MEASURE on every qubit (tfg.py:56-65)."""
    return _measured(notQCorrelated(nParties, nQubits), "Not Q-Correlated Circuit")
