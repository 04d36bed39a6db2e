"""Dense numpy statevector for the reference's gate lists.

TEST INFRASTRUCTURE ONLY (see oracle/tfg_oracle.py header).

Convention (same as the product engine): qubit 0 is the most significant bit
of the basis index, so for the reference's layout (group g owns qubits
g*nQ .. g*nQ+nQ-1, MSB first, tfg.py:34,49-50,81-82) a basis index is the
base-w concatenation L0 L1 ... Ln of the measured values.

Gates are (name, target, control) with control = -1 for none; "X" with a
control is the reference's ``add_operation("X", targets=t, controls=c)``
(tfg.py:21, 39).  Amplitudes stay real for H/X/CX, so the state is float64.
"""
from __future__ import annotations

from typing import Iterable, Sequence, Tuple

import numpy as np

INV_SQRT2 = 1.0 / np.sqrt(2.0)


def run(gates: Iterable[Tuple[str, int, int]], nqubits: int) -> np.ndarray:
    psi = np.zeros(2 ** nqubits, np.float64)
    psi[0] = 1.0
    t = psi.reshape((2,) * nqubits)  # axis i == qubit i (MSB first)
    for name, tgt, ctl in gates:
        if name == "H":
            if ctl >= 0:
                raise ValueError("controlled H not used by the reference")
            a0 = np.take(t, 0, axis=tgt)
            a1 = np.take(t, 1, axis=tgt)
            t = np.stack([(a0 + a1) * INV_SQRT2, (a0 - a1) * INV_SQRT2], axis=tgt)
        elif name == "X":
            if ctl < 0:
                t = np.flip(t, axis=tgt)
            else:
                sl1 = [slice(None)] * nqubits
                sl1[ctl] = 1
                sub = t[tuple(sl1)]
                ax = tgt - (1 if tgt > ctl else 0)
                t = t.copy()
                t[tuple(sl1)] = np.flip(sub, axis=ax)
        else:
            raise ValueError(f"gate {name} not in the reference's gate set")
    return np.ascontiguousarray(t).reshape(-1)


def probabilities(psi: np.ndarray) -> np.ndarray:
    return psi * psi


def support(probs: np.ndarray, eps: float = 0.0):
    idx = np.nonzero(probs > eps)[0]
    return idx.astype(np.int64), probs[idx]


def register_gates(gates: Sequence[Tuple[str, int, int]], qubits: Sequence[int]):
    """Restrict a gate list to a qubit subset, renumbered 0..len-1 in ascending order."""
    pos = {q: i for i, q in enumerate(sorted(qubits))}
    out = []
    for name, tgt, ctl in gates:
        if tgt in pos and (ctl < 0 or ctl in pos):
            out.append((name, pos[tgt], pos[ctl] if ctl >= 0 else -1))
        elif tgt in pos or ctl in pos:
            raise ValueError("gate straddles the register boundary")
    return out
