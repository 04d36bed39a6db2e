# qba_stub.py -- drop next to tfg.py: the reference's hot path on an MI355X
# through libqba's C ABI (include/qba.h) with nothing but ctypes and torch
# (device buffers).  INTEGRATION.md embeds this file; tests/test_integration.py
# runs it against the oracle.
import ctypes as C
import os

import numpy as np
import torch

LIB = os.environ.get("QBA_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                             "tfg---quantum-byzantine-agreement_amd", "_build", "libqba.so"))
lib = C.CDLL(LIB)
lib.qba_last_error.restype = C.c_char_p
ctx = C.c_void_p()
i32p = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
dev = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731


def _ok(rc):
    if rc != 0:
        raise RuntimeError(lib.qba_last_error().decode())


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def init(device=0):
    torch.cuda.set_device(device)
    _ok(lib.qba_init(device, C.byref(ctx)))


def _triples(ops):  # [(gate, target, control|-1)] as tfg.py adds them -> int32 {kind, t, c}
    return np.ascontiguousarray([(0 if g == "H" else 1, t, c) for g, t, c in ops], np.int32).reshape(-1, 3)


def compile_resource(nParties, nQubits):
    """tfg.py:15-65 once per run: the gate lists of notQCorrelated and
    qCorrelated (pi = identity; the engine redraws pi per entry), exactly as
    tfg.py builds them, compiled into the sampler's program.  Call before
    generacionListas."""
    total = (nParties + 1) * nQubits
    notq = [("H", q, -1) for q in range(nQubits, total)] + [("X", j, nQubits + j) for j in range(nQubits)]
    q = [("H", j, -1) for j in range(nQubits)]
    for g in range(1, nParties + 1):
        q += [("X", g * nQubits + j, -1) for j, b in enumerate(format(g, f"0{nQubits}b")) if b == "1"]
    q += [("X", t, t % nQubits) for t in range(nQubits, total)]
    g0, g1 = _triples(notq), _triples(q)
    perm = np.arange(1, nParties + 1, dtype=np.int32)
    _ok(lib.qba_resource_compile(ctx, nParties, 0, i32p(g0), len(g0), None))
    _ok(lib.qba_resource_compile(ctx, nParties, 1, i32p(g1), len(g1), i32p(perm)))


def generacionListas(nParties, size, nQubits, w, seed=0):
    """tfg.py:68-84: rawS as the reference returns it -- int64 (n+1, nQubits*size),
    one measured bit per element, MSB first -- so rank 0's Isend of rawS[i]
    (tfg.py:142-145) and the receivers' buffers stay byte-identical."""
    ld = (size + 4095) // 4096 * 4096
    lists = torch.empty((nParties + 1, ld), dtype=torch.uint8, device="cuda")
    _ok(lib.qba_sample(ctx, nParties, C.c_uint64(seed), C.c_uint64(0), C.c_uint64(size), dev(lists),
                       C.c_uint64(ld), stream()))
    raw = torch.empty((nParties + 1, nQubits * size), dtype=torch.int64, device="cuda")
    for g in range(nParties + 1):
        _ok(lib.qba_values_to_bits(ctx, dev(lists[g]), C.c_uint64(size), nQubits, dev(raw[g]), stream()))
    return raw.cpu().numpy()


def measure_to_ints(raw, sizeL, nQubits):
    """tfg.py:128-129 on the device; returns the DEVICE list (uint8) that
    own_tuple / check_packet read -- print it with .tolist()."""
    bits = torch.as_tensor(np.ascontiguousarray(raw, np.int64), device="cuda")
    out = torch.empty(sizeL, dtype=torch.uint8, device="cuda")
    _ok(lib.qba_bits_to_values(ctx, dev(bits), C.c_uint64(sizeL), nQubits, dev(out), stream()))
    return out


def add_own_and_check(Li_dev, P, v, L, w):
    """tfg.py:189-192 / 291-294: L.add(tuple(Li[j] for j in P)); consistent(v, L, w)
    -- the gather and Cond2/Cond3 in ONE launch (qba_check_packet); Cond1 and
    the set stay in Python.  Returns consistent(...)."""
    order = np.fromiter(P, np.int64, len(P))  # this process's set-iteration order
    rows = [t for t in L if len(t) == len(order)]
    same = len(rows) == len(L)
    m, ln = (len(rows) if same else 0), len(order)
    stage = torch.as_tensor(np.concatenate([order] + ([np.asarray(rows, np.int64).ravel()] if m and ln else [])),
                            device="cuda") if ln else torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.empty(ln + 3 + m, dtype=torch.int64, device="cuda")
    _ok(lib.qba_check_packet(ctx, dev(Li_dev), C.c_uint64(Li_dev.numel()), dev(stage), C.c_int64(m),
                             C.c_int64(ln), C.c_int64(int(v)), C.c_int64(w), dev(out), stream()))
    o = out.cpu().numpy()
    if o[ln]:
        raise IndexError("P holds an index outside the list")
    eq = o[ln + 3:]
    ok = (not o[ln + 1] and not o[ln + 2] and bool(np.all((eq == 0) | (eq == ln)))) or (m > 0 and ln == 0)
    L.add(tuple(o[:ln].tolist()))
    return bool(ok and same)
