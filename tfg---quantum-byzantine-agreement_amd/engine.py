"""Device engine: torch-tensor front end of libqba (include/qba.h).

PyTorch is used only for device memory, streams and torch.distributed; every
computation on lists, counts and statevectors runs in the HIP kernels of
libqba.  Constructing an :class:`Engine` without the library or without a
gfx950 GPU raises :class:`QbaError` -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch

from . import resource
from ._lib import KIND_NOTQ, KIND_Q, MAX_PARTIES, QbaError, call, lib


def _ptr(t: torch.Tensor) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


def _i32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


@dataclass
class Counts:
    """Count-mode result of one pass (see qba.h): int64 device tensors."""

    H: torch.Tensor  # [w][n+1][w]
    C: torch.Tensor  # [w][n+1][n+1]
    P: torch.Tensor  # [w]

    def numpy(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        return self.H.cpu().numpy(), self.C.cpu().numpy(), self.P.cpu().numpy()


class Engine:
    """One libqba context bound to one GPU."""

    def __init__(self, device: int = 0):
        if not torch.cuda.is_available():
            raise QbaError("no GPU visible: the qba engine has no CPU fallback")
        self.device = torch.device("cuda", device)
        self.index = device
        handle = C.c_void_p()
        torch.cuda.set_device(device)
        call("qba_init", device, C.byref(handle))
        self._ctx = handle
        self._prepared: Dict[int, dict] = {}

    # -- lifetime ----------------------------------------------------------
    def close(self) -> None:
        if self._ctx:
            torch.cuda.synchronize(self.device)
            call("qba_destroy", self._ctx)
            self._ctx = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            if getattr(self, "_ctx", None):
                lib().qba_destroy(self._ctx)
        except Exception:
            pass

    @property
    def ctx(self) -> C.c_void_p:
        if not self._ctx:
            raise QbaError("engine closed")
        return self._ctx

    def stream(self) -> C.c_void_p:
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # -- sizes --------------------------------------------------------------
    @staticmethod
    def sizes(n: int) -> Tuple[int, int]:
        nq = resource.n_qubits(n)
        return nq, 1 << nq

    @staticmethod
    def _check_n(n: int) -> None:
        if not 1 <= n <= MAX_PARTIES:
            raise QbaError(f"n_parties={n} outside [1, {MAX_PARTIES}]")

    # -- (A1/A2) resource preparation ------------------------------------------
    def prepare(self, n: int, perm: Optional[Sequence[int]] = None) -> dict:
        """Compile both reference circuits for n parties (tfg.py:15-65).

        The Q circuit is built with permutation ``perm`` (default: identity);
        its X gates are verified by the library to be the classical mask the
        sampler redraws for every entry.
        """
        self._check_n(n)
        if n in self._prepared and perm is None:
            return self._prepared[n]
        nq, _ = self.sizes(n)
        notq = resource.notQCorrelated(n, nq)
        q = resource.qCorrelated(n, nq, perm=list(range(1, n + 1)) if perm is None else perm)
        return self.compile(n, notq, q)

    def compile(self, n: int, notq: "resource.Gate", q: "resource.Gate") -> dict:
        """Compile a (not-Q, Q) circuit pair for n parties and make it the
        program that sample / sample_check use for n.  ``q.perm`` is the
        permutation its X gates encode.  Returns the program info (tables and
        the sampler flags: canonical table layout, closed form)."""
        self._check_n(n)
        nq, _ = self.sizes(n)
        g0 = np.ascontiguousarray(notq.triples())
        g1 = np.ascontiguousarray(q.triples())
        p1 = np.ascontiguousarray(np.asarray(q.perm, dtype=np.int32))
        call("qba_resource_compile", self.ctx, n, KIND_NOTQ, _i32p(g0), len(g0), None)
        call("qba_resource_compile", self.ctx, n, KIND_Q, _i32p(g1), len(g1), _i32p(p1))
        flags = np.zeros(6, np.int32)
        call("qba_program_flags", self.ctx, n, _i32p(flags))
        info = {"n": n, "nq": nq, "notq": self.program(n, KIND_NOTQ), "q": self.program(n, KIND_Q),
                "canonical": bool(flags[0]), "closed": bool(flags[1])}
        self._prepared[n] = info
        return info

    def program(self, n: int, kind: int) -> dict:
        nf = C.c_int32()
        tl = C.c_int32()
        desc = np.zeros((16, 6), np.int32)
        cap = 8192
        pat = np.zeros(cap, np.uint64)
        apat = np.zeros(cap, np.uint64)
        thr = np.zeros(cap, np.uint64)
        u64p = C.POINTER(C.c_uint64)
        call("qba_program_export", self.ctx, n, kind, C.byref(nf), _i32p(desc),
             pat.ctypes.data_as(u64p), apat.ctypes.data_as(u64p), thr.ctypes.data_as(u64p), cap,
             C.byref(tl))
        t = tl.value
        return {"nfac": nf.value, "desc": desc[: nf.value].copy(), "pat": pat[:t].copy(),
                "apat": apat[:t].copy(), "thr": thr[:t].copy()}

    # -- buffers -----------------------------------------------------------------
    def alloc_lists(self, n: int, count: int) -> torch.Tensor:
        # rows start 4 KiB-aligned: the 8-B-per-lane row stores then never
        # straddle a partial line at a row start (1.3% over 64-B alignment at
        # n = 11, measured in round 2)
        ld = max(4096, (count + 4095) // 4096 * 4096)
        return torch.empty((n + 1, ld), dtype=torch.uint8, device=self.device)

    def alloc_packed(self, n: int, count: int) -> torch.Tensor:
        """Nibble rows (qba.h "packed lists"): (count + 1) // 2 bytes per row,
        rows 4 KiB-aligned like alloc_lists."""
        nb = (count + 1) // 2
        ld = max(4096, (nb + 4095) // 4096 * 4096)
        return torch.empty((n + 1, ld), dtype=torch.uint8, device=self.device)

    def alloc_counts(self, n: int) -> Counts:
        _, w = self.sizes(n)
        z = lambda *s: torch.zeros(s, dtype=torch.int64, device=self.device)  # noqa: E731
        return Counts(z(w, n + 1, w), z(w, n + 1, n + 1), z(w))

    @staticmethod
    def _lists_ok(lists: torch.Tensor, n: int, count: int) -> int:
        if lists.dtype != torch.uint8 or lists.dim() != 2 or lists.shape[0] != n + 1:
            raise QbaError("lists must be a uint8 [n+1, ld] device tensor")
        if lists.stride(1) != 1 or lists.shape[1] < count:
            raise QbaError("lists rows must be contiguous and hold `count` entries")
        return lists.stride(0)

    @staticmethod
    def _packed_ok(packed: torch.Tensor, rows: int, count: int) -> int:
        if packed.dtype != torch.uint8 or packed.dim() != 2 or packed.shape[0] != rows:
            raise QbaError(f"packed lists must be a uint8 [{rows}, ld] device tensor")
        if packed.stride(1) != 1 or packed.shape[1] < (count + 1) // 2:
            raise QbaError("packed rows must be contiguous and hold (count + 1) // 2 bytes")
        return packed.stride(0)

    # -- (A3/A4) sampling ---------------------------------------------------------
    def sample(self, n: int, seed: int, first: int, count: int,
               lists: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Lists of entries [first, first+count) (tfg.py:68-84, 128-129)."""
        self.prepare(n)
        if lists is None:
            lists = self.alloc_lists(n, count)
        ld = self._lists_ok(lists, n, count)
        call("qba_sample", self.ctx, n, seed, first, count, _ptr(lists), ld, self.stream())
        return lists

    def sample_check(self, n: int, seed: int, first: int, count: int,
                     lists: Optional[torch.Tensor] = None, counts: Optional[Counts] = None,
                     accumulate: bool = False, deferred: bool = False) -> Tuple[torch.Tensor, Counts]:
        """deferred: qba_sample_check_deferred -- the counts are complete only
        after the next deferred call or flush_deferred() (include/qba.h)."""
        self.prepare(n)
        if lists is None:
            lists = self.alloc_lists(n, count)
        if counts is None:
            counts = self.alloc_counts(n)
        ld = self._lists_ok(lists, n, count)
        call("qba_sample_check_deferred" if deferred else "qba_sample_check", self.ctx, n, seed, first, count,
             _ptr(lists), ld, _ptr(counts.H), _ptr(counts.C), _ptr(counts.P), int(accumulate), self.stream())
        return lists, counts

    def flush_deferred(self) -> None:
        """Launch the pending deferred reduction (on its call's stream)."""
        call("qba_flush_deferred", self.ctx)

    def sample_packed(self, n: int, seed: int, first: int, count: int,
                      packed: Optional[torch.Tensor] = None) -> torch.Tensor:
        """sample() into nibble rows."""
        self.prepare(n)
        if packed is None:
            packed = self.alloc_packed(n, count)
        ld = self._packed_ok(packed, n + 1, count)
        call("qba_sample_packed", self.ctx, n, seed, first, count, _ptr(packed), ld, self.stream())
        return packed

    def sample_check_packed(self, n: int, seed: int, first: int, count: int,
                            packed: Optional[torch.Tensor] = None, counts: Optional[Counts] = None,
                            accumulate: bool = False, deferred: bool = False) -> Tuple[torch.Tensor, Counts]:
        """The fused hot path writing nibble rows (half the bytes of
        sample_check; same lists and counts).  deferred: as sample_check."""
        self.prepare(n)
        if packed is None:
            packed = self.alloc_packed(n, count)
        if counts is None:
            counts = self.alloc_counts(n)
        ld = self._packed_ok(packed, n + 1, count)
        call("qba_sample_check_packed_deferred" if deferred else "qba_sample_check_packed", self.ctx, n, seed,
             first, count, _ptr(packed), ld, _ptr(counts.H), _ptr(counts.C), _ptr(counts.P), int(accumulate),
             self.stream())
        return packed, counts

    def sample_check_batched(self, n: int, seed_base: int, n_inst: int, count: int,
                             lists: Optional[torch.Tensor] = None,
                             packed: bool = False) -> Tuple[torch.Tensor, Counts]:
        """n_inst independent runs (key seed_base + i) of `count` entries each.
        Returns lists [n_inst, n+1, ld] (nibble rows when packed) and
        per-instance counts [n_inst, ...]."""
        self.prepare(n)
        _, w = self.sizes(n)
        # rows start 4 KiB-aligned: the 8-B-per-lane row stores then never
        # straddle a partial line at a row start (1.3% over 64-B alignment at
        # n = 11, measured in round 2)
        nb = (count + 1) // 2 if packed else count
        ld = max(4096, (nb + 4095) // 4096 * 4096)
        if lists is None:
            lists = torch.empty((n_inst, n + 1, ld), dtype=torch.uint8, device=self.device)
        if lists.dim() != 3 or lists.shape[:2] != (n_inst, n + 1) or lists.stride(2) != 1:
            raise QbaError("lists must be a uint8 [n_inst, n+1, ld] tensor")
        z = lambda *s: torch.empty(s, dtype=torch.int64, device=self.device)  # noqa: E731
        counts = Counts(z(n_inst, w, n + 1, w), z(n_inst, w, n + 1, n + 1), z(n_inst, w))
        if lists.shape[2] < nb:
            raise QbaError("lists rows too short for `count` entries")
        call("qba_sample_check_batched_packed" if packed else "qba_sample_check_batched", self.ctx, n,
             seed_base, n_inst, count, _ptr(lists),
             lists.stride(1), lists.stride(0), _ptr(counts.H), _ptr(counts.C), _ptr(counts.P),
             self.stream())
        return lists, counts

    # -- (A5-A8) count mode -------------------------------------------------------
    def check_counts(self, lists: torch.Tensor, n: int, count: int,
                     counts: Optional[Counts] = None, accumulate: bool = False) -> Counts:
        self._check_n(n)
        if counts is None:
            counts = self.alloc_counts(n)
        ld = self._lists_ok(lists, n, count)
        call("qba_check_counts", self.ctx, n, _ptr(lists), count, ld, _ptr(counts.H),
             _ptr(counts.C), _ptr(counts.P), int(accumulate), self.stream())
        return counts

    def check_counts_packed(self, packed: torch.Tensor, n: int, count: int,
                            counts: Optional[Counts] = None, accumulate: bool = False) -> Counts:
        self._check_n(n)
        if counts is None:
            counts = self.alloc_counts(n)
        ld = self._packed_ok(packed, n + 1, count)
        call("qba_check_counts_packed", self.ctx, n, _ptr(packed), count, ld, _ptr(counts.H),
             _ptr(counts.C), _ptr(counts.P), int(accumulate), self.stream())
        return counts

    def pack(self, lists: torch.Tensor, rows: int, count: int,
             packed: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Byte rows -> nibble rows on the device; raises when a value > 15."""
        if lists.dtype != torch.uint8 or lists.dim() != 2 or lists.shape[0] < rows or \
                lists.stride(1) != 1 or lists.shape[1] < count:
            raise QbaError("lists must be a uint8 [>= rows, >= count] device tensor")
        if packed is None:
            nb = (count + 1) // 2
            packed = torch.empty((rows, max(4096, (nb + 4095) // 4096 * 4096)), dtype=torch.uint8,
                                 device=self.device)
        ldp = self._packed_ok(packed, rows, count)
        bad = torch.empty(1, dtype=torch.int64, device=self.device)
        call("qba_lists_pack", self.ctx, _ptr(lists), lists.stride(0), rows, count, _ptr(packed), ldp,
             _ptr(bad), self.stream())
        if int(bad.item()):
            raise QbaError(f"{int(bad.item())} values > 15 cannot be stored as nibbles")
        return packed

    def unpack(self, packed: torch.Tensor, rows: int, count: int,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Nibble rows -> byte rows [rows, ld] on the device."""
        ldp = self._packed_ok(packed, rows, count)
        if out is None:
            out = torch.empty((rows, max(4096, (count + 4095) // 4096 * 4096)), dtype=torch.uint8,
                              device=self.device)
        if out.dtype != torch.uint8 or out.dim() != 2 or out.shape[0] < rows or out.stride(1) != 1 or \
                out.shape[1] < count:
            raise QbaError("out must be a uint8 [>= rows, >= count] device tensor")
        call("qba_lists_unpack", self.ctx, _ptr(packed), ldp, rows, count, _ptr(out), out.stride(0),
             self.stream())
        return out

    def count_tables(self, n: int, sizeL: int, seed: int = 0, lists: Optional[np.ndarray] = None,
                     chunk: int = 1 << 27, first: int = 0, device_out: bool = False):
        """Flat int64 [H | C | P] over entries [first, first + sizeL): injected
        host lists (shape (n+1, sizeL)) are checked on the device, otherwise
        entries are sampled and checked in chunks of `chunk` (lists are written
        once to a reused buffer).  device_out returns the device tensor (for a
        collective) instead of a host copy."""
        self._check_n(n)
        _, w = self.sizes(n)
        g = n + 1
        h, c = w * g * w, w * g * g
        flat = torch.zeros(h + c + w, dtype=torch.int64, device=self.device)
        counts = Counts(flat[:h].view(w, g, w), flat[h:h + c].view(w, g, g), flat[h + c:])
        if lists is not None:
            arr = np.ascontiguousarray(lists, dtype=np.uint8)
            if arr.shape != (g, sizeL):
                raise QbaError(f"lists must have shape {(g, sizeL)}")
            dev = self.alloc_lists(n, sizeL)
            dev[:, :sizeL] = torch.from_numpy(arr).to(self.device)
            self.check_counts(dev, n, sizeL, counts)
        else:
            # the lists are sampled, counted and dropped: nibble rows (half the
            # bytes written)
            chunk = max(8, chunk & ~7)
            buf = self.alloc_packed(n, min(chunk, max(sizeL, 1)))
            for off in range(0, sizeL, chunk):
                self.sample_check_packed(n, seed, first + off, min(chunk, sizeL - off), buf, counts,
                                         accumulate=off > 0)
        if sizeL and self.last_stats()[0] != 0:
            raise QbaError("lists hold values >= w at Q-correlated positions: count mode "
                           "cannot evaluate them (the reference never produces such lists)")
        return flat if device_out else flat.cpu().numpy()

    def last_stats(self) -> np.ndarray:
        out = np.zeros(2, np.int64)
        call("qba_last_stats", self.ctx, out.ctypes.data_as(C.POINTER(C.c_int64)))
        return out

    def reserve(self, n: int, max_blocks: int) -> None:
        call("qba_reserve", self.ctx, n, max_blocks)

    # -- (A5-A8) exact-order mode -----------------------------------------------
    def to_device(self, arr) -> torch.Tensor:
        return torch.as_tensor(np.ascontiguousarray(arr)).to(self.device, non_blocking=False)

    @staticmethod
    def to_host(t: torch.Tensor) -> np.ndarray:
        return t.cpu().numpy()

    def isq_indices(self, li: torch.Tensor, lc: torch.Tensor) -> np.ndarray:
        """Ascending {k : Li[k] != Lc[k]} (tfg.py:327)."""
        count = li.numel()
        out = np.empty(max(count, 1), np.int64)
        found = C.c_int64()
        call("qba_isq_indices_host", self.ctx, _ptr(li), _ptr(lc), count, out.ctypes.data, count,
             C.byref(found), self.stream())
        return out[: found.value]

    def select_eq(self, order: np.ndarray, lc: torch.Tensor, v: int) -> np.ndarray:
        """[x for x in order if Lc[x] == v], order kept (tfg.py:182)."""
        m = len(order)
        if m == 0:
            return np.zeros(0, np.int64)
        h_order = np.ascontiguousarray(order, dtype=np.int64)
        out = np.empty(m, np.int64)
        found = C.c_int64()
        call("qba_select_eq_host", self.ctx, h_order.ctypes.data, m, _ptr(lc), lc.numel(), int(v),
             out.ctypes.data, C.byref(found), self.stream())
        return out[: found.value]

    def gather(self, li: torch.Tensor, order: np.ndarray) -> np.ndarray:
        """Li[j] for j in order (tfg.py:189, 291)."""
        m = len(order)
        if m == 0:
            return np.zeros(0, np.int64)
        d_idx = self.to_device(np.asarray(order, dtype=np.int64))
        out = torch.empty(m, dtype=torch.int64, device=self.device)
        call("qba_gather", self.ctx, _ptr(li), li.numel(), _ptr(d_idx), m, _ptr(out), self.stream())
        return out.cpu().numpy()

    def check_packet(self, li: torch.Tensor, order: np.ndarray, rows: Sequence[Sequence[int]], v: int,
                     w: int) -> Tuple[tuple, bool]:
        """One packet of the exact-order protocol (tfg.py:189-192, 291-294):
        own = tuple(Li[j] for j in order) and Cond2/Cond3 of
        consistent(v, rows | {own}, w), in one launch and one host sync
        (qba_check_packet_host).  All rows must have len(order) entries
        (Cond1 stays with the caller)."""
        ln, m = len(order), len(rows)
        stage = np.empty(ln * (m + 1), np.int64)
        stage[:ln] = order
        if m and ln:
            for a, t in enumerate(rows):
                stage[ln * (a + 1):ln * (a + 2)] = t if isinstance(t, np.ndarray) else \
                    np.fromiter(t, dtype=np.int64, count=ln)
        o = np.empty(ln + 3 + m, np.int64)
        call("qba_check_packet_host", self.ctx, _ptr(li), li.numel(), stage.ctypes.data, m, ln, int(v), int(w),
             o.ctypes.data, self.stream())
        if o[ln]:
            raise QbaError("qba_check_packet: index outside the list")
        eq = o[ln + 3:]
        ok = not o[ln + 1] and not o[ln + 2] and bool(np.all((eq == 0) | (eq == ln)))
        if m and not ln:  # every tuple empty: the set is {()}, vacuously consistent
            ok = True
        return tuple(o[:ln].tolist()), ok

    def check_packets(self, li: torch.Tensor, reqs: Sequence[Tuple[np.ndarray, Sequence, int]],
                      w: int) -> list:
        """A round's packets (tfg.py:337-348 -> 289-294) in one device round
        trip (qba_check_packets_host): reqs = [(order, rows, v)], each as
        :meth:`check_packet`; returns [(own, ok, own_wire)] in the same order
        (own_wire: the own tuple as the int64 array it travels as)."""
        if not reqs:
            return []
        dims = [(len(o), len(r)) for o, r, _ in reqs]
        nin = sum(ln * (m + 1) for ln, m in dims)
        stage = np.empty(max(nin, 1), np.int64)
        desc = np.empty(3 * len(reqs), np.int64)
        off = 0
        for i, ((order, rows, v), (ln, m)) in enumerate(zip(reqs, dims)):
            desc[3 * i:3 * i + 3] = (m, ln, int(v))
            stage[off:off + ln] = order
            for a, t in enumerate(rows):
                stage[off + ln * (a + 1):off + ln * (a + 2)] = t if isinstance(t, np.ndarray) else \
                    np.fromiter(t, dtype=np.int64, count=ln)
            off += ln * (m + 1)
        out = np.empty(sum(ln + 3 + m for ln, m in dims), np.int64)
        call("qba_check_packets_host", self.ctx, _ptr(li), li.numel(), stage.ctypes.data, desc.ctypes.data,
             len(reqs), int(w), out.ctypes.data, self.stream())
        res, o = [], 0
        for ln, m in dims:
            if out[o + ln]:
                raise QbaError("qba_check_packets_host: index outside the list")
            eq = out[o + ln + 3:o + ln + 3 + m]
            ok = not out[o + ln + 1] and not out[o + ln + 2] and bool(np.all((eq == 0) | (eq == ln)))
            if m and not ln:  # every tuple empty: the set is {()}, vacuously consistent
                ok = True
            own = out[o:o + ln]
            res.append((tuple(own.tolist()), ok, own))
            o += ln + 3 + m
        return res

    def check_gather(self, lists: torch.Tensor, count: int, idx: np.ndarray, party: Sequence[int], v: int,
                     w: int) -> bool:
        """consistent(v, L, w) (tfg.py:87-98) over the tuples
        L = {tuple(lists[party[a]][j] for j in idx[a])}, gathered and checked on
        the device (qba_check_gather; identical tuples collapse as in the
        reference's set).  idx: int64 [m, len]."""
        idx_d = torch.as_tensor(np.ascontiguousarray(idx, dtype=np.int64), device=self.device)
        m = idx_d.shape[0]
        ln = idx_d.shape[1] if idx_d.dim() == 2 else 0
        party_d = torch.as_tensor(np.asarray(party, dtype=np.int32), device=self.device)
        ok = torch.empty(1, dtype=torch.int32, device=self.device)
        call("qba_check_gather", self.ctx, _ptr(lists), lists.stride(0), lists.shape[0], count, _ptr(idx_d),
             _ptr(party_d), m, ln, int(v), int(w), _ptr(ok), self.stream())
        r = int(ok.item())
        if r < 0:
            raise QbaError("qba_check_gather: index or party outside the lists")
        return bool(r)

    def lists_to_bits(self, lists: torch.Tensor, rows: int, count: int, nq: int) -> np.ndarray:
        """rawS (tfg.py:81-84): rows [0, rows) encoded, host int64 [rows, count*nq]."""
        out = np.empty((rows, count * nq), np.int64)
        call("qba_lists_to_bits_host", self.ctx, _ptr(lists), lists.stride(0), rows, count, nq,
             out.ctypes.data, self.stream())
        return out

    def bits_to_values_host(self, raw: np.ndarray, count: int, nq: int) -> torch.Tensor:
        """measure_to_ints (tfg.py:158, 161) of a received host buffer -> device list."""
        raw = np.ascontiguousarray(raw, dtype=np.int64)
        out = torch.empty(max(count, 1), dtype=torch.uint8, device=self.device)
        call("qba_bits_to_values_host", self.ctx, raw.ctypes.data, count, nq, _ptr(out), self.stream())
        return out[:count]

    def allreduce_i64(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the RCCL communicator of rccl_init (qba_allreduce_i64)."""
        if t.dtype != torch.int64 or not t.is_contiguous() or t.device != self.device:
            raise QbaError("allreduce_i64 needs a contiguous int64 tensor on this engine's device")
        call("qba_allreduce_i64", self.ctx, _ptr(t), t.numel(), self.stream())
        return t

    @staticmethod
    def rccl_unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        call("qba_rccl_unique_id", buf)
        return bytes(buf)

    def rccl_init(self, uid: bytes, nranks: int, rank: int) -> None:
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        call("qba_rccl_init", self.ctx, buf, nranks, rank)

    def consistent_rows(self, rows: np.ndarray, v: int, w: int) -> bool:
        """Cond2 and Cond3 of tfg.py:93-98 over an (m, len) int64 matrix."""
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        m, ln = rows.shape
        d = self.to_device(rows) if ln > 0 else torch.zeros(1, dtype=torch.int64, device=self.device)
        ok = C.c_int32()
        call("qba_consistent", self.ctx, _ptr(d), m, ln, int(v), int(w), C.byref(ok), self.stream())
        return bool(ok.value)

    # -- codec (rawS wire layout) ----------------------------------------------
    def bits_to_values(self, raw: torch.Tensor, count: int, nq: int) -> torch.Tensor:
        out = torch.empty(max(count, 1), dtype=torch.uint8, device=self.device)
        call("qba_bits_to_values", self.ctx, _ptr(raw), count, nq, _ptr(out), self.stream())
        return out[:count]

    def values_to_bits(self, values: torch.Tensor, count: int, nq: int) -> torch.Tensor:
        out = torch.empty(max(count * nq, 1), dtype=torch.int64, device=self.device)
        call("qba_values_to_bits", self.ctx, _ptr(values), count, nq, _ptr(out), self.stream())
        return out[: count * nq]

    # -- statevector -------------------------------------------------------------
    def statevector(self, nqubits: int, gates: np.ndarray,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
        sv = out if out is not None else torch.empty(1 << nqubits, dtype=torch.float64, device=self.device)
        g = np.ascontiguousarray(gates, dtype=np.int32).reshape(-1, 3)
        call("qba_sv_prepare", self.ctx, _ptr(sv), nqubits, _i32p(g), len(g), self.stream())
        return sv

    def statevector_unfused(self, nqubits: int, gates: np.ndarray,
                            out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """qba_sv_init + qba_sv_apply: no folding of the single-qubit layer into
        the init pass (the H/X/CX run fusion of qba_sv_apply still applies)."""
        sv = out if out is not None else torch.empty(1 << nqubits, dtype=torch.float64, device=self.device)
        g = np.ascontiguousarray(gates, dtype=np.int32).reshape(-1, 3)
        call("qba_sv_init", self.ctx, _ptr(sv), nqubits, self.stream())
        call("qba_sv_apply", self.ctx, _ptr(sv), nqubits, _i32p(g), len(g), self.stream())
        return sv

    def apply_gates(self, sv: torch.Tensor, nqubits: int, gates: np.ndarray) -> None:
        g = np.ascontiguousarray(gates, dtype=np.int32).reshape(-1, 3)
        call("qba_sv_apply", self.ctx, _ptr(sv), nqubits, _i32p(g), len(g), self.stream())

    def support(self, sv: torch.Tensor, nqubits: int, eps: float = 1e-24,
                cap: int = 1 << 20) -> Tuple[np.ndarray, np.ndarray]:
        idx = torch.empty(cap, dtype=torch.int64, device=self.device)
        prob = torch.empty(cap, dtype=torch.float64, device=self.device)
        cnt = C.c_int64()
        call("qba_sv_support", self.ctx, _ptr(sv), nqubits, float(eps), _ptr(idx), _ptr(prob), cap,
             C.byref(cnt), self.stream())
        k = min(cnt.value, cap)
        if cnt.value > cap:
            raise QbaError(f"support of {cnt.value} outcomes exceeds cap={cap}")
        return idx[:k].cpu().numpy(), prob[:k].cpu().numpy()

    # -- test helpers -------------------------------------------------------------
    def set_test_knobs(self, chunk: int = 0, pb_min: int = -1, list_grid: int = 0) -> "Engine":
        """qba_test_set_knobs: launch-shape knobs for the GPU tests (0 / -1 / 0
        = the shipped selection).  Results never change, only which kernel
        path computes them."""
        call("qba_test_set_knobs", self.ctx, chunk, pb_min, list_grid)
        return self

    def philox(self, ctr: np.ndarray, key: int) -> np.ndarray:
        ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
        d_ctr = self.to_device(ctr.view(np.int32))
        out = torch.empty_like(d_ctr)
        call("qba_philox_dev", self.ctx, _ptr(d_ctr), len(ctr), int(key), _ptr(out), self.stream())
        return out.cpu().numpy().view(np.uint32)


def unpack_nibbles(packed: np.ndarray, count: int) -> np.ndarray:
    """Host view of nibble rows [rows, >= (count+1)//2] as byte rows [rows, count]."""
    p = np.asarray(packed, dtype=np.uint8)
    out = np.empty((p.shape[0], 2 * ((count + 1) // 2)), dtype=np.uint8)
    out[:, 0::2] = p[:, :(count + 1) // 2] & 15
    out[:, 1::2] = p[:, :(count + 1) // 2] >> 4
    return out[:, :count]


def alias_build(probs: Sequence[float]) -> Tuple[np.ndarray, np.ndarray]:
    """Host Vose alias table (exported for tests): (thr u64 in [0, 2^32], alias i32)."""
    p = np.ascontiguousarray(probs, dtype=np.float64)
    thr = np.zeros(len(p), np.uint64)
    alias = np.zeros(len(p), np.int32)
    call("qba_alias_build", p.ctypes.data_as(C.POINTER(C.c_double)), len(p),
         thr.ctypes.data_as(C.POINTER(C.c_uint64)), alias.ctypes.data_as(C.POINTER(C.c_int32)))
    return thr, alias
