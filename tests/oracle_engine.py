"""A numpy stand-in for Engine's exact-mode methods, built on the oracle.

TEST INFRASTRUCTURE ONLY: lets the CPU suite exercise the protocol host's
logic (set hops, RNG order, rounds) without a GPU.  The product never uses it;
the GPU suite runs the same tests with the real Engine.
"""
import numpy as np

import tfg_oracle as orc


class OracleEngine:
    def to_device(self, arr):
        return np.array(arr, copy=True)

    @staticmethod
    def to_host(arr):
        return np.asarray(arr)

    def values_to_bits(self, values, count, nq):
        return orc.lists_to_raw(np.asarray(values)[None, :count], nq)[0]

    def bits_to_values(self, raw, count, nq):
        return np.asarray(orc.measure_to_ints(np.asarray(raw), count, nq), dtype=np.uint8)

    def isq_indices(self, li, lc):
        return orc.is_qcorr_indices(li, lc)

    def select_eq(self, order, lc, v):
        return np.asarray(orc.p_filter(order, lc, v), dtype=np.int64)

    def gather(self, li, order):
        return np.asarray(orc.gather(li, order), dtype=np.int64)

    def consistent_rows(self, rows, v, w):
        return orc.consistent(v, {tuple(r) for r in rows.tolist()}, w) if len(rows) else True

    def count_tables(self, n, sizeL, seed=0, lists=None, chunk=None, first=0, device_out=False):
        if lists is None:  # sampled: the C twin's closed-form schedule (n <= 11)
            import oracle_lib
            dummy = {"nfac": 0, "desc": np.zeros((0, 6), np.int32), "pat": np.zeros(1, np.uint64),
                     "apat": np.zeros(1, np.uint64), "thr": np.zeros(1, np.uint64)}
            H, C, P, bad = oracle_lib.stream_counts(n, seed, first, sizeL, dummy, dummy, closed=True)
        else:
            H, C, P = orc.counts(np.asarray(lists), n)
        return np.concatenate([H.ravel(), C.ravel(), P.ravel()])
