"""ctypes binding of libqba.so (include/qba.h).

The library is built in-tree (``csrc/Makefile`` -> ``_build/libqba.so``) by
``__graft_entry__.build()``.  There is no CPU fallback: if the library or a
gfx950 device is missing, :func:`lib` / :class:`Context` raise
:class:`QbaError` immediately.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("QBA_LIB", _HERE / "_build" / "libqba.so"))
# QBA_LIB naming a tools/exp/build.sh library (_build/exp/): an A/B build
EXPERIMENT_LIB = LIB_PATH.parent.name == "exp"

QBA_OK, QBA_EINVAL, QBA_EHIP, QBA_ENOMEM, QBA_EUNSUPPORTED, QBA_ESTATE = 0, -1, -2, -3, -4, -5
KIND_NOTQ, KIND_Q = 0, 1
GATE_H, GATE_X = 0, 1
MAX_PARTIES = 15

_i32, _i64, _u64, _f64 = C.c_int32, C.c_int64, C.c_uint64, C.c_double
_p = C.c_void_p
_pi32, _pi64, _pu64, _pf64 = C.POINTER(_i32), C.POINTER(_i64), C.POINTER(_u64), C.POINTER(_f64)

# name -> argtypes (restype is int unless listed in _RESTYPE)
SIGNATURES = {
    "qba_last_error": [],
    "qba_version": [],
    "qba_build_flags": [],
    "qba_init": [C.c_int, C.POINTER(_p)],
    "qba_destroy": [_p],
    "qba_reserve": [_p, C.c_int, _i64],
    "qba_sv_init": [_p, _p, C.c_int, _p],
    "qba_sv_apply": [_p, _p, C.c_int, _pi32, C.c_int, _p],
    "qba_sv_prepare": [_p, _p, C.c_int, _pi32, C.c_int, _p],
    "qba_sv_support": [_p, _p, C.c_int, _f64, _p, _p, _i64, _pi64, _p],
    "qba_resource_compile": [_p, C.c_int, C.c_int, _pi32, C.c_int, _pi32],
    "qba_program_export": [_p, C.c_int, C.c_int, _pi32, _pi32, _pu64, _pu64, _pu64, _i32, _pi32],
    "qba_program_flags": [_p, C.c_int, _pi32],
    "qba_perm_tables": [C.c_int, _p, _i32, _pi32],
    "qba_sample": [_p, C.c_int, _u64, _u64, _u64, _p, _u64, _p],
    "qba_check_counts": [_p, C.c_int, _p, _u64, _u64, _p, _p, _p, C.c_int, _p],
    "qba_last_stats": [_p, _pi64],
    "qba_sample_check": [_p, C.c_int, _u64, _u64, _u64, _p, _u64, _p, _p, _p, C.c_int, _p],
    "qba_sample_packed": [_p, C.c_int, _u64, _u64, _u64, _p, _u64, _p],
    "qba_sample_check_packed": [_p, C.c_int, _u64, _u64, _u64, _p, _u64, _p, _p, _p, C.c_int, _p],
    "qba_sample_check_deferred": [_p, C.c_int, _u64, _u64, _u64, _p, _u64, _p, _p, _p, C.c_int, _p],
    "qba_sample_check_packed_deferred": [_p, C.c_int, _u64, _u64, _u64, _p, _u64, _p, _p, _p, C.c_int, _p],
    "qba_flush_deferred": [_p],
    "qba_check_counts_packed": [_p, C.c_int, _p, _u64, _u64, _p, _p, _p, C.c_int, _p],
    "qba_lists_pack": [_p, _p, _u64, C.c_int, _u64, _p, _u64, _p, _p],
    "qba_lists_unpack": [_p, _p, _u64, C.c_int, _u64, _p, _u64, _p],
    "qba_sample_check_batched": [_p, C.c_int, _u64, _i64, _u64, _p, _u64, _u64, _p, _p, _p, _p],
    "qba_sample_check_batched_packed": [_p, C.c_int, _u64, _i64, _u64, _p, _u64, _u64, _p, _p, _p, _p],
    "qba_isq_indices": [_p, _p, _p, _u64, _p, _i64, _pi64, _p],
    "qba_select_eq": [_p, _p, _i64, _p, _u64, _i64, _p, _pi64, _p],
    "qba_isq_indices_host": [_p, _p, _p, _u64, _p, _i64, _pi64, _p],
    "qba_select_eq_host": [_p, _p, _i64, _p, _u64, _i64, _p, _pi64, _p],
    "qba_check_gather": [_p, _p, C.c_uint64, C.c_int, C.c_uint64, _p, _p, _i64, _i64, _i64, _i64, _p, _p],
    "qba_check_packet": [_p, _p, _u64, _p, _i64, _i64, _i64, _i64, _p, _p],
    "qba_check_packet_host": [_p, _p, _u64, _p, _i64, _i64, _i64, _i64, _p, _p],
    "qba_check_packets_host": [_p, _p, _u64, _p, _p, _i64, _i64, _p, _p],
    "qba_host_pyset_order": [_p, _i64, _p, _p],
    "qba_host_pytuple_hash": [_p, _i64, _p],
    "qba_lists_to_bits_host": [_p, _p, _u64, C.c_int, _u64, C.c_int, _p, _p],
    "qba_bits_to_values_host": [_p, _p, _u64, C.c_int, _p, _p],
    "qba_rccl_unique_id": [_p],
    "qba_rccl_init": [_p, _p, C.c_int, C.c_int],
    "qba_allreduce_i64": [_p, _p, _i64, _p],
    "qba_gather": [_p, _p, _u64, _p, _i64, _p, _p],
    "qba_consistent": [_p, _p, _i64, _i64, _i64, _i64, _pi32, _p],
    "qba_bits_to_values": [_p, _p, _u64, C.c_int, _p, _p],
    "qba_values_to_bits": [_p, _p, _u64, C.c_int, _p, _p],
    "qba_alias_build": [_pf64, _i32, _pu64, _pi32],
    "qba_philox_dev": [_p, _p, _i64, _u64, _p, _p],
    "qba_test_set_knobs": [_p, _u64, _i64, C.c_int],
}
_RESTYPE = {"qba_last_error": C.c_char_p}


class QbaError(RuntimeError):
    """A libqba call failed (or the library / a gfx950 device is unavailable)."""

    def __init__(self, msg: str, code: int = QBA_EHIP):
        super().__init__(msg)
        self.code = code


_lock = threading.Lock()
_lib = None


def lib() -> C.CDLL:
    """Load libqba.so (once).  Raises QbaError if it is missing."""
    global _lib
    with _lock:
        if _lib is None:
            if not LIB_PATH.exists():
                raise QbaError(f"libqba.so not built at {LIB_PATH}; run __graft_entry__.build()",
                               QBA_ESTATE)
            handle = C.CDLL(str(LIB_PATH))
            for name, args in SIGNATURES.items():
                if EXPERIMENT_LIB and not hasattr(handle, name):
                    continue  # an A/B build of an older tree (tools/exp) may predate a symbol
                fn = getattr(handle, name)
                fn.argtypes = args
                fn.restype = _RESTYPE.get(name, C.c_int)
            _lib = handle
        return _lib


def check(rc: int, what: str) -> None:
    if rc != QBA_OK:
        msg = lib().qba_last_error().decode(errors="replace")
        raise QbaError(f"{what} failed ({rc}): {msg}", rc)


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
