"""ctypes binding of the C ABI in include/lcv.h (liblcv.so, HIP/gfx950).

`load()` returns the product library that sits next to this file and raises `LcvUnavailable`
(loudly) if it is missing or cannot be loaded — there is no CPU fallback anywhere in `lcv`.
`Lib(path)` binds any library exporting the same ABI; the test suite uses it to drive the
host-simulation build of the same per-item code (never used by the product path).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblcv.so")

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)


class LcvUnavailable(RuntimeError):
    """liblcv.so (the HIP extension) is missing, unloadable, or no GPU is present."""


class LcvError(RuntimeError):
    pass


class HeaderCols(C.Structure):
    _fields_ = [("beacon", u8p), ("execution", u8p), ("exec_branch", u8p)]


class UpdateBatch(C.Structure):
    _fields_ = [
        ("attested", HeaderCols),
        ("finalized", HeaderCols),
        ("nsc_pool", u8p),
        ("nsc_index", u32p),
        ("nsc_branch", u8p),
        ("finality_branch", u8p),
        ("sync_bits", u8p),
        ("sync_signature", u8p),
        ("signature_slot", u64p),
        ("n", C.c_uint64),
        ("npool", C.c_uint64),
    ]


# name -> (restype, argtypes); must match include/lcv.h exactly (tests/test_abi.py checks it)
SIGNATURES = {
    "lcv_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "lcv_init": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "lcv_destroy": (None, [C.c_void_p]),
    "lcv_last_error": (C.c_char_p, [C.c_void_p]),
    "lcv_set_store": (C.c_int, [C.c_void_p, C.c_uint64, u8p, u8p, u8p]),
    "lcv_validate_updates": (C.c_int, [C.c_void_p, C.POINTER(UpdateBatch), C.c_uint64, u8p, u8p, u8p]),
    "lcv_batch_upload": (C.c_int, [C.c_void_p, C.POINTER(UpdateBatch), C.POINTER(C.c_void_p)]),
    "lcv_batch_free": (None, [C.c_void_p, C.c_void_p]),
    "lcv_validate_resident": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, u8p, u8p, u8p]),
    "lcv_validate_resident_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, u8p, C.c_void_p]),
    "lcv_validate_resident_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, u8p, C.c_int]),
    "lcv_slot_wait": (C.c_int, [C.c_void_p, C.c_int, C.c_uint64, u8p, u8p]),
    "lcv_slot_allgather": (C.c_int, [C.c_void_p, C.c_int, C.c_uint64, C.c_uint64, u8p]),
    "lcv_validate_async": (C.c_int, [C.c_void_p, C.POINTER(UpdateBatch), C.c_uint64, u8p, C.c_int]),
    "lcv_comm_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "lcv_debug_event_pool": (C.c_int, [C.c_void_p, u64p]),
    "lcv_debug_set_chunk": (C.c_int, [C.c_void_p, C.c_uint64]),
    "lcv_debug_work_check": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int]),
    "lcv_debug_hold_slot": (C.c_int, [C.c_void_p, C.c_int, C.c_double]),
    "lcv_debug_release_slots": (C.c_int, [C.c_void_p]),
    "lcv_build_id": (C.c_int, [C.c_char_p, C.c_uint64]),
    "lcv_last_timings": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int)]),
    "lcv_set_pipeline": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "lcv_set_latency_mode": (C.c_int, [C.c_void_p, C.c_uint64]),
    "lcv_debug_engine_log": (C.c_int, [C.c_void_p, u64p, C.c_int]),
    "lcv_set_config": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]),
    "lcv_stage_name": (C.c_char_p, [C.c_int]),
    "lcv_comm_unique_id": (C.c_int, [u8p]),
    "lcv_comm_init": (C.c_int, [C.c_void_p, C.c_int, C.c_int, u8p]),
    "lcv_comm_destroy": (C.c_int, [C.c_void_p]),
    "lcv_validate_sharded": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, u8p, C.c_uint64, u8p]),
    "lcv_comm_allreduce_max": (C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    "lcv_comm_set_timeout": (C.c_int, [C.c_void_p, C.c_double]),
    "lcv_comm_shrink": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "lcv_comm_abort": (C.c_int, [C.c_void_p]),
    "lcv_fast_aggregate_verify": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u8p, C.c_uint64, u8p, C.POINTER(C.c_int)]),
    "lcv_fast_aggregate_verify_batch": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u32p, u8p, u8p, u8p, C.c_uint64, u8p]),
    "lcv_merkle_branch_batch": (C.c_int, [C.c_void_p, u8p, u8p, C.c_uint32, C.c_uint64, u8p, C.c_uint64, u8p]),
    "lcv_htr_sync_committee_batch": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u8p]),
    "lcv_bootstrap_check_batch": (C.c_int, [C.c_void_p, u8p, u8p, u8p, u8p, u8p, u8p, C.c_uint64, u8p]),
    "lcv_ssz_decode_updates": (C.c_int, [u8p, u64p, u64p, C.c_uint64, C.c_int, C.c_int, C.POINTER(UpdateBatch),
                                         u64p, u64p, u8p]),
    "lcv_ssz_decode_updates_mixed": (C.c_int, [u8p, u64p, u64p, C.c_uint64, C.c_int, u8p, C.POINTER(UpdateBatch),
                                               u64p, u64p, u8p]),
    "lcv_ssz_decode_bootstrap": (C.c_int, [u8p, C.c_uint64, C.c_int, u8p, u8p, u8p, u8p, u8p, u8p]),
    "lcv_sk_to_pk_batch": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u8p]),
    "lcv_sign_batch": (C.c_int, [C.c_void_p, u8p, u8p, C.c_uint64, u8p]),
    "lcv_debug_fp": (C.c_int, [C.c_void_p, u8p, u8p, C.c_uint64, u8p, u8p]),
    "lcv_debug_fp_pow": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u8p]),
    "lcv_debug_hash_to_g2": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u8p, u8p]),
    "lcv_debug_g2_decompress": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u8p, u8p]),
    "lcv_debug_aggregate": (C.c_int, [C.c_void_p, u8p, C.c_uint64, u32p, u8p, C.c_uint64, u8p, u8p]),
    "lcv_debug_pairing": (C.c_int, [C.c_void_p, u8p, u8p, C.c_uint64, u8p]),
}


def as_u8(buf) -> np.ndarray:
    a = np.ascontiguousarray(np.frombuffer(buf, dtype=np.uint8) if isinstance(buf, (bytes, bytearray)) else buf)
    if a.dtype != np.uint8:
        a = a.view(np.uint8)
    return a


def ptr(a: np.ndarray, ctype=C.c_uint8):
    return a.ctypes.data_as(C.POINTER(ctype))


class Lib:
    def __init__(self, path: str):
        if not os.path.exists(path):
            raise LcvUnavailable(f"{path} not found — build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            self.dll = C.CDLL(path)
        except OSError as e:
            raise LcvUnavailable(f"cannot load {path}: {e}") from e
        self.path = path
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(self.dll, name)
            fn.restype = res
            fn.argtypes = args

    def __getattr__(self, name):
        return getattr(self.dll, name)

    def build_id(self) -> str:
        """The source hash compiled into the library (tools/build_id.py at build time)."""
        buf = C.create_string_buffer(64)
        if self.dll.lcv_build_id(buf, 64) != 0:
            raise LcvError("lcv_build_id failed")
        return buf.value.decode()


_lib = None
_lock = threading.Lock()


def load() -> Lib:
    """The product HIP library (raises LcvUnavailable if absent)."""
    global _lib
    with _lock:
        if _lib is None:
            _lib = Lib(LIB_PATH)
        return _lib
