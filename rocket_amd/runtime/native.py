"""ctypes bindings of ``librocket_runtime.so`` (``native/runtime/*.cpp``): RCCL communicator +
bucket reducer (comm.cpp) and the host batch assembler (loader.cpp)."""

from __future__ import annotations

import ctypes

from rocket_amd.ops import _lib

c_void_p, c_int, c_int64, c_char_p = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_char_p
P = ctypes.POINTER(ctypes.c_void_p)

RUNTIME_SIGS = {
    "rkr_last_error": (c_char_p, []),
    "rkr_unique_id_bytes": (c_int, []),
    "rkr_unique_id": (c_int, [c_void_p]),
    "rkr_comm_init": (c_int, [P, c_int, c_int, c_void_p, c_int]),
    "rkr_comm_destroy": (c_int, [c_void_p]),
    "rkr_comm_abort": (c_int, [c_void_p]),
    "rkr_all_reduce": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "rkr_broadcast": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "rkr_all_gather": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "rkr_reduce_scatter": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "rkr_reducer_create": (c_int, [P, c_void_p, c_int]),
    "rkr_reducer_set_bucket": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int]),
    "rkr_reducer_launch": (c_int, [c_void_p, c_int, c_void_p]),
    "rkr_reducer_join": (c_int, [c_void_p, c_void_p]),
    "rkr_reducer_destroy": (c_int, [c_void_p]),
    "rkl_create": (c_int, [P, c_int, c_void_p, c_void_p, c_int64, c_int, c_int]),
    "rkl_submit": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_void_p]),
    "rkl_wait": (c_int, [c_void_p, c_int]),
    "rkl_destroy": (c_int, [c_void_p]),
}


class RuntimeError_(RuntimeError):
    pass


def runtime():
    return _lib._load("rocket_runtime", RUNTIME_SIGS)


def check(code: int, what: str) -> None:
    if code != 0:
        msg = runtime().rkr_last_error()
        raise RuntimeError_(f"{what} failed ({code}): {msg.decode() if msg else ''}")
