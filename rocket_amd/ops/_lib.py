"""ctypes bindings of the in-tree native libraries.

The HIP kernels are plain ``extern "C"`` entry points in
``rocket_amd/_lib/librocket_kernels.so`` (built by :mod:`rocket_amd.native.build`).
They receive raw device pointers and the *current* PyTorch HIP stream, so every
launch is stream-ordered with PyTorch work and is captured by HIP graphs.

``torch`` is imported first so its HIP runtime is the one our library binds to
(both carry the ``libamdhip64.so.7`` SONAME).  On a machine with a GPU a
missing or unloadable library is an error (:func:`require_native`), never a
silent fallback.
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede loading the HIP library)

_HERE = os.path.dirname(os.path.abspath(__file__))
# ROCKET_LIBDIR: load the native libraries from another directory (A/B of two builds in one tree)
LIBDIR = os.environ.get("ROCKET_LIBDIR") or os.path.join(os.path.dirname(_HERE), "_lib")
_lock = threading.Lock()
_libs: dict = {}

c_void_p, c_int, c_int64, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float

# name -> (restype, argtypes)
KERNEL_SIGS = {
    "rk_ce_fwd": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int64, c_float, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "rk_ce_bwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int64, c_float, c_void_p, c_void_p, c_int, c_void_p]),
    "rk_ce_partials_needed": (c_int, [c_int, c_int]),
    "rk_ce_train": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int64, c_float, c_float, c_void_p,
                            c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_float, c_int, c_void_p]),
    "rk_optim_chunk": (c_int, []),
    "rk_gemm": (c_int, [c_void_p, c_int, c_int64, c_int, c_void_p, c_int, c_int64, c_int, c_void_p, c_int, c_int64,
                        c_int, c_void_p, c_int, c_int64, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int,
                        c_int, c_int, c_void_p]),
    "rk_mgemm": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_int64, c_int, c_void_p, c_int, c_int64, c_void_p, c_void_p,
                         c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "rk_xgemm": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_int64, c_int, c_void_p, c_int, c_int64, c_void_p, c_void_p,
                         c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "rk_xgemm_set_dbg": (c_int, [c_int]),
    "rk_xgemm4_set_dbg": (c_int, [c_int]),
    "rk_xgemm5_set_shape": (c_int, [c_int]),
    "rk_xgemm5": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int, c_void_p, c_int, c_int, c_int,
                          c_void_p]),
    "rk_xgemm4_set_trace": (c_int, [c_void_p]),
    "rk_xgemm4": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int, c_void_p, c_int, c_int, c_int,
                          c_void_p]),
    "rk_xgemm4_epi": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "rk_transpose16": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "rk_slab_acc": (c_int, [c_void_p, c_int, c_int, c_int64, c_void_p, c_int, c_void_p]),
    "rk_conv_fwd": (c_int, [c_int] + [c_void_p, c_void_p, c_void_p, c_int, c_void_p] + [c_int] * 11 + [c_void_p, c_void_p]),
    "rk_conv_fwd_c8": (c_int, [c_int] + [c_void_p, c_void_p, c_void_p] + [c_int] * 10 + [c_void_p, c_void_p]),
    "rk_pad_c8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int64, c_int64, c_int64, c_void_p]),
    "rk_bn_finalize": (c_int, [c_void_p, c_int, c_int, c_int64, c_int] + [c_void_p] * 9 + [c_float, c_float, c_void_p,
                                                                                            c_void_p, c_void_p]),
    "rk_conv_set_lds_epi": (c_int, [c_int]),
    "rk_conv_set_bn_prologue": (c_int, [c_void_p]),
    "rk_conv_set_tile_group": (c_int, [c_int]),
    "rk_conv_set_cfg": (c_int, [c_int]),
    "rk_mlp3_set_trace": (None, [c_void_p]),
    "rk_conv_dgrad_bn": (c_int, [c_int] + [c_void_p] * 3 + [c_int] * 9 + [c_void_p] * 6),
    "rk_bn_bwd_partials": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int64, c_int] + [c_void_p] * 11),
    "rk_conv_dgrad": (c_int, [c_int] + [c_void_p, c_void_p, c_void_p, c_int, c_int] + [c_int] * 11 + [c_void_p]),
    "rk_conv_wgrad": (c_int, [c_int] + [c_void_p, c_void_p, c_void_p, c_int, c_void_p] + [c_int] * 12 + [c_void_p, c_void_p]),
    "rk_conv_defer_reduce": (c_int, [c_int]),
    "rk_conv_flush_reduce": (c_int, [c_void_p]),
    "rk_conv_tail_counts": (c_int, [c_void_p]),
    "rk_head_fwd": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                            c_void_p]),
    "rk_head_bwd": (c_int, [c_int] + [c_void_p] * 6 + [c_int] * 5 + [c_void_p] * 2 + [c_int, c_void_p]),
    "rk_head_bwd_scratch": (c_int64, [c_int, c_int, c_int]),
    "rk_conv_pool_fwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p] + [c_int] * 7 + [c_void_p]),
    "rk_conv_pool_wgrad": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p] + [c_int] * 7 + [c_void_p]),
    "rk_conv_pool_dgrad": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int] + [c_int] * 7 + [c_void_p]),
    "rk_lenet_conv_fwd": (c_int, [c_void_p] * 9 + [c_int, c_void_p]),
    "rk_lenet_conv_bwd": (c_int, [c_void_p] * 10 + [c_int, c_int, c_void_p]),
    "rk_lenet_prep": (c_int, [c_void_p] * 7),
    "rk_lenet_frag_bytes": (c_int, []),
    "rk_lenet_set_trace": (None, [c_void_p, c_void_p]),
    "rk_lenet_fwd": (c_int, [c_void_p] * 16 + [c_int, c_void_p]),
    "rk_lenet_bwd": (c_int, [c_void_p] * 13 + [c_int, c_int, c_void_p, c_void_p]),
    "rk_lenet_slab_width": (c_int, []),
    "rk_lenet_slab_cols": (c_int, []),
    "rk_mlp3_fwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                            c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "rk_mlp3_dgrad": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int,
                              c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "rk_mlp3_wgrad": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                              c_int, c_void_p, c_void_p, c_void_p]),
    "rk_mlp3_wgrad_loss": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                   c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_void_p]),
    "rk_lenet_train": (c_int, [c_void_p] * 18 + [c_int, c_void_p, c_void_p, c_void_p]),
    "rk_optim_mt": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_int, c_int, c_void_p]),
    "rk_amp_check": (c_int, [c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "rk_host_mapped_alloc": (c_void_p, [c_int64, c_void_p]),
    "rk_gap_fwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "rk_patchify": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "rk_gap_bwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "rk_host_mapped_free": (None, [c_void_p]),
    "rk_optim_chunk_for": (c_int, [c_int64]),
    "rk_gather_rows": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "rk_loss_accum": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_float, c_int, c_void_p]),
    "rk_bn_workspace": (c_int64, [c_int64, c_int]),
    "rk_bn_stats": (c_int, [c_int, c_void_p, c_int64, c_int] + [c_void_p] * 9 + [c_float, c_float, c_void_p, c_void_p,
                                                                                  c_void_p]),
    "rk_bn_apply": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int,
                            c_int, c_void_p]),
    "rk_bn_counters": (c_int, [c_int]),
    "rk_bn_relu_maxpool": (c_int, [c_int] + [c_void_p] * 5 + [c_int] * 6 + [c_void_p]),
    "rk_maxpool_bwd": (c_int, [c_int] + [c_void_p] * 3 + [c_int] * 6 + [c_void_p]),
    "rk_colsum_acc": (c_int, [c_int, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_gelu_bwd_colsum16": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
    "rk_gelu_bwd_colsum": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
    "rk_bn_bwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int] + [c_void_p] * 11),
    "rk_ln_fwd": (c_int, [c_int, c_int] + [c_void_p] * 8 + [c_int64, c_int, c_float, c_void_p]),
    "rk_ln_workspace": (c_int64, [c_int64, c_int]),
    "rk_ln_set_bwd_cfg": (c_int, [c_int, c_int]),
    "rk_attn_max_len": (c_int, []),
    "rk_attn_set_waves": (c_int, [c_int, c_int, c_int]),
    "rk_attn_set_bwd_fused": (c_int, [c_int]),
    "rk_attn_set_stamps": (c_int, [c_void_p]),
    "rk_spin": (c_int, [ctypes.c_double, c_int, c_void_p, c_void_p]),
    "rk_gap_write": (c_int, [c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p]),
    "rk_gap_stamp": (c_int, [c_int, c_void_p, c_int, c_void_p]),
    "rk_gather_rows_any_order": (None, []),
    "rk_gather_set_trace": (None, [c_void_p]),
    "rk_rows_next": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "rk_mlp3_set_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int]),
    "rk_mlp3_set_amp_found": (c_int, [c_void_p]),
    "rk_gap_stamp_big": (c_int, [c_int, c_void_p, c_int, c_void_p]),
    "rk_attn_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_float,
                            c_void_p]),
    "rk_attn_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p]),
    "rk_attn_fwd16": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                              c_float, c_void_p]),
    "rk_attn_bwd16": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p]),
    "rk_gelu_fwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p]),
    "rk_gelu_bwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "rk_softmax_fwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int64, c_int, c_float, c_void_p]),
    "rk_softmax_bwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_float, c_void_p]),
    "rk_p2p_handle_bytes": (c_int, []),
    "rk_p2p_chunk": (c_int, []),
    "rk_p2p_create": (c_int, [c_int, c_int, c_int64, c_void_p, c_void_p]),
    "rk_p2p_open": (c_int, [c_void_p, c_void_p]),
    "rk_p2p_allreduce": (c_int, [c_void_p, c_void_p, c_int64, c_float, c_void_p]),
    "rk_p2p_allreduce_adam": (c_int, [c_void_p, c_void_p, c_int64, c_float, c_void_p, c_int, c_void_p, c_int,
                                      c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "rk_p2p_error": (c_int, [c_void_p]),
    "rk_p2p_set_timeout": (c_int, [c_void_p, ctypes.c_double]),
    "rk_p2p_set_skip": (c_int, [c_void_p, c_void_p, c_void_p]),
    "rk_p2p_set_loss_ring": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int64]),
    "rk_p2p_clear_error": (c_int, [c_void_p]),
    "rk_p2p_error_ptr": (c_void_p, [c_void_p]),
    "rk_p2p_destroy": (c_int, [c_void_p]),
    "rk_ln_bwd": (c_int, [c_int, c_int] + [c_void_p] * 12 + [c_int64, c_int, c_void_p, c_void_p, c_void_p]),
}

# fp16 builds of the fused LeNet kernels (lenet_conv_h.hip / mlp_h.hip): same signatures
KERNEL_SIGS.update({n + "_h": KERNEL_SIGS[n] for n in (
    "rk_lenet_conv_fwd", "rk_lenet_conv_bwd", "rk_lenet_prep", "rk_lenet_fwd", "rk_lenet_bwd", "rk_lenet_train",
    "rk_mlp3_fwd", "rk_mlp3_dgrad", "rk_mlp3_wgrad", "rk_mlp3_wgrad_loss", "rk_mlp3_set_rows",
    "rk_mlp3_set_amp_found")})


class NativeError(RuntimeError):
    pass


def _load(name: str, sigs: dict, build_if_missing: bool = True):
    with _lock:
        if name in _libs:
            return _libs[name]
        path = os.path.join(LIBDIR, f"lib{name}.so")
        if not os.path.exists(path) and build_if_missing:
            from rocket_amd.native import build as _build

            _build.build(verbose=False)
        if not os.path.exists(path):
            raise NativeError(f"{path} is missing; run `python -m rocket_amd.native.build`")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        for fn, (res, args) in sigs.items():
            f = getattr(lib, fn, None)
            if f is None:
                continue
            f.restype, f.argtypes = res, args
        _libs[name] = lib
        return lib


def kernels():
    return _load("rocket_kernels", KERNEL_SIGS)


def available() -> bool:
    try:
        kernels()
        return True
    except Exception:
        return False


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None) -> int:
    """hipStream_t of the current stream (a raw-handle lookup: ~10x cheaper on the host than
    materialising a ``torch.cuda.Stream``, which matters for a ~60 µs launch-bound step)."""
    if _raw_stream is None:
        return torch.cuda.current_stream(device).cuda_stream
    if device is None:
        return _raw_stream(torch.cuda.current_device())
    if isinstance(device, int):
        return _raw_stream(device)
    if not isinstance(device, torch.device):
        device = torch.device(device)
    return _raw_stream(device.index if device.index is not None else torch.cuda.current_device())


# Serialised debug mode: ROCKET_DEBUG_SYNC=1 synchronises the device after every
# native launch outside graph capture, so an asynchronous fault (out-of-bounds access, failed
# assertion in a kernel) is reported at the launch that caused it, by name.  runtime/hipenv.py also
# turns on the runtime's own kernel serialisation for that mode.
DEBUG_SYNC = os.environ.get("ROCKET_DEBUG_SYNC", "0") == "1"


def check(code: int, what: str) -> None:
    if code != 0:
        raise NativeError(f"{what} failed with hipError {code}")
    if DEBUG_SYNC and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:  # the fault surfaced here: name the launch
            raise NativeError(f"{what}: device error after launch (ROCKET_DEBUG_SYNC): {e}") from e


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float16:
        return 2
    raise NativeError(f"unsupported dtype {t.dtype}")


class Workspace:
    """Per-device scratch: zero-initialised ticket counters for in-launch grid reductions.

    Kernels on one stream run in order and every last-arriving block resets its
    counter to zero, so one counter per kernel family per device suffices.
    """

    _per_device: dict = {}
    SIZE = 65536  # counters are reset by their last block, so one slot per (op, call-site) suffices

    def __init__(self, device: torch.device):
        self.counters = torch.zeros(self.SIZE, dtype=torch.int32, device=device)
        self._next = 0
        self._named: dict = {}

    @classmethod
    def get(cls, device) -> "Workspace":
        device = torch.device(device)
        key = (device.type, device.index)
        ws = cls._per_device.get(key)
        if ws is None:
            ws = cls._per_device[key] = Workspace(device)
        return ws

    def counter_array(self, name: str, n: int) -> int:
        """Pointer to ``n`` consecutive zeroed counters reserved under ``name``."""
        key = (name, n)
        idx = self._named.get(key)
        if idx is None:
            idx = self._named[key] = self._next
            self._next += n
            if self._next > self.counters.numel():
                self._grow(self._next)
        return self.counters.data_ptr() + 4 * idx

    def _grow(self, need: int) -> None:
        raise NativeError(f"workspace counters exhausted ({need} > {self.counters.numel()}); "
                          "raise Workspace.SIZE before the first launch")

    def counter(self, name: str) -> int:
        idx = self._named.get(name)
        if idx is None:
            idx = self._named[name] = self._next
            self._next += 1
            if self._next > self.counters.numel():
                raise NativeError("workspace counters exhausted")
        return self.counters.data_ptr() + 4 * idx
