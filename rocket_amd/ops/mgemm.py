"""Host side of the large MFMA GEMM (``native/kernels/mgemm.hip``).

``mgemm(a, b, c, ...)`` computes ``C[M,N] (op)= epi(sum_k A(m,k) B(n,k))`` on bf16 operands with
f32 accumulation.  Each operand is either *row* (``A(m,k) = a[m*lda + k]``, K contiguous) or
*kmaj* (``A(m,k) = a[k*lda + m]``), so the three products of a linear layer need no transposes:

=========  ===========================  ============================
forward    ``Y = X W^T``                 A = X (row), B = W (row)
dgrad      ``dX = dY W``                 A = dY (row), B = W (kmaj)
wgrad      ``dW = dY^T X``               A = dY (kmaj), B = X (kmaj)
=========  ===========================  ============================

Tile choice (:func:`pick_tile`) models the grid as waves of resident blocks over 256 CUs: the
256x256 tile is the fastest per CU but a small grid leaves CUs idle in its last wave, so the
model prices every tile's wave quantisation and takes the cheapest.
"""

from __future__ import annotations

import torch

from rocket_amd.ops import _lib

EPI = {"none": 0, "relu": 1, "gelu": 2, "mul_gelu_grad": 3, "mul_relu_grad": 4}
# tile id -> (BM, BN, resident blocks per CU, relative per-CU throughput); see rk_mgemm
TILES = {0: (128, 128, 2, 0.85), 4: (128, 128, 2, 0.85), 5: (128, 128, 2, 0.8), 6: (256, 256, 1, 1.0),
         7: (256, 128, 1, 0.9), 8: (256, 256, 1, 1.0), 9: (256, 128, 1, 0.9)}
N_CU = 256
# tile ids >= XTILE select the macro-tile kernels of native/kernels/xgemm.hip (config = id - XTILE)
XTILE = 20
XTILES = {20: (256, 256, 1, 1.0), 21: (256, 128, 1, 0.9)}  # + 16: fp16 operands


def _cost(M: int, N: int, K: int, tile: int, splitk: int = 1) -> float:
    bm, bn, occ, rate = TILES[tile]
    blocks = -(-M // bm) * -(-N // bn) * splitk
    waves = -(-blocks // (N_CU * occ))
    return waves * bm * bn * occ * (K / splitk) / rate


def pick_tile(M: int, N: int, K: int) -> int:
    return min(TILES, key=lambda t: (_cost(M, N, K, t), t))


def pick_split(M: int, N: int, K: int, max_split: int = 16) -> tuple[int, int]:
    """(tile, splitk) for a long-K / few-tile product (weight gradients): split K over blocks so
    the grid fills the chip; the partial tiles go to f32 slabs that a second launch sums."""
    best = None
    for t in (0,):  # the 8-wave 128x128 tile measured fastest for every K-major x K-major product
        for s in range(1, max_split + 1):
            # every split writes and re-reads one more f32 slab
            c = _cost(M, N, K, t, s) * (1.0 + 0.06 * (s - 1))
            if best is None or c < best[0]:
                best = (c, t, s)
    return best[1], best[2]


_slabs: dict = {}
_retired: list = []  # outgrown slabs: captured HIP graphs may still write into them on replay


def _slab(device: torch.device, numel: int) -> torch.Tensor:
    """Split-K scratch, one per device, grown on demand (stream-ordered reuse: every launch on
    the stream consumes its slab before the next one writes it).

    A slab that is outgrown is retired, never freed: graphs captured while it was current keep
    its raw pointer and write their split-K partials into it on every replay, so returning it to
    the caching allocator would let another tensor alias those writes."""
    key = (device.type, device.index)
    buf = _slabs.get(key)
    if buf is None or buf.numel() < numel:
        if buf is not None:
            _retired.append(buf)
        buf = _slabs[key] = torch.empty(numel, dtype=torch.float32, device=device)
    return buf


def supported(*tensors: torch.Tensor) -> bool:
    return all(t.dtype == torch.bfloat16 and t.is_cuda and t.data_ptr() % 16 == 0 for t in tensors)


def mgemm(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, *, M: int, N: int, K: int, lda: int, ldb: int, ldc: int,
          a_kmaj: bool = False, b_kmaj: bool = False, c_pre: torch.Tensor | None = None,
          bias: torch.Tensor | None = None, aux: torch.Tensor | None = None, epi: str = "none",
          accumulate: bool = False, rowsum: torch.Tensor | None = None, splitk: int = 1,
          tile: int | None = None) -> torch.Tensor:
    if tile is None:
        tile = pick_tile(M, N, K // max(splitk, 1))
    slab = _slab(c.device, splitk * M * N) if splitk > 1 else None
    lib = _lib.kernels()
    fn, name, t = (lib.rk_xgemm, "rk_xgemm", tile - XTILE) if tile >= XTILE else (lib.rk_mgemm, "rk_mgemm", tile)
    _lib.check(
        fn(a.data_ptr(), lda, int(a_kmaj), b.data_ptr(), ldb, int(b_kmaj), c.data_ptr(), _lib.dtype_code(c),
                     ldc, _lib.ptr(c_pre), _lib.ptr(bias), _lib.ptr(aux), EPI[epi], int(accumulate), _lib.ptr(rowsum),
                     M, N, K, splitk, t, _lib.ptr(slab), _lib.stream_ptr(c.device)),
        name,
    )
    return c
