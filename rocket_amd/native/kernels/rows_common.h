// Device-side batch cursor of deferred device-loader batches (runtime/data.py PendingRows), shared
// by the stand-alone launch (data.hip rk_rows_next) and the fused LeNet weight-gradient launch
// (mlp.hip), which advances it as the step's last kernel.
#pragma once
#include "rk_common.h"

// One block: meta = {cursor, table length}; cursor += n_cur, then rows[i] = table[cursor + i] for
// i < min(bs, length - cursor).  The cursor store and the rows stores are by distinct threads of
// this one block after a barrier, so every thread reads the old cursor.
__device__ __forceinline__ void rows_next_block(const int64_t* __restrict__ table, int64_t* meta,
                                                int64_t* __restrict__ rows, int n_cur, int bs) {
  const int64_t c = meta[0] + n_cur, len = meta[1];
  __syncthreads();
  if (threadIdx.x == 0) meta[0] = c;
  const int64_t n = c < len ? (len - c < bs ? len - c : bs) : 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) rows[i] = table[c + i];
}
