// Host entry of the macro-tile GEMM (kernels: xgemm_impl.h, instantiated per operand layout in
// xgemm_l{0,1,2}.hip so the three compile in parallel).
#include "xgemm_impl.h"

namespace {
int xg_num_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cus[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

int g_dbg = 0;  // rk_xgemm_set_dbg

}  // namespace

// Diagnostics only (timing what each part of the main loop costs; results are garbage): bit 0
// skips the LDS-DMA, 1 the barrier, 2 the fragment reads, 3 the MFMAs.
RK_API int rk_xgemm_set_dbg(int bits) {
  g_dbg = bits;
  return 0;
}

// Configs (block tile, waves; one persistent block per CU, 4-slot ring of 32-deep k-units):
//   0: 256 x 256, 8 waves (2 x 4), 128 x 64 per wave   (128 KiB LDS)
//   1: 256 x 128, 8 waves (4 x 2),  64 x 64 per wave   (96 KiB)
// cfg + 16: fp16 operands (v_mfma_f32_16x16x32_f16), else bf16.
RK_API int rk_xgemm(const void* a, int64_t lda, int a_kmaj, const void* b, int64_t ldb, int b_kmaj, void* c, int c_dt,
                    int64_t ldc, void* c_pre, const float* bias, const void* aux, int epi, int accumulate,
                    float* rowsum, int M, int N, int K, int splitk, int cfg, float* slab, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  const bool h = cfg >= 16;
  cfg &= 15;
  if (cfg > 1 || (a_kmaj && !b_kmaj)) return (int)hipErrorInvalidValue;
  if (K <= 0 || ((!a_kmaj || !b_kmaj) && K % 32) || N % 8 || (a_kmaj && M % 8) || ldc % 4)
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)a | (uintptr_t)b) % 16 || (lda * 2) % 16 || (ldb * 2) % 16) return (int)hipErrorInvalidValue;
  if (epi != kNone || c_pre) return (int)hipErrorInvalidValue;  // activation epilogues: rk_mgemm
  const int BM = kXBM[cfg], BN = kXBN[cfg];
  // operand extents in bytes (row: rows x ld; kmaj: K rows x ld) and the largest per-lane offset
  const int64_t a_bytes = a_kmaj ? (int64_t)K * lda * 2 : (int64_t)M * lda * 2;
  const int64_t b_bytes = b_kmaj ? (int64_t)K * ldb * 2 : (int64_t)N * ldb * 2;
  const int64_t a_off_max = a_kmaj ? (int64_t)32 * lda * 2 + (M + BM) * 2 : (int64_t)(M + BM) * lda * 2;
  const int64_t b_off_max = b_kmaj ? (int64_t)32 * ldb * 2 + (N + BN) * 2 : (int64_t)(N + BN) * ldb * 2;
  if (a_off_max >= (1ll << 31) || b_off_max >= (1ll << 31)) return (int)hipErrorInvalidValue;
  MArgs g;
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c; g.c_pre = c_pre; g.bias = bias;
  g.aux = (const uint16_t*)aux; g.rowsum = rowsum; g.slab = slab;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.c_dt = c_dt; g.epi = epi; g.accumulate = accumulate;
  g.lds_epi = 0;
  g.tgroup = 1;  // (the persistent walk places tiles itself)
  g.dbg = g_dbg;
  if (splitk < 1) splitk = 1;
  const int kq = 32;  // split boundaries on whole units
  const int kps = ((K + kq - 1) / kq + splitk - 1) / splitk * kq;
  splitk = (K + kps - 1) / kps;
  if (splitk > 1 && (slab == nullptr || epi != kNone || c_pre)) return (int)hipErrorInvalidValue;
  g.splitk = splitk;
  g.k_per_split = kps;
  const int nc = xg_num_cus();
  const int rc = !a_kmaj && !b_kmaj ? rkx_launch_l0(&g, cfg, h, a_bytes, b_bytes, nc, s)
                 : !a_kmaj          ? rkx_launch_l1(&g, cfg, h, a_bytes, b_bytes, nc, s)
                                    : rkx_launch_l2(&g, cfg, h, a_bytes, b_bytes, nc, s);
  if (rc || splitk == 1) return rc;
  launch_mgemm_reduce(slab, splitk, M, N, bias, c, c_dt, ldc, accumulate, s);
  return (int)hipGetLastError();
}
