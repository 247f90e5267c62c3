// Implicit-GEMM convolutions (NHWC bf16 or fp16, f32 accumulation) on the MFMA GEMM core (mgemm_core.h)
// for the ResNet configs (reference anchor examples/mnist.py:47-48).
//
// Tensors are channels-last: X [N][H][W][C], weights [Cout][R][S][Cin] (the memory order of a
// channels_last nn.Conv2d weight), Y [N][OH][OW][Cout].  No im2col buffer: the LDS-DMA stager of
// the gathered operand computes every 16-byte chunk's source pixel itself, and chunks that fall
// into the zero padding (or past the last pixel) are DMA'd from a zero page.
//
//   forward  Y  = X (*) W      GEMM M = N*OH*OW pixels, N = Cout, K = R*S*Cin (r, s, ci order)
//            A(m, k) = X[n, oh*st - pad + r, ow*st - pad + s, ci]          gathered, row image
//            B(co, k) = W[co][r][s][ci]                                     plain row image
//   dgrad    dX = dY (*) W^T   (stride 1) GEMM M = N*H*W, N = Cin, K = R*S*Cout (r, s, co order)
//            A(m, k) = dY[n, ih + pad - r, iw + pad - s, co]               gathered, row image
//            B(ci, k) = W[co][r][s][ci]                                     K-major, per-tile base
//   wgrad    dW = dY^T (*) X   GEMM M = Cout, N = R*S*Cin, K = N*OH*OW pixels (split-K)
//            A(co, m) = dY[m][co]                                           plain K-major image
//            B(k', m) = X[n, oh*st - pad + r, ow*st - pad + s, ci]          gathered, K-major image
//
// A k-tile (64 deep) must sit inside one (r, s) tap: Cin % 64 == 0 (forward / wgrad columns:
// Cin % 8), Cout % 64 == 0 for the dgrad.  So the tap (r, s, c0) of a k-tile is wave-uniform
// (scalar), and a lane only adds it to its precomputed pixel coordinates.
// Tile: 128 x 128 x 64, 8 waves (2 x 4), two blocks per CU, 2-slot LDS ring (mgemm.hip tile 0).
#include "mgemm_core.h"

using namespace rk;

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

enum ConvMode : int { kConvFwd = 0, kConvDgrad = 1, kConvWgrad = 2, kConvDgradS = 3, kConvFwdC8 = 4 };

// Strided input gradient, one GEMM per parity class (py, px) of the dX pixels: pixel
// (2*gi + py, 2*gj + px) receives only the taps r = r0y + 2j, s = r0x + 2l (those with
// ih + pad - r even), from dY pixel (gi + hoff - j, gj + woff - l) — a stride-1 gather over a
// (GH x GW) sub-grid with Rv x Sv taps.  The four classes share one launch (interleaved blocks).
struct DgCls {
  int M, K;            // N*GH*GW rows, Rv*Sv*Cout reduction
  int GH, GW, Sv;      // sub-grid, taps per row
  int r0y, r0x;        // first tap of the class
  int hoff, woff;      // dY row/col of (gi, gj) at tap (j, l) = (gi + hoff - j, gj + woff - l)
  int py, px;          // parity of the class's dX pixels
};

struct ConvGeom {
  int N, H, W, C;        // the gathered tensor (fwd/wgrad: X; dgrad: dY), NHWC
  int GH, GW;            // the pixel grid the GEMM rows/k run over (fwd/wgrad: OH x OW; dgrad: H x W)
  int R, S, stride, pad;
  int taps_c;            // channels per tap of the GEMM K order (fwd: Cin; dgrad: Cout)
  int64_t w_tap_stride;  // dgrad: elements between taps in W (= Cin); wgrad/fwd unused
  int64_t w_co_stride;   // dgrad: elements between output channels in W (= R*S*Cin)
  float inv_gw, inv_gh;  // 1/GW, 1/GH (pixel decomposition of the wgrad k index)
  float inv_s;           // 1/S (tap decomposition of the C = 8 stem gather)
  float* bnpart;         // forward: per row-tile BatchNorm partials [tiles_m][2][Cout] (tile mean, M2) or null
  int hoff, woff;        // dgrad: dY pixel of grid pixel (gh, gw) at tap (tr, ts) = (gh + hoff - tr, gw + woff - ts)
  int dx_h, dx_w;        // strided dgrad: dX extent (the epilogue's pixel map)
  // stride-1 dgrad whose dX is the gradient of a BatchNorm(+ReLU) output (ResNet: every conv input
  // but the stem's): the epilogue applies that BatchNorm's ReLU mask, stores the masked dX and writes
  // per-128-row-tile partials (sum dX', sum dX' * xhat) of the BatchNorm backward, [tiles][2][C]
  const uint16_t* bnb_x;   // the BatchNorm's input [M][C] (bf16), or null: no BN epilogue
  const uint8_t* bnb_mask; // its ReLU mask [M][C/8] (bit k: channel 8*(c/8) + k), or null
  const float* bnb_mean;
  const float* bnb_invstd;
  float* bnb_part;
  // BatchNorm-apply prologue (fwd A / wgrad B gather): the gathered tensor is a BatchNorm's INPUT z
  // and the operand is relu(z*scale + shift) [2][C] (scale, shift), formed in registers between the
  // load and the LDS write; padding chunks stay zero.  bnb_ss (BNB dgrad): the ReLU mask is
  // recomputed from bnb_x the same way instead of read from bnb_mask.
  const float* pro_ss;
  const float* bnb_ss;
  int w_s;               // strided dgrad: the weight's full kernel width S (tap index r*S + s)
  int ncls;              // strided dgrad: parity classes in the launch
  int zero_nb;           // strided dgrad, 1x1 kernel: only class (0, 0) has taps; its tiles also zero
                         // the three odd-parity neighbours of each of their pixels
  int st_nt;             // row-chunk tile stores (store_tile_lds) nontemporal (ROCKET_CONV_NT)
  DgCls cls[4];
  // tail-reduce job (rk_conv_defer_reduce): the split-K combine of a preceding weight gradient, run
  // by tr_blocks extra blocks appended to this launch (mgemm_core.h reduce_slabs; dW[tr_M][tr_N] f32)
  const float* tr_slab;
  float* tr_c;
  int tr_splitk, tr_M, tr_N, tr_acc, tr_blocks, tr_g4;
};

// (n, gh, gw) of grid pixel m (exact for m < 2^24 after the correction steps)
__device__ __forceinline__ void split_pixel(int m, const ConvGeom& cg, int& n, int& gh, int& gw) {
  int q = (int)((float)m * cg.inv_gw);
  q -= (q * cg.GW > m);
  q += ((q + 1) * cg.GW <= m);
  gw = m - q * cg.GW;
  int nn = (int)((float)q * cg.inv_gh);
  nn -= (nn * cg.GH > q);
  nn += ((nn + 1) * cg.GH <= q);
  gh = q - nn * cg.GH;
  n = nn;
}

// relu(z*scale + shift) of 8 16-bit channels (scale / shift: 8 f32 at sc / sc + C in LDS), or zero
// for a padding chunk — the same fp32 expression (and rounding) as norm.hip bn_apply_kernel
constexpr int kProMaxC = 512;  // channels of a prologue's scale / shift table (LDS, host-checked)
template <bool H>
__device__ __forceinline__ u32x4 bn_relu8(u32x4 v, const float* sc, int C, bool ok) {
  const f32x4 a0 = *(const f32x4*)sc, a1 = *(const f32x4*)(sc + 4);
  const f32x4 b0 = *(const f32x4*)(sc + C), b1 = *(const f32x4*)(sc + C + 4);
  const float a[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
  const float b[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  u32x4 o;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float lo = fmaxf(__builtin_fmaf(lo16t<H>(v[p]), a[2 * p], b[2 * p]), 0.f);
    const float hi = fmaxf(__builtin_fmaf(hi16t<H>(v[p]), a[2 * p + 1], b[2 * p + 1]), 0.f);
    o[p] = ok ? pack16t<H>(lo, hi) : 0u;
  }
  return o;
}

// Gathered row-image operand (forward / dgrad A): rows are grid pixels, k runs over (r, s, c).
// A lane's rows are fixed for the whole block, only the k-tile's tap (r, s) and channel offset c0
// change (wave-uniform): so the per-lane work of a k-tile is one pointer add of a scalar offset, a
// bit test in the lane's precomputed tap-validity mask (R*S <= 32 taps, host-checked) and a select
// — no per-k-tile multiplies, 64-bit index math or branches around the DMAs.
template <int R, int BK, int NW, int MODE>
struct GatherRows {
  static constexpr int NI = R * BK / (512 * NW), CPR = BK / 8;
  const char* p0[NI];  // the lane's chunk at tap (0, 0), c0 = 0 (may point outside x: never read then)
  uint32_t vmask[NI];  // bit r*S + s: tap (r, s) inside the image, and the row inside M
  int chl[NI];         // the lane's channel offset within a k-tile (prologue scale / shift index)
  __device__ __forceinline__ void init(const uint16_t* x, const ConvGeom& cg, int row0, int M, int wid, int lane) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = (wid * NI + i) * 64 + lane;
      const int r = q / CPR, c = q % CPR;
      const int m = row0 + r;
      const int mm = m < M ? m : 0;
      const int gw = mm % cg.GW, t = mm / cg.GW;
      const int gh = t % cg.GH, n = t / cg.GH;
      int h0, w0;
      if (MODE == kConvFwd) {
        h0 = gh * cg.stride - cg.pad;
        w0 = gw * cg.stride - cg.pad;
      } else {  // dgrad (stride 1: hoff = woff = pad; strided: per parity class)
        h0 = gh + cg.hoff;
        w0 = gw + cg.woff;
      }
      chl[i] = (c ^ rswz<BK>(r)) * 8;
      const int64_t e = ((int64_t)(n * cg.H + h0) * cg.W + w0) * cg.C + chl[i];
      p0[i] = (const char*)x + e * 2;
      uint32_t v = 0;
      if (m < M) {
        for (int tr = 0; tr < cg.R; ++tr)
          for (int ts = 0; ts < cg.S; ++ts) {
            const int h = MODE == kConvFwd ? h0 + tr : h0 - tr;
            const int w = MODE == kConvFwd ? w0 + ts : w0 - ts;
            if ((unsigned)h < (unsigned)cg.H && (unsigned)w < (unsigned)cg.W) v |= 1u << (tr * cg.S + ts);
          }
      }
      vmask[i] = v;
    }
  }
  // k-tile at tap (tr, ts), channel offset c0
  __device__ __forceinline__ void issue(const ConvGeom& cg, int tr, int ts, int c0, char* lds, int wid,
                                        const char* zero) const {
    // wave-uniform byte offset of (tr, ts, c0) from tap (0, 0)
    const int64_t tap_off = (int64_t)(tr * cg.W + ts) * cg.C;
    const int64_t soff = ((MODE == kConvFwd ? tap_off : -tap_off) + c0) * 2;
    const int bit = tr * cg.S + ts;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const bool ok = (vmask[i] >> bit) & 1u;
      const char* src = ok ? p0[i] + soff : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + (wid * NI + i) * 1024), 16, 0, 0);
    }
  }
  // prologue form: the k-tile's chunks into registers (padding: the zero page, flagged in okm)
  __device__ __forceinline__ void load(const ConvGeom& cg, int tr, int ts, int c0, const char* zero, u32x4 (&v)[NI],
                                       uint32_t& okm) const {
    const int64_t tap_off = (int64_t)(tr * cg.W + ts) * cg.C;
    const int64_t soff = ((MODE == kConvFwd ? tap_off : -tap_off) + c0) * 2;
    const int bit = tr * cg.S + ts;
    okm = 0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const bool ok = (vmask[i] >> bit) & 1u;
      okm |= (uint32_t)ok << i;
      v[i] = *(const u32x4*)(ok ? p0[i] + soff : zero);
    }
  }
  // ... transformed and written to the k-tile's LDS image (the DMA's lane-linear layout)
  template <bool H>
  __device__ __forceinline__ void put(char* lds, int wid, int lane, const u32x4 (&v)[NI], uint32_t okm,
                                      const float* tab, int C, int c0) const {
#pragma unroll
    for (int i = 0; i < NI; ++i)
      *(u32x4*)(lds + (wid * NI + i) * 1024 + lane * 16) = bn_relu8<H>(v[i], tab + c0 + chl[i], C, (okm >> i) & 1u);
  }
};

// Gathered row image for a stem conv on a channel-padded image (C = 8: the 3 image channels + 5
// zero channels, one 16-byte chunk per pixel): a 64-deep k-tile spans 8 taps, so every chunk of a
// row is its own tap, (k0 / 8 + chunk).  K = R*S*8 is padded to whole k-tiles: taps >= R*S (and
// pixels outside the image) come from the zero page, the weights' pad columns are zero.
template <int R, int BK, int NW>
struct GatherRowsC8 {
  static constexpr int NI = R * BK / (512 * NW), CPR = BK / 8;
  int pix[NI], h0[NI], w0[NI], j[NI];
  bool mok[NI];
  __device__ __forceinline__ void init(const ConvGeom& cg, int row0, int M, int wid, int lane) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = (wid * NI + i) * 64 + lane;
      const int r = q / CPR, c = q % CPR;
      const int m = row0 + r;
      mok[i] = m < M;
      const int mm = mok[i] ? m : 0;
      const int gw = mm % cg.GW, t = mm / cg.GW;
      const int gh = t % cg.GH, n = t / cg.GH;
      pix[i] = n * cg.H;
      h0[i] = gh * cg.stride - cg.pad;
      w0[i] = gw * cg.stride - cg.pad;
      j[i] = c ^ rswz<BK>(r);  // the logical chunk (tap offset within the k-tile) this lane fetches
    }
  }
  __device__ __forceinline__ void issue(const uint16_t* x, const ConvGeom& cg, int k0, char* lds, int wid,
                                        const char* zero) const {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int tap = (k0 >> 3) + j[i];
      const int tr = (int)((float)tap * cg.inv_s);  // tap < 2^12: the float quotient is exact after the fixup
      const int trc = tr - (tr * cg.S > tap) + ((tr + 1) * cg.S <= tap);
      const int ts = tap - trc * cg.S;
      const int h = h0[i] + trc, w = w0[i] + ts;
      const bool ok = mok[i] && tap < cg.R * cg.S && (unsigned)h < (unsigned)cg.H && (unsigned)w < (unsigned)cg.W;
      const int64_t e = ((int64_t)(pix[i] + h) * cg.W + w) * 8;
      const char* src = ok ? (const char*)(x + e) : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + (wid * NI + i) * 1024), 16, 0, 0);
    }
  }
};

// Gathered K-major operand (wgrad B): k rows are output pixels, columns are (r, s, ci) chunks.
// A lane's column (tap, channel chunk) is fixed for the block and its k row moves by BK pixels per
// k-tile (the tiles of a split are issued in order): the pixel's (n, oh, ow) digits, its window
// position and its element offset are carried from k-tile to k-tile by mixed-radix increments with
// wave-uniform deltas — adds, compares and selects only, no per-k-tile divisions or multiplies.
template <int R, int BK, int NW>
struct GatherCols {
  static constexpr int NI = R * BK / (512 * NW), CPR = R / 8;
  int m[NI], oh[NI], ow[NI], hs[NI], ws[NI];  // pixel, its output row / col, window row / col + tap
  int64_t e[NI];                              // element offset of the lane's chunk at that pixel
  bool cok[NI];
  int chn[NI];                                // the lane's channel (prologue scale / shift index)
  // per-k-tile increments (wave-uniform): BK pixels = qn images + qh rows + qw columns
  int qw, qh, qn;
  int64_t d_w, d_wc, d_h, d_hc, d_n;
  __device__ __forceinline__ void init(const ConvGeom& cg, int col0, int Ncols, int kb, int wid, int lane) {
    const int st = cg.stride;
    qw = BK % cg.GW;
    qh = (BK / cg.GW) % cg.GH;
    qn = BK / (cg.GW * cg.GH);
    d_w = (int64_t)qw * st * cg.C;                              // ow += qw
    d_wc = ((int64_t)st * cg.W - (int64_t)cg.GW * st) * cg.C;   // ow wraps: next output row
    d_h = (int64_t)qh * st * cg.W * cg.C;                       // oh += qh
    d_hc = ((int64_t)cg.H - (int64_t)cg.GH * st) * cg.W * cg.C; // oh wraps: next image
    d_n = (int64_t)qn * cg.H * cg.W * cg.C;                     // n += qn
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = (wid * NI + i) * 64 + lane;
      const int k = q / CPR, c = q % CPR;
      const int col = col0 + (c ^ kswz<R>(k)) * 8;
      cok[i] = col < Ncols;
      const int cc = cok[i] ? col : 0;
      const int tap = cc / cg.C;
      const int ci = cc - tap * cg.C;
      chn[i] = ci;
      const int tr = tap / cg.S, ts = tap - tr * cg.S;
      m[i] = kb + k;
      int n, h, w;
      split_pixel(m[i], cg, n, h, w);
      oh[i] = h;
      ow[i] = w;
      hs[i] = h * st - cg.pad + tr;
      ws[i] = w * st - cg.pad + ts;
      e[i] = ((int64_t)(n * cg.H + hs[i]) * cg.W + ws[i]) * cg.C + ci;
    }
  }
  // the current k-tile (rows m .. of every lane), then advance every lane's row by BK pixels
  __device__ __forceinline__ void issue(const uint16_t* x, const ConvGeom& cg, int kend, char* lds, int wid,
                                        const char* zero) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const bool ok = cok[i] && m[i] < kend && (unsigned)hs[i] < (unsigned)cg.H && (unsigned)ws[i] < (unsigned)cg.W;
      const char* src = ok ? (const char*)(x + e[i]) : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + (wid * NI + i) * 1024), 16, 0, 0);
    }
    advance(cg);
  }
  // prologue form of issue: the chunks into registers (zero page + okm flag for padding / tails)
  __device__ __forceinline__ void load(const uint16_t* x, const ConvGeom& cg, int kend, const char* zero,
                                       u32x4 (&v)[NI], uint32_t& okm) {
    okm = 0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const bool ok = cok[i] && m[i] < kend && (unsigned)hs[i] < (unsigned)cg.H && (unsigned)ws[i] < (unsigned)cg.W;
      okm |= (uint32_t)ok << i;
      v[i] = *(const u32x4*)(ok ? (const char*)(x + e[i]) : zero);
    }
    advance(cg);
  }
  template <bool H>
  __device__ __forceinline__ void put(char* lds, int wid, int lane, const u32x4 (&v)[NI], uint32_t okm,
                                      const float* tab, int C) const {
#pragma unroll
    for (int i = 0; i < NI; ++i)
      *(u32x4*)(lds + (wid * NI + i) * 1024 + lane * 16) = bn_relu8<H>(v[i], tab + chn[i], C, (okm >> i) & 1u);
  }
  // every lane's row moves on by BK pixels
  __device__ __forceinline__ void advance(const ConvGeom& cg) {
    const int st = cg.stride;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      m[i] += BK;
      int w = ow[i] + qw, h = oh[i] + qh;
      int64_t ee = e[i] + d_w + d_h + d_n;
      int hh = hs[i] + qh * st, ww = ws[i] + qw * st;
      if (w >= cg.GW) {  // column carry into the row digit
        w -= cg.GW;
        ++h;
        ee += d_wc;
        ww -= cg.GW * st;
        hh += st;
      }
      if (h >= cg.GH) {  // row carry into the image digit
        h -= cg.GH;
        ee += d_hc;
        hh -= cg.GH * st;
      }
      ow[i] = w;
      oh[i] = h;
      hs[i] = hh;
      ws[i] = ww;
      e[i] = ee;
    }
  }
};

// BatchNorm statistics of the forward output, from the accumulators (rounded to the bf16 the tile
// is stored as, so they describe exactly the tensor the BatchNorm normalises): every wave writes,
// per channel of its columns, the sum and sum of squares of its TM-row slice of the tile — one
// register pass and a 16-lane xor-shuffle reduction, no LDS, no barrier.  The following BatchNorm
// merges these (rk_bn_finalize, pivoted on slice 0's mean) instead of re-reading the activation.
template <int BM, int BN, int WM, int WN, int FM, int FN, bool H>
__device__ __forceinline__ void tile_bn_stats(const MArgs& g, const ConvGeom& cg, f32x4 (&acc)[FM][FN], int tm,
                                              int row0, int col0, int wm, int wn, int lane) {
  constexpr int TM = BM / WM, TN = BN / WN;
  const int mbase = row0 + wm * TM;
  float s1[FN][4], s2[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) s1[j][e] = s2[j][e] = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const bool ok = mbase + i * 16 + (lane & 15) < g.M;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = ok ? round16t<H>(acc[i][j][e]) : 0.f;
        s1[j][e] += v;
        s2[j][e] = __builtin_fmaf(v, v, s2[j][e]);
      }
  }
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[j][e] += __shfl_xor(s1[j][e], o, 64);
        s2[j][e] += __shfl_xor(s2[j][e], o, 64);
      }
  if ((lane & 15) == 0) {
    float* part = cg.bnpart + (int64_t)(tm * WM + wm) * 2 * g.N;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = col0 + wn * TN + j * 16 + 4 * (lane >> 4);
      if (n < g.N) {  // N % 4 == 0: all four columns in
        *(float4*)(part + n) = make_float4(s1[j][0], s1[j][1], s1[j][2], s1[j][3]);
        *(float4*)(part + g.N + n) = make_float4(s2[j][0], s2[j][1], s2[j][2], s2[j][3]);
      }
    }
  }
}

// Block barrier for LDS hand-offs only: waits for this wave's LDS operations, not for the tile's
// global stores already issued (__syncthreads() would drain vmcnt: a memory round trip per slice)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Row-coalesced bf16 tile store through LDS (plain / accumulate, no bias / activation / split-K):
// the accumulators are parked in an f32 LDS image and every thread then moves 16-byte (8-channel)
// row chunks, so a wave instruction covers whole row segments instead of the MFMA layout's 16 rows x
// 32 bytes (which streamed at about half of HBM bandwidth on the memory-bound 1x1 convs).  One pass
// per wave row (wm): its TM x BN f32 slice fits in the dead operand stages.  Values are rounded to
// bf16 once, after the optional accumulate.  Called by all threads after the main loop.
//
// BNB (stride-1 dgrad, ConvGeom::bnb_x): the stored dX' = ReLU-mask * dX (+ old dX) also feeds the
// BatchNorm backward's reduction — each thread owns one 8-channel column chunk for the whole tile,
// reads the BN input / mask byte of its chunks row-contiguously like the store, and the per-thread
// sums are combined (xor-shuffles over the lanes sharing the chunk, then LDS over the waves) into one
// [2][BN] partial row per 128-row tile.
template <int BM, int BN, int WM, int WN, int FM, int FN, bool BNB, bool H, typename RowMap, bool BNX = false>
__device__ __forceinline__ void store_tile_lds(const MArgs& g, const ConvGeom& cg, f32x4 (&acc)[FM][FN], char* smem,
                                               int row0, int col0, int tm, int wm, int wn, int lane,
                                               const RowMap& rowmap) {
  constexpr int TM = BM / WM, TN = BN / WN, LS = BN + 4, NT = 64 * WM * WN, CPR = BN / 8;
  static_assert(TM * CPR % NT == 0 && NT % CPR == 0 && CPR <= 64, "whole chunk passes, fixed chunk column");
  float* img = (float*)smem;
  const int cc = ((int)threadIdx.x % CPR) * 8;  // this thread's chunk column (fixed: NT % CPR == 0)
  float s1[8], s2[8], mu[8], is[8], qa[BNX ? 8 : 1], qb[BNX ? 8 : 1];
  if constexpr (BNB) {
    const int n = min(col0 + cc, g.N - 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] = s2[e] = 0.f;
      mu[e] = cg.bnb_mean[n + e];
      is[e] = cg.bnb_invstd[n + e];
    }
    if (BNX) {  // the mask is recomputed from the BN input: scale / shift of these channels
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        qa[e] = cg.bnb_ss[n + e];
        qb[e] = cg.bnb_ss[g.N + n + e];
      }
    }
  }
  // side inputs of every chunk this thread stores (the BN input and ReLU-mask byte of BNB, the old
  // output of an accumulate), all issued now: their memory latency overlaps the LDS image passes
  // instead of stalling each chunk's store in turn
  // (each optional input under ONE uniform branch around its whole loop: a per-element
  // condition would make hipcc wait for every load separately)
  constexpr int KI = TM * CPR / NT;
  uint4 xz[WM][KI], old[WM][KI];
  unsigned mbv[WM][KI];
  int64_t offs[WM][KI];
  int mrow[WM][KI];
  const int ncl = min(col0 + cc, g.N - 8);
#pragma unroll
  for (int h = 0; h < WM; ++h)
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int r = (k * NT + (int)threadIdx.x) / CPR;
      mrow[h][k] = min(row0 + h * TM + r, g.M - 1);
      offs[h][k] = rowmap(mrow[h][k]) * g.ldc + ncl;
      xz[h][k] = old[h][k] = make_uint4(0u, 0u, 0u, 0u);
      mbv[h][k] = 0xFFu;
    }
  if constexpr (BNB) {
#pragma unroll
    for (int h = 0; h < WM; ++h)
#pragma unroll
      for (int k = 0; k < KI; ++k) xz[h][k] = *(const uint4*)(cg.bnb_x + offs[h][k]);
    if (cg.bnb_mask) {
#pragma unroll
      for (int h = 0; h < WM; ++h)
#pragma unroll
        for (int k = 0; k < KI; ++k) mbv[h][k] = cg.bnb_mask[(int64_t)mrow[h][k] * (g.N >> 3) + (ncl >> 3)];
    }
  }
  if (g.accumulate) {
#pragma unroll
    for (int h = 0; h < WM; ++h)
#pragma unroll
      for (int k = 0; k < KI; ++k) old[h][k] = *(const uint4*)((const uint16_t*)g.c + offs[h][k]);
  }
#pragma unroll
  for (int h = 0; h < WM; ++h) {
    lds_barrier();  // operand stages (h = 0) / the previous slice's image (h > 0) are dead
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          *(f32x4*)(img + (i * 16 + (lane & 15)) * LS + wn * TN + j * 16 + 4 * (lane >> 4)) = acc[i][j];
    }
    lds_barrier();
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int r = (k * NT + (int)threadIdx.x) / CPR;
      const int m = row0 + h * TM + r, n = col0 + cc;
      if (m >= g.M || n >= g.N) continue;  // N % 8 == 0: a chunk is all in or all out
      const int64_t off = rowmap(m) * g.ldc + n;
      unsigned mb = mbv[h][k];
      if constexpr (BNB) {
        if constexpr (BNX) {  // [relu(x*scale + shift) > 0], the fp32 expression of the forward's prologue
          const uint32_t px[4] = {xz[h][k].x, xz[h][k].y, xz[h][k].z, xz[h][k].w};
          mb = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = (e & 1) ? hi16t<H>(px[e >> 1]) : lo16t<H>(px[e >> 1]);
            mb |= (__builtin_fmaf(x, qa[e], qb[e]) > 0.f ? 1u : 0u) << e;
          }
        }
      }
      const f32x4 a = *(const f32x4*)(img + r * LS + cc), b = *(const f32x4*)(img + r * LS + cc + 4);
      float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
      uint16_t* dst = (uint16_t*)g.c + off;
      if (g.accumulate) {
        const uint32_t po[4] = {old[h][k].x, old[h][k].y, old[h][k].z, old[h][k].w};
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          v[2 * w] += lo16t<H>(po[w]);
          v[2 * w + 1] += hi16t<H>(po[w]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ((mb >> e) & 1u) ? v[e] : 0.f;
      const uint32_t pk[4] = {pack16t<H>(v[0], v[1]), pack16t<H>(v[2], v[3]), pack16t<H>(v[4], v[5]),
                              pack16t<H>(v[6], v[7])};
      if constexpr (BNB) {
        const uint32_t px[4] = {xz[h][k].x, xz[h][k].y, xz[h][k].z, xz[h][k].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = (e & 1) ? hi16t<H>(px[e >> 1]) : lo16t<H>(px[e >> 1]);
          const float rr = (e & 1) ? hi16t<H>(pk[e >> 1]) : lo16t<H>(pk[e >> 1]);
          s1[e] += rr;
          s2[e] = __builtin_fmaf(rr, (x - mu[e]) * is[e], s2[e]);
        }
      }
      if (cg.st_nt) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u32x4{pk[0], pk[1], pk[2], pk[3]}, (u32x4*)dst);
      } else {
        *(uint4*)dst = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      }
    }
  }
  if constexpr (BNB) {
    // lanes sharing the chunk column: lane % CPR equal
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    constexpr int NW = WM * WN;
    float* red = img;  // [NW][2][BN]
    lds_barrier();     // the last slice's image is dead
    const int w = (int)threadIdx.x >> 6;
    if (lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(w * 2) * BN + cc + e] = s1[e];
        red[(w * 2 + 1) * BN + cc + e] = s2[e];
      }
    }
    lds_barrier();
    for (int t = (int)threadIdx.x; t < 2 * BN; t += NT) {
      const int which = t / BN, c = t % BN;
      if (col0 + c >= g.N) continue;
      float u = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) u += red[(ww * 2 + which) * BN + c];
      cg.bnb_part[((int64_t)tm * 2 + which) * g.N + col0 + c] = u;
    }
  }
}

// 16x16x32 MFMA on 16-bit operands held as raw bits: bf16 or (H) fp16
template <bool H>
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (H) {
    typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
}

// dX row of sub-grid pixel m of a strided-dgrad parity class
struct ClsRow {
  int GH, GW, H, W, py, px;
  __device__ __forceinline__ int64_t operator()(int m) const {
    const int gj = m % GW, t = m / GW;
    const int gi = t % GH, n = t / GH;
    return ((int64_t)n * H + 2 * gi + py) * W + 2 * gj + px;
  }
};

// H: fp16 operands (MFMA f16; storage / rounding by g.c_dt), else bf16
// BK x NS: k-tile depth x LDS ring slots (NS - 1 k-tiles in flight while one is consumed); OCC:
// resident blocks per CU the register budget is sized for
// PRO: BatchNorm-apply prologue on the gathered operand (forward A / wgrad B; ConvGeom::pro_ss):
// that operand is loaded into registers one k-tile ahead (together with the other operand's DMA),
// transformed after the current k-tile's MFMAs and written into the free ring slot with ds_write_b128
template <int MODE, int BM, int BN, int WM, int WN, bool H, int BK = 64, int NS = 2, int OCC = 2, bool PRO = false>
__global__ void __launch_bounds__(64 * WM * WN, OCC * WM * WN / 4) conv_kernel(MArgs g, const ConvGeom cg0) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16, KK = BK / 32;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr bool FWD = MODE == kConvFwd || MODE == kConvFwdC8;
  constexpr bool AK = MODE == kConvWgrad;   // A K-major (dY read pixel-major)
  constexpr bool BKM = !FWD;                // B K-major (dgrad: W per tap; wgrad: gathered X)
  constexpr int NL = (BM + BN) * BK / (512 * NW);  // LDS-DMA instructions per wave per k-tile
  static_assert(NS * STAGE_BYTES >= (BM / WM) * (BN + 4) * 4, "the LDS epilogue image fits in the ring");
  // PRO on the stride-1 dgrad: its BatchNorm epilogue recomputes the ReLU mask (ConvGeom::bnb_ss)
  static_assert(!PRO || ((MODE == kConvFwd || MODE == kConvWgrad || MODE == kConvDgrad) && NS == 2),
                "prologue: fwd / wgrad / BNB dgrad, 2-slot ring");
  constexpr bool PL = PRO && MODE != kConvDgrad;  // an operand goes through registers
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE_BYTES];
  __shared__ __attribute__((aligned(16))) float pro_tab[PL ? 2 * kProMaxC : 4];  // [scale C][shift C]

  if (cg0.tr_blocks) {  // appended blocks: the deferred split-K combine (independent of the tiles)
    const int nmain = (int)gridDim.x - cg0.tr_blocks;
    if ((int)blockIdx.x >= nmain) {
      if (cg0.tr_g4)
        reduce_slabs<4>(cg0.tr_slab, cg0.tr_splitk, cg0.tr_M, cg0.tr_N, nullptr, cg0.tr_c, F32, cg0.tr_N, cg0.tr_acc,
                        (int)blockIdx.x - nmain, cg0.tr_blocks, 64 * NW);
      else
        reduce_slabs<1>(cg0.tr_slab, cg0.tr_splitk, cg0.tr_M, cg0.tr_N, nullptr, cg0.tr_c, F32, cg0.tr_N, cg0.tr_acc,
                        (int)blockIdx.x - nmain, cg0.tr_blocks, 64 * NW);
      return;
    }
  }
  int lin = xcd_remap(blockIdx.x, (int)gridDim.x - cg0.tr_blocks);
  ConvGeom cg = cg0;
  int r0y = 0, r0x = 0;
  ClsRow crow = {};
  if constexpr (MODE == kConvDgradS) {  // find this block's parity class; specialise the geometry
    // constant-index field selects only: a runtime index into the argument struct (or a select of
    // whole structs) puts the geometry in scratch memory
    // classes interleaved block by block (class = lin % ncls): every XCD's share of the grid mixes
    // the heavy classes (most taps) with the light ones (1x1 stride 2: three classes of zeros)
    const int c = lin % cg0.ncls;
    lin /= cg0.ncls;
#define RK_SEL(f) (c == 0 ? cg0.cls[0].f : c == 1 ? cg0.cls[1].f : c == 2 ? cg0.cls[2].f : cg0.cls[3].f)
    g.M = RK_SEL(M); g.K = RK_SEL(K); g.k_per_split = g.K;
    cg.GH = RK_SEL(GH); cg.GW = RK_SEL(GW); cg.S = RK_SEL(Sv); cg.hoff = RK_SEL(hoff); cg.woff = RK_SEL(woff);
    r0y = RK_SEL(r0y); r0x = RK_SEL(r0x);
    crow = ClsRow{cg.GH, cg.GW, cg0.dx_h, cg0.dx_w, RK_SEL(py), RK_SEL(px)};
#undef RK_SEL
  }
  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  if (MODE == kConvDgradS && lin >= ntiles) return;  // this class has fewer tiles than the largest
  const int split = lin / ntiles;
  const int tile = lin % ntiles;
  int tm, tn;
  grouped_tile(tile, tiles_m, tiles_n, g.tgroup, tm, tn);
  const int row0 = tm * BM, col0 = tn * BN;
  const int kb = split * g.k_per_split;
  const int ke = min(g.K, kb + g.k_per_split);
  const int nt = (ke - kb + BK - 1) / BK;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const char* zero = (const char*)g_mgemm_zero;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // operand stagers per mode
  GatherRows<BM, BK, NW, MODE == kConvFwd ? kConvFwd : kConvDgrad> ga;  // fwd/dgrad A
  GatherRowsC8<BM, BK, NW> ga8;                                            // stem fwd A (C = 8)
  Stager<BM, BK, true, NW> sa_k;                                      // wgrad A (dY K-major)
  Stager<BN, BK, false, NW> sb_row;                                    // fwd B (W rows)
  Stager<BN, BK, true, NW> sb_k;                                       // dgrad B (W per tap)
  GatherCols<BN, BK, NW> gb;                                           // wgrad B
  if constexpr (MODE == kConvWgrad) {
    sa_k.init(g.lda, row0, g.M, wid, lane);
    gb.init(cg, col0, g.N, kb, wid, lane);
  } else if constexpr (MODE == kConvFwdC8) {
    ga8.init(cg, row0, g.M, wid, lane);
    sb_row.init(g.ldb, col0, g.N, wid, lane);
  } else {
    ga.init(g.a, cg, row0, g.M, wid, lane);
    if constexpr (MODE == kConvFwd) sb_row.init(g.ldb, col0, g.N, wid, lane);
    else sb_k.init(g.ldb, col0, g.N, wid, lane);
  }

  // prologue operand of the k-tile in flight (registers), its padding flags and channel offset
  constexpr int PNI = MODE == kConvWgrad ? GatherCols<BN, BK, NW>::NI : GatherRows<BM, BK, NW, kConvFwd>::NI;
  u32x4 pv[PNI];
  uint32_t pok = 0;
  int pc0 = 0;
  if constexpr (PL) {
    for (int i = (int)threadIdx.x; i < 2 * cg.C; i += 64 * NW) pro_tab[i] = cg.pro_ss[i];
    __syncthreads();
  }
  auto issue = [&](int t) {
    char* buf = smem + (t % NS) * STAGE_BYTES;
    const int k0 = kb + t * BK;
    if constexpr (MODE == kConvWgrad) {
      // (prologue: the register loads first, so the DMAs after them are the only vm ops a wait for
      // the registers has to let through)
      if constexpr (PL) gb.load(g.b, cg, ke, zero, pv, pok);
      if (k0 + BK <= ke) sa_k.issue((const char*)g.a + (int64_t)k0 * g.lda * 2, buf, wid);
      else sa_k.issue_tail((const char*)g.a + (int64_t)k0 * g.lda * 2, buf, wid, lane, ke - k0, zero);
      if constexpr (!PL) gb.issue(g.b, cg, ke, buf + A_BYTES, wid, zero);  // k-tiles are issued in order: its rows are k0..
    } else if constexpr (MODE == kConvFwdC8) {
      ga8.issue(g.a, cg, k0, buf, wid, zero);
      sb_row.issue((const char*)g.b + (int64_t)k0 * 2, buf + A_BYTES, wid);
    } else {
      const int tap = k0 / cg.taps_c, c0 = k0 - tap * cg.taps_c;
      const int tr = tap / cg.S, ts = tap - tr * cg.S;
      if constexpr (PL) {
        ga.load(cg, tr, ts, c0, zero, pv, pok);
        pc0 = c0;
      } else {
        ga.issue(cg, tr, ts, c0, buf, wid, zero);
      }
      if constexpr (MODE == kConvFwd)
        sb_row.issue((const char*)g.b + (int64_t)k0 * 2, buf + A_BYTES, wid);
      else {  // W[co][tap][ci]: k-tile rows co = c0.., columns ci (strided: the class's tap (j, l))
        const int wtap = MODE == kConvDgradS ? (r0y + 2 * tr) * cg.w_s + r0x + 2 * ts : tap;
        sb_k.issue((const char*)g.b + ((int64_t)wtap * cg.w_tap_stride + (int64_t)c0 * cg.w_co_stride) * 2,
                   buf + A_BYTES, wid);
      }
    }
  };
  FragReader<BM, BK, AK, FM> ra;
  FragReader<BN, BK, BKM, FN> rb;
  ra.init(wm * TM, lane);
  rb.init(wn * TN, lane);

  const bool want_rows = g.rowsum != nullptr && tn == 0;
  constexpr int FR = (FM + WN - 1) / WN;
  f32x4 racc[FR];
#pragma unroll
  for (int i = 0; i < FR; ++i) racc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;  // 1.0 in the operand format
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = __builtin_bit_cast(__bf16, (uint16_t)(H ? 0x3C00u : 0x3F80u));

  // PRO: the registers of k-tile t, transformed, into its slot
  auto put = [&](int t) {
    char* buf = smem + (t % NS) * STAGE_BYTES;
    if constexpr (MODE == kConvWgrad) gb.template put<H>(buf + A_BYTES, wid, lane, pv, pok, pro_tab, cg.C);
    else ga.template put<H>(buf, wid, lane, pv, pok, pro_tab, cg.C, pc0);
  };

  // prologue: NS - 1 k-tiles in flight
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nt) issue(t);
  if constexpr (PL) {
    if (nt > 0) put(0);
  }
  for (int t = 0; t < nt; ++t) {
    // tile t has landed once at most the tiles issued after it (up to t + NS - 2) are outstanding
    // (PRO: its DMA'd operand; the register-staged one was written by put(t) — waited for here)
    wait_vm(PL ? 0 : (min(nt - 1, t + NS - 2) - t) * NL);
    if constexpr (PL) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // every wave's share of tile t is in LDS and every wave has consumed tile t - 1: refill its
    // slot with tile t + NS - 1
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + NS - 1 < nt) issue(t + NS - 1);
    const char* As = smem + (t % NS) * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = rb.get(Bs, j, kk);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = ra.get(As, i, kk);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma16<H>(bfr[j], af[i], acc[i][j]);
      if (want_rows) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
          if (i % WN == wn) racc[i / WN] = mfma16<H>(ones, af[i], racc[i / WN]);
      }
    }
    if constexpr (PL) {
      if (t + 1 < nt) put(t + 1);
    }
  }
  if (want_rows && lane < 16) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = row0 + wm * TM + i * 16 + lane;
      if (i % WN == wn && m < g.M) atomicAdd(g.rowsum + m, racc[i / WN][0]);
    }
  }
  if constexpr (FWD) {
    if (cg.bnpart != nullptr) tile_bn_stats<BM, BN, WM, WN, FM, FN, H>(g, cg, acc, tm, row0, col0, wm, wn, lane);
  }
  const uint2 nos[FM][FN] = {};
  if constexpr (MODE == kConvDgradS) {
    if (g.lds_epi)
      store_tile_lds<BM, BN, WM, WN, FM, FN, false, H>(g, cg, acc, smem, row0, col0, tm, wm, wn, lane, crow);
    else
      store_tile<FM, FN, false, ClsRow>(g, acc, nos, row0 + wm * TM, col0 + wn * TN, lane, split, crow);
    if (cg0.zero_nb && !g.accumulate) {  // classes without taps: zeros next to this tile's pixels
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = col0 + wn * TN + j * 16 + 4 * (lane >> 4);
        if (n >= g.N) continue;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = row0 + wm * TM + i * 16 + (lane & 15);
          if (m >= g.M) continue;
          const int gj = m % crow.GW, t = m / crow.GW;
          const int gi = t % crow.GH, img = t / crow.GH;
          const int64_t p0 = ((int64_t)img * crow.H + 2 * gi) * crow.W + 2 * gj;
          const bool right = 2 * gj + 1 < crow.W, down = 2 * gi + 1 < crow.H;
          uint16_t* c = (uint16_t*)g.c + n;
          if (right) *(uint2*)(c + (p0 + 1) * g.ldc) = make_uint2(0u, 0u);
          if (down) *(uint2*)(c + (p0 + crow.W) * g.ldc) = make_uint2(0u, 0u);
          if (right && down) *(uint2*)(c + (p0 + crow.W + 1) * g.ldc) = make_uint2(0u, 0u);
        }
      }
    }
  } else if (MODE == kConvDgrad && cg.bnb_x != nullptr) {
    store_tile_lds<BM, BN, WM, WN, FM, FN, true, H, IdRow, PRO>(g, cg, acc, smem, row0, col0, tm, wm, wn, lane, IdRow());
  } else if (MODE != kConvWgrad && g.lds_epi) {
    store_tile_lds<BM, BN, WM, WN, FM, FN, false, H>(g, cg, acc, smem, row0, col0, tm, wm, wn, lane, IdRow());
  } else
    store_tile<FM, FN, false>(g, acc, nos, row0 + wm * TM, col0 + wn * TN, lane, split);
}

// tiles of a launch: one GEMM, or (strided dgrad) the parity classes' GEMMs back to back
template <int MODE>
int conv_tiles(const MArgs& g, const ConvGeom& cg, int bm, int bn) {
  if constexpr (MODE == kConvDgradS) {  // classes interleaved: ncls x the largest class's tiles
    int t = 0;
    for (int c = 0; c < cg.ncls; ++c) t = std::max(t, ((cg.cls[c].M + bm - 1) / bm) * ((g.N + bn - 1) / bn));
    return t * cg.ncls;
  }
  return ((g.M + bm - 1) / bm) * ((g.N + bn - 1) / bn);
}

int g_conv_cfg = 0;  // rk_conv_set_cfg: k-tile pipeline of the bf16 kernels

// The deferred split-K combine of the last rk_conv_wgrad (rk_conv_defer_reduce(1)): the next conv
// launch on the same stream runs it in appended blocks (the stride-1 dgrad of the same backward:
// iconv.py issues the wgrad first), rk_conv_flush_reduce launches it on its own otherwise.  One
// launch and its ~5 us floor fewer per ResNet conv backward, the combine overlapping the dgrad's
// last wave.  Host-side state, one pending job (the backward issues its launches in order).
struct TailJob {
  const float* slab = nullptr;
  float* c = nullptr;
  int splitk = 0, M = 0, N = 0, acc = 0;
  hipStream_t s = nullptr;
  bool pending = false;
};
TailJob g_tail;
int g_defer_reduce = 0;
int64_t g_tail_attached = 0, g_tail_flushed = 0;  // rk_conv_tail_counts (tests)

void attach_tail(ConvGeom& cg, hipStream_t s, int nt) {
  cg.tr_blocks = 0;
  if (!g_tail.pending || g_tail.s != s) return;
  const int64_t nq = (int64_t)g_tail.M * g_tail.N / 4;
  const int G = g_tail.splitk >= 8 ? 4 : 1;
  cg.tr_slab = g_tail.slab; cg.tr_c = g_tail.c; cg.tr_splitk = g_tail.splitk;
  cg.tr_M = g_tail.M; cg.tr_N = g_tail.N; cg.tr_acc = g_tail.acc; cg.tr_g4 = G == 4;
  cg.tr_blocks = (int)std::max<int64_t>(1, std::min<int64_t>((nq * G + nt - 1) / nt, 1024));
  g_tail.pending = false;
  ++g_tail_attached;
}

template <int MODE, bool H, int BK, int NS, int OCC, int WN128 = 4, bool PRO = false>
int launch_conv_p(const MArgs& g, const ConvGeom& cg_in, hipStream_t s) {
  // (the forward's wave row slice is 64 pixels in every variant: the BatchNorm partials rely on it)
  // 64-wide GEMM side (Cout / Cin = 64 layers): a 64-wide tile with 4 waves instead of half an
  // empty 128-wide one; everything else 128 x 128 with 8 waves
  ConvGeom cg = cg_in;
  if (MODE != kConvWgrad && g.N <= 64) {
    const int tiles = conv_tiles<MODE>(g, cg, 128, 64);
    attach_tail(cg, s, 256);
    conv_kernel<MODE, 128, 64, 2, 2, H, BK, NS, OCC, PRO><<<tiles * g.splitk + cg.tr_blocks, 256, 0, s>>>(g, cg);
  } else if (MODE == kConvWgrad && g.M <= 64) {
    const int tiles = ((g.M + 63) / 64) * ((g.N + 127) / 128);
    attach_tail(cg, s, 256);
    conv_kernel<MODE, 64, 128, 2, 2, H, BK, NS, OCC, PRO><<<tiles * g.splitk + cg.tr_blocks, 256, 0, s>>>(g, cg);
  } else {
    const int tiles = conv_tiles<MODE>(g, cg, 128, 128);
    attach_tail(cg, s, 128 * WN128);
    conv_kernel<MODE, 128, 128, 2, WN128, H, BK, NS, OCC, PRO>
        <<<tiles * g.splitk + cg.tr_blocks, 128 * WN128, 0, s>>>(g, cg);
  }
  return (int)hipGetLastError();
}

template <int MODE, bool H>
int launch_conv_t(const MArgs& g, ConvGeom cg, hipStream_t s) {
  if constexpr (MODE == kConvFwd || MODE == kConvWgrad || MODE == kConvDgrad) {
    if (cg.pro_ss || cg.bnb_ss) return launch_conv_p<MODE, H, 64, 2, 2, 4, true>(g, cg, s);  // the default pipeline only
  }
  if constexpr (!H) {
    switch (g_conv_cfg) {
      case 1: return launch_conv_p<MODE, H, 64, 3, 1>(g, cg, s);
      case 2: return launch_conv_p<MODE, H, 32, 4, 2>(g, cg, s);
      case 3: return launch_conv_p<MODE, H, 32, 3, 3>(g, cg, s);
      case 4: return launch_conv_p<MODE, H, 64, 2, 2, 2>(g, cg, s);
      case 5: return launch_conv_p<MODE, H, 32, 3, 3, 2>(g, cg, s);
      default: break;
    }
  }
  return launch_conv_p<MODE, H, 64, 2, 2>(g, cg, s);
}
// operand dtype dt: BF16 or F16 (anything else is refused by the entry points)
template <int MODE>
int launch_conv(const MArgs& g, ConvGeom cg, int dt, hipStream_t s) {
  return dt == F16 ? launch_conv_t<MODE, true>(g, cg, s) : launch_conv_t<MODE, false>(g, cg, s);
}

ConvGeom geom(int N, int H, int W, int C, int GH, int GW, int R, int S, int stride, int pad, int taps_c) {
  ConvGeom cg;
  cg.N = N; cg.H = H; cg.W = W; cg.C = C; cg.GH = GH; cg.GW = GW;
  cg.R = R; cg.S = S; cg.stride = stride; cg.pad = pad; cg.taps_c = taps_c;
  cg.w_tap_stride = 0; cg.w_co_stride = 0; cg.bnpart = nullptr;
  cg.bnb_x = nullptr; cg.bnb_mask = nullptr; cg.bnb_mean = nullptr; cg.bnb_invstd = nullptr; cg.bnb_part = nullptr;
  cg.pro_ss = nullptr; cg.bnb_ss = nullptr;
  cg.hoff = cg.woff = pad; cg.dx_h = cg.dx_w = 0; cg.w_s = S; cg.ncls = 0; cg.zero_nb = 0;
  cg.tr_slab = nullptr; cg.tr_c = nullptr;
  cg.tr_splitk = cg.tr_M = cg.tr_N = cg.tr_acc = cg.tr_blocks = cg.tr_g4 = 0;
  // the tile's outputs stream to HBM (ResNet activations are far larger than L2) and their next
  // reader is another launch: nontemporal stores (ROCKET_CONV_NT=0: plain)
  static const int nt = getenv("ROCKET_CONV_NT") ? atoi(getenv("ROCKET_CONV_NT")) : 1;
  cg.st_nt = nt;
  cg.inv_gw = 1.f / (float)GW;
  cg.inv_gh = 1.f / (float)GH;
  cg.inv_s = 1.f / (float)S;
  return cg;
}

int g_tile_group = 4;  // rk_conv_set_tile_group: tile-rows per group of the conv tile walk (1: row-major)

MArgs margs(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int c_dt, int64_t ldc, int M, int N,
            int K) {
  MArgs g = {};
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.M = M; g.N = N; g.K = K; g.c_dt = c_dt;
  g.splitk = 1; g.k_per_split = K;
  g.tgroup = g_tile_group;
  return g;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int g_lds_epi = 1;  // rk_conv_set_lds_epi
// rk_conv_set_bn_prologue: [2][C] scale / shift for the NEXT rk_conv_fwd / rk_conv_wgrad /
// rk_conv_dgrad_bn call on this host thread (consumed by it)
thread_local const float* g_pro_ss = nullptr;
const float* take_pro() {
  const float* p = g_pro_ss;
  g_pro_ss = nullptr;
  return p;
}

}  // namespace

// Operand dtype `dt` (every entry point below): BF16 or F16 — X, W, dY and the 16-bit outputs all
// in that format (MFMA bf16 / f16, f32 accumulation).
static bool dt_ok(int dt) { return dt == BF16 || dt == F16; }

// Y[N*OH*OW][Cout] (dt or f32) = conv(X, W) (+ bias[Cout]).  Cin % 64 == 0, Cout % 8 == 0, R*S <= 32.
// bnpart (optional): f32 [ceil(N*OH*OW / 64)][2][Cout] per 64-pixel slice (sum, sum of squares)
// BatchNorm partials for rk_bn_finalize.
RK_API int rk_conv_fwd(int dt, const void* x, const void* w, void* y, int y_dt, const float* bias, int N, int H, int W,
                       int Cin, int Cout, int R, int S, int stride, int pad, int OH, int OW, float* bnpart,
                       hipStream_t s) {
  const float* pro = take_pro();
  if (!dt_ok(dt) || (y_dt != F32 && y_dt != dt)) return (int)hipErrorInvalidValue;
  if (pro && (Cin > kProMaxC || !aligned16(pro))) return (int)hipErrorInvalidValue;
  if (Cin % 64 || Cout % 8 || R * S > 32 || !aligned16(x) || !aligned16(w) || !aligned16(y)) return (int)hipErrorInvalidValue;
  if (OH != (H + 2 * pad - R) / stride + 1 || OW != (W + 2 * pad - S) / stride + 1) return (int)hipErrorInvalidValue;
  const int M = N * OH * OW, K = R * S * Cin;
  MArgs g = margs(x, 0, w, K, y, y_dt, Cout, M, Cout, K);
  g.bias = bias;
  g.lds_epi = g_lds_epi && y_dt != F32 && bias == nullptr;
  ConvGeom cg = geom(N, H, W, Cin, OH, OW, R, S, stride, pad, Cin);
  cg.bnpart = bnpart;
  cg.pro_ss = pro;
  return launch_conv<kConvFwd>(g, cg, dt, s);
}

// Stem conv on a channel-padded image: X8 [N][H][W][8] (image channels + zeros), W8 [Cout][Kp]
// with the taps' 8 channels in (r, s, c) order and Kp = R*S*8 rounded up to 64 (zero pad
// columns).  Otherwise as rk_conv_fwd (Y in dt, BatchNorm partials).
RK_API int rk_conv_fwd_c8(int dt, const void* x8, const void* w8, void* y, int N, int H, int W, int Cout, int R,
                          int S, int stride, int pad, int OH, int OW, float* bnpart, hipStream_t s) {
  if (!dt_ok(dt) || Cout % 8 || !aligned16(x8) || !aligned16(w8) || !aligned16(y) || R * S > 4096) return (int)hipErrorInvalidValue;
  if (OH != (H + 2 * pad - R) / stride + 1 || OW != (W + 2 * pad - S) / stride + 1) return (int)hipErrorInvalidValue;
  const int M = N * OH * OW, Kp = (R * S * 8 + 63) / 64 * 64;
  MArgs g = margs(x8, 0, w8, Kp, y, dt, Cout, M, Cout, Kp);
  g.lds_epi = g_lds_epi;
  ConvGeom cg = geom(N, H, W, 8, OH, OW, R, S, stride, pad, 8);
  cg.bnpart = bnpart;
  return launch_conv<kConvFwdC8>(g, cg, dt, s);
}

// Image [N][C][H][W] in any memory layout (element (n, c, pixel) at n*sn + c*sc + pixel*sp; C <= 8,
// 2-byte elements) -> [N][H][W][8] with zero channels C..7 (the stem operand of rk_conv_fwd_c8 /
// rk_conv_wgrad): one pixel per thread, one 16-byte store.  Reads NCHW batches directly, so the
// image needs no channels_last copy first.
__global__ void __launch_bounds__(256) pad_c8_kernel(const uint16_t* __restrict__ x, uint4* __restrict__ y,
                                                     int64_t pixels, int hw, int C, int64_t sn, int64_t sc, int64_t sp) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= pixels) return;
  const int64_t n = p / hw, q = p - n * hw;
  const uint16_t* src = x + n * sn + q * sp;
  uint16_t v[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) v[c] = c < C ? src[c * sc] : (uint16_t)0;
  y[p] = make_uint4((uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                    (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16));
}

RK_API int rk_pad_c8(const void* x, void* y, int N, int C, int H, int W, int64_t sn, int64_t sc, int64_t sp,
                     hipStream_t s) {
  if (C < 1 || C > 8 || !aligned16(y)) return (int)hipErrorInvalidValue;
  const int64_t pixels = (int64_t)N * H * W;
  if (pixels <= 0) return 0;
  pad_c8_kernel<<<(unsigned)((pixels + 255) / 256), 256, 0, s>>>((const uint16_t*)x, (uint4*)y, pixels, H * W, C,
                                                                  sn, sc, sp);
  return (int)hipGetLastError();
}

// dX[N*H*W][Cin] (bf16/f32) (+)= conv_transpose(dY, W), stride 1 or 2.  Cout % 64 == 0, Cin % 8 == 0.
// accumulate: dX += (e.g. the residual-branch gradient already in dX).  Stride 2: the four parity
// classes of dX pixels as four stride-1 gathers in one launch (classes without taps store zeros).
// 1 (default): bf16 forward / input-gradient tiles are stored through LDS in row-contiguous 16-byte
// chunks; 0: straight from the MFMA accumulator layout (A/B switch, ROCKET_CONV_LDS_EPI)
// BatchNorm-apply prologue of the next conv call on this host thread (see g_pro_ss): the gathered
// input X (fwd / wgrad) is the BatchNorm's input z and the conv reads relu(z*scale + shift),
// ss = [2][Cin] f32 (scale, shift; Cin <= 512); rk_conv_dgrad_bn: the ReLU mask from bn_x and ss
RK_API int rk_conv_set_bn_prologue(const float* ss) {
  g_pro_ss = ss;
  return 0;
}
RK_API int rk_conv_set_tile_group(int gh) {
  g_tile_group = gh < 1 ? 1 : gh;
  return 0;
}
RK_API int rk_conv_set_lds_epi(int on) {
  g_lds_epi = on != 0;
  return 0;
}

// k-tile pipeline of the bf16 conv kernels: 0 = 64-deep k-tiles, 2-slot ring, 2 blocks/CU;
// 1 = 64-deep, 3 slots, 1 block/CU; 2 = 32-deep, 4 slots, 2 blocks/CU; 3 = 32-deep, 3 slots, 3 blocks/CU;
// 4 / 5 = 0 / 3 with 4-wave 128 x 128 tiles (64 x 64 per wave: half the LDS reads per MFMA)
RK_API int rk_conv_set_cfg(int cfg) {
  if (cfg < 0 || cfg > 5) return (int)hipErrorInvalidValue;
  g_conv_cfg = cfg;
  return 0;
}

// Stride-1 dX of a conv whose input is a BatchNorm(+ReLU) output, fused with that BatchNorm's
// backward reduction: dX' = relu-mask * dX (+ old dX) is stored (bf16) and part (f32
// [ceil(N*H*W / 128)][2][Cin]) receives per-128-pixel (sum dX', sum dX' * (x - mean) * invstd) for
// rk_bn_bwd_partials.  mask may be null (BatchNorm without ReLU).
RK_API int rk_conv_dgrad_bn(int dt, const void* dy, const void* w, void* dx, int accumulate, int N, int H, int W,
                            int Cin, int Cout, int R, int S, int pad, const void* bn_x, const void* bn_mask,
                            const float* mean, const float* invstd, float* part, hipStream_t s) {
  const float* pro = take_pro();
  if (pro && (bn_mask || !aligned16(pro))) return (int)hipErrorInvalidValue;
  if (!dt_ok(dt) || Cout % 64 || Cin % 8 || R * S > 32 || !aligned16(dy) || !aligned16(w) || !aligned16(dx) || !aligned16(bn_x) || !part ||
      !aligned16(mean) || !aligned16(invstd) || !aligned16(part))
    return (int)hipErrorInvalidValue;
  const int OH = H + 2 * pad - R + 1, OW = W + 2 * pad - S + 1;
  if (OH <= 0 || OW <= 0) return (int)hipErrorInvalidValue;
  const int M = N * H * W, K = R * S * Cout;
  MArgs g = margs(dy, 0, w, (int64_t)R * S * Cin, dx, dt, Cin, M, Cin, K);
  g.accumulate = accumulate;
  ConvGeom cg = geom(N, OH, OW, Cout, H, W, R, S, 1, pad, Cout);
  cg.w_tap_stride = Cin;
  cg.w_co_stride = (int64_t)R * S * Cin;
  cg.bnb_x = (const uint16_t*)bn_x;
  cg.bnb_mask = (const uint8_t*)bn_mask;
  cg.bnb_mean = mean;
  cg.bnb_invstd = invstd;
  cg.bnb_part = part;
  cg.bnb_ss = pro;
  return launch_conv<kConvDgrad>(g, cg, dt, s);
}

RK_API int rk_conv_dgrad(int dt, const void* dy, const void* w, void* dx, int dx_dt, int accumulate, int N, int H,
                         int W, int Cin, int Cout, int R, int S, int stride, int pad, int OH, int OW, hipStream_t s) {
  if (!dt_ok(dt) || (dx_dt != F32 && dx_dt != dt)) return (int)hipErrorInvalidValue;
  if ((stride != 1 && stride != 2) || Cout % 64 || Cin % 8 || R * S > 32 || !aligned16(dy) || !aligned16(w) || !aligned16(dx))
    return (int)hipErrorInvalidValue;
  if (OH != (H + 2 * pad - R) / stride + 1 || OW != (W + 2 * pad - S) / stride + 1) return (int)hipErrorInvalidValue;
  const int M = N * H * W, K = R * S * Cout;
  MArgs g = margs(dy, 0, w, (int64_t)R * S * Cin, dx, dx_dt, Cin, M, Cin, K);
  g.accumulate = accumulate;
  g.lds_epi = g_lds_epi && dx_dt != F32;
  ConvGeom cg = geom(N, OH, OW, Cout, H, W, R, S, stride, pad, Cout);
  cg.w_tap_stride = Cin;
  cg.w_co_stride = (int64_t)R * S * Cin;
  if (stride == 1) return launch_conv<kConvDgrad>(g, cg, dt, s);
  cg.dx_h = H;
  cg.dx_w = W;
  cg.ncls = 0;
  for (int py = 0; py < 2; ++py)
    for (int px = 0; px < 2; ++px) {
      DgCls k = {};
      k.py = py; k.px = px;
      k.GH = (H - py + 1) / 2;
      k.GW = (W - px + 1) / 2;
      k.r0y = (py + pad) & 1;
      k.r0x = (px + pad) & 1;
      const int rv = k.r0y < R ? (R - k.r0y + 1) / 2 : 0, sv = k.r0x < S ? (S - k.r0x + 1) / 2 : 0;
      k.Sv = sv > 0 ? sv : 1;
      k.hoff = (py + pad - k.r0y) / 2;
      k.woff = (px + pad - k.r0x) / 2;
      k.M = N * k.GH * k.GW;
      k.K = rv * sv * Cout;
      if (k.M > 0 && k.K > 0) cg.cls[cg.ncls++] = k;
    }
  // a 1x1 kernel (pad 0) leaves three classes without taps: class (0, 0)'s tiles zero them (a
  // tile launch per zero class measured ~3x slower than the whole GEMM)
  if (R == 1 && S == 1 && pad == 0) {
    if (cg.ncls != 1 || dx_dt == F32) return (int)hipErrorInvalidValue;
    cg.zero_nb = 1;
  } else if (cg.ncls != 4) {
    return (int)hipErrorInvalidValue;  // every class must have taps (or be zeroed by its neighbour)
  }
  return launch_conv<kConvDgradS>(g, cg, dt, s);
}

// dW[Cout][R*S*Cin] f32 (+)= dY^T (*) X; split-K over the N*OH*OW pixels into `slab`
// (splitk*Cout*R*S*Cin floats) + one combine launch.  Cin % 8 == 0, Cout % 8 == 0.
// db (optional, f32 [Cout]) += column sums of dY (the bias gradient) from the same launch.
RK_API int rk_conv_wgrad(int dt, const void* dy, const void* x, float* dw, int accumulate, float* db, int N, int H,
                         int W, int Cin, int Cout, int R, int S, int stride, int pad, int OH, int OW, int splitk,
                         float* slab, hipStream_t s) {
  const float* pro = take_pro();
  if (!dt_ok(dt) || Cin % 8 || Cout % 8 || !aligned16(dy) || !aligned16(x)) return (int)hipErrorInvalidValue;
  if (pro && (Cin > kProMaxC || !aligned16(pro))) return (int)hipErrorInvalidValue;
  const int P = N * OH * OW, Ncol = R * S * Cin;
  MArgs g = margs(dy, Cout, x, 0, dw, F32, Ncol, Cout, Ncol, P);
  g.rowsum = db;
  g.accumulate = accumulate;
  if (splitk < 1) splitk = 1;
  int kps = ((P + 63) / 64 + splitk - 1) / splitk * 64;
  splitk = (P + kps - 1) / kps;
  if (splitk > 1 && slab == nullptr) return (int)hipErrorInvalidValue;
  g.splitk = splitk;
  g.k_per_split = kps;
  g.slab = slab;
  ConvGeom cg = geom(N, H, W, Cin, OH, OW, R, S, stride, pad, Cin);
  cg.pro_ss = pro;
  int rc = launch_conv<kConvWgrad>(g, cg, dt, s);
  if (rc || splitk == 1) return rc;
  if (g_defer_reduce) {  // the next conv launch on this stream (or rk_conv_flush_reduce) combines
    g_tail.slab = slab; g_tail.c = dw; g_tail.splitk = splitk; g_tail.M = Cout; g_tail.N = Ncol;
    g_tail.acc = accumulate; g_tail.s = s; g_tail.pending = true;
    return 0;
  }
  launch_mgemm_reduce(slab, splitk, Cout, Ncol, nullptr, dw, F32, Ncol, accumulate, s);
  return (int)hipGetLastError();
}

// 1: the next rk_conv_wgrad leaves its split-K combine to the following conv launch (TailJob)
RK_API int rk_conv_defer_reduce(int on) {
  g_defer_reduce = on;
  return 0;
}

// deferred combines run by a conv launch's appended blocks / flushed on their own, since load
RK_API int rk_conv_tail_counts(int64_t* out) {
  out[0] = g_tail_attached;
  out[1] = g_tail_flushed;
  return 0;
}

// launch a still-pending deferred combine on its own (no-op when a conv launch took it)
RK_API int rk_conv_flush_reduce(hipStream_t s) {
  if (!g_tail.pending) return 0;
  g_tail.pending = false;
  ++g_tail_flushed;
  launch_mgemm_reduce(g_tail.slab, g_tail.splitk, g_tail.M, g_tail.N, nullptr, g_tail.c, F32, g_tail.N, g_tail.acc,
                      g_tail.s);
  (void)s;
  return (int)hipGetLastError();
}
