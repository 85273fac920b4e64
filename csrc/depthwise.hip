// Depthwise convolution (groups == channels) on bf16 NHWC — SURVEY §2.7 K6 (MobileNet V1
// R/MobileNet/pytorch/models/mobilenet_v1.py:109-133, Keras DepthwiseConv2D in
// R/MobileNet/tensorflow/models/mobilenet_v1.py:7-25).
//
// Depthwise conv has no reduction over channels, so there is nothing for MFMA to do: it is a
// bandwidth-bound stencil and every kernel here is built to touch each byte of HBM once:
//   * one thread = 8 consecutive channels (16-B vectors) x a strip of QT output pixels along W;
//     per filter row the strip's input columns ((QT-1)*SW + KS of them) are loaded ONCE and
//     feed every (output, tap) pair that uses them (compile-time stride SW: no divisions);
//   * the filter taps of the thread's 8 channels live in registers (fp32 master weights read
//     directly: no bf16 weight-prep launch);
//   * 2-D grid: blockIdx.y = a slab of up to 64 x 8 channels (one wave-width of vectors per
//     pixel), blockIdx.x = a range of pixel strips, so every layer (32 channels @112 to 1024
//     channels @7) launches a few thousand blocks;
//   * forward epilogue: bias, ReLU / LeakyReLU and per-channel BatchNorm partial statistics
//     (LDS reduction over the block's strips, channel-contiguous atomics into the shards);
//   * dgrad: stride 1 = the forward stencil with the filter flipped; stride 2 = a gather whose
//     output-parity pattern is uniform per launch (QT even), unrolled per parity;
//   * wgrad: per-thread KS*KS x 8 partials over the strips, per-tap LDS reduction, one
//     channel-contiguous atomic row per tap per block (256-B coalesced atomic rows).
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;
constexpr int SLAB = 64;  // channel groups (of 8) per block slab

DV_DEVICE void ld8(const u16* p, float* v) {
  uint4 r = *reinterpret_cast<const uint4*>(p); uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = bf2f(w[i] & 0xffff); v[2 * i + 1] = bf2f(w[i] >> 16); }
}
DV_DEVICE void st8(u16* p, const float* v) {
  uint4 r; r.x = pack2bf(v[0], v[1]); r.y = pack2bf(v[2], v[3]); r.z = pack2bf(v[4], v[5]); r.w = pack2bf(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = r;
}

struct DwGeo {
  int N, H, W, C, ldx, P, Q, ldy, sh, sw, ph, pw;
  FastDiv fd_strips, fd_rows;  // strip decode: strip -> (row index, strip in row) -> (image, row)
};

// Packed-fp32 forms (v_pk_fma_f32 / v_pk_add_f32: two channels per VALU instruction; the strip
// kernels are VALU-issue-bound -- 1,760 VALU per wave for 128 outputs on the 112x112x32 forward
// before, profiles/pmc_dw_*): a 16-B bf16 vector unpacks to 4 channel pairs
typedef float f32x2 __attribute__((ext_vector_type(2)));
DV_DEVICE void ld8p(const u16* p, f32x2* v) {
  const uint4 r = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = f32x2{__uint_as_float(w[i] << 16), __uint_as_float(w[i] & 0xffff0000u)};
}
DV_DEVICE void st8p(u16* p, const f32x2* v) {
  uint4 r; r.x = pack2bf(v[0].x, v[0].y); r.y = pack2bf(v[1].x, v[1].y); r.z = pack2bf(v[2].x, v[2].y); r.w = pack2bf(v[3].x, v[3].y);
  *reinterpret_cast<uint4*>(p) = r;
}
DV_DEVICE f32x2 pfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// Fused BatchNorm-backward reduction in a depthwise dgrad epilogue (the dgrad output is the
// incoming gradient of the BatchNorm that feeds this depthwise conv, MobileNet's pw -> BN -> ReLU
// -> dw): sum dz and sum dz*(x - mean) of the STORED bf16 gradient, dz = act'(x*scale + shift)*d
// (mode 2) or d (mode 1) -- what csrc/bn.hip bn_bwd_reduce would read back -- into the BN's
// [SHARDS][2][C] accumulator (the invstd factor is applied once per channel at the end).
struct DwBnr {
  const u16* x;       // BN input, dense NHWC like dx
  const float* prm;   // [4][C]: scale, shift, mean, invstd
  float* acc;         // [SHARDS][2][C]
  int mode, act;      // mode 1: no activation, 2: mask recomputed from x
  float slope;
  float* det = nullptr;  // deterministic mode: per-block slab rows (kernels.h DetStats)
};
struct DwBnrLane {  // this thread's 8 channels
  f32x2 ms[4], mh[4], mu[4], s[4], q[4];
  DV_DEVICE void init(const DwBnr& b, int C, int c0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + 2 * k;
      ms[k] = f32x2{b.prm[c], b.prm[c + 1]};
      mh[k] = f32x2{b.prm[C + c], b.prm[C + c + 1]};
      mu[k] = f32x2{b.prm[2 * C + c], b.prm[2 * C + c + 1]};
      s[k] = f32x2{0.f, 0.f}; q[k] = f32x2{0.f, 0.f};
    }
  }
  // v: the 8 fp32 gradient values about to be stored; xr: the BN input at the same element
  // offset, loaded when the strip started (a load issued here would stall every strip on a
  // full memory round trip)
  DV_DEVICE void add(const DwBnr& b, const f32x2* v, const uint4& xr) {
    f32x2 xv[4];
    const uint32_t w[4] = {xr.x, xr.y, xr.z, xr.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) xv[i] = f32x2{__uint_as_float(w[i] << 16), __uint_as_float(w[i] & 0xffff0000u)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x2 d{bf2f(f2bf(v[k].x)), bf2f(f2bf(v[k].y))};  // the bf16 value the store writes
      if (b.mode == 2) {
        const f32x2 z = pfma(xv[k], ms[k], mh[k]);
        const f32x2 neg = b.act == 2 ? d * b.slope : f32x2{0.f, 0.f};
        d.x = z.x > 0.f ? d.x : neg.x;
        d.y = z.y > 0.f ? d.y : neg.y;
      }
      s[k] += d;
      q[k] = pfma(d, xv[k] - mu[k], q[k]);
    }
  }
};
// block-wide: [NT][8] lanes -> per-channel sums of the slab -> one coalesced atomic row per block
DV_DEVICE void bnr_commit(const DwBnr& b, const DwBnrLane& l, int C, int tpr, int rpi, float* sh0, float* sh1) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    sh0[threadIdx.x * 8 + 2 * k] = l.s[k].x; sh0[threadIdx.x * 8 + 2 * k + 1] = l.s[k].y;
    sh1[threadIdx.x * 8 + 2 * k] = l.q[k].x; sh1[threadIdx.x * 8 + 2 * k + 1] = l.q[k].y;
  }
  __syncthreads();
  const int sw = tpr * 8;
  float* a = stat_row(b.acc, b.det, blockIdx.x, C);
  const int cbase = (int)blockIdx.y * SLAB * 8;
  for (int ch = threadIdx.x; ch < sw; ch += NT) {
    float s1v = 0.f, s2v = 0.f;
    for (int rr = 0; rr < rpi; ++rr) { s1v += sh0[rr * sw + ch]; s2v += sh1[rr * sw + ch]; }
    atomicAdd(a + cbase + ch, s1v);
    atomicAdd(a + C + cbase + ch, s2v * b.prm[3 * C + cbase + ch]);  // sum dz*(x-mean) * invstd
  }
}

// thread -> (channel group, strip lane) inside the block's slab
struct DwTile {
  int tpr, rpi, lane_c, lane_r, cg, c0;
  DV_DEVICE DwTile(int C) {
    const int cgn = C / 8, rem = cgn - (int)blockIdx.y * SLAB;
    tpr = rem < SLAB ? rem : SLAB;
    rpi = NT / tpr;
    lane_c = threadIdx.x % tpr; lane_r = threadIdx.x / tpr;
    cg = (int)blockIdx.y * SLAB + lane_c;
    c0 = cg * 8;
  }
  DV_DEVICE bool active() const { return lane_r < rpi; }
};

// ---------------------------------------------------------------- forward (and stride-1 dgrad)
// FLIP: correlate with the spatially flipped filter (dgrad of a stride-1 conv); then the caller
// passes the flipped padding KS-1-p and the output grid is the input grid.
template <int KS, int SW, int QT, bool FLIP, int OCC = 1, bool BNR = false>
__global__ __launch_bounds__(NT, OCC) void dw_fwd_kernel(const u16* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ bias, u16* __restrict__ y, DwGeo g,
                                                      int act, float slope, float* __restrict__ stats,
                                                      int strips_per_block, DwBnr bnr, float* __restrict__ sdet) {
  __shared__ float sh[2][NT * 8];
  DwTile t(g.C);
  DwBnrLane bl;
  if constexpr (BNR) bl.init(bnr, g.C, t.c0);
  constexpr int NCOL = (QT - 1) * SW + KS;
  f32x2 wr[KS * KS][4];
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int wt = FLIP ? KS * KS - 1 - tp : tp;
      wr[tp][k] = f32x2{w[(t.c0 + 2 * k) * KS * KS + wt], w[(t.c0 + 2 * k + 1) * KS * KS + wt]};
    }
  f32x2 bv[4], ssum[4], ssq[4], nkq[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    bv[k] = bias ? f32x2{bias[t.c0 + 2 * k], bias[t.c0 + 2 * k + 1]} : f32x2{0.f, 0.f};
    ssum[k] = f32x2{0.f, 0.f}; ssq[k] = f32x2{0.f, 0.f};
    // shifted statistics (bn.hip): sums of (v - K)
    nkq[k] = stats ? -f32x2{stat_shift(stats, g.C)[t.c0 + 2 * k], stat_shift(stats, g.C)[t.c0 + 2 * k + 1]}
                   : f32x2{0.f, 0.f};
  }
  const int qstrips = (g.Q + QT - 1) / QT;
  const int nstrips = g.N * g.P * qstrips;
  const int s0 = blockIdx.x * strips_per_block, s1 = min(nstrips, s0 + strips_per_block);
  if (t.active()) {
    for (int s = s0 + t.lane_r; s < s1; s += t.rpi) {
      const int np = (int)fdiv((uint32_t)s, g.fd_strips);
      const int qs = s - np * qstrips;
      const int n = (int)fdiv((uint32_t)np, g.fd_rows);
      const int p = np - n * g.P;
      const int q0 = qs * QT;
      uint4 bx[BNR ? QT : 1];
      if constexpr (BNR) {
#pragma unroll
        for (int i = 0; i < QT; ++i) {
          const int qq = min(q0 + i, g.Q - 1);
          bx[i] = *reinterpret_cast<const uint4*>(bnr.x + (((int64_t)n * g.P + p) * g.Q + qq) * g.ldy + t.c0);
        }
      }
      f32x2 acc[QT][4];
#pragma unroll
      for (int i = 0; i < QT; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[i][k] = bv[k];
      // every load is unconditional: out-of-image taps read the zero page (a branch around a
      // load makes hipcc wait for it on the spot -- one serial HBM round trip per tap)
#pragma unroll
      for (int r = 0; r < KS; ++r) {
        const int h = p * g.sh - g.ph + r;
        const bool hv = h >= 0 && h < g.H;
        const u16* xrow = x + ((int64_t)n * g.H + (hv ? h : 0)) * g.W * g.ldx + t.c0;
        const int wbase = q0 * SW - g.pw;
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          const int ww = wbase + j;
          const bool ok = hv && ww >= 0 && ww < g.W;
          f32x2 v[4];
          ld8p(ok ? xrow + (int64_t)ww * g.ldx : reinterpret_cast<const u16*>(dv_zero_page), v);
#pragma unroll
          for (int i = 0; i < QT; ++i) {
            const int sx = j - i * SW;  // compile-time
            if (sx >= 0 && sx < KS) {
#pragma unroll
              for (int k = 0; k < 4; ++k) acc[i][k] = pfma(v[k], wr[r * KS + sx][k], acc[i][k]);
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < QT; ++i) {
        const int q = q0 + i;
        if (q >= g.Q) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          f32x2 v = acc[i][k];
          if (act == 1) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); }
          else if (act == 2) { v.x = v.x > 0.f ? v.x : v.x * slope; v.y = v.y > 0.f ? v.y : v.y * slope; }
          acc[i][k] = v;
          const f32x2 d = v + nkq[k];
          ssum[k] += d; ssq[k] = pfma(d, d, ssq[k]);
        }
        const int64_t off = (((int64_t)n * g.P + p) * g.Q + q) * g.ldy + t.c0;
        st8p(y + off, acc[i]);
        if constexpr (BNR) bl.add(bnr, acc[i], bx[i]);
      }
    }
  }
  if constexpr (BNR) {
    bnr_commit(bnr, bl, g.C, t.tpr, t.rpi, sh[0], sh[1]);
    return;
  }
  if (stats) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sh[0][threadIdx.x * 8 + 2 * k] = ssum[k].x; sh[0][threadIdx.x * 8 + 2 * k + 1] = ssum[k].y;
      sh[1][threadIdx.x * 8 + 2 * k] = ssq[k].x; sh[1][threadIdx.x * 8 + 2 * k + 1] = ssq[k].y;
    }
    __syncthreads();
    const int sw = t.tpr * 8;  // slab width in channels; sh is [strip lane][slab channel]
    float* a = stat_row(stats, sdet, blockIdx.x, g.C);
    const int cbase = (int)blockIdx.y * SLAB * 8;
    for (int ch = threadIdx.x; ch < sw; ch += NT) {
      float s1v = 0.f, s2v = 0.f;
      for (int rr = 0; rr < t.rpi; ++rr) { s1v += sh[0][rr * sw + ch]; s2v += sh[1][rr * sw + ch]; }
      atomicAdd(a + cbase + ch, s1v);
      atomicAdd(a + g.C + cbase + ch, s2v);
    }
  }
}

// ---------------------------------------------------------------- stride-2 dgrad
// dx[n][h][w][c] = sum over taps (r, s) with (h+ph-r), (w+pw-s) even of
//                  dy[n][(h+ph-r)/2][(w+pw-s)/2][c] * w[c][r][s]
// QT (even) consecutive w per thread: the parity of (w0 + pw) is the same for every thread, so
// each parity is a fully unrolled body with compile-time register indices.
// With B = w0 + pw = 2b + PAR, output i and tap s read q = (B + i - s) / 2 when B + i - s is
// even; relative to qb = floor((B - (KS-1)) / 2) that column is
//   j = ((PAR + i - s) >> 1) - ((PAR - KS + 1) >> 1)      (compile-time for a fixed PAR)
template <int KS, int QT, int PAR>
DV_DEVICE void dgrad2_row(const u16* __restrict__ dyrow, bool rv, int w0, const DwGeo& g, const f32x2 (*wr)[4],
                          int r, f32x2 (*acc)[4]) {
  const int qb = (w0 + g.pw - (KS - 1)) >> 1;  // arithmetic shift: floor for negatives too
  constexpr int J0 = (PAR - KS + 1) >> 1;
  constexpr int NQ = ((PAR + QT - 1) >> 1) - J0 + 1;
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    const int q = qb + j;
    f32x2 v[4];
    ld8p(rv && q >= 0 && q < g.Q ? dyrow + (int64_t)q * g.ldy : reinterpret_cast<const u16*>(dv_zero_page), v);
#pragma unroll
    for (int i = 0; i < QT; ++i)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (((PAR + i - s) & 1) == 0 && ((PAR + i - s) >> 1) - J0 == j) {
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[i][k] = pfma(v[k], wr[r * KS + s][k], acc[i][k]);
        }
      }
  }
}

template <int KS, int QT, int OCC = 1, bool BNR = false>
__global__ __launch_bounds__(NT, OCC) void dw_dgrad2_kernel(const u16* __restrict__ dy, const float* __restrict__ w,
                                                         u16* __restrict__ dx, DwGeo g, int strips_per_block, DwBnr bnr) {
  __shared__ float sh[BNR ? 2 : 1][BNR ? NT * 8 : 1];
  DwTile t(g.C);
  DwBnrLane bl;
  if constexpr (BNR) bl.init(bnr, g.C, t.c0);
  if (!t.active()) {
    if constexpr (BNR) bnr_commit(bnr, bl, g.C, t.tpr, t.rpi, sh[0], sh[1]);  // zero partials, joins the barrier
    return;
  }
  f32x2 wr[KS * KS][4];
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
    for (int k = 0; k < 4; ++k) wr[tp][k] = f32x2{w[(t.c0 + 2 * k) * KS * KS + tp], w[(t.c0 + 2 * k + 1) * KS * KS + tp]};
  const int wstrips = (g.W + QT - 1) / QT;
  const int nstrips = g.N * g.H * wstrips;
  const int s0 = blockIdx.x * strips_per_block, s1 = min(nstrips, s0 + strips_per_block);
  const int par = g.pw & 1;  // parity of w0 + pw (w0 is a multiple of the even QT)
  for (int s = s0 + t.lane_r; s < s1; s += t.rpi) {
    const int nh = (int)fdiv((uint32_t)s, g.fd_strips);
    const int ws = s - nh * wstrips;
    const int n = (int)fdiv((uint32_t)nh, g.fd_rows);
    const int h = nh - n * g.H;
    const int w0 = ws * QT;
    uint4 bx[BNR ? QT : 1];
    if constexpr (BNR) {
#pragma unroll
      for (int i = 0; i < QT; ++i)
        bx[i] = *reinterpret_cast<const uint4*>(bnr.x + (((int64_t)n * g.H + h) * g.W + min(w0 + i, g.W - 1)) * g.ldx + t.c0);
    }
    f32x2 acc[QT][4];
#pragma unroll
    for (int i = 0; i < QT; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[i][k] = f32x2{0.f, 0.f};
#pragma unroll
    for (int r = 0; r < KS; ++r) {
      const int hn = h + g.ph - r;
      const int p = hn >> 1;
      const bool rv = hn >= 0 && !(hn & 1) && p < g.P;  // invalid rows read the zero page
      const u16* dyrow = dy + ((int64_t)n * g.P + (rv ? p : 0)) * g.Q * g.ldy + t.c0;
      if (par == 0) dgrad2_row<KS, QT, 0>(dyrow, rv, w0, g, wr, r, acc);
      else dgrad2_row<KS, QT, 1>(dyrow, rv, w0, g, wr, r, acc);
    }
#pragma unroll
    for (int i = 0; i < QT; ++i)
      if (w0 + i < g.W) {
        const int64_t off = (((int64_t)n * g.H + h) * g.W + w0 + i) * g.ldx + t.c0;
        st8p(dx + off, acc[i]);
        if constexpr (BNR) bl.add(bnr, acc[i], bx[i]);
      }
  }
  if constexpr (BNR) bnr_commit(bnr, bl, g.C, t.tpr, t.rpi, sh[0], sh[1]);
}

// ---------------------------------------------------------------- wgrad
// dw[c][r][s] += sum_{n,p,q} dy[n][p][q][c] * x[n][p*sh-ph+r][q*SW-pw+s][c]
template <int KS, int SW, int QT, int OCC = 1>
__global__ __launch_bounds__(NT, OCC) void dw_wgrad_kernel(const u16* __restrict__ x, const u16* __restrict__ dy,
                                                        float* __restrict__ dw, DwGeo g, int strips_per_block,
                                                        float* __restrict__ slabs) {
  __shared__ float sh[NT * 8];
  __shared__ float red[SLAB * 8 * KS * KS];
  DwTile t(g.C);
  constexpr int NCOL = (QT - 1) * SW + KS;
  f32x2 acc2[KS * KS][4];
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc2[tp][k] = f32x2{0.f, 0.f};
  const int qstrips = (g.Q + QT - 1) / QT;
  const int nstrips = g.N * g.P * qstrips;
  const int s0 = blockIdx.x * strips_per_block, s1 = min(nstrips, s0 + strips_per_block);
  if (t.active()) {
    for (int s = s0 + t.lane_r; s < s1; s += t.rpi) {
      const int np = (int)fdiv((uint32_t)s, g.fd_strips);
      const int qs = s - np * qstrips;
      const int n = (int)fdiv((uint32_t)np, g.fd_rows);
      const int p = np - n * g.P;
      const int q0 = qs * QT;
      f32x2 d[QT][4];
#pragma unroll
      for (int i = 0; i < QT; ++i)
        ld8p(q0 + i < g.Q ? dy + (((int64_t)n * g.P + p) * g.Q + q0 + i) * g.ldy + t.c0
                          : reinterpret_cast<const u16*>(dv_zero_page), d[i]);
#pragma unroll
      for (int r = 0; r < KS; ++r) {
        const int h = p * g.sh - g.ph + r;
        const bool hv = h >= 0 && h < g.H;
        const u16* xrow = x + ((int64_t)n * g.H + (hv ? h : 0)) * g.W * g.ldx + t.c0;
        const int wbase = q0 * SW - g.pw;
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          const int ww = wbase + j;
          const bool ok = hv && ww >= 0 && ww < g.W;
          f32x2 v[4];
          ld8p(ok ? xrow + (int64_t)ww * g.ldx : reinterpret_cast<const u16*>(dv_zero_page), v);
#pragma unroll
          for (int i = 0; i < QT; ++i) {
            const int sx = j - i * SW;
            if (sx >= 0 && sx < KS) {
#pragma unroll
              for (int k = 0; k < 4; ++k) acc2[r * KS + sx][k] = pfma(d[i][k], v[k], acc2[r * KS + sx][k]);
            }
          }
        }
      }
    }
  }
  float acc[KS * KS][8];
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
    for (int k = 0; k < 4; ++k) { acc[tp][2 * k] = acc2[tp][k].x; acc[tp][2 * k + 1] = acc2[tp][k].y; }
  // per tap: strip lanes -> LDS -> per-channel sums into red[channel][tap]
  const int sw = t.tpr * 8;
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp) {
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[threadIdx.x * 8 + k] = acc[tp][k];
    __syncthreads();
    for (int ch = threadIdx.x; ch < sw; ch += NT) {
      float sum = 0.f;
      for (int rr = 0; rr < t.rpi; ++rr) sum += sh[rr * sw + ch];
      red[ch * KS * KS + tp] = sum;
    }
    __syncthreads();
  }
  // dw is [C][KS*KS]: the slab's block of sw*KS*KS floats is contiguous -> coalesced atomics.
  // Deterministic mode: this block's partial goes to its own [C][KS*KS] slab (row blockIdx.x),
  // summed in block order by dv_slab_reduce -- reproducible bits, no atomics.
  const int64_t coff = (int64_t)blockIdx.y * SLAB * 8 * KS * KS;
  if (slabs) {
    float* dst = slabs + (int64_t)blockIdx.x * g.C * KS * KS + coff;
    for (int e = threadIdx.x; e < sw * KS * KS; e += NT) dst[e] = red[e];
    return;
  }
  float* dst = dw + coff;
  for (int e = threadIdx.x; e < sw * KS * KS; e += NT) atomicAdd(dst + e, red[e]);
}


// ---------------------------------------------------------------- small planes (<= 14x14 outputs)
// One block = one image x 64 channels x the WHOLE output plane. The input window the plane needs
// ((P-1)*sh + KS rows x (Q-1)*SW + KS columns, zero outside the image) is staged once in LDS with
// 16-B loads issued all at once; every tap is then an LDS read. The strip kernels above re-read
// each input pixel ~4.5x through L1/L2 and, on 14x14 / 7x7 layers, ran at 1.2-2 TB/s
// (profiles/archive/dw_bench_r2.txt). Thread = 8 channels (cg = tid % 8) x output pixels pl, pl + 32, ...
constexpr int PL_CH = 64;              // channels per block
constexpr int PL_LANES = NT / 8;       // pixel lanes
constexpr int PLANE_MAX_OUT = 196;     // 14 x 14
inline int plane_win(int P, int s, int KS) { return (P - 1) * s + KS; }
inline size_t plane_lds(int P, int Q, int sh, int sw, int KS) {
  return (size_t)plane_win(P, sh, KS) * plane_win(Q, sw, KS) * PL_CH * 2;
}

template <int KS>
DV_DEVICE void plane_stage(const u16* __restrict__ x, const DwGeo& g, int n, int c0, u16* win, int WR, int WC) {
  const int total = WR * WC * 8;  // 16-B pieces
  for (int base = threadIdx.x; base < total; base += 8 * NT) {
    uint4 v[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {  // all loads in flight before the LDS writes
      const int i = min(base + b * NT, total - 1);
      const int pix = i >> 3, cg = i & 7;
      const int wr = pix / WC, wc = pix - wr * WC;
      const int h = wr - g.ph, w = wc - g.pw;
      const bool ok = h >= 0 && h < g.H && w >= 0 && w < g.W;
      const u16* src = ok ? x + (((int64_t)n * g.H + h) * g.W + w) * g.ldx + c0 + cg * 8
                          : reinterpret_cast<const u16*>(dv_zero_page);
      v[b] = *reinterpret_cast<const uint4*>(src);
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int i = base + b * NT;
      if (i < total) *reinterpret_cast<uint4*>(win + (int64_t)(i >> 3) * PL_CH + (i & 7) * 8) = v[b];
    }
  }
}

template <int KS, int SW, bool FLIP>
__global__ __launch_bounds__(NT) void dw_plane_fwd_kernel(const u16* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ bias, u16* __restrict__ y, DwGeo g,
                                                          int act, float slope, float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  u16* win = reinterpret_cast<u16*>(smem);
  const int slabs = g.C / PL_CH;
  const int n = blockIdx.x / slabs, c0 = (blockIdx.x - n * slabs) * PL_CH;
  const int WR = (g.P - 1) * g.sh + KS, WC = (g.Q - 1) * SW + KS;
  const int cg = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int c = c0 + cg * 8;
  float wr[KS * KS][8], bv[8], ssum[8], ssq[8], kq[8];
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
    for (int k = 0; k < 8; ++k) wr[tp][k] = w[(c + k) * KS * KS + (FLIP ? KS * KS - 1 - tp : tp)];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    bv[k] = bias ? bias[c + k] : 0.f;
    ssum[k] = 0.f; ssq[k] = 0.f;
    kq[k] = stats ? stat_shift(stats, g.C)[c + k] : 0.f;
  }
  plane_stage<KS>(x, g, n, c0, win, WR, WC);
  __syncthreads();
  const int npix = g.P * g.Q;
  for (int o = pl; o < npix; o += PL_LANES) {
    const int p = o / g.Q, q = o - p * g.Q;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = bv[k];
#pragma unroll
    for (int r = 0; r < KS; ++r)
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        float v[8];
        ld8(win + ((p * g.sh + r) * WC + q * SW + s2) * PL_CH + cg * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(v[k], wr[r * KS + s2][k], acc[k]);
      }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = acc[k];
      if (act == 1) v = fmaxf(v, 0.f);
      else if (act == 2) v = v > 0.f ? v : v * slope;
      acc[k] = v;
      const float d = v - kq[k];
      ssum[k] += d; ssq[k] = fmaf(d, d, ssq[k]);
    }
    st8(y + ((int64_t)n * npix + o) * g.ldy + c, acc);
  }
  if (!stats) return;
  // shifted BN partial statistics: the 32 pixel lanes of each channel meet in LDS (the window
  // is no longer read), one coalesced atomic row per block
  __syncthreads();
  float* sh = reinterpret_cast<float*>(smem);  // [2][PL_LANES][PL_CH]
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sh[pl * PL_CH + cg * 8 + k] = ssum[k];
    sh[PL_LANES * PL_CH + pl * PL_CH + cg * 8 + k] = ssq[k];
  }
  __syncthreads();
  if (threadIdx.x < 2 * PL_CH) {
    const int which = threadIdx.x / PL_CH, ch = threadIdx.x % PL_CH;
    float t = 0.f;
    for (int l = 0; l < PL_LANES; ++l) t += sh[which * PL_LANES * PL_CH + l * PL_CH + ch];
    atomicAdd(stats + (int64_t)(blockIdx.x % DV_STAT_SHARDS) * 2 * g.C + which * g.C + c0 + ch, t);
  }
}

// dw[c][r][s] += sum over the images of this block and the output plane of
//                dy[n][p][q][c] * x[n][p*sh - ph + r][q*SW - pw + s][c]
template <int KS, int SW>
__global__ __launch_bounds__(NT) void dw_plane_wgrad_kernel(const u16* __restrict__ x, const u16* __restrict__ dy,
                                                            float* __restrict__ dw, DwGeo g, int imgs_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  u16* win = reinterpret_cast<u16*>(smem);
  const int slabs = g.C / PL_CH;
  const int nb = blockIdx.x / slabs, c0 = (blockIdx.x - nb * slabs) * PL_CH;
  const int WR = (g.P - 1) * g.sh + KS, WC = (g.Q - 1) * SW + KS;
  const int cg = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int c = c0 + cg * 8;
  const int npix = g.P * g.Q;
  float acc[KS * KS][8];
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[tp][k] = 0.f;
  const int n0 = nb * imgs_per_block, n1 = min(g.N, n0 + imgs_per_block);
  for (int n = n0; n < n1; ++n) {
    __syncthreads();  // the previous image's window is no longer read
    plane_stage<KS>(x, g, n, c0, win, WR, WC);
    __syncthreads();
    for (int o = pl; o < npix; o += PL_LANES) {
      const int p = o / g.Q, q = o - p * g.Q;
      float d[8];
      ld8(dy + ((int64_t)n * npix + o) * g.ldy + c, d);
#pragma unroll
      for (int r = 0; r < KS; ++r)
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          float v[8];
          ld8(win + ((p * g.sh + r) * WC + q * SW + s2) * PL_CH + cg * 8, v);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[r * KS + s2][k] = fmaf(d[k], v[k], acc[r * KS + s2][k]);
        }
    }
  }
  // the 8 pixel lanes of a wave (lane bits 3-5) by butterfly, then the 4 waves in LDS
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int off = 8; off < 64; off <<= 1) acc[tp][k] += __shfl_xor(acc[tp][k], off, 64);
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][KS*KS][PL_CH]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < 8) {
#pragma unroll
    for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
      for (int k = 0; k < 8; ++k) red[(wv * KS * KS + tp) * PL_CH + cg * 8 + k] = acc[tp][k];
  }
  __syncthreads();
  // dw is [C][KS*KS]: this slab's block of PL_CH * KS*KS floats is contiguous
  for (int e = threadIdx.x; e < PL_CH * KS * KS; e += NT) {
    const int ch = e / (KS * KS), tp = e - ch * (KS * KS);
    float t = 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) t += red[(v * KS * KS + tp) * PL_CH + ch];
    atomicAdd(dw + (int64_t)(c0 + ch) * KS * KS + tp, t);
  }
}

template <int KS, int SW, bool FLIP>
bool plane_fwd(const void* x, const float* w, const float* bias, void* y, const DwGeo& g, int act, float slope,
               float* stats, hipStream_t st) {
  if constexpr (KS > 3) return false;  // the 5x5 / 7x7 filters' registers do not fit this layout
  const size_t lds = plane_lds(g.P, g.Q, g.sh, SW, KS);
  const size_t need = std::max(lds, stats ? (size_t)2 * PL_LANES * PL_CH * 4 : (size_t)0);
  if (g.C % PL_CH || g.P * g.Q > PLANE_MAX_OUT || need > 64 * 1024 || g.sh != SW) return false;
  dw_plane_fwd_kernel<KS, SW, FLIP><<<g.N * (g.C / PL_CH), NT, need, st>>>((const u16*)x, w, bias, (u16*)y, g, act,
                                                                              slope, stats);
  return true;
}
template <int KS, int SW>
bool plane_wgrad(const void* x, const void* dy, float* dw, const DwGeo& g, hipStream_t st) {
  if constexpr (KS > 3) return false;
  const size_t lds = std::max(plane_lds(g.P, g.Q, g.sh, SW, KS), (size_t)4 * KS * KS * PL_CH * 4);
  if (g.C % PL_CH || g.P * g.Q > PLANE_MAX_OUT || lds > 64 * 1024 || g.sh != SW) return false;
  const int slabs = g.C / PL_CH;
  // ~512 blocks: each adds its 64 x KS*KS tile into dw once
  const int ipb = std::max(1, (g.N * slabs + 511) / 512);
  const int nblk = (g.N + ipb - 1) / ipb;
  dw_plane_wgrad_kernel<KS, SW><<<nblk * slabs, NT, lds, st>>>((const u16*)x, (const u16*)dy, dw, g, ipb);
  return true;
}

// Benchmark override of (strip length QT, minimum waves per SIMD) for the 3x3 strip kernels:
// 0 = heuristic, 1 = (4, 4), 2 = (2, 4), 3 = (8, 2), 4 = (4, 2), 5 = (2, 2); 60 = LDS-tiled
// kernels everywhere (stride 1 and 2), 61 = the strip / plane kernels everywhere, 62 = tiled with 4 rows
// per thread.
int g_dw_variant = 0;

// ---------------------------------------------------------------- LDS-tiled stride 1 (fwd, dgrad)
// One block = one image x NG*8 channels x a tile of RB*TH output rows x TW output columns. The
// input halo ((RB*TH + KS-1) x (TW + KS-1) pixels x NG*8 channels, bf16) is staged ONCE by LDS-DMA
// (global_load_lds_dwordx4: no VGPR staging, the zero page for the padding, one piece = 16 B = 8
// channels of one pixel, pieces in (row, column, group) order so each 1-KB wave-instruction is 64
// consecutive pieces). Then thread = (8-channel group, output column of a row band) streams its TH
// output rows down the tile: every input row's KS columns are read from LDS once (ds_read_b128)
// and feed up to KS output rows held in registers. Per output and 8 channels: KS LDS reads, 4*KS
// unpacks and 4*KS*KS packed FMAs -- against the strip kernel's 4.5 global loads per output, each
// with its own bounds / 64-bit address VALU (1,368 VALU per wave there, VALU-issue- and
// latency-bound at 2-3 TB/s: profiles/pmc_dw_r5.txt).
//
// Stride 2 (STR = 2, forward and weight gradient): the halo is (RB*TH-1)*2 + KS rows x (TW-1)*2 + KS
// columns, and each staged row keeps its even input columns first and its odd ones after them (NE
// even positions): thread column c reads input columns 2c + s at positions c + s/2 (even s) and
// NE + c + s/2 (odd s), so the 16 lanes of one ds_read_b128 cycle hit 256 consecutive bytes.
struct DwTileGeo {
  int TW, RB, LCOLS, pieces, ncolt, nrowt, NE;
  FastDiv fd_lcols;
};
// LDS column position -> input column offset in the halo (the even / odd split of stride 2)
template <int STR>
DV_DEVICE int halo_col(int lc, int NE) {
  if constexpr (STR == 1) return lc;
  else return lc < NE ? 2 * lc : 2 * (lc - NE) + 1;
}
// input column offset s of a thread's window -> LDS position offset (from the thread's base c)
template <int STR>
DV_DEVICE int halo_pos(int s, int NE) {
  if constexpr (STR == 1) return s;
  else return (s & 1) ? NE + (s >> 1) : (s >> 1);
}

template <int KS, bool FLIP, bool BNR, int NG, int TH, int STR = 1>
__global__ __launch_bounds__(NT) void dw_tile_kernel(const u16* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ bias, u16* __restrict__ y, DwGeo g,
                                                     DwTileGeo tg, int act, float slope, float* __restrict__ stats,
                                                     DwBnr bnr, float* __restrict__ sdet) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CW = NG * 8;  // channels per block
  const int cb = (int)blockIdx.y * CW;
  const int ct = (int)blockIdx.x % tg.ncolt, rest = (int)blockIdx.x / tg.ncolt;
  const int rt = rest % tg.nrowt, n = rest / tg.nrowt;
  const int p0 = rt * tg.RB * TH, q0 = ct * tg.TW;
  const int h0 = p0 * STR - g.ph, w0 = q0 * STR - g.pw;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // ---- stage the halo: chunk k = pieces [64k, 64k + 64), one LDS-DMA wave-instruction ----
  {
    const u16* xb = x + (int64_t)n * g.H * g.W * g.ldx + cb;
    const int nchunks = (tg.pieces + 63) >> 6;
    for (int k = wid; k < nchunks; k += NT / 64) {
      const int piece = k * 64 + lane;
      const int pix = piece / NG, gi = piece & (NG - 1);
      const int lr = (int)fdiv((uint32_t)pix, tg.fd_lcols), lc = pix - lr * tg.LCOLS;
      const int h = h0 + lr, ww = w0 + halo_col<STR>(lc, tg.NE);
      const bool ok = piece < tg.pieces && (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
      const u16* src = ok ? xb + ((int64_t)h * g.W + ww) * g.ldx + gi * 8 : reinterpret_cast<const u16*>(dv_zero_page);
      __builtin_amdgcn_global_load_lds(GLB_PTR(src), LDS_PTR(smem + k * 1024), 16, 0, 0);
    }
  }
  const int gi = threadIdx.x & (NG - 1), pl = threadIdx.x / NG;
  const int band = pl / tg.TW, c = pl - band * tg.TW;
  const bool active = band < tg.RB;
  const int c0 = cb + gi * 8;
  f32x2 wr[KS * KS][4];
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int wt = FLIP ? KS * KS - 1 - tp : tp;
      wr[tp][k] = f32x2{w[(c0 + 2 * k) * KS * KS + wt], w[(c0 + 2 * k + 1) * KS * KS + wt]};
    }
  f32x2 bv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) bv[k] = bias ? f32x2{bias[c0 + 2 * k], bias[c0 + 2 * k + 1]} : f32x2{0.f, 0.f};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int q = q0 + c;
  const int pb = p0 + band * TH;  // first output row of this thread's band
  // BN input of the fused BN-backward reduction at this thread's outputs, in flight during the FMAs
  uint4 bxv[BNR ? TH : 1];
  if constexpr (BNR) {
#pragma unroll
    for (int i = 0; i < TH; ++i) {
      const bool ok = active && pb + i < g.P && q < g.Q;
      bxv[i] = ok ? *reinterpret_cast<const uint4*>(bnr.x + (((int64_t)n * g.P + pb + i) * g.Q + q) * g.ldy + c0)
                  : uint4{0u, 0u, 0u, 0u};
    }
  }
  f32x2 acc[TH][4];
#pragma unroll
  for (int i = 0; i < TH; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[i][k] = bv[k];
  if (active) {
    const char* rp = smem + ((band * TH * STR * tg.LCOLS + c) * NG + gi) * 16;
    const int rowb = tg.LCOLS * NG * 16;
#pragma unroll
    for (int ir = 0; ir < (TH - 1) * STR + KS; ++ir) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        f32x2 v[4];
        ld8p(reinterpret_cast<const u16*>(rp + halo_pos<STR>(s, tg.NE) * NG * 16), v);
#pragma unroll
        for (int r = 0; r < KS; ++r) {
          const int i = (ir - r) / STR;  // compile-time
          if (ir >= r && (ir - r) % STR == 0 && i < TH) {
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[i][k] = pfma(v[k], wr[r * KS + s][k], acc[i][k]);
          }
        }
      }
      rp += rowb;
    }
  }
  f32x2 ssum[4], ssq[4], nkq[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    ssum[k] = f32x2{0.f, 0.f}; ssq[k] = f32x2{0.f, 0.f};
    nkq[k] = stats ? -f32x2{stat_shift(stats, g.C)[c0 + 2 * k], stat_shift(stats, g.C)[c0 + 2 * k + 1]}
                   : f32x2{0.f, 0.f};
  }
  DwBnrLane bl;
  if constexpr (BNR) bl.init(bnr, g.C, c0);
  if (active && q < g.Q) {
#pragma unroll
    for (int i = 0; i < TH; ++i) {
      if (pb + i >= g.P) break;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f32x2 v = acc[i][k];
        if (act == 1) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); }
        else if (act == 2) { v.x = v.x > 0.f ? v.x : v.x * slope; v.y = v.y > 0.f ? v.y : v.y * slope; }
        acc[i][k] = v;
        if (stats) { const f32x2 d = v + nkq[k]; ssum[k] += d; ssq[k] = pfma(d, d, ssq[k]); }
      }
      st8p(y + (((int64_t)n * g.P + pb + i) * g.Q + q) * g.ldy + c0, acc[i]);
      if constexpr (BNR) bl.add(bnr, acc[i], bxv[i]);
    }
  }
  if (!stats && !BNR) return;
  // ---- per-channel block sums (the tile is no longer read) -> one coalesced atomic row ----
  __syncthreads();
  float* sh0 = reinterpret_cast<float*>(smem);
  float* sh1 = sh0 + NT * 8;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 a = BNR ? bl.s[k] : ssum[k], b = BNR ? bl.q[k] : ssq[k];
    sh0[pl * CW + gi * 8 + 2 * k] = a.x; sh0[pl * CW + gi * 8 + 2 * k + 1] = a.y;
    sh1[pl * CW + gi * 8 + 2 * k] = b.x; sh1[pl * CW + gi * 8 + 2 * k + 1] = b.y;
  }
  __syncthreads();
  if (threadIdx.x < CW) {
    const int ch = threadIdx.x;
    float s1v = 0.f, s2v = 0.f;
    for (int r = 0; r < NT / NG; ++r) { s1v += sh0[r * CW + ch]; s2v += sh1[r * CW + ch]; }
    if constexpr (BNR) {
      float* a = stat_row(bnr.acc, bnr.det, blockIdx.x, g.C);
      atomicAdd(a + cb + ch, s1v);
      atomicAdd(a + g.C + cb + ch, s2v * bnr.prm[3 * g.C + cb + ch]);  // sum dz*(x-mean) * invstd
    } else {
      float* a = stat_row(stats, sdet, blockIdx.x, g.C);
      atomicAdd(a + cb + ch, s1v);
      atomicAdd(a + g.C + cb + ch, s2v);
    }
  }
}

// Weight gradient on the same tiles: dw[c][r][s] += sum_{n,p,q} dy[n][p][q][c] * x[n][p-ph+r][q-pw+s][c].
// A block walks `tpb` tiles; per tile the x halo and the dy tile are staged by LDS-DMA, then the
// thread streams its column down the band: each input row's KS columns (read once) meet the dy of
// the KS output rows that use them (a rolling 3-row dy window in registers), into KS*KS x 8
// per-thread tap partials. One LDS reduction over the pixel lanes and one coalesced atomic row
// (or, deterministic mode, one slab row) per block.
template <int KS, int NG, int TH, int STR = 1>
__global__ __launch_bounds__(NT) void dw_tile_wgrad_kernel(const u16* __restrict__ x, const u16* __restrict__ dy,
                                                           float* __restrict__ dw, DwGeo g, DwTileGeo tg, int tpb,
                                                           float* __restrict__ slabs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CW = NG * 8;
  const int cb = (int)blockIdx.y * CW;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int gi = threadIdx.x & (NG - 1), pl = threadIdx.x / NG;
  const int band = pl / tg.TW, c = pl - band * tg.TW;
  const bool active = band < tg.RB;
  const int xchunks = (tg.pieces + 63) >> 6;
  const int dpieces = tg.RB * TH * tg.TW * NG, dchunks = (dpieces + 63) >> 6;
  char* dimg = smem + xchunks * 1024;
  const int ntiles = g.N * tg.nrowt * tg.ncolt;
  f32x2 acc[KS * KS][4];
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[tp][k] = f32x2{0.f, 0.f};
  const int t0 = (int)blockIdx.x * tpb, t1 = min(ntiles, t0 + tpb);
  for (int t = t0; t < t1; ++t) {
    const int ct = t % tg.ncolt, rest = t / tg.ncolt;
    const int rt = rest % tg.nrowt, n = rest / tg.nrowt;
    const int p0 = rt * tg.RB * TH, q0 = ct * tg.TW;
    const int h0 = p0 * STR - g.ph, w0 = q0 * STR - g.pw;
    if (t != t0) __syncthreads();  // the previous tile's LDS reads are done
    const u16* xb = x + (int64_t)n * g.H * g.W * g.ldx + cb;
    for (int k = wid; k < xchunks; k += NT / 64) {
      const int piece = k * 64 + lane;
      const int pix = piece / NG, pg = piece & (NG - 1);
      const int lr = (int)fdiv((uint32_t)pix, tg.fd_lcols), lc = pix - lr * tg.LCOLS;
      const int h = h0 + lr, ww = w0 + halo_col<STR>(lc, tg.NE);
      const bool ok = piece < tg.pieces && (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
      const u16* src = ok ? xb + ((int64_t)h * g.W + ww) * g.ldx + pg * 8 : reinterpret_cast<const u16*>(dv_zero_page);
      __builtin_amdgcn_global_load_lds(GLB_PTR(src), LDS_PTR(smem + k * 1024), 16, 0, 0);
    }
    const u16* db = dy + (int64_t)n * g.P * g.Q * g.ldy + cb;
    for (int k = wid; k < dchunks; k += NT / 64) {
      const int piece = k * 64 + lane;
      const int pix = piece / NG, pg = piece & (NG - 1);
      const int lr = pix / tg.TW, lc = pix - lr * tg.TW;
      const int p = p0 + lr, q = q0 + lc;
      const bool ok = piece < dpieces && p < g.P && q < g.Q;  // outside the output grid: zero gradient
      const u16* src = ok ? db + ((int64_t)p * g.Q + q) * g.ldy + pg * 8 : reinterpret_cast<const u16*>(dv_zero_page);
      __builtin_amdgcn_global_load_lds(GLB_PTR(src), LDS_PTR(dimg + k * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (STR != 1 && active) {
      // stride 2: the TH dy rows of the band in registers (TH <= 4), each input row meets the
      // (up to two) output rows whose taps reach it
      const char* xp = smem + ((band * TH * STR * tg.LCOLS + c) * NG + gi) * 16;
      const char* dp = dimg + ((band * TH * tg.TW + c) * NG + gi) * 16;
      const int xrowb = tg.LCOLS * NG * 16, drowb = tg.TW * NG * 16;
      f32x2 d[TH][4];
#pragma unroll
      for (int i = 0; i < TH; ++i) ld8p(reinterpret_cast<const u16*>(dp + i * drowb), d[i]);
#pragma unroll
      for (int ir = 0; ir < (TH - 1) * STR + KS; ++ir) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          f32x2 v[4];
          ld8p(reinterpret_cast<const u16*>(xp + halo_pos<STR>(s, tg.NE) * NG * 16), v);
#pragma unroll
          for (int r = 0; r < KS; ++r) {
            const int i = (ir - r) / STR;  // compile-time
            if (ir >= r && (ir - r) % STR == 0 && i < TH) {
#pragma unroll
              for (int k = 0; k < 4; ++k) acc[r * KS + s][k] = pfma(v[k], d[i][k], acc[r * KS + s][k]);
            }
          }
        }
        xp += xrowb;
      }
    } else if (active) {
      const char* xp = smem + ((band * TH * tg.LCOLS + c) * NG + gi) * 16;
      const char* dp = dimg + ((band * TH * tg.TW + c) * NG + gi) * 16;
      const int xrowb = tg.LCOLS * NG * 16, drowb = tg.TW * NG * 16;
      f32x2 d[KS][4];  // dy of output rows ir, ir-1, ..., ir-KS+1 (slot i % KS)
#pragma unroll
      for (int ir = 0; ir < TH + KS - 1; ++ir) {
        if (ir < TH) ld8p(reinterpret_cast<const u16*>(dp + ir * drowb), d[ir % KS]);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          f32x2 v[4];
          ld8p(reinterpret_cast<const u16*>(xp + s * NG * 16), v);
#pragma unroll
          for (int r = 0; r < KS; ++r) {
            const int i = ir - r;  // compile-time
            if (i >= 0 && i < TH) {
#pragma unroll
              for (int k = 0; k < 4; ++k) acc[r * KS + s][k] = pfma(v[k], d[i % KS][k], acc[r * KS + s][k]);
            }
          }
        }
        xp += xrowb;
      }
    }
  }
  // ---- per-tap sums over the pixel lanes (LDS, tap by tap) -> [CW][KS*KS] -> one row per block ----
  __syncthreads();
  float* sh = reinterpret_cast<float*>(smem);  // [NT/NG][CW]
  float* red = sh + NT * 8;                    // [CW][KS*KS]
#pragma unroll
  for (int tp = 0; tp < KS * KS; ++tp) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sh[pl * CW + gi * 8 + 2 * k] = acc[tp][k].x;
      sh[pl * CW + gi * 8 + 2 * k + 1] = acc[tp][k].y;
    }
    __syncthreads();
    if (threadIdx.x < CW) {
      float sum = 0.f;
      for (int r = 0; r < NT / NG; ++r) sum += sh[r * CW + threadIdx.x];
      red[threadIdx.x * KS * KS + tp] = sum;
    }
    __syncthreads();
  }
  const int64_t coff = (int64_t)cb * KS * KS;
  if (slabs) {
    float* dst = slabs + (int64_t)blockIdx.x * g.C * KS * KS + coff;
    for (int e = threadIdx.x; e < CW * KS * KS; e += NT) dst[e] = red[e];
    return;
  }
  for (int e = threadIdx.x; e < CW * KS * KS; e += NT) atomicAdd(dw + coff + e, red[e]);
}

inline DwTileGeo make_tile_geo(const DwGeo& g, int NG, int TH, int KS, int STR = 1) {
  const int PL = NT / NG;
  DwTileGeo tg{};
  tg.TW = std::min(g.Q, PL);
  tg.RB = PL / tg.TW;
  tg.LCOLS = (tg.TW - 1) * STR + KS;
  tg.NE = (tg.LCOLS + 1) / 2;
  tg.pieces = ((tg.RB * TH - 1) * STR + KS) * tg.LCOLS * NG;
  tg.ncolt = (g.Q + tg.TW - 1) / tg.TW;
  tg.nrowt = (g.P + tg.RB * TH - 1) / (tg.RB * TH);
  tg.fd_lcols = make_fastdiv((uint32_t)tg.LCOLS);
  return tg;
}

template <int KS, int NG, int TH, int STR = 1>
void tile_wgrad_launch(const void* x, const void* dy, float* dw, const DwGeo& g, hipStream_t st) {
  const DwTileGeo tg = make_tile_geo(g, NG, TH, KS, STR);
  const int ntiles = g.N * tg.nrowt * tg.ncolt, nslab = g.C / (NG * 8);
  // ~768 blocks (3 per CU): every block ends in KS*KS LDS reductions + one atomic row, so a block
  // walks several tiles
  const int tpb = std::max(1, (ntiles * nslab + 767) / 768);
  const dim3 grid((unsigned)((ntiles + tpb - 1) / tpb), (unsigned)nslab);
  const size_t xb = (size_t)((tg.pieces + 63) / 64) * 1024;
  const size_t db = (size_t)((tg.RB * TH * tg.TW * NG + 63) / 64) * 1024;
  const size_t lds = std::max(xb + db, (size_t)(NT * 8 + NG * 8 * KS * KS) * 4);
  float* ws = nullptr;
  const int64_t n = (int64_t)g.C * KS * KS;
  if (dv_deterministic()) ws = dv_slab_workspace((size_t)grid.x * n, st);
  dw_tile_wgrad_kernel<KS, NG, TH, STR><<<grid, NT, lds, st>>>((const u16*)x, (const u16*)dy, dw, g, tg, tpb, ws);
  if (ws) dv_slab_reduce(ws, dw, n, (int)grid.x, 1, st);
}

template <int KS, bool FLIP, int NG, int TH, int STR = 1>
void tile_launch(const void* x, const float* w, const float* bias, void* y, const DwGeo& g, int act, float slope,
                 float* stats, hipStream_t st, const DwBnr* bnr) {
  const DwTileGeo tg = make_tile_geo(g, NG, TH, KS, STR);
  const dim3 grid((unsigned)(g.N * tg.nrowt * tg.ncolt), (unsigned)(g.C / (NG * 8)));
  const size_t lds = std::max<size_t>((size_t)((tg.pieces + 63) / 64) * 1024, (size_t)2 * NT * 8 * 4);
  const DetStats det((bnr || stats) ? grid.x : 0, g.C, st);
  if (bnr) {
    DwBnr b = *bnr;
    b.det = det.slab;
    dw_tile_kernel<KS, FLIP, true, NG, TH, STR><<<grid, NT, lds, st>>>((const u16*)x, w, bias, (u16*)y, g, tg, act, slope,
                                                                  stats, b, nullptr);
    det.fold(bnr->acc);
  } else {
    dw_tile_kernel<KS, FLIP, false, NG, TH, STR><<<grid, NT, lds, st>>>((const u16*)x, w, bias, (u16*)y, g, tg, act, slope,
                                                                   stats, DwBnr{}, det.slab);
    det.fold(stats);
  }
}
// rows per thread: the candidate that covers P (in bands of RB rows) with the fewest idle rows
inline int tile_th(int P, int Q, int NG) {
  const int PL = NT / NG, TW = std::min(Q, PL), RB = PL / TW;
  int best = 8, waste = 1 << 30;
  for (int th : {8, 7, 4, 2}) {
    const int rows = RB * th, wst = (P + rows - 1) / rows * rows - P;
    if (wst < waste) { waste = wst; best = th; }
  }
  return best;
}
// stride 2: rows per thread (4 or 2) with the fewest idle rows whose tile fits `cap` bytes of LDS
// (the halo is ~4x the output tile); 0 = none fits
inline int tile_th2(const DwGeo& g, int NG, int KS, int cap, bool with_dy) {
  const int PL = NT / NG, TW = std::min(g.Q, PL), RB = PL / TW, LCOLS = (TW - 1) * 2 + KS;
  int best = 0, waste = 1 << 30;
  for (int th : {4, 2}) {
    const int rows = RB * th;
    const int lds = (((rows - 1) * 2 + KS) * LCOLS * NG + (with_dy ? rows * TW * NG : 0)) * 16;
    const int wst = (g.P + rows - 1) / rows * rows - g.P;
    if (lds <= cap && wst < waste) { waste = wst; best = th; }
  }
  return best;
}
template <int KS>
bool tile_fwd2(const void* x, const float* w, const float* bias, void* y, const DwGeo& g, int act, float slope,
               float* stats, hipStream_t st) {
  if constexpr (KS != 3) {
    return false;
  } else {
    if (g.sh != 2 || g.sw != 2 || g.ldx % 8 || g.ldy % 8) return false;
    const int NG = g.C % 64 == 0 ? 8 : (g.C % 32 == 0 ? 4 : 0);
    if (!NG) return false;
    const int th = tile_th2(g, NG, KS, 80 * 1024, false);
    if (NG == 8 && th == 4) { tile_launch<KS, false, 8, 4, 2>(x, w, bias, y, g, act, slope, stats, st, nullptr); return true; }
    if (NG == 8 && th == 2) { tile_launch<KS, false, 8, 2, 2>(x, w, bias, y, g, act, slope, stats, st, nullptr); return true; }
    if (NG == 4 && th == 4) { tile_launch<KS, false, 4, 4, 2>(x, w, bias, y, g, act, slope, stats, st, nullptr); return true; }
    if (NG == 4 && th == 2) { tile_launch<KS, false, 4, 2, 2>(x, w, bias, y, g, act, slope, stats, st, nullptr); return true; }
    return false;
  }
}
template <int KS>
bool tile_wgrad2(const void* x, const void* dy, float* dw, const DwGeo& g, hipStream_t st) {
  if constexpr (KS != 3) {
    return false;
  } else {
    if (g.sh != 2 || g.sw != 2 || g.ldx % 8 || g.ldy % 8) return false;
    const int NG = g.C % 64 == 0 ? 8 : (g.C % 32 == 0 ? 4 : 0);
    if (!NG) return false;
    const int th = tile_th2(g, NG, KS, 60 * 1024, true);
    if (NG == 8 && th == 4) { tile_wgrad_launch<KS, 8, 4, 2>(x, dy, dw, g, st); return true; }
    if (NG == 8 && th == 2) { tile_wgrad_launch<KS, 8, 2, 2>(x, dy, dw, g, st); return true; }
    if (NG == 4 && th == 4) { tile_wgrad_launch<KS, 4, 4, 2>(x, dy, dw, g, st); return true; }
    if (NG == 4 && th == 2) { tile_wgrad_launch<KS, 4, 2, 2>(x, dy, dw, g, st); return true; }
    return false;
  }
}

template <int KS, bool FLIP>
bool tile_fwd(const void* x, const float* w, const float* bias, void* y, const DwGeo& g, int act, float slope,
              float* stats, hipStream_t st, const DwBnr* bnr) {
  if constexpr (KS != 3) {
    return false;
  } else {
    if (g.sh != 1 || g.sw != 1 || g.ldx % 8 || g.ldy % 8) return false;
    const int NG = g.C % 64 == 0 ? 8 : (g.C % 32 == 0 ? 4 : 0);
    if (!NG) return false;
    const int th = g_dw_variant == 62 ? 4 : tile_th(g.P, g.Q, NG);
#define DW_TILE(NGV, THV) \
  if (NG == NGV && th == THV) { tile_launch<KS, FLIP, NGV, THV>(x, w, bias, y, g, act, slope, stats, st, bnr); return true; }
    DW_TILE(8, 8) DW_TILE(8, 7) DW_TILE(8, 4) DW_TILE(8, 2)
    DW_TILE(4, 8) DW_TILE(4, 7) DW_TILE(4, 4) DW_TILE(4, 2)
#undef DW_TILE
    return false;
  }
}

template <int KS>
bool tile_wgrad(const void* x, const void* dy, float* dw, const DwGeo& g, hipStream_t st) {
  if constexpr (KS != 3) {
    return false;
  } else {
    if (g.sh != 1 || g.sw != 1 || g.ldx % 8 || g.ldy % 8) return false;
    const int NG = g.C % 64 == 0 ? 8 : (g.C % 32 == 0 ? 4 : 0);
    if (!NG) return false;
    const int th = g_dw_variant == 62 ? 4 : tile_th(g.P, g.Q, NG);
#define DW_TILE(NGV, THV) \
  if (NG == NGV && th == THV) { tile_wgrad_launch<KS, NGV, THV>(x, dy, dw, g, st); return true; }
    DW_TILE(8, 8) DW_TILE(8, 7) DW_TILE(8, 4) DW_TILE(8, 2)
    DW_TILE(4, 8) DW_TILE(4, 7) DW_TILE(4, 4) DW_TILE(4, 2)
#undef DW_TILE
    return false;
  }
}

int64_t per_block(int64_t nstrips, int rpi, int slabs, int64_t target_blocks) {
  // ~target blocks in total over the slabs, a whole number of strip passes per block
  int64_t spb = std::max<int64_t>(rpi, (nstrips * slabs + target_blocks - 1) / target_blocks);
  return (spb + rpi - 1) / rpi * rpi;
}
// strip decode divisors of a launch: strips per row (rows = images x rows per image)
inline DwGeo with_strips(DwGeo g, int strips_per_row, int rows_per_img) {
  g.fd_strips = make_fastdiv((uint32_t)strips_per_row);
  g.fd_rows = make_fastdiv((uint32_t)rows_per_img);
  return g;
}
inline int slabs_of(int C) { return (C / 8 + SLAB - 1) / SLAB; }
inline int rpi_of(int C) {
  const int cgn = C / 8, tpr = cgn < SLAB ? cgn : SLAB;
  return NT / tpr;
}

template <int KS, int SW, bool FLIP, int QT, int OCC>
void fwd_launch(const void* x, const float* w, const float* bias, void* y, const DwGeo& g, int act, float slope,
                float* stats, int target, hipStream_t st, const DwBnr* bnr = nullptr) {
  const int slabs = slabs_of(g.C), rpi = rpi_of(g.C);
  const int64_t nstrips = (int64_t)g.N * g.P * ((g.Q + QT - 1) / QT);
  const int64_t spb = per_block(nstrips, rpi, slabs, target);
  const dim3 grid((unsigned)((nstrips + spb - 1) / spb), (unsigned)slabs);
  const DwGeo gs = with_strips(g, (g.Q + QT - 1) / QT, g.P);
  const DetStats det((bnr || stats) ? grid.x : 0, g.C, st);
  if (bnr) {
    DwBnr b = *bnr;
    b.det = det.slab;
    dw_fwd_kernel<KS, SW, QT, FLIP, OCC, true><<<grid, NT, 0, st>>>((const u16*)x, w, bias, (u16*)y, gs, act, slope,
                                                                     stats, (int)spb, b, nullptr);
    det.fold(bnr->acc);
  } else {
    dw_fwd_kernel<KS, SW, QT, FLIP, OCC><<<grid, NT, 0, st>>>((const u16*)x, w, bias, (u16*)y, gs, act, slope, stats,
                                                             (int)spb, DwBnr{}, det.slab);
    det.fold(stats);
  }
}
template <int KS, int SW, bool FLIP>
void fwd_variants(const void* x, const float* w, const float* bias, void* y, const DwGeo& g, int act, float slope,
                  float* stats, hipStream_t st, const DwBnr* bnr = nullptr) {
  // LDS-tiled for stride 1 down to 14x14 outputs (18-40 % faster than the strip kernel there); the
  // strip kernel keeps 7x7 (the 9x9 halo of a 7x7 tile costs more than it saves: profiles/dw_tile_r5.txt)
  const bool tiled = g_dw_variant == 60 || g_dw_variant == 62 || (g_dw_variant == 0 && g.P * g.Q >= 196);
  if (tiled && tile_fwd<KS, FLIP>(x, w, bias, y, g, act, slope, stats, st, bnr)) return;
  // stride 2 on LDS tiles (the even / odd split halo), every map size; variant 63 = strip kernel
  if constexpr (SW == 2 && !FLIP) {
    // measured no faster than the strip kernel on any MobileNet stride-2 layer (the strip kernel
    // already streams the big ones at ~4 TB/s; profiles/dw_tile_stride2.txt): variant 60 only
    if (!bnr && g_dw_variant == 60 && tile_fwd2<KS>(x, w, bias, y, g, act, slope, stats, st)) return;
  }
  if (bnr) return fwd_launch<KS, SW, FLIP, 4, 1>(x, w, bias, y, g, act, slope, stats, 4096, st, bnr);
  if constexpr (KS == 3) {
    switch (g_dw_variant) {
      case 1: return fwd_launch<KS, SW, FLIP, 4, 4>(x, w, bias, y, g, act, slope, stats, 8192, st);
      case 2: return fwd_launch<KS, SW, FLIP, 2, 4>(x, w, bias, y, g, act, slope, stats, 8192, st);
      case 3: return fwd_launch<KS, SW, FLIP, 8, 2>(x, w, bias, y, g, act, slope, stats, 4096, st);
      case 4: return fwd_launch<KS, SW, FLIP, 4, 2>(x, w, bias, y, g, act, slope, stats, 8192, st);
      case 5: return fwd_launch<KS, SW, FLIP, 2, 2>(x, w, bias, y, g, act, slope, stats, 8192, st);
      default: break;
    }
  }
  // the whole-plane forward measured no faster on 14x14 and slower on 7x7 outputs than the strip
  // kernel (profiles/archive/dw_bench_r3.txt): benchmark variant 51 only
  if (g_dw_variant == 51 && !dv_deterministic() && plane_fwd<KS, SW, FLIP>(x, w, bias, y, g, act, slope, stats, st)) return;
  fwd_launch<KS, SW, FLIP, 4, 1>(x, w, bias, y, g, act, slope, stats, 4096, st);
}
template <int KS, int SW, int QT, int OCC>
void wgrad_launch(const void* x, const void* dy, float* dw, const DwGeo& g, int target, hipStream_t st) {
  const int slabs = slabs_of(g.C), rpi = rpi_of(g.C);
  const int64_t nstrips = (int64_t)g.N * g.P * ((g.Q + QT - 1) / QT);
  // >= 4 strips per thread: every block ends in KS*KS reductions + C*KS*KS atomics (on the
  // 1024-channel 7x7 layer those dominated a one-strip-per-thread grid)
  const int64_t spb = std::max<int64_t>(per_block(nstrips, rpi, slabs, target), 4 * rpi);
  const dim3 grid((unsigned)((nstrips + spb - 1) / spb), (unsigned)slabs);
  float* ws = nullptr;
  const int64_t n = (int64_t)g.C * KS * KS;
  if (dv_deterministic()) ws = dv_slab_workspace((size_t)grid.x * n, st);
  dw_wgrad_kernel<KS, SW, QT, OCC><<<grid, NT, 0, st>>>((const u16*)x, (const u16*)dy, dw,
                                                        with_strips(g, (g.Q + QT - 1) / QT, g.P), (int)spb, ws);
  if (ws) dv_slab_reduce(ws, dw, n, (int)grid.x, 1, st);
}
template <int KS, int SW>
void wgrad_variants(const void* x, const void* dy, float* dw, const DwGeo& g, hipStream_t st) {
  if constexpr (SW == 1) {
    // tiled weight gradient for outputs up to 14x14 (28-30 % faster than the plane / strip kernels
    // there); larger maps keep the strip kernel, whose blocks overlap loads with FMAs across strips
    const bool tiled = g_dw_variant == 60 || g_dw_variant == 62 || (g_dw_variant == 0 && g.P * g.Q <= 196);
    if (tiled && tile_wgrad<KS>(x, dy, dw, g, st)) return;
  } else {
    // outputs up to 14x14: 12-20 % faster than the strip / plane kernels; the 56x56 and 28x28
    // outputs keep the strip kernel (profiles/dw_tile_stride2.txt)
    const bool tiled = g_dw_variant == 60 || (g_dw_variant == 0 && g.P * g.Q <= 196);
    if (tiled && tile_wgrad2<KS>(x, dy, dw, g, st)) return;
  }
  if constexpr (KS == 3) {
    switch (g_dw_variant) {
      case 1: return wgrad_launch<KS, SW, 4, 4>(x, dy, dw, g, 2048, st);
      case 2: return wgrad_launch<KS, SW, 2, 4>(x, dy, dw, g, 2048, st);
      case 3: return wgrad_launch<KS, SW, 8, 2>(x, dy, dw, g, 1024, st);
      case 4: return wgrad_launch<KS, SW, 4, 2>(x, dy, dw, g, 2048, st);
      case 5: return wgrad_launch<KS, SW, 2, 2>(x, dy, dw, g, 2048, st);
      default: break;
    }
  }
  if (g_dw_variant != 50 && !dv_deterministic() && plane_wgrad<KS, SW>(x, dy, dw, g, st)) return;
  wgrad_launch<KS, SW, 4, 1>(x, dy, dw, g, 512, st);
}
template <int KS, int QT, int OCC>
void dgrad2_launch(const void* dy, const float* w, void* dx, const DwGeo& g, int target, hipStream_t st,
                   const DwBnr* bnr = nullptr) {
  const int slabs = slabs_of(g.C), rpi = rpi_of(g.C);
  const int64_t nstrips = (int64_t)g.N * g.H * ((g.W + QT - 1) / QT);
  const int64_t spb = per_block(nstrips, rpi, slabs, target);
  const dim3 grid((unsigned)((nstrips + spb - 1) / spb), (unsigned)slabs);
  const DwGeo gs = with_strips(g, (g.W + QT - 1) / QT, g.H);
  if (bnr) {
    const DetStats det(grid.x, g.C, st);
    DwBnr b = *bnr;
    b.det = det.slab;
    dw_dgrad2_kernel<KS, QT, OCC, true><<<grid, NT, 0, st>>>((const u16*)dy, w, (u16*)dx, gs, (int)spb, b);
    det.fold(bnr->acc);
  } else
    dw_dgrad2_kernel<KS, QT, OCC><<<grid, NT, 0, st>>>((const u16*)dy, w, (u16*)dx, gs, (int)spb, DwBnr{});
}
template <int KS>
void dgrad2_variants(const void* dy, const float* w, void* dx, const DwGeo& g, hipStream_t st, const DwBnr* bnr = nullptr) {
  if (bnr) return dgrad2_launch<KS, 4, 2>(dy, w, dx, g, 8192, st, bnr);  // 8-pixel strips + BN state: 256 VGPRs
  if constexpr (KS == 3) {
    switch (g_dw_variant) {
      case 1: return dgrad2_launch<KS, 4, 4>(dy, w, dx, g, 8192, st);
      case 2: return dgrad2_launch<KS, 2, 4>(dy, w, dx, g, 8192, st);
      case 3: return dgrad2_launch<KS, 8, 2>(dy, w, dx, g, 4096, st);
      case 4: return dgrad2_launch<KS, 4, 2>(dy, w, dx, g, 8192, st);
      case 5: return dgrad2_launch<KS, 2, 2>(dy, w, dx, g, 8192, st);
      default: break;
    }
  }
  // 8-pixel strips: measured 15-27 % faster than 4 on every MobileNet stride-2 layer (tools/dw_bench.py)
  dgrad2_launch<KS, 8, 1>(dy, w, dx, g, 4096, st);
}

}  // namespace

#define DW_KS(K, BODY)                        \
  switch (K) {                                \
    case 3: { constexpr int KS = 3; BODY; } break; \
    case 5: { constexpr int KS = 5; BODY; } break; \
    case 1: { constexpr int KS = 1; BODY; } break; \
    case 7: { constexpr int KS = 7; BODY; } break; \
    default: return -1;                       \
  }

// every block's slab must be a whole number of 8-channel groups; partial last slabs are fine
static inline bool dw_shape_ok(int C, int ldx, int ldy) { return C % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0; }

void dv_dw_variant(int v) { g_dw_variant = v; }

int dv_dw_fwd(const void* x, const float* w, const float* bias, void* y, int N, int H, int W, int C, int ldx, int P,
              int Q, int ldy, int K, int sh, int sw, int ph, int pw, int act, float slope, float* stats, hipStream_t st) {
  if (!dw_shape_ok(C, ldx, ldy) || (sw != 1 && sw != 2)) return -1;
  DwGeo g{N, H, W, C, ldx, P, Q, ldy, sh, sw, ph, pw, {}, {}};
  if (sw == 1) {
    DW_KS(K, (fwd_variants<KS, 1, false>(x, w, bias, y, g, act, slope, stats, st)))
  } else {
    DW_KS(K, (fwd_variants<KS, 2, false>(x, w, bias, y, g, act, slope, stats, st)))
  }
  return 0;
}

int dv_dw_dgrad(const void* dy, const float* w, void* dx, int N, int H, int W, int C, int ldx, int P, int Q, int ldy,
                int K, int sh, int sw, int ph, int pw, hipStream_t st, const void* bnx, const float* bnprm, float* bnacc,
                int bnmode, int bnact, float bnslope) {
  if (!dw_shape_ok(C, ldx, ldy)) return -1;
  // fused BN-backward reduction: dense dx and BN input (element offsets shared), modes 1 / 2
  DwBnr b{(const u16*)bnx, bnprm, bnacc, bnmode, bnact, bnslope};
  const DwBnr* bp = (bnmode == 1 || bnmode == 2) && bnx && bnprm && bnacc && ldx == C ? &b : nullptr;
  if (bnmode && !bp) return -1;
  if (sh == 1 && sw == 1) {
    // correlation of dY with the flipped filter, padding K-1-p, output grid = input grid
    DwGeo g{N, P, Q, C, ldy, H, W, ldx, 1, 1, K - 1 - ph, K - 1 - pw, {}, {}};
    DW_KS(K, (fwd_variants<KS, 1, true>(dy, w, nullptr, dx, g, 0, 0.f, nullptr, st, bp)))
    return 0;
  }
  if (sh != 2 || sw != 2) return -1;
  DwGeo g{N, H, W, C, ldx, P, Q, ldy, sh, sw, ph, pw, {}, {}};
  DW_KS(K, (dgrad2_variants<KS>(dy, w, dx, g, st, bp)))
  return 0;
}

int dv_dw_wgrad(const void* x, const void* dy, float* dw, int N, int H, int W, int C, int ldx, int P, int Q, int ldy,
                int K, int sh, int sw, int ph, int pw, int accumulate, hipStream_t st) {
  if (!dw_shape_ok(C, ldx, ldy) || (sw != 1 && sw != 2)) return -1;
  DwGeo g{N, H, W, C, ldx, P, Q, ldy, sh, sw, ph, pw, {}, {}};
  if (!accumulate) (void)hipMemsetAsync(dw, 0, (size_t)C * K * K * sizeof(float), st);
  if (sw == 1) {
    DW_KS(K, (wgrad_variants<KS, 1>(x, dy, dw, g, st)))
  } else {
    DW_KS(K, (wgrad_variants<KS, 2>(x, dy, dw, g, st)))
  }
  return 0;
}
