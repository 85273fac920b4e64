// Pooling / resampling kernels on bf16 NHWC.
//   maxpool fwd writes a u8 window-position index per output element; the backward is a
//   gather over the (<= ceil(k/s)^2) outputs covering each input — no atomics, no int64 index.
//   avgpool follows torch semantics (ceil_mode, count_include_pad, divisor_override).
//   Global average pool accumulates in fp32. Nearest upsample by an integer factor.
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

template <int VEC> struct V;
template <> struct V<8> {
  using raw = uint4;
  DV_DEVICE static void ld(const u16* p, float* v) {
    uint4 r = *reinterpret_cast<const uint4*>(p); uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[2 * i] = bf2f(w[i] & 0xffff); v[2 * i + 1] = bf2f(w[i] >> 16); }
  }
  DV_DEVICE static void st(u16* p, const float* v) {
    uint4 r; r.x = pack2bf(v[0], v[1]); r.y = pack2bf(v[2], v[3]); r.z = pack2bf(v[4], v[5]); r.w = pack2bf(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = r;
  }
};
template <> struct V<1> {
  DV_DEVICE static void ld(const u16* p, float* v) { v[0] = bf2f(*p); }
  DV_DEVICE static void st(u16* p, const float* v) { *p = f2bf(v[0]); }
};

struct PoolGeo { int N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw; };

// Fused BatchNorm statistics of a grid-stride kernel's output (the consumer BN then skips its own
// statistics pass; models/hourglass.py pooled / upsampled block inputs): with C / VEC dividing NT
// a thread keeps one channel group for the whole grid-stride loop, sums d = v - K and d^2 (K: the
// BN's shift row, ops.bn) of the stored bf16 values, and the block's NT / cg threads of a channel
// group meet in LDS -> one coalesced atomic row per block into the [SHARDS][2][C] accumulator.
struct PoolStats {
  float* acc;  // nullptr: no statistics
  float* det;  // deterministic mode: this launch's per-block rows
};
template <int VEC>
DV_DEVICE void pool_stats_commit(const float* s, const float* q, const PoolStats& ps, int C) {
  __shared__ float sh[2][NT * VEC];
  const int tid = threadIdx.x, cg = C / VEC, rpi = NT / cg;
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sh[0][tid * VEC + i] = s[i]; sh[1][tid * VEC + i] = q[i]; }
  __syncthreads();
  float* a = stat_row(ps.acc, ps.det, blockIdx.x, C);
  for (int ch = tid; ch < C; ch += NT) {
    const int gi = ch / VEC, i = ch - gi * VEC;
    float ss = 0.f, qq = 0.f;
    for (int r = 0; r < rpi; ++r) { ss += sh[0][(r * cg + gi) * VEC + i]; qq += sh[1][(r * cg + gi) * VEC + i]; }
    atomicAdd(a + ch, ss);
    atomicAdd(a + C + ch, qq);
  }
}

template <int VEC>
__global__ __launch_bounds__(NT) void maxpool_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y,
                                                           uint8_t* __restrict__ idx, PoolGeo g, int64_t total,
                                                           PoolStats ps) {
  const int cg = g.C / VEC;
  float ss[VEC], sq[VEC], kq[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    ss[i] = 0.f; sq[i] = 0.f;
    kq[i] = ps.acc ? stat_shift(ps.acc, g.C)[(threadIdx.x % cg) * VEC + i] : 0.f;
  }
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c = (int)(t % cg) * VEC;
    int64_t pix = t / cg;
    const int q = (int)(pix % g.Q); pix /= g.Q;
    const int p = (int)(pix % g.P); const int n = (int)(pix / g.P);
    float best[VEC]; int bi[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) { best[i] = -INFINITY; bi[i] = 0; }
    for (int r = 0; r < g.kh; ++r) {
      const int h = p * g.sh - g.ph + r;
      if (h < 0 || h >= g.H) continue;
      for (int s = 0; s < g.kw; ++s) {
        const int w = q * g.sw - g.pw + s;
        if (w < 0 || w >= g.W) continue;
        float v[VEC];
        V<VEC>::ld(x + (((int64_t)n * g.H + h) * g.W + w) * g.C + c, v);
#pragma unroll
        for (int i = 0; i < VEC; ++i) if (v[i] > best[i] || (v[i] != v[i] && best[i] == best[i])) { best[i] = v[i]; bi[i] = r * g.kw + s; }
      }
    }
    const int64_t o = (((int64_t)n * g.P + p) * g.Q + q) * g.C + c;
    V<VEC>::st(y + o, best);
    if (idx) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) idx[o + i] = (uint8_t)bi[i];
    }
    if (ps.acc) {  // the window maxima are bf16 values already
#pragma unroll
      for (int i = 0; i < VEC; ++i) { const float d = best[i] - kq[i]; ss[i] += d; sq[i] = fmaf(d, d, sq[i]); }
    }
  }
  if (ps.acc) pool_stats_commit<VEC>(ss, sq, ps, g.C);
}

template <int VEC>
__global__ __launch_bounds__(NT) void maxpool_bwd_kernel(const u16* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                           u16* __restrict__ dx, PoolGeo g, int64_t total) {
  const int cg = g.C / VEC;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c = (int)(t % cg) * VEC;
    int64_t pix = t / cg;
    const int w = (int)(pix % g.W); pix /= g.W;
    const int h = (int)(pix % g.H); const int n = (int)(pix / g.H);
    float acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
    // outputs p with p*sh - ph <= h <= p*sh - ph + kh - 1
    int p_lo = (h + g.ph - g.kh + 1 + g.sh - 1); p_lo = p_lo < 0 ? 0 : p_lo / g.sh;
    int p_hi = (h + g.ph) / g.sh; if (p_hi > g.P - 1) p_hi = g.P - 1;
    int q_lo = (w + g.pw - g.kw + 1 + g.sw - 1); q_lo = q_lo < 0 ? 0 : q_lo / g.sw;
    int q_hi = (w + g.pw) / g.sw; if (q_hi > g.Q - 1) q_hi = g.Q - 1;
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * g.sh - g.ph);
      if (r < 0 || r >= g.kh) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int s = w - (q * g.sw - g.pw);
        if (s < 0 || s >= g.kw) continue;
        const int64_t o = (((int64_t)n * g.P + p) * g.Q + q) * g.C + c;
        float d[VEC];
        V<VEC>::ld(dy + o, d);
        const int pos = r * g.kw + s;
#pragma unroll
        for (int i = 0; i < VEC; ++i) if (idx[o + i] == pos) acc[i] += d[i];
      }
    }
    V<VEC>::st(dx + (((int64_t)n * g.H + h) * g.W + w) * g.C + c, acc);
  }
}

DV_DEVICE void avg_window(const PoolGeo& g, int p, int q, int cip, int divover, int& h0, int& h1, int& w0, int& w1,
                          float& inv) {
  int hs = p * g.sh - g.ph, ws = q * g.sw - g.pw;
  int he = min(hs + g.kh, g.H + g.ph), we = min(ws + g.kw, g.W + g.pw);
  const int pool = (he - hs) * (we - ws);
  hs = max(hs, 0); ws = max(ws, 0); he = min(he, g.H); we = min(we, g.W);
  h0 = hs; h1 = he; w0 = ws; w1 = we;
  const int div = divover > 0 ? divover : (cip ? pool : (he - hs) * (we - ws));
  inv = div > 0 ? 1.f / (float)div : 0.f;
}

template <int VEC>
__global__ __launch_bounds__(NT) void avgpool_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y, PoolGeo g,
                                                           int cip, int divover, int64_t total) {
  const int cg = g.C / VEC;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c = (int)(t % cg) * VEC;
    int64_t pix = t / cg;
    const int q = (int)(pix % g.Q); pix /= g.Q;
    const int p = (int)(pix % g.P); const int n = (int)(pix / g.P);
    int h0, h1, w0, w1; float inv;
    avg_window(g, p, q, cip, divover, h0, h1, w0, w1, inv);
    float acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) {
        float v[VEC];
        V<VEC>::ld(x + (((int64_t)n * g.H + h) * g.W + w) * g.C + c, v);
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] += v[i];
      }
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] *= inv;
    V<VEC>::st(y + (((int64_t)n * g.P + p) * g.Q + q) * g.C + c, acc);
  }
}

template <int VEC>
__global__ __launch_bounds__(NT) void avgpool_bwd_kernel(const u16* __restrict__ dy, u16* __restrict__ dx, PoolGeo g,
                                                           int cip, int divover, int64_t total) {
  const int cg = g.C / VEC;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c = (int)(t % cg) * VEC;
    int64_t pix = t / cg;
    const int w = (int)(pix % g.W); pix /= g.W;
    const int h = (int)(pix % g.H); const int n = (int)(pix / g.H);
    float acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
    int p_lo = (h + g.ph - g.kh + 1 + g.sh - 1); p_lo = p_lo < 0 ? 0 : p_lo / g.sh;
    int p_hi = (h + g.ph) / g.sh; if (p_hi > g.P - 1) p_hi = g.P - 1;
    int q_lo = (w + g.pw - g.kw + 1 + g.sw - 1); q_lo = q_lo < 0 ? 0 : q_lo / g.sw;
    int q_hi = (w + g.pw) / g.sw; if (q_hi > g.Q - 1) q_hi = g.Q - 1;
    for (int p = p_lo; p <= p_hi; ++p)
      for (int q = q_lo; q <= q_hi; ++q) {
        int h0, h1, w0, w1; float inv;
        avg_window(g, p, q, cip, divover, h0, h1, w0, w1, inv);
        if (h < h0 || h >= h1 || w < w0 || w >= w1) continue;
        float d[VEC];
        V<VEC>::ld(dy + (((int64_t)n * g.P + p) * g.Q + q) * g.C + c, d);
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] += d[i] * inv;
      }
    V<VEC>::st(dx + (((int64_t)n * g.H + h) * g.W + w) * g.C + c, acc);
  }
}

// global average pool: x [N][HW][C] -> y [N][C] (bf16 out, fp32 accumulate)
template <int VEC>
__global__ __launch_bounds__(NT) void gap_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y, int N, int HW, int C) {
  const int cg = C / VEC;
  const int64_t total = (int64_t)N * cg;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c = (int)(t % cg) * VEC; const int n = (int)(t / cg);
    float acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
    const u16* base = x + (int64_t)n * HW * C + c;
    for (int r = 0; r < HW; ++r) {
      float v[VEC];
      V<VEC>::ld(base + (int64_t)r * C, v);
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] += v[i];
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] *= inv;
    V<VEC>::st(y + (int64_t)n * C + c, acc);
  }
}

template <int VEC>
__global__ __launch_bounds__(NT) void gap_bwd_kernel(const u16* __restrict__ dy, u16* __restrict__ dx, int N, int HW, int C) {
  const int cg = C / VEC;
  const int64_t total = (int64_t)N * HW * cg;
  const float inv = 1.f / (float)HW;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c = (int)(t % cg) * VEC; const int64_t row = t / cg; const int n = (int)(row / HW);
    float d[VEC];
    V<VEC>::ld(dy + (int64_t)n * C + c, d);
#pragma unroll
    for (int i = 0; i < VEC; ++i) d[i] *= inv;
    V<VEC>::st(dx + row * C + c, d);
  }
}

template <int VEC>
__global__ __launch_bounds__(NT) void upsample_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y, int N, int H,
                                                            int W, int C, int f) {
  const int cg = C / VEC, OH = H * f, OW = W * f;
  const int64_t total = (int64_t)N * OH * OW * cg;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c = (int)(t % cg) * VEC; int64_t pix = t / cg;
    const int ow = (int)(pix % OW); pix /= OW; const int oh = (int)(pix % OH); const int n = (int)(pix / OH);
    const u16* src = x + (((int64_t)n * H + oh / f) * W + ow / f) * C + c;
    u16* dst = y + (((int64_t)n * OH + oh) * OW + ow) * C + c;
    if (VEC == 8) *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    else *dst = *src;
  }
}

// y = upsample_nearest(x, f) + r (Stacked Hourglass level merge, models/hourglass.py): one pass
// instead of an upsample pass + an add pass over the upsampled tensor (16 per step)
template <int VEC>
__global__ __launch_bounds__(NT) void upsample_add_kernel(const u16* __restrict__ x, const u16* __restrict__ r,
                                                            u16* __restrict__ y, int N, int H, int W, int C, int f,
                                                            PoolStats ps) {
  const int cg = C / VEC, OH = H * f, OW = W * f;
  const int64_t total = (int64_t)N * OH * OW * cg;
  float ss[VEC], sq[VEC], kq[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    ss[i] = 0.f; sq[i] = 0.f;
    kq[i] = ps.acc ? stat_shift(ps.acc, C)[(threadIdx.x % cg) * VEC + i] : 0.f;
  }
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c = (int)(t % cg) * VEC; int64_t pix = t / cg;
    const int ow = (int)(pix % OW); pix /= OW; const int oh = (int)(pix % OH); const int n = (int)(pix / OH);
    const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c;
    float a[VEC], b[VEC];
    V<VEC>::ld(x + (((int64_t)n * H + oh / f) * W + ow / f) * C + c, a);
    V<VEC>::ld(r + o, b);
#pragma unroll
    for (int i = 0; i < VEC; ++i) a[i] += b[i];
    V<VEC>::st(y + o, a);
    if (ps.acc) {  // statistics of the stored (bf16-rounded) sums
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const float d = bf2f(f2bf(a[i])) - kq[i];
        ss[i] += d; sq[i] = fmaf(d, d, sq[i]);
      }
    }
  }
  if (ps.acc) pool_stats_commit<VEC>(ss, sq, ps, C);
}

template <int VEC>
__global__ __launch_bounds__(NT) void upsample_bwd_kernel(const u16* __restrict__ dy, u16* __restrict__ dx, int N, int H,
                                                            int W, int C, int f) {
  const int cg = C / VEC, OH = H * f, OW = W * f;
  const int64_t total = (int64_t)N * H * W * cg;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c = (int)(t % cg) * VEC; int64_t pix = t / cg;
    const int w = (int)(pix % W); pix /= W; const int h = (int)(pix % H); const int n = (int)(pix / H);
    float acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
    for (int a = 0; a < f; ++a)
      for (int b = 0; b < f; ++b) {
        float d[VEC];
        V<VEC>::ld(dy + (((int64_t)n * OH + h * f + a) * OW + w * f + b) * C + c, d);
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] += d[i];
      }
    V<VEC>::st(dx + (((int64_t)n * H + h) * W + w) * C + c, acc);
  }
}

// ---- BatchNorm apply + activation + max pool as one pass: the conv -> BN -> ReLU -> MaxPool stem
// (R/ResNet/pytorch/models/resnet50.py:33-35,72-75). The BN output (411 MB for the ResNet-50 stem
// at batch 256) is never written, and the backward never materialises its gradient.
DV_DEVICE float pool_act(float z, int act, float slope) {
  if (act == 1) return fmaxf(z, 0.f);
  if (act == 2) return z > 0.f ? z : z * slope;
  return z;
}

// Window geometry: compile-time for the 3x3 / stride-2 stem pool (KH = 0: runtime g.kh ...). Every
// input row / column is covered by at most WIN = ceil(k / s) windows per dimension.
template <int KH, int KW, int SH, int SW>
struct PoolWin {
  DV_DEVICE static int kh(const PoolGeo& g) { return KH ? KH : g.kh; }
  DV_DEVICE static int kw(const PoolGeo& g) { return KW ? KW : g.kw; }
  DV_DEVICE static int sh(const PoolGeo& g) { return SH ? SH : g.sh; }
  DV_DEVICE static int sw(const PoolGeo& g) { return SW ? SW : g.sw; }
  static constexpr int WH = KH ? (KH + SH - 1) / SH : 16;  // loop bound (runtime form breaks out early)
  static constexpr int WW = KW ? (KW + SW - 1) / SW : 16;
};

// Forward: out = max over the window of bf16(act(x*scale + shift)). The bf16 rounding of the
// unfused BN pass is applied before the comparison, so values and window indices are exactly the
// unfused ones. One thread per (n, p, q, 8-channel group), grid-stride (stride % cg == 0: a
// thread keeps its channels and their scale/shift); every window load is issued before the max.
// RELU (compiled windows): the comparison runs on one integer key per element, bf16(z) bits in the
// high half and (last window index - index) in the low bits -- a signed max picks the largest value and,
// on ties, the first window position (the unfused pool's strict '>'); negative z (ReLU zeros, whose
// gradient is zero whichever position is kept) order below every non-negative key and leave as +0.
// (v_perm_b32 byte selects: one op per key; bytes 4-7 are pk, 0-3 lowc, 0x0c reads zero)
DV_DEVICE uint32_t pool_pk_bf16(float a, float b) {  // one v_cvt_pk_bf16_f32, a in the low half
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){a, b}, b2));
}
DV_DEVICE uint32_t pool_key_lo(uint32_t pk, uint32_t lowc) { return __builtin_amdgcn_perm(pk, lowc, 0x05040c00u); }
DV_DEVICE uint32_t pool_key_hi(uint32_t pk, uint32_t lowc) { return __builtin_amdgcn_perm(pk, lowc, 0x07060c00u); }

template <int KH, int KW, int SH, int SW, bool RELU>
__global__ __launch_bounds__(NT) void bn_act_maxpool_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y,
                                                                uint8_t* __restrict__ idx, PoolGeo g, FastDiv div_cg,
                                                                FastDiv div_q, FastDiv div_p, int64_t total,
                                                                const float* __restrict__ scale,
                                                                const float* __restrict__ shift, int act, float slope) {
  using Wn = PoolWin<KH, KW, SH, SW>;
  const int kh = Wn::kh(g), kw = Wn::kw(g), sh = Wn::sh(g), sw = Wn::sw(g);
  const uint32_t t0 = blockIdx.x * NT + threadIdx.x;
  const int lc = (int)(t0 - fdiv(t0, div_cg) * div_cg.d), c = lc * 8;
  float sc[8], sf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { sc[i] = scale[c + i]; sf[i] = shift[c + i]; }
  for (uint32_t t = t0; t < total; t += gridDim.x * NT) {
    const uint32_t pix = fdiv(t, div_cg);
    const uint32_t row = fdiv(pix, div_q);
    const int q = (int)(pix - row * div_q.d);
    const int n = (int)fdiv(row, div_p), p = (int)(row - n * div_p.d);
    const int h0 = p * sh - g.ph, w0 = q * sw - g.pw;
    if constexpr (RELU) {
      static_assert(KH != 0 && KW != 0, "integer-key path is for compiled windows");
      const u16* xb = x + ((int64_t)n * g.H * g.W) * g.C + c;
      uint4 raw[KH * KW];
      bool ok[KH * KW];
#pragma unroll
      for (int r = 0; r < KH; ++r)
#pragma unroll
        for (int s = 0; s < KW; ++s) {  // all window loads in flight together
          const int h = h0 + r, w = w0 + s;
          ok[r * KW + s] = h >= 0 && h < g.H && w >= 0 && w < g.W;
          raw[r * KW + s] = ok[r * KW + s] ? *reinterpret_cast<const uint4*>(xb + ((int64_t)h * g.W + w) * g.C)
                                           : uint4{0u, 0u, 0u, 0u};
        }
      int key[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) key[i] = INT32_MIN;
#pragma unroll
      for (int k = 0; k < KH * KW; ++k) {
        if (!ok[k]) continue;
        const uint32_t lowc = (uint32_t)(KH * KW - 1 - k);  // an inline constant (VOP3 takes no literal)
        const uint32_t wd[4] = {raw[k].x, raw[k].y, raw[k].z, raw[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = __uint_as_float(wd[e] << 16), hi = __uint_as_float(wd[e] & 0xffff0000u);
          const uint32_t pk = pool_pk_bf16(fmaf(lo, sc[2 * e], sf[2 * e]), fmaf(hi, sc[2 * e + 1], sf[2 * e + 1]));
          key[2 * e] = max(key[2 * e], (int)pool_key_lo(pk, lowc));
          key[2 * e + 1] = max(key[2 * e + 1], (int)pool_key_hi(pk, lowc));
        }
      }
      const int64_t o = (int64_t)pix * g.C + c;
      uint4 out;
      uint32_t ow[4], iw[2] = {0u, 0u};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        ow[e] = ((uint32_t)max(key[2 * e], 0) >> 16) | ((uint32_t)max(key[2 * e + 1], 0) & 0xffff0000u);
#pragma unroll
      for (int i = 0; i < 8; ++i) iw[i >> 2] |= ((uint32_t)(KH * KW - 1) - ((uint32_t)key[i] & 0xffu)) << (8 * (i & 3));
      out.x = ow[0]; out.y = ow[1]; out.z = ow[2]; out.w = ow[3];
      *reinterpret_cast<uint4*>(y + o) = out;
      *reinterpret_cast<uint2*>(idx + o) = uint2{iw[0], iw[1]};
      continue;
    }
    float best[8]; int bi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { best[i] = -INFINITY; bi[i] = 0; }
    const u16* xb = x + ((int64_t)n * g.H * g.W) * g.C + c;
#pragma unroll
    for (int r = 0; r < (KH ? KH : 16); ++r) {
      if (!KH && r >= kh) break;
      const int h = h0 + r;
      uint4 raw[KW ? KW : 1];
      bool ok[KW ? KW : 1];
      if constexpr (KW != 0) {
#pragma unroll
        for (int s = 0; s < KW; ++s) {  // issue the row's loads together
          const int w = w0 + s;
          ok[s] = h >= 0 && h < g.H && w >= 0 && w < g.W;
          raw[s] = ok[s] ? *reinterpret_cast<const uint4*>(xb + ((int64_t)h * g.W + w) * g.C) : uint4{0u, 0u, 0u, 0u};
        }
      }
      for (int s = 0; s < kw; ++s) {
        const int w = w0 + s;
        float v[8];
        if constexpr (KW != 0) {
          if (!ok[s]) continue;
          const uint32_t wd[4] = {raw[s].x, raw[s].y, raw[s].z, raw[s].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[2 * e] = bf2f(wd[e] & 0xffff); v[2 * e + 1] = bf2f(wd[e] >> 16); }
        } else {
          if (h < 0 || h >= g.H || w < 0 || w >= g.W) continue;
          V<8>::ld(xb + ((int64_t)h * g.W + w) * g.C, v);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float a = bf2f(f2bf(pool_act(fmaf(v[i], sc[i], sf[i]), act, slope)));
          if (a > best[i] || (a != a && best[i] == best[i])) { best[i] = a; bi[i] = r * kw + s; }
        }
      }
    }
    const int64_t o = (int64_t)pix * g.C + c;
    V<8>::st(y + o, best);
    uint2 pk;
    pk.x = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
    pk.y = (uint32_t)bi[4] | ((uint32_t)bi[5] << 8) | ((uint32_t)bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = pk;
  }
}

// Backward, per input element: da = sum of the pooled gradients whose window index points at it
// (the maxpool gather, bf16-rounded like the unfused pass's stored da), dz = act'(z) * da with
// z = x*mscale + mshift recomputed from the BN input.
//   REDUCE: per-channel (sum dz, sum dz*(x-mean)*invstd) into the BN shard accumulator
//           acc[SHARDS][2][C] (csrc/bn.hip layout; bn_bwd_finalize folds it);
//   APPLY : dx = kA*dz + kB*x + kC (coefficients from bn_bwd_finalize).
// One thread per (n, h, w, 8-channel group), grid-stride (cg | 256, so a thread's channels are
// fixed and the block's partial sums meet in LDS for one coalesced atomic row per block).
template <bool APPLY, int KH, int KW, int SH, int SW>
__global__ __launch_bounds__(NT) void bn_act_maxpool_bwd_kernel(const u16* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                                const u16* __restrict__ x, u16* __restrict__ dx, PoolGeo g,
                                                                FastDiv div_cg, FastDiv div_w, FastDiv div_h, int64_t total,
                                                                const float* __restrict__ prm,
                                                                const float* __restrict__ coef, int act, float slope,
                                                                float* __restrict__ acc, float* __restrict__ det) {
  using Wn = PoolWin<KH, KW, SH, SW>;
  const int kh = Wn::kh(g), kw = Wn::kw(g), sh = Wn::sh(g), sw = Wn::sw(g);
  const int cg = g.C / 8;
  const uint32_t t0 = blockIdx.x * NT + threadIdx.x;
  const int lc = (int)(t0 - fdiv(t0, div_cg) * div_cg.d), c = lc * 8;
  // prm = [scale; shift; mean; invstd] x C, coef = [kA; kB; kC] x C
  float ms[8], mh[8], k0[8], k1[8], k2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ms[i] = prm[c + i]; mh[i] = prm[g.C + c + i];
    if (APPLY) { k0[i] = coef[c + i]; k1[i] = coef[g.C + c + i]; k2[i] = coef[2 * g.C + c + i]; }
    else { k0[i] = prm[2 * g.C + c + i]; k1[i] = prm[3 * g.C + c + i]; k2[i] = 0.f; }
  }
  float s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { s1[i] = 0.f; s2[i] = 0.f; }
  for (uint32_t t = t0; t < total; t += gridDim.x * NT) {
    const uint32_t pix = fdiv(t, div_cg);
    const uint32_t row = fdiv(pix, div_w);
    const int w = (int)(pix - row * div_w.d);
    const int n = (int)fdiv(row, div_h), h = (int)(row - n * div_h.d);
    // windows covering (h, w): p*sh - ph <= h <= p*sh - ph + kh - 1
    const int hp = h + g.ph, wp = w + g.pw;
    const int p_hi = min(hp / sh, g.P - 1), q_hi = min(wp / sw, g.Q - 1);
    const int64_t xo = (int64_t)pix * g.C + c;
    float xv[8];
    V<8>::ld(x + xo, xv);
    float da[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) da[i] = 0.f;
#pragma unroll
    for (int a = 0; a < Wn::WH; ++a) {
      const int p = p_hi - a, r = hp - p * sh;
      if (!KH && r >= kh) break;
      if (p < 0 || r >= kh) continue;
#pragma unroll
      for (int b = 0; b < Wn::WW; ++b) {
        const int q = q_hi - b, s = wp - q * sw;
        if (!KW && s >= kw) break;
        if (q < 0 || s >= kw) continue;
        const int64_t o = (((int64_t)n * g.P + p) * g.Q + q) * g.C + c;
        float d[8];
        V<8>::ld(dy + o, d);
        const uint2 ib = *reinterpret_cast<const uint2*>(idx + o);
        const uint32_t pos = (uint32_t)(r * kw + s);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t bsel = ((i < 4 ? ib.x : ib.y) >> (8 * (i & 3))) & 0xffu;
          if (bsel == pos) da[i] += d[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = bf2f(f2bf(da[i]));
      const float z = fmaf(xv[i], ms[i], mh[i]);
      const float dz = act == 1 ? (z > 0.f ? d : 0.f) : (act == 2 ? (z > 0.f ? d : d * slope) : d);
      if (APPLY) da[i] = fmaf(k0[i], dz, fmaf(k1[i], xv[i], k2[i]));
      else { s1[i] += dz; s2[i] += dz * (xv[i] - k0[i]) * k1[i]; }
    }
    if (APPLY) V<8>::st(dx + xo, da);
  }
  if (APPLY) return;
  // per-channel totals over the block's pixel lanes, one coalesced atomic row per block
  __shared__ float sh_[2][NT * 8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { sh_[0][threadIdx.x * 8 + i] = s1[i]; sh_[1][threadIdx.x * 8 + i] = s2[i]; }
  __syncthreads();
  const int lanes = NT / cg;
  float* a = stat_row(acc, det, blockIdx.x, g.C);
  for (int ch = threadIdx.x; ch < g.C; ch += NT) {
    const int gi = ch / 8, e = ch % 8;
    float t1 = 0.f, t2 = 0.f;
    for (int l = 0; l < lanes; ++l) {
      t1 += sh_[0][(l * cg + gi) * 8 + e];
      t2 += sh_[1][(l * cg + gi) * 8 + e];
    }
    atomicAdd(a + ch, t1);
    atomicAdd(a + g.C + ch, t2);
  }
}

// Backward for the 3x3 / stride-2 / pad-1 window with H = 2P, W = 2Q (the ResNet stem), one thread
// per (n, p, q, 8-channel group) owning the 2x2 input block rows {2p, 2p+1} x cols {2q, 2q+1}: row
// 2p lies only in window row p (r = 1), row 2p+1 in window rows p (r = 2) and p+1 (r = 0), columns
// alike -- the block's gradients come from windows (p,q), (p,q+1), (p+1,q), (p+1,q+1), nine
// (input, window) pairs per channel, branch-free (a window past the edge reads as never selected).
// Same REDUCE / APPLY contract as bn_act_maxpool_bwd_kernel; REDUCE accumulates dz*(x-mean) and
// scales by invstd once per thread.
DV_DEVICE float pool_pick(uint32_t iw, int i, uint32_t pos, float d) {
  return ((iw >> (8 * (i & 3))) & 0xffu) == pos ? d : 0.f;
}
DV_DEVICE float half_bf(uint32_t w, int hi) { return __uint_as_float(hi ? (w & 0xffff0000u) : (w << 16)); }

template <bool APPLY, int ACT>
__global__ __launch_bounds__(NT) void bn_act_maxpool_bwd_s2_kernel(const u16* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                                   const u16* __restrict__ x, u16* __restrict__ dx,
                                                                   PoolGeo g, FastDiv div_cg, FastDiv div_q, FastDiv div_p,
                                                                   int64_t total, const float* __restrict__ prm,
                                                                   const float* __restrict__ coef, float slope,
                                                                   float* __restrict__ acc, float* __restrict__ det) {
  const int cg = g.C / 8;
  const uint32_t t0 = blockIdx.x * NT + threadIdx.x;
  const int lc = (int)(t0 - fdiv(t0, div_cg) * div_cg.d), c = lc * 8;
  float ms[8], mh[8], k0[8], k1[8], k2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ms[i] = prm[c + i]; mh[i] = prm[g.C + c + i];
    if (APPLY) { k0[i] = coef[c + i]; k1[i] = coef[g.C + c + i]; k2[i] = coef[2 * g.C + c + i]; }
    else { k0[i] = prm[2 * g.C + c + i]; k1[i] = prm[3 * g.C + c + i]; k2[i] = 0.f; }
  }
  float s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { s1[i] = 0.f; s2[i] = 0.f; }
  const int64_t rowC = (int64_t)g.W * g.C;
  for (uint32_t t = t0; t < total; t += gridDim.x * NT) {
    const uint32_t pix = fdiv(t, div_cg);
    const uint32_t row = fdiv(pix, div_q);
    const int q = (int)(pix - row * div_q.d);
    const int n = (int)fdiv(row, div_p), p = (int)(row - n * div_p.d);
    const bool pr = p + 1 < g.P, qr = q + 1 < g.Q;
    const int64_t o = (int64_t)pix * g.C + c, oq = (int64_t)g.Q * g.C;
    const uint4 z4{0u, 0u, 0u, 0u};
    const uint2 none{0xffffffffu, 0xffffffffu};
    const uint4 d00 = *reinterpret_cast<const uint4*>(dy + o);
    const uint4 d01 = qr ? *reinterpret_cast<const uint4*>(dy + o + g.C) : z4;
    const uint4 d10 = pr ? *reinterpret_cast<const uint4*>(dy + o + oq) : z4;
    const uint4 d11 = pr && qr ? *reinterpret_cast<const uint4*>(dy + o + oq + g.C) : z4;
    const uint2 i00 = *reinterpret_cast<const uint2*>(idx + o);
    const uint2 i01 = qr ? *reinterpret_cast<const uint2*>(idx + o + g.C) : none;
    const uint2 i10 = pr ? *reinterpret_cast<const uint2*>(idx + o + oq) : none;
    const uint2 i11 = pr && qr ? *reinterpret_cast<const uint2*>(idx + o + oq + g.C) : none;
    const int64_t xo = (((int64_t)n * g.H + 2 * p) * g.W + 2 * q) * g.C + c;
    uint4 xr[4];
    xr[0] = *reinterpret_cast<const uint4*>(x + xo);
    xr[1] = *reinterpret_cast<const uint4*>(x + xo + g.C);
    xr[2] = *reinterpret_cast<const uint4*>(x + xo + rowC);
    xr[3] = *reinterpret_cast<const uint4*>(x + xo + rowC + g.C);
    uint32_t ow[4][4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = i >> 1, hi = i & 1;
      const uint32_t w00 = (&d00.x)[e], w01 = (&d01.x)[e], w10 = (&d10.x)[e], w11 = (&d11.x)[e];
      const uint32_t j00 = i < 4 ? i00.x : i00.y, j01 = i < 4 ? i01.x : i01.y;
      const uint32_t j10 = i < 4 ? i10.x : i10.y, j11 = i < 4 ? i11.x : i11.y;
      const float g00 = half_bf(w00, hi), g01 = half_bf(w01, hi), g10 = half_bf(w10, hi), g11 = half_bf(w11, hi);
      float da[4];
      da[0] = pool_pick(j00, i, 4, g00);
      da[1] = pool_pick(j00, i, 5, g00) + pool_pick(j01, i, 3, g01);
      da[2] = pool_pick(j00, i, 7, g00) + pool_pick(j10, i, 1, g10);
      da[3] = (pool_pick(j00, i, 8, g00) + pool_pick(j01, i, 6, g01)) + (pool_pick(j10, i, 2, g10) + pool_pick(j11, i, 0, g11));
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float xv = half_bf((&xr[b].x)[e], hi);
        const float d = bf2f(f2bf(da[b]));
        const float z = fmaf(xv, ms[i], mh[i]);
        const float dz = ACT == 1 ? (z > 0.f ? d : 0.f) : (ACT == 2 ? (z > 0.f ? d : d * slope) : d);
        if (APPLY) {
          const uint32_t v = f2bf(fmaf(k0[i], dz, fmaf(k1[i], xv, k2[i])));
          ow[b][e] = hi ? (ow[b][e] | (v << 16)) : v;
        } else {
          s1[i] += dz;
          s2[i] = fmaf(dz, xv - k0[i], s2[i]);
        }
      }
    }
    if (APPLY) {
      *reinterpret_cast<uint4*>(dx + xo) = uint4{ow[0][0], ow[0][1], ow[0][2], ow[0][3]};
      *reinterpret_cast<uint4*>(dx + xo + g.C) = uint4{ow[1][0], ow[1][1], ow[1][2], ow[1][3]};
      *reinterpret_cast<uint4*>(dx + xo + rowC) = uint4{ow[2][0], ow[2][1], ow[2][2], ow[2][3]};
      *reinterpret_cast<uint4*>(dx + xo + rowC + g.C) = uint4{ow[3][0], ow[3][1], ow[3][2], ow[3][3]};
    }
  }
  if (APPLY) return;
  __shared__ float sh_[2][NT * 8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { sh_[0][threadIdx.x * 8 + i] = s1[i]; sh_[1][threadIdx.x * 8 + i] = s2[i] * k1[i]; }
  __syncthreads();
  const int lanes = NT / cg;
  float* a = stat_row(acc, det, blockIdx.x, g.C);
  for (int ch = threadIdx.x; ch < g.C; ch += NT) {
    const int gi = ch / 8, e = ch % 8;
    float t1 = 0.f, t2 = 0.f;
    for (int l = 0; l < lanes; ++l) {
      t1 += sh_[0][(l * cg + gi) * 8 + e];
      t2 += sh_[1][(l * cg + gi) * 8 + e];
    }
    atomicAdd(a + ch, t1);
    atomicAdd(a + g.C + ch, t2);
  }
}

inline int grid_for(int64_t total) {
  int64_t g = (total + NT - 1) / NT;
  return (int)std::min<int64_t>(std::max<int64_t>(g, 1), 256 * 16);
}
}  // namespace

#define VDISPATCH(C, K, ...) do { if ((C) % 8 == 0) K<8> __VA_ARGS__; else K<1> __VA_ARGS__; } while (0)

// statistics-fused launches (stats != nullptr): C % 8 == 0 with C / 8 dividing NT (else -1, no
// launch), a grid of at most 1,024 blocks (one atomic row each)
static bool pool_stats_ok(int C) { return C % 8 == 0 && NT % (C / 8) == 0; }
static int stats_grid(int64_t total) { return (int)std::min<int64_t>(grid_for(total), 1024); }

int dv_maxpool_fwd(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                   int sh, int sw, int ph, int pw, float* stats, hipStream_t st) {
  PoolGeo g{N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw};
  const int v = C % 8 == 0 ? 8 : 1;
  const int64_t total = (int64_t)N * P * Q * (C / v);
  if (stats) {
    if (!pool_stats_ok(C)) return -1;
    const int grid = stats_grid(total);
    DetStats d(grid, C, st);
    maxpool_fwd_kernel<8><<<grid, NT, 0, st>>>((const u16*)x, (u16*)y, idx, g, total, PoolStats{stats, d.slab});
    d.fold(stats);
    return 0;
  }
  VDISPATCH(C, maxpool_fwd_kernel, <<<grid_for(total), NT, 0, st>>>((const u16*)x, (u16*)y, idx, g, total, PoolStats{nullptr, nullptr}));
  return 0;
}
void dv_maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C, int P, int Q, int kh,
                    int kw, int sh, int sw, int ph, int pw, hipStream_t st) {
  PoolGeo g{N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw};
  const int v = C % 8 == 0 ? 8 : 1;
  const int64_t total = (int64_t)N * H * W * (C / v);
  VDISPATCH(C, maxpool_bwd_kernel, <<<grid_for(total), NT, 0, st>>>((const u16*)dy, idx, (u16*)dx, g, total));
}
// fused BN-apply + activation + max pool: C % 8 == 0 and C/8 a divisor of 256 (else -1); the
// 3x3 / stride-2 window (ResNet / Inception stems) is compiled, other windows take the runtime form
static bool stem_window(int kh, int kw, int sh, int sw) { return kh == 3 && kw == 3 && sh == 2 && sw == 2; }

int dv_bn_act_maxpool_fwd(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                          int sh, int sw, int ph, int pw, const float* scale, const float* shift, int act, float slope,
                          hipStream_t st) {
  const int64_t total = (int64_t)N * P * Q * (C / 8);
  if (C % 8 || NT % (C / 8) || kh * kw > 255 || kh > 16 || total >= (1ll << 31)) return -1;
  PoolGeo g{N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw};
  const FastDiv dc = make_fastdiv(C / 8), dq = make_fastdiv(Q), dp = make_fastdiv(P);
  const int grid = (int)std::min<int64_t>((total + NT - 1) / NT, 256 * 32);
#define FWD_ARGS <<<grid, NT, 0, st>>>((const u16*)x, (u16*)y, idx, g, dc, dq, dp, total, scale, shift, act, slope)
  if (stem_window(kh, kw, sh, sw) && act == 1) bn_act_maxpool_fwd_kernel<3, 3, 2, 2, true> FWD_ARGS;
  else if (stem_window(kh, kw, sh, sw)) bn_act_maxpool_fwd_kernel<3, 3, 2, 2, false> FWD_ARGS;
  else bn_act_maxpool_fwd_kernel<0, 0, 0, 0, false> FWD_ARGS;
#undef FWD_ARGS
  return 0;
}
int dv_bn_act_maxpool_bwd(const void* dy, const uint8_t* idx, const void* x, void* dx, int N, int H, int W, int C, int P,
                          int Q, int kh, int kw, int sh, int sw, int ph, int pw, const float* prm, const float* coef,
                          int act, float slope, float* acc, int apply, hipStream_t st) {
  const int64_t total = (int64_t)N * H * W * (C / 8);
  if (C % 8 || NT % (C / 8) || kh * kw > 255 || kh > 16 || total >= (1ll << 31)) return -1;
  PoolGeo g{N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw};
  if (stem_window(kh, kw, sh, sw) && ph == 1 && pw == 1 && H == 2 * P && W == 2 * Q && act >= 0 && act <= 2) {
    // 2x2 input block per thread (bn_act_maxpool_bwd_s2_kernel)
    const int64_t blocks = (int64_t)N * P * Q * (C / 8);
    const FastDiv dc = make_fastdiv(C / 8), dq = make_fastdiv(Q), dp = make_fastdiv(P);
    const int grid = (int)std::min<int64_t>((blocks + NT - 1) / NT, apply ? 256 * 32 : 2048);
    const DetStats det(apply ? 0 : grid, C, st);
#define S2_ARGS <<<grid, NT, 0, st>>>((const u16*)dy, idx, (const u16*)x, (u16*)dx, g, dc, dq, dp, blocks, prm, coef, slope, acc, det.slab)
#define S2_ACT(A) do { if (act == 0) bn_act_maxpool_bwd_s2_kernel<A, 0> S2_ARGS; \
                       else if (act == 1) bn_act_maxpool_bwd_s2_kernel<A, 1> S2_ARGS; \
                       else bn_act_maxpool_bwd_s2_kernel<A, 2> S2_ARGS; } while (0)
    if (apply) S2_ACT(true);
    else S2_ACT(false);
#undef S2_ACT
#undef S2_ARGS
    det.fold(acc);
    return 0;
  }
  const FastDiv dc = make_fastdiv(C / 8), dw = make_fastdiv(W), dh = make_fastdiv(H);
  // the reduction's atomics are one row per block: a bounded grid (~2k blocks) keeps them cheap
  const int grid = (int)std::min<int64_t>((total + NT - 1) / NT, apply ? 256 * 32 : 2048);
  const DetStats det(apply ? 0 : grid, C, st);
#define BWD_ARGS <<<grid, NT, 0, st>>>((const u16*)dy, idx, (const u16*)x, (u16*)dx, g, dc, dw, dh, total, prm, coef, act, slope, acc, det.slab)
  const bool stem = stem_window(kh, kw, sh, sw);
  if (apply) {
    if (stem) bn_act_maxpool_bwd_kernel<true, 3, 3, 2, 2> BWD_ARGS;
    else bn_act_maxpool_bwd_kernel<true, 0, 0, 0, 0> BWD_ARGS;
  } else {
    if (stem) bn_act_maxpool_bwd_kernel<false, 3, 3, 2, 2> BWD_ARGS;
    else bn_act_maxpool_bwd_kernel<false, 0, 0, 0, 0> BWD_ARGS;
  }
#undef BWD_ARGS
  det.fold(acc);
  return 0;
}
void dv_avgpool_fwd(const void* x, void* y, int N, int H, int W, int C, int P, int Q, int kh, int kw, int sh, int sw,
                    int ph, int pw, int cip, int divover, hipStream_t st) {
  PoolGeo g{N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw};
  const int v = C % 8 == 0 ? 8 : 1;
  const int64_t total = (int64_t)N * P * Q * (C / v);
  VDISPATCH(C, avgpool_fwd_kernel, <<<grid_for(total), NT, 0, st>>>((const u16*)x, (u16*)y, g, cip, divover, total));
}
void dv_avgpool_bwd(const void* dy, void* dx, int N, int H, int W, int C, int P, int Q, int kh, int kw, int sh, int sw,
                    int ph, int pw, int cip, int divover, hipStream_t st) {
  PoolGeo g{N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw};
  const int v = C % 8 == 0 ? 8 : 1;
  const int64_t total = (int64_t)N * H * W * (C / v);
  VDISPATCH(C, avgpool_bwd_kernel, <<<grid_for(total), NT, 0, st>>>((const u16*)dy, (u16*)dx, g, cip, divover, total));
}
void dv_gap_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st) {
  const int v = C % 8 == 0 ? 8 : 1;
  VDISPATCH(C, gap_fwd_kernel, <<<grid_for((int64_t)N * C / v), NT, 0, st>>>((const u16*)x, (u16*)y, N, HW, C));
}
void dv_gap_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st) {
  const int v = C % 8 == 0 ? 8 : 1;
  VDISPATCH(C, gap_bwd_kernel, <<<grid_for((int64_t)N * HW * C / v), NT, 0, st>>>((const u16*)dy, (u16*)dx, N, HW, C));
}
void dv_upsample_fwd(const void* x, void* y, int N, int H, int W, int C, int f, hipStream_t st) {
  const int v = C % 8 == 0 ? 8 : 1;
  VDISPATCH(C, upsample_fwd_kernel, <<<grid_for((int64_t)N * H * W * f * f * C / v), NT, 0, st>>>((const u16*)x, (u16*)y, N, H, W, C, f));
}
int dv_upsample_add(const void* x, const void* r, void* y, int N, int H, int W, int C, int f, float* stats,
                    hipStream_t st) {
  const int v = C % 8 == 0 ? 8 : 1;
  const int64_t total = (int64_t)N * H * W * f * f * C / v;
  if (stats) {
    if (!pool_stats_ok(C)) return -1;
    const int grid = stats_grid(total);
    DetStats d(grid, C, st);
    upsample_add_kernel<8><<<grid, NT, 0, st>>>((const u16*)x, (const u16*)r, (u16*)y, N, H, W, C, f, PoolStats{stats, d.slab});
    d.fold(stats);
    return 0;
  }
  VDISPATCH(C, upsample_add_kernel, <<<grid_for(total), NT, 0, st>>>((const u16*)x, (const u16*)r, (u16*)y, N, H, W, C, f, PoolStats{nullptr, nullptr}));
  return 0;
}
void dv_upsample_bwd(const void* dy, void* dx, int N, int H, int W, int C, int f, hipStream_t st) {
  const int v = C % 8 == 0 ? 8 : 1;
  VDISPATCH(C, upsample_bwd_kernel, <<<grid_for((int64_t)N * H * W * C / v), NT, 0, st>>>((const u16*)dy, (u16*)dx, N, H, W, C, f));
}
