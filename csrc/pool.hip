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

template <int VEC>
__global__ __launch_bounds__(NT) void maxpool_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y,
                                                           uint8_t* __restrict__ idx, PoolGeo g, int64_t total) {
  const int cg = g.C / VEC;
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
  }
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

inline int grid_for(int64_t total) {
  int64_t g = (total + NT - 1) / NT;
  return (int)std::min<int64_t>(std::max<int64_t>(g, 1), 256 * 16);
}
}  // namespace

#define VDISPATCH(C, K, ...) do { if ((C) % 8 == 0) K<8> __VA_ARGS__; else K<1> __VA_ARGS__; } while (0)

void dv_maxpool_fwd(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                    int sh, int sw, int ph, int pw, hipStream_t st) {
  PoolGeo g{N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw};
  const int v = C % 8 == 0 ? 8 : 1;
  const int64_t total = (int64_t)N * P * Q * (C / v);
  VDISPATCH(C, maxpool_fwd_kernel, <<<grid_for(total), NT, 0, st>>>((const u16*)x, (u16*)y, idx, g, total));
}
void dv_maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C, int P, int Q, int kh,
                    int kw, int sh, int sw, int ph, int pw, hipStream_t st) {
  PoolGeo g{N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw};
  const int v = C % 8 == 0 ? 8 : 1;
  const int64_t total = (int64_t)N * H * W * (C / v);
  VDISPATCH(C, maxpool_bwd_kernel, <<<grid_for(total), NT, 0, st>>>((const u16*)dy, idx, (u16*)dx, g, total));
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
void dv_upsample_bwd(const void* dy, void* dx, int N, int H, int W, int C, int f, hipStream_t st) {
  const int v = C % 8 == 0 ? 8 : 1;
  VDISPATCH(C, upsample_bwd_kernel, <<<grid_for((int64_t)N * H * W * C / v), NT, 0, st>>>((const u16*)dy, (u16*)dx, N, H, W, C, f));
}
