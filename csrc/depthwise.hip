// Depthwise convolution (groups == channels) on bf16 NHWC — SURVEY §2.7 K6 (MobileNet V1
// R/MobileNet/pytorch/models/mobilenet_v1.py:109-133, Keras DepthwiseConv2D in
// R/MobileNet/tensorflow/models/mobilenet_v1.py:7-25).
//
// Depthwise conv has no reduction over channels, so there is nothing for MFMA to do: it is a
// bandwidth-bound stencil. Design:
//   * one thread = 8 consecutive channels (16-B loads/stores) x a strip of QT output pixels
//     along W; the weights of its 8 channels live in registers (read once, fp32 master
//     weights directly — no bf16 weight-prep launch);
//   * the input row segment shared by the strip is loaded once per filter row and reused
//     from registers for all QT outputs (stride 1 reuses (QT+S-1)/ (QT*S) of the loads);
//   * forward epilogue: optional bias, ReLU, and per-channel BatchNorm partial statistics
//     (thread partials -> LDS reduction over the block's pixel rows -> sharded atomics),
//     so the following BN needs no statistics pass;
//   * dgrad: the transposed stencil (divisibility gather for stride 2);
//   * wgrad: per-thread 8ch x R x S partials over a pixel range, LDS tree over the block,
//     one fp32 atomic per (channel, tap) per block into dW (plain accumulate into the live
//     gradient when requested).
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;
constexpr int QT = 4;  // output pixels per thread along W (forward)

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
};

// thread layout: TPR = C/8 channel groups per pixel strip (capped at NT), RPI strips per pass
template <int KS>
__global__ __launch_bounds__(NT) void dw_fwd_kernel(const u16* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ bias, u16* __restrict__ y, DwGeo g,
                                                      int act, float slope, float* __restrict__ stats, int strips_per_block) {
  __shared__ float sh[2][NT * 8];
  const int cgn = g.C / 8;
  const int tpr = cgn < NT ? cgn : NT, rpi = NT / tpr;
  const int lane_c = threadIdx.x % tpr, lane_r = threadIdx.x / tpr;
  const int qstrips = (g.Q + QT - 1) / QT;
  const int64_t nstrips = (int64_t)g.N * g.P * qstrips;
  const int64_t s0 = (int64_t)blockIdx.x * strips_per_block;
  const int64_t s1 = min(nstrips, s0 + strips_per_block);
  for (int cgi = lane_c; cgi < cgn; cgi += tpr) {
    const int c0 = cgi * 8;
    float wr[KS * KS][8];
#pragma unroll
    for (int t = 0; t < KS * KS; ++t)
#pragma unroll
      for (int k = 0; k < 8; ++k) wr[t][k] = w[(c0 + k) * KS * KS + t];
    float bv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) bv[k] = bias ? bias[c0 + k] : 0.f;
    float ssum[8], ssq[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { ssum[k] = 0.f; ssq[k] = 0.f; }
    if (lane_r < rpi) {
      for (int64_t s = s0 + lane_r; s < s1; s += rpi) {
        const int qs = (int)(s % qstrips);
        const int64_t np = s / qstrips;
        const int p = (int)(np % g.P), n = (int)(np / g.P);
        const int q0 = qs * QT;
        float acc[QT][8];
#pragma unroll
        for (int i = 0; i < QT; ++i)
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[i][k] = bv[k];
#pragma unroll
        for (int r = 0; r < KS; ++r) {
          const int h = p * g.sh - g.ph + r;
          if (h < 0 || h >= g.H) continue;
          const u16* xrow = x + ((int64_t)n * g.H + h) * g.W * g.ldx + c0;
#pragma unroll
          for (int i = 0; i < QT; ++i) {
            const int q = q0 + i;
#pragma unroll
            for (int sx = 0; sx < KS; ++sx) {
              const int ww = q * g.sw - g.pw + sx;
              if (q >= g.Q || ww < 0 || ww >= g.W) continue;
              float v[8];
              ld8(xrow + (int64_t)ww * g.ldx, v);
#pragma unroll
              for (int k = 0; k < 8; ++k) acc[i][k] = fmaf(v[k], wr[r * KS + sx][k], acc[i][k]);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < QT; ++i) {
          const int q = q0 + i;
          if (q >= g.Q) continue;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            float t = acc[i][k];
            if (act == 1) t = fmaxf(t, 0.f);
            else if (act == 2) t = t > 0.f ? t : t * slope;
            acc[i][k] = t;
            ssum[k] += t; ssq[k] += t * t;
          }
          st8(y + (((int64_t)n * g.P + p) * g.Q + q) * g.ldy + c0, acc[i]);
        }
      }
    }
    if (stats) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) { sh[0][threadIdx.x * 8 + k] = ssum[k]; sh[1][threadIdx.x * 8 + k] = ssq[k]; }
      __syncthreads();
      if (lane_r == 0) {
        for (int rr = 1; rr < rpi; ++rr)
#pragma unroll
          for (int k = 0; k < 8; ++k) { ssum[k] += sh[0][(rr * tpr + lane_c) * 8 + k]; ssq[k] += sh[1][(rr * tpr + lane_c) * 8 + k]; }
        float* a = stats + (int64_t)(blockIdx.x % DV_STAT_SHARDS) * 2 * g.C;
#pragma unroll
        for (int k = 0; k < 8; ++k) { atomicAdd(a + c0 + k, ssum[k]); atomicAdd(a + g.C + c0 + k, ssq[k]); }
      }
    }
  }
}

// dx[n][h][w][c] = sum_{r,s} dy[n][(h+ph-r)/sh][(w+pw-s)/sw][c] * w[c][r][s]
template <int KS>
__global__ __launch_bounds__(NT) void dw_dgrad_kernel(const u16* __restrict__ dy, const float* __restrict__ w,
                                                        u16* __restrict__ dx, DwGeo g) {
  const int cgn = g.C / 8;
  const int64_t total = (int64_t)g.N * g.H * g.W * cgn;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cgi = (int)(t % cgn);
    int64_t pix = t / cgn;
    const int ww = (int)(pix % g.W); pix /= g.W;
    const int h = (int)(pix % g.H); const int n = (int)(pix / g.H);
    const int c0 = cgi * 8;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
    for (int r = 0; r < KS; ++r) {
      const int hn = h + g.ph - r;
      if (hn < 0 || hn % g.sh) continue;
      const int p = hn / g.sh;
      if (p >= g.P) continue;
#pragma unroll
      for (int sx = 0; sx < KS; ++sx) {
        const int wn = ww + g.pw - sx;
        if (wn < 0 || wn % g.sw) continue;
        const int q = wn / g.sw;
        if (q >= g.Q) continue;
        float v[8];
        ld8(dy + (((int64_t)n * g.P + p) * g.Q + q) * g.ldy + c0, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(v[k], w[(c0 + k) * KS * KS + r * KS + sx], acc[k]);
      }
    }
    st8(dx + (((int64_t)n * g.H + h) * g.W + ww) * g.ldx + c0, acc);
  }
}

// dw[c][r][s] += sum_{n,p,q} dy[n][p][q][c] * x[n][p*sh-ph+r][q*sw-pw+s][c]
template <int KS>
__global__ __launch_bounds__(NT) void dw_wgrad_kernel(const u16* __restrict__ x, const u16* __restrict__ dy,
                                                        float* __restrict__ dw, DwGeo g, int64_t pix_per_block) {
  __shared__ float sh[NT * 8];
  const int cgn = g.C / 8;
  const int tpr = cgn < NT ? cgn : NT, rpi = NT / tpr;
  const int lane_c = threadIdx.x % tpr, lane_r = threadIdx.x / tpr;
  const int64_t npix = (int64_t)g.N * g.P * g.Q;
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_block, p1 = min(npix, p0 + pix_per_block);
  for (int cgi = lane_c; cgi < cgn; cgi += tpr) {
    const int c0 = cgi * 8;
    float acc[KS * KS][8];
#pragma unroll
    for (int t = 0; t < KS * KS; ++t)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[t][k] = 0.f;
    if (lane_r < rpi) {
      for (int64_t pi = p0 + lane_r; pi < p1; pi += rpi) {
        const int q = (int)(pi % g.Q);
        const int64_t np = pi / g.Q;
        const int p = (int)(np % g.P), n = (int)(np / g.P);
        float d[8];
        ld8(dy + pi * g.ldy + c0, d);
#pragma unroll
        for (int r = 0; r < KS; ++r) {
          const int h = p * g.sh - g.ph + r;
          if (h < 0 || h >= g.H) continue;
#pragma unroll
          for (int sx = 0; sx < KS; ++sx) {
            const int ww = q * g.sw - g.pw + sx;
            if (ww < 0 || ww >= g.W) continue;
            float v[8];
            ld8(x + (((int64_t)n * g.H + h) * g.W + ww) * g.ldx + c0, v);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[r * KS + sx][k] = fmaf(d[k], v[k], acc[r * KS + sx][k]);
          }
        }
      }
    }
    // block reduction per tap over the rpi pixel lanes sharing these channels
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) sh[threadIdx.x * 8 + k] = acc[t][k];
      __syncthreads();
      if (lane_r == 0) {
        float s[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] = acc[t][k];
        for (int rr = 1; rr < rpi; ++rr)
#pragma unroll
          for (int k = 0; k < 8; ++k) s[k] += sh[(rr * tpr + lane_c) * 8 + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) atomicAdd(dw + (c0 + k) * KS * KS + t, s[k]);
      }
    }
  }
}

inline int grid_for(int64_t total) {
  int64_t gsz = (total + NT - 1) / NT;
  return (int)std::min<int64_t>(std::max<int64_t>(gsz, 1), 256 * 16);
}
}  // namespace

#define DW_KS_DISPATCH(K, KERNEL, ...)                                  \
  switch (K) {                                                          \
    case 3: KERNEL<3> __VA_ARGS__; break;                               \
    case 5: KERNEL<5> __VA_ARGS__; break;                               \
    case 1: KERNEL<1> __VA_ARGS__; break;                               \
    case 7: KERNEL<7> __VA_ARGS__; break;                               \
    default: return -1;                                                 \
  }

// the block-wide barriers inside the channel-group loop need a uniform trip count
static inline bool dw_shape_ok(int C, int ldx, int ldy) {
  const int cgn = C / 8;
  return C % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && (cgn <= NT || cgn % NT == 0);
}

int dv_dw_fwd(const void* x, const float* w, const float* bias, void* y, int N, int H, int W, int C, int ldx, int P,
              int Q, int ldy, int K, int sh, int sw, int ph, int pw, int act, float slope, float* stats, hipStream_t st) {
  if (!dw_shape_ok(C, ldx, ldy)) return -1;
  DwGeo g{N, H, W, C, ldx, P, Q, ldy, sh, sw, ph, pw};
  const int cgn = C / 8, tpr = cgn < NT ? cgn : NT, rpi = NT / tpr;
  const int64_t nstrips = (int64_t)N * P * ((Q + QT - 1) / QT);
  // channel groups beyond NT threads are looped inside the block
  int64_t spb = std::max<int64_t>(rpi, (nstrips + 2047) / 2048);
  spb = (spb + rpi - 1) / rpi * rpi;
  const int blocks = (int)((nstrips + spb - 1) / spb);
  DW_KS_DISPATCH(K, dw_fwd_kernel, <<<blocks, NT, 0, st>>>((const u16*)x, w, bias, (u16*)y, g, act, slope, stats, (int)spb))
  return 0;
}

int dv_dw_dgrad(const void* dy, const float* w, void* dx, int N, int H, int W, int C, int ldx, int P, int Q, int ldy,
                int K, int sh, int sw, int ph, int pw, hipStream_t st) {
  if (C % 8 || ldx % 8 || ldy % 8) return -1;
  DwGeo g{N, H, W, C, ldx, P, Q, ldy, sh, sw, ph, pw};
  const int64_t total = (int64_t)N * H * W * (C / 8);
  DW_KS_DISPATCH(K, dw_dgrad_kernel, <<<grid_for(total), NT, 0, st>>>((const u16*)dy, w, (u16*)dx, g))
  return 0;
}

int dv_dw_wgrad(const void* x, const void* dy, float* dw, int N, int H, int W, int C, int ldx, int P, int Q, int ldy,
                int K, int sh, int sw, int ph, int pw, int accumulate, hipStream_t st) {
  if (!dw_shape_ok(C, ldx, ldy)) return -1;
  DwGeo g{N, H, W, C, ldx, P, Q, ldy, sh, sw, ph, pw};
  if (!accumulate) (void)hipMemsetAsync(dw, 0, (size_t)C * K * K * sizeof(float), st);
  const int64_t npix = (int64_t)N * P * Q;
  int64_t ppb = std::max<int64_t>(256, (npix + 1023) / 1024);
  const int blocks = (int)((npix + ppb - 1) / ppb);
  DW_KS_DISPATCH(K, dw_wgrad_kernel, <<<blocks, NT, 0, st>>>((const u16*)x, (const u16*)dy, dw, g, ppb))
  return 0;
}
