// Local Response Normalisation across channels on bf16 NHWC.
//
//   out_c = a_c * D_c^-beta,  D_c = k + alpha_eff * sum_{j = c-lo}^{c+hi} a_j^2   (clipped window)
//
// torch.nn.LocalResponseNorm(size, alpha, beta, k): lo = size/2, hi = (size-1)/2,
//   alpha_eff = alpha/size (R/AlexNet/pytorch/models/alexnet_v1.py:41 uses size = C).
// tf.nn.local_response_normalization(depth_radius r, bias, alpha, beta): lo = hi = r,
//   alpha_eff = alpha (R/AlexNet/tensorflow/models/alexnet_v2.py:9-22).
//
// Backward:  da_c = g_c D_c^-beta - 2 beta alpha_eff a_c * sum_{j = c-hi}^{c+lo} g_j a_j D_j^(-beta-1).
//
// One wave per pixel: NHWC makes a pixel's channels contiguous, each lane owns CPL consecutive
// channels; window sums come from an inclusive prefix sum (in-lane serial + wave shuffle scan)
// staged in LDS so any lane can read P[c+hi+1] - P[c-lo]. O(C) per pixel for any window size
// (the reference's size == C window would be O(C^2) directly).
#include "common.h"
#include "kernels.h"

namespace {
constexpr int WPB = 4;  // waves per block

template <int CPL>
DV_DEVICE void wave_prefix(const float (&v)[CPL], float* P, int C, int lane) {
  // P[0] = 0, P[i+1] = sum_{j<=i} v_j  for the lane-chunked vector
  float run[CPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) { s += v[i]; run[i] = s; }
  float incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const float excl = incl - s;
  if (lane == 0) P[0] = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane * CPL + i;
    if (c < C) P[c + 1] = excl + run[i];
  }
}

template <int CPL>
__global__ __launch_bounds__(WPB * 64) void lrn_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y, int64_t npix,
                                                             int C, int lo, int hi, float alpha, float beta, float kk) {
  __shared__ float Pbuf[WPB][CPL * 64 + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* P = Pbuf[wv];
  for (int64_t pix = (int64_t)blockIdx.x * WPB + wv; pix < npix; pix += (int64_t)gridDim.x * WPB) {
    const u16* xr = x + pix * C;
    float a[CPL], sq[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane * CPL + i;
      a[i] = c < C ? bf2f(xr[c]) : 0.f;
      sq[i] = a[i] * a[i];
    }
    wave_prefix<CPL>(sq, P, C, lane);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane * CPL + i;
      if (c >= C) continue;
      const int l = max(0, c - lo), h = min(C, c + hi + 1);
      const float D = kk + alpha * (P[h] - P[l]);
      y[pix * C + c] = f2bf(a[i] * __powf(D, -beta));
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <int CPL>
__global__ __launch_bounds__(WPB * 64) void lrn_bwd_kernel(const u16* __restrict__ x, const u16* __restrict__ dy,
                                                             u16* __restrict__ dx, int64_t npix, int C, int lo, int hi,
                                                             float alpha, float beta, float kk) {
  __shared__ float Pbuf[WPB][CPL * 64 + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* P = Pbuf[wv];
  for (int64_t pix = (int64_t)blockIdx.x * WPB + wv; pix < npix; pix += (int64_t)gridDim.x * WPB) {
    float a[CPL], g[CPL], t[CPL], D[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane * CPL + i;
      a[i] = c < C ? bf2f(x[pix * C + c]) : 0.f;
      g[i] = c < C ? bf2f(dy[pix * C + c]) : 0.f;
      t[i] = a[i] * a[i];
    }
    wave_prefix<CPL>(t, P, C, lane);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane * CPL + i;
      float d = 1.f;
      if (c < C) {
        const int l = max(0, c - lo), h = min(C, c + hi + 1);
        d = kk + alpha * (P[h] - P[l]);
      }
      D[i] = d;
      t[i] = g[i] * a[i] * __powf(d, -beta - 1.f);
    }
    __builtin_amdgcn_wave_barrier();
    wave_prefix<CPL>(t, P, C, lane);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane * CPL + i;
      if (c >= C) continue;
      const int l = max(0, c - hi), h = min(C, c + lo + 1);
      const float T = P[h] - P[l];
      dx[pix * C + c] = f2bf(g[i] * __powf(D[i], -beta) - 2.f * beta * alpha * a[i] * T);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

inline int blocks_for(int64_t npix) {
  int64_t b = (npix + WPB - 1) / WPB;
  return (int)std::min<int64_t>(std::max<int64_t>(b, 1), 256 * 32);
}
}  // namespace

#define LRN_DISPATCH(C, KERNEL, ...)                                        \
  if ((C) <= 128) KERNEL<2> __VA_ARGS__;                                     \
  else if ((C) <= 256) KERNEL<4> __VA_ARGS__;                                \
  else if ((C) <= 512) KERNEL<8> __VA_ARGS__;                                \
  else if ((C) <= 1024) KERNEL<16> __VA_ARGS__;                              \
  else return -1;

int dv_lrn_fwd(const void* x, void* y, int64_t npix, int C, int lo, int hi, float alpha, float beta, float k,
               hipStream_t st) {
  LRN_DISPATCH(C, lrn_fwd_kernel, <<<blocks_for(npix), WPB * 64, 0, st>>>((const u16*)x, (u16*)y, npix, C, lo, hi, alpha, beta, k))
  return 0;
}

int dv_lrn_bwd(const void* x, const void* dy, void* dx, int64_t npix, int C, int lo, int hi, float alpha, float beta,
               float k, hipStream_t st) {
  LRN_DISPATCH(C, lrn_bwd_kernel, <<<blocks_for(npix), WPB * 64, 0, st>>>((const u16*)x, (const u16*)dy, (u16*)dx, npix, C, lo, hi, alpha, beta, k))
  return 0;
}
