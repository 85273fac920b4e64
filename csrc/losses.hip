// Pointwise training losses with their gradient (CenterNet focal/L1):
// one memory-bound pass over (rows x C) NHWC elements computes sum(loss) (and the positive
// count for the focal loss) and, in the backward launch, writes d(loss)/d(pred) scaled by the
// upstream gradient read from device memory (no host sync anywhere).
//
//   WMSE   l = w (p - t)^2,  w = 1 + a [t > 0]        Hourglass heatmaps (R/Hourglass/tensorflow/train.py:65-76)
//   MSE    l = (p - t)^2                              LSGAN (R/CycleGAN/tensorflow/train.py:53-62)
//   L1     l = |p - t|                                cycle / identity (R/CycleGAN/tensorflow/train.py:64-72)
//   BCEL   l = max(z,0) - z t + log(1 + e^-|z|)       BCE-from-logits (R/DCGAN/tensorflow/main.py:42-53)
//   FOCAL  penalty-reduced focal loss on sigmoid(z) (CenterNet, Zhou et al. 2019 eq. 1; the reference
//          trainer has no loss):  t == 1: -(1-p)^a log p ;  else -(1-t)^b p^a log(1-p)
//          with p clamped to [1e-4, 1-1e-4]; sums[1] counts the positives (t == 1)
//
// Layout: pred / target / grad are row-major (rows, ld) with C valid channels per row (padded NHWC
// channel strides are honoured, padding channels of the gradient are written as zeros). The
// target is fp32, bf16 or a scalar constant (GAN labels); an optional fp32 weight tensor (target
// layout) scales each element's loss and gradient (CenterNet's masked size / offset L1).
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;
enum { K_WMSE = 0, K_MSE = 1, K_L1 = 2, K_BCEL = 3, K_FOCAL = 4 };

template <typename T> DV_DEVICE float ldv(const T* p, int64_t i);
template <> DV_DEVICE float ldv<float>(const float* p, int64_t i) { return p[i]; }
template <> DV_DEVICE float ldv<u16>(const u16* p, int64_t i) { return bf2f(p[i]); }
template <typename T> DV_DEVICE void stv(T* p, int64_t i, float v);
template <> DV_DEVICE void stv<float>(float* p, int64_t i, float v) { p[i] = v; }
template <> DV_DEVICE void stv<u16>(u16* p, int64_t i, float v) { p[i] = f2bf(v); }

DV_DEVICE void pw_eval(int kind, float p, float t, float a, float b, float& l, float& g, float& pos) {
  pos = 0.f;
  switch (kind) {
    case K_WMSE: {
      const float w = 1.f + (t > 0.f ? a : 0.f), d = p - t;
      l = w * d * d; g = 2.f * w * d; break;
    }
    case K_MSE: { const float d = p - t; l = d * d; g = 2.f * d; break; }
    case K_L1: { const float d = p - t; l = fabsf(d); g = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); break; }
    case K_BCEL: {
      l = fmaxf(p, 0.f) - p * t + log1pf(__expf(-fabsf(p)));
      g = 1.f / (1.f + __expf(-p)) - t; break;
    }
    default: {  // K_FOCAL, p is the logit
      const float s = 1.f / (1.f + __expf(-p));
      const bool clamped = s < 1e-4f || s > 1.f - 1e-4f;
      const float q = fminf(fmaxf(s, 1e-4f), 1.f - 1e-4f);
      if (t >= 1.f) {
        pos = 1.f;
        const float om = 1.f - q, lq = __logf(q);
        l = -__powf(om, a) * lq;
        // d/dq [-(1-q)^a log q] = a (1-q)^(a-1) log q - (1-q)^a / q ; dq/dz = q (1-q)
        g = clamped ? 0.f : (a * __powf(om, a - 1.f) * lq - __powf(om, a) / q) * q * om;
      } else {
        const float nw = __powf(1.f - t, b), pa = __powf(q, a), l1q = __logf(1.f - q);
        l = -nw * pa * l1q;
        // d/dq [-nw q^a log(1-q)] = -nw (a q^(a-1) log(1-q) - q^a / (1-q))
        g = clamped ? 0.f : -nw * (a * __powf(q, a - 1.f) * l1q - pa / (1.f - q)) * q * (1.f - q);
      }
    }
  }
}

template <typename TP, typename TT>
__global__ __launch_bounds__(NT) void pw_loss_kernel(int kind, const TP* __restrict__ pred, const TT* __restrict__ tgt,
                                                     float tval, const float* __restrict__ wt, int64_t rows, int C,
                                                     int ldp, int ldt, float a, float b, float* __restrict__ sums,
                                                     TP* __restrict__ grad, const float* __restrict__ gscale,
                                                     float hscale, float* __restrict__ det) {
  __shared__ float sh[NT / 64];
  const int ldg = ldp;
  const int64_t total = rows * ldg;
  const float sc = grad ? (gscale ? gscale[0] : 1.f) * hscale : 0.f;
  float ls = 0.f, ps = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / ldg;
    const int c = (int)(i - r * ldg);
    if (c >= C) {
      if (grad) stv<TP>(grad, i, 0.f);
      continue;
    }
    const float p = ldv<TP>(pred, i);
    const float t = tgt ? ldv<TT>(tgt, r * ldt + c) : tval;
    float l, g, pos;
    pw_eval(kind, p, t, a, b, l, g, pos);
    if (wt) {
      const float w = wt[r * ldt + c];
      l *= w; g *= w;
    }
    ls += l; ps += pos;
    if (grad) stv<TP>(grad, i, g * sc);
  }
  if (sums) {
    ls = block_sum<NT>(ls, sh);
    if (kind == K_FOCAL) ps = block_sum<NT>(ps, sh);
    if (threadIdx.x == 0) {
      float* d = det ? det + blockIdx.x * (kind == K_FOCAL ? 2 : 1) : sums;  // deterministic mode: this block's slab row
      atomicAdd(d, ls);
      if (kind == K_FOCAL) atomicAdd(d + 1, ps);
    }
  }
}

template <typename TP, typename TT>
void launch(int kind, const void* pred, const void* tgt, float tval, const float* wt, int64_t rows, int C, int ldp,
            int ldt, float a, float b, float* sums, void* grad, const float* gscale, float hscale, hipStream_t st) {
  const int64_t total = rows * ldp;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + NT - 1) / NT, 2048));
  float* det = (sums && dv_deterministic()) ? dv_det_workspace((size_t)blocks * 2, st) : nullptr;
  pw_loss_kernel<TP, TT><<<blocks, NT, 0, st>>>(kind, (const TP*)pred, (const TT*)tgt, tval, wt, rows, C, ldp, ldt, a,
                                                b, sums, (TP*)grad, gscale, hscale, det);
  if (det) dv_det_sum(det, blocks, kind == K_FOCAL ? 2 : 1, sums, st);
}
}  // namespace

// tgt_type: 0 fp32, 1 bf16, 2 scalar (tval). wt: optional fp32 per-element weight in the target's layout.
void dv_pw_loss(int kind, const void* pred, int pred_bf16, const void* tgt, int tgt_type, float tval, const float* wt,
                int64_t rows, int C, int ldp, int ldt, float a, float b, float* sums, void* grad, const float* gscale,
                float hscale, hipStream_t st) {
  const void* t = tgt_type == 2 ? nullptr : tgt;
  if (pred_bf16) {
    if (tgt_type == 1) launch<u16, u16>(kind, pred, t, tval, wt, rows, C, ldp, ldt, a, b, sums, grad, gscale, hscale, st);
    else launch<u16, float>(kind, pred, t, tval, wt, rows, C, ldp, ldt, a, b, sums, grad, gscale, hscale, st);
  } else {
    if (tgt_type == 1) launch<float, u16>(kind, pred, t, tval, wt, rows, C, ldp, ldt, a, b, sums, grad, gscale, hscale, st);
    else launch<float, float>(kind, pred, t, tval, wt, rows, C, ldp, ldt, a, b, sums, grad, gscale, hscale, st);
  }
}
