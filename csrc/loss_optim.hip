// Softmax cross-entropy and fused optimizers over flat fp32 buffers (K20).
//
// softmax_xent: one block per row; single pass over the logits computes the row max and the
//   log-sum-exp (online), the loss, and writes d(loss)/d(logits) = (softmax - onehot) * scale
//   in the same launch, so the backward is free (the autograd node only rescales when the
//   upstream gradient is not 1).
// optimizers: one grid-stride launch updates every parameter of the model (flat buffer):
//   SGD      d = g*gs + wd*p ; buf = m*buf + (1-dampening)*d (first step buf = d) ; p -= lr*(nesterov ? d + m*buf : buf)
//   Adam     PyTorch semantics incl. bias correction, optional decoupled (AdamW) decay
//   RMSprop  PyTorch semantics (alpha, eps, momentum, centered)
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

template <bool BF16>
__global__ __launch_bounds__(NT) void softmax_xent_kernel(const void* __restrict__ logits, const int64_t* __restrict__ labels,
                                                            int C, float* __restrict__ loss_rows, void* __restrict__ grad,
                                                            float grad_scale, float label_smoothing) {
  __shared__ float sh[NT / 64];
  const int row = blockIdx.x;
  const int64_t base = (int64_t)row * C;
  auto ld = [&](int c) -> float {
    if (BF16) return bf2f(reinterpret_cast<const u16*>(logits)[base + c]);
    return reinterpret_cast<const float*>(logits)[base + c];
  };
  float m = -INFINITY, s = 0.f, sumx = 0.f;
  for (int c = threadIdx.x; c < C; c += NT) {
    const float v = ld(c);
    sumx += v;
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; } else s += __expf(v - m);
  }
  // combine (m, s) across the block
  float gm = wave_max(m);
  {
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[w] = gm;
    __syncthreads();
    gm = sh[0];
#pragma unroll
    for (int i = 1; i < NT / 64; ++i) gm = fmaxf(gm, sh[i]);
    __syncthreads();
  }
  float ss = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  ss = block_sum<NT>(ss, sh);
  const float lse = gm + __logf(ss);
  const int64_t lab = labels[row];
  const bool valid = lab >= 0 && lab < C;
  float sx = (label_smoothing > 0.f) ? block_sum<NT>(sumx, sh) : 0.f;
  if (threadIdx.x == 0) {
    float l = valid ? (lse - ld((int)lab)) : 0.f;
    if (label_smoothing > 0.f) l = (1.f - label_smoothing) * l + label_smoothing * (lse - sx / C);
    loss_rows[row] = l;
  }
  if (grad) {
    const float off = label_smoothing / C;
    for (int c = threadIdx.x; c < C; c += NT) {
      float g = __expf(ld(c) - lse);
      if (label_smoothing > 0.f) g -= off + (c == lab ? (1.f - label_smoothing) : 0.f);
      else if (c == lab) g -= 1.f;
      if (!valid) g = 0.f;
      g *= grad_scale;
      if (BF16) reinterpret_cast<u16*>(grad)[base + c] = f2bf(g);
      else reinterpret_cast<float*>(grad)[base + c] = g;
    }
  }
}

// hp (optional, device): [lr, bc1, bc2, step] written by the host before a HIP-graph replay, so a
// captured optimizer step follows LR schedules / Adam bias correction without re-capture
__global__ __launch_bounds__(NT) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                                                   int64_t n, float lr, float momentum, float dampening, float wd,
                                                   int nesterov, int first, float gscale, const float* __restrict__ hp,
                                                   const float* __restrict__ skip) {
  if (skip && *skip != 0.f) return;  // device non-finite guard: the step is a no-op
  if (hp) lr = hp[0];
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const float pv = p[i];
    float d = g[i] * gscale + wd * pv;
    if (momentum != 0.f) {
      float b = first ? d : momentum * buf[i] + (1.f - dampening) * d;
      buf[i] = b;
      d = nesterov ? d + momentum * b : b;
    }
    p[i] = pv - lr * d;
  }
}

__global__ __launch_bounds__(NT) void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                                                    float wd, int decoupled, float bc1, float bc2, float gscale,
                                                    const float* __restrict__ hp, const float* __restrict__ skip) {
  if (skip && *skip != 0.f) return;
  if (hp) { lr = hp[0]; bc1 = hp[1]; bc2 = hp[2]; }
  if (hp && skip) {  // device guard: the bias corrections count the steps actually applied (guard[4])
    const float t = skip[4] + 1.f;
    bc1 = 1.f - powf(b1, t);
    bc2 = 1.f - powf(b2, t);
  }
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    float pv = p[i];
    float gv = g[i] * gscale;
    if (decoupled) pv *= (1.f - lr * wd); else gv += wd * pv;
    const float mv = b1 * m[i] + (1.f - b1) * gv;
    const float vv = b2 * v[i] + (1.f - b2) * gv * gv;
    m[i] = mv; v[i] = vv;
    const float denom = sqrtf(vv / bc2) + eps;
    p[i] = pv - (lr / bc1) * mv / denom;
  }
}

__global__ __launch_bounds__(NT) void rmsprop_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ sq,
                                                       float* __restrict__ mom, float* __restrict__ gavg, int64_t n, float lr,
                                                       float alpha, float eps, float wd, float momentum, int centered, float gscale,
                                                       const float* __restrict__ hp, const float* __restrict__ skip) {
  if (skip && *skip != 0.f) return;
  if (hp) lr = hp[0];
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const float pv = p[i];
    const float gv = g[i] * gscale + wd * pv;
    const float s = alpha * sq[i] + (1.f - alpha) * gv * gv;
    sq[i] = s;
    float avg;
    if (centered) { const float ga = alpha * gavg[i] + (1.f - alpha) * gv; gavg[i] = ga; avg = sqrtf(s - ga * ga) + eps; }
    else avg = sqrtf(s) + eps;
    if (momentum > 0.f) { const float b = momentum * mom[i] + gv / avg; mom[i] = b; p[i] = pv - lr * b; }
    else p[i] = pv - lr * gv / avg;
  }
}

// sum of squares (grad-norm / non-finite detection): block partials -> atomic
__global__ __launch_bounds__(NT) void sumsq_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out,
                                                   float* __restrict__ det) {
  __shared__ float sh[NT / 64];
  float s = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) { const float v = x[i]; s += v * v; }
  s = block_sum<NT>(s, sh);
  if (threadIdx.x == 0) atomicAdd(det ? det + blockIdx.x : out, s);  // det: this block's slab row
}

// Device-side non-finite guard (graph-captured steps: no host sync). guard = [flag, skipped total,
// consecutive skips, last step's flag, steps applied]. nonfinite_check ORs "any non-finite gradient" into flag
// (every finder stores the same 1.0: plain vector stores, no atomics); the optimizer kernels
// read flag and skip the whole update; nonfinite_tally, the step's last launch, folds flag into
// the counters and re-arms it for the next step. In a data-parallel step the checked buffer is
// the all-reduced gradient, identical on every rank, so every rank skips or steps together.
template <bool V4>
__global__ __launch_bounds__(NT) void nonfinite_check_kernel(const float* __restrict__ g, int64_t n,
                                                               float* __restrict__ guard) {
  bool bad = false;
  if constexpr (V4) {  // 16-B aligned buffer: float4 body + scalar tail
    const int64_t n4 = n >> 2;
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT) {
      const float4 v = g4[i];
      bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) bad |= !isfinite(g[n4 * 4 + threadIdx.x]);
  } else {
    for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) bad |= !isfinite(g[i]);
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0) guard[0] = 1.f;
}

__global__ void nonfinite_tally_kernel(float* __restrict__ guard) {
  const float f = guard[0] != 0.f ? 1.f : 0.f;
  guard[1] += f;
  guard[2] = f != 0.f ? guard[2] + 1.f : 0.f;
  guard[3] = f;
  guard[4] += 1.f - f;  // Adam's bias corrections under the guard count applied steps only
  guard[0] = 0.f;
}

inline int grid_for(int64_t n) {
  int64_t g = (n + NT - 1) / NT;
  return (int)std::min<int64_t>(std::max<int64_t>(g, 1), 256 * 8);
}
}  // namespace

void dv_softmax_xent(const void* logits, int is_bf16, const int64_t* labels, int rows, int C, float* loss_rows, void* grad,
                     float grad_scale, float label_smoothing, hipStream_t st) {
  if (is_bf16) softmax_xent_kernel<true><<<rows, NT, 0, st>>>(logits, labels, C, loss_rows, grad, grad_scale, label_smoothing);
  else softmax_xent_kernel<false><<<rows, NT, 0, st>>>(logits, labels, C, loss_rows, grad, grad_scale, label_smoothing);
}
// out = in * (*s): the cross-entropy backward's upstream-gradient scale, read on the device (no
// host sync) -- one vectorised launch instead of a broadcasting torch multiply with type promotion
template <bool BF>
__global__ __launch_bounds__(NT) void scale_by_kernel(const void* __restrict__ in, void* __restrict__ out, int64_t n,
                                                      const float* __restrict__ s) {
  const float k = *s;
  const int64_t i0 = ((int64_t)blockIdx.x * NT + threadIdx.x) * 8;
  if (i0 >= n) return;
  if constexpr (BF) {
    const u16* a = reinterpret_cast<const u16*>(in) + i0;
    u16* o = reinterpret_cast<u16*>(out) + i0;
    if (i0 + 8 <= n) {
      const uint4 v = *reinterpret_cast<const uint4*>(a);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      uint32_t r[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = pack2bf(bf2f(w[e] & 0xffff) * k, bf2f(w[e] >> 16) * k);
      *reinterpret_cast<uint4*>(o) = uint4{r[0], r[1], r[2], r[3]};
    } else {
      for (int64_t i = 0; i < n - i0; ++i) o[i] = f2bf(bf2f(a[i]) * k);
    }
  } else {
    const float* a = reinterpret_cast<const float*>(in) + i0;
    float* o = reinterpret_cast<float*>(out) + i0;
    for (int64_t i = 0; i < 8 && i0 + i < n; ++i) o[i] = a[i] * k;
  }
}
void dv_scale_by(const void* in, void* out, int64_t n, int is_bf16, const float* s, hipStream_t st) {
  const unsigned g = (unsigned)((n + NT * 8 - 1) / (NT * 8));
  if (is_bf16) scale_by_kernel<true><<<g, NT, 0, st>>>(in, out, n, s);
  else scale_by_kernel<false><<<g, NT, 0, st>>>(in, out, n, s);
}
void dv_sgd(float* p, const float* g, float* buf, int64_t n, float lr, float momentum, float dampening, float wd,
            int nesterov, int first, float gscale, const float* hp, hipStream_t st, const float* skip) {
  sgd_kernel<<<grid_for(n), NT, 0, st>>>(p, g, buf, n, lr, momentum, dampening, wd, nesterov, first, gscale, hp, skip);
}
void dv_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2, float eps, float wd,
             int decoupled, float bc1, float bc2, float gscale, const float* hp, hipStream_t st, const float* skip) {
  adam_kernel<<<grid_for(n), NT, 0, st>>>(p, g, m, v, n, lr, b1, b2, eps, wd, decoupled, bc1, bc2, gscale, hp, skip);
}
void dv_rmsprop(float* p, const float* g, float* sq, float* mom, float* gavg, int64_t n, float lr, float alpha, float eps,
                float wd, float momentum, int centered, float gscale, const float* hp, hipStream_t st, const float* skip) {
  rmsprop_kernel<<<grid_for(n), NT, 0, st>>>(p, g, sq, mom, gavg, n, lr, alpha, eps, wd, momentum, centered, gscale, hp,
                                             skip);
}
void dv_nonfinite_check(const float* g, int64_t n, float* guard, hipStream_t st) {
  if (((uintptr_t)g & 15) == 0) nonfinite_check_kernel<true><<<std::min(grid_for((n + 3) / 4), 1024), NT, 0, st>>>(g, n, guard);
  else nonfinite_check_kernel<false><<<std::min(grid_for(n), 1024), NT, 0, st>>>(g, n, guard);
}
void dv_nonfinite_tally(float* guard, hipStream_t st) { nonfinite_tally_kernel<<<1, 1, 0, st>>>(guard); }
void dv_sumsq(const float* x, int64_t n, float* out, hipStream_t st) {
  const int grid = std::min(grid_for(n), 1024);
  float* det = dv_deterministic() ? dv_det_workspace((size_t)grid, st) : nullptr;
  sumsq_kernel<<<grid, NT, 0, st>>>(x, n, out, det);
  if (det) dv_det_sum(det, grid, 1, out, st);
}
