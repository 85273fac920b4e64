// BatchNorm2d (training + eval) on bf16 NHWC activations, fp32 statistics.
// per-channel batch statistics, fused BN-apply + ReLU/LeakyReLU
// (+ residual add) forward, fused activation-backward + BN-backward.
//
// Statistics travel through a sharded fp32 accumulator `acc[SHARDS][2][C]` + a shift row `[C]`
// (kernels.h DV_STAT_ROWS):
//   * the conv epilogue (conv_fwd.hip), the depthwise forward or `bn_stats_kernel` atomically
//     adds per-block partial sums of d = x - K and d^2 into shard blockIdx % SHARDS (spreads
//     same-address atomics 64 ways), K = the shift row: this BN's previous batch mean;
//   * `bn_finalize_kernel` folds the shards into mean = K + E[d], var = E[d^2] - E[d]^2,
//     invstd / scale / shift, updates the running statistics with PyTorch semantics (unbiased
//     running_var) and stores the batch mean as the next shift. With K = 0 (first step) this is
//     the plain single-pass form; afterwards the E[x^2] - mean^2 cancellation (large |mean| /
//     std) is gone.
// Backward uses the same shard layout for (sum dz, sum dz*xhat).
#include <cstdlib>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace {
constexpr int SHARDS = DV_STAT_SHARDS;
constexpr int NT = 256;

template <int VEC> struct VecIO;
template <> struct VecIO<8> {
  DV_DEVICE static void load(const u16* p, float* v) {
    uint4 r = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[2 * i] = bf2f(w[i] & 0xffff); v[2 * i + 1] = bf2f(w[i] >> 16); }
  }
  // streaming read of an apply pass's input (read once by this pass): non-temporal policy
  DV_DEVICE static void load_nt(const u16* p, float* v) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[2 * i] = bf2f(w[i] & 0xffff); v[2 * i + 1] = bf2f(w[i] >> 16); }
  }
  DV_DEVICE static void store(u16* p, const float* v) {
    uint4 r; r.x = pack2bf(v[0], v[1]); r.y = pack2bf(v[2], v[3]); r.z = pack2bf(v[4], v[5]); r.w = pack2bf(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = r;
  }
};
template <> struct VecIO<4> {
  DV_DEVICE static void load_nt(const u16* p, float* v) { load(p, v); }
  DV_DEVICE static void load(const u16* p, float* v) {
    uint2 r = *reinterpret_cast<const uint2*>(p);
    v[0] = bf2f(r.x & 0xffff); v[1] = bf2f(r.x >> 16); v[2] = bf2f(r.y & 0xffff); v[3] = bf2f(r.y >> 16);
  }
  DV_DEVICE static void store(u16* p, const float* v) {
    uint2 r; r.x = pack2bf(v[0], v[1]); r.y = pack2bf(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = r;
  }
};
template <> struct VecIO<2> {
  DV_DEVICE static void load_nt(const u16* p, float* v) { load(p, v); }
  DV_DEVICE static void load(const u16* p, float* v) {
    uint32_t r = *reinterpret_cast<const uint32_t*>(p); v[0] = bf2f(r & 0xffff); v[1] = bf2f(r >> 16);
  }
  DV_DEVICE static void store(u16* p, const float* v) { *reinterpret_cast<uint32_t*>(p) = pack2bf(v[0], v[1]); }
};
template <> struct VecIO<1> {
  DV_DEVICE static void load_nt(const u16* p, float* v) { load(p, v); }
  DV_DEVICE static void load(const u16* p, float* v) { v[0] = bf2f(*p); }
  DV_DEVICE static void store(u16* p, const float* v) { *p = f2bf(v[0]); }
};

// The apply passes stream tensors far larger than the 256 MB MALL at the big layers: their
// once-read inputs go through the non-temporal policy there (512x28x28 / 1024x14x14 at batch 256:
// 15-22 % faster, profiles/bn_apply_nt.txt) and through the default policy for tensors small
// enough to still sit in the MALL from their producer (2048x7x7: 12 % slower with nt).
const int64_t NT_LOAD_MIN_ELEMS = [] {
  const char* v = std::getenv("DV_NT_MIN");  // benchmarking override (elements)
  return v ? (int64_t)std::atoll(v) : (24ll << 20);
}();
template <bool NTL, int VEC>
DV_DEVICE void ldv(const u16* p, float* v) {
  if constexpr (NTL) VecIO<VEC>::load_nt(p, v);
  else VecIO<VEC>::load(p, v);
}

DV_DEVICE float act_fwd(float z, int act, float slope) {
  if (act == 1) return fmaxf(z, 0.f);
  if (act == 2) return z > 0.f ? z : z * slope;
  return z;
}
// derivative from the activation OUTPUT (relu: out>0; leaky: out>0 ? 1 : slope)
DV_DEVICE float act_bwd(float dout, float out, int act, float slope) {
  if (act == 1) return out > 0.f ? dout : 0.f;
  if (act == 2) return out > 0.f ? dout : dout * slope;
  return dout;
}

// ---- statistics of an NHWC tensor: rows x C -> shard accumulators ----
// 2-D grid: blockIdx.y = channel slab of up to 64 x VEC channels (one wave-width of 16-B vectors
// per row), blockIdx.x = row range. TPR threads cover the slab of one row, RPI = NT/TPR rows per
// iteration. Wide layers (C = 1024 / 2048 at 14x14 / 7x7) have few rows: slabs keep >= ~4
// blocks per CU in flight there instead of a few hundred row blocks.
constexpr int SLAB_TPR = 64;
struct SlabTile {
  int cg, tpr, rpi, lane_c, lane_r, g;
  int64_t r0, r1;
  DV_DEVICE SlabTile(int C, int VEC, int64_t rows) {
    cg = C / VEC; tpr = cg < SLAB_TPR ? cg : SLAB_TPR; rpi = NT / tpr;
    lane_c = threadIdx.x % tpr; lane_r = threadIdx.x / tpr;
    g = blockIdx.y * tpr + lane_c;
    const int64_t rpb = (rows + gridDim.x - 1) / gridDim.x;
    r0 = blockIdx.x * rpb; r1 = min(rows, r0 + rpb);
  }
  DV_DEVICE bool active() const { return lane_r < rpi && g < cg; }
};

// per-block partial sums of the slab -> LDS -> per-channel totals over the RPI row lanes ->
// shard atomics with consecutive lanes on consecutive channels (256-B coalesced atomic rows;
// lane-strided atomics run ~8x slower, MI355X_MICROARCH.md "Global float atomics")
template <int VEC>
DV_DEVICE void slab_commit(const SlabTile& t, float* s, float* q, float* __restrict__ acc, int C, float* det) {
  __shared__ float sh[2][NT * VEC];
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sh[0][tid * VEC + i] = s[i]; sh[1][tid * VEC + i] = q[i]; }
  __syncthreads();
  const int sw = t.tpr * VEC;  // slab width (channels); sh is [row lane][slab channel]
  const int c0 = blockIdx.y * sw;
  float* a = stat_row(acc, det, blockIdx.x, C);
  for (int ch = tid; ch < sw; ch += NT) {
    if (c0 + ch < C) {
      float ss = 0.f, qq = 0.f;
      for (int rr = 0; rr < t.rpi; ++rr) { ss += sh[0][rr * sw + ch]; qq += sh[1][rr * sw + ch]; }
      atomicAdd(a + c0 + ch, ss);
      atomicAdd(a + C + c0 + ch, qq);
    }
  }
}

template <int VEC>
__global__ __launch_bounds__(NT) void bn_stats_kernel(const u16* __restrict__ x, int64_t rows, int C,
                                                        float* __restrict__ acc, float* __restrict__ det) {
  SlabTile t(C, VEC, rows);
  float s[VEC], q[VEC], kq[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { s[i] = 0.f; q[i] = 0.f; kq[i] = 0.f; }
  if (t.active()) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) kq[i] = stat_shift(acc, C)[t.g * VEC + i];
#pragma unroll 2
    for (int64_t r = t.r0 + t.lane_r; r < t.r1; r += t.rpi) {
      float v[VEC];
      VecIO<VEC>::load(x + r * C + t.g * VEC, v);
#pragma unroll
      for (int i = 0; i < VEC; ++i) { const float d = v[i] - kq[i]; s[i] += d; q[i] = fmaf(d, d, q[i]); }
    }
  }
  slab_commit<VEC>(t, s, q, acc, C, det);
}

// Fold the SHARDS partial (a, b) pairs of channel blockIdx.x*64 + (tid & 63) and re-zero them
// (the accumulator is persistent and self-cleaning: no memset launch). 256 threads = 64 channels
// x 4 shard groups, so each thread issues 16 independent coalesced loads instead of a serial
// 64-deep chain. Returns true on the thread that holds the channel's totals.
DV_DEVICE bool fold_shards(float* __restrict__ acc, int C, double& s, double& q) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  constexpr int PER = SHARDS / 4;
  double a = 0.0, b = 0.0;
  if (c < C) {
    float va[PER], vb[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const float* p = acc + (int64_t)(grp * PER + i) * 2 * C + c;
      va[i] = p[0]; vb[i] = p[C];
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      float* p = acc + (int64_t)(grp * PER + i) * 2 * C + c;
      p[0] = 0.f; p[C] = 0.f;
      a += va[i]; b += vb[i];
    }
  }
  red[0][grp][cl] = a; red[1][grp][cl] = b;
  __syncthreads();
  if (grp != 0 || c >= C) return false;
  s = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
  q = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
  return true;
}

// ---- fold shards -> mean/invstd/scale/shift, update running stats ----
__global__ void bn_finalize_kernel(float* __restrict__ acc, int C, double count, float eps,
                                   float momentum, const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ running_mean, float* __restrict__ running_var,
                                   float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                   float* __restrict__ scale, float* __restrict__ shift) {
  // the per-channel operands are fetched before the shard fold: one memory round trip for all of
  // them instead of a second, dependent one after the fold's barrier (the finalizes are pure
  // latency: ~4.5 -> ~3 us each, 53 + 53 of them per ResNet-50 step)
  const int c = blockIdx.x * 64 + threadIdx.x;
  const bool own = threadIdx.x < 64 && c < C;
  float* shiftp = stat_shift(acc, C) + c;
  float k = 0.f, g = 1.f, b = 0.f, rm0 = 0.f, rv0 = 0.f;
  if (own) {
    k = *shiftp;
    if (gamma) g = gamma[c];
    if (beta) b = beta[c];
    if (running_mean) { rm0 = running_mean[c]; rv0 = running_var[c]; }
  }
  double s, q;
  if (!fold_shards(acc, C, s, q)) return;
  // the producers summed d = x - K and d^2 with the per-channel shift K: var = E[d^2] - E[d]^2
  // cancels only by (mean - K)^2 / var, which is small once K tracks the batch mean
  const double dm = s / count;
  const double mean = (double)k + dm;
  double var = q / count - dm * dm;
  if (var < 0) var = 0;
  // the next batch's shift; a non-finite batch (skipped by the trainer's NaN guard) must not
  // poison every later batch's statistics through it: reset to 0 (the unshifted sums)
  *shiftp = isfinite(mean) ? (float)mean : 0.f;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  save_mean[c] = (float)mean; save_invstd[c] = invstd;
  scale[c] = g * invstd; shift[c] = b - (float)mean * g * invstd;
  // a non-finite batch (the step the non-finite guard skips) leaves the running statistics as they
  // were, so evaluation after a skipped step is not poisoned either
  if (running_mean && isfinite(mean) && isfinite(var)) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    running_mean[c] = (1.f - momentum) * rm0 + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * rv0 + momentum * (float)unb;
  }
}

// eval-mode scale/shift from running statistics
__global__ void bn_eval_prep_kernel(int C, float eps, const float* gamma, const float* beta, const float* rm,
                                    const float* rv, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = rsqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * inv; shift[c] = b - rm[c] * g * inv;
}

// Row x channel-group tiling shared by the memory-bound BN passes: TPR = C/VEC threads cover
// one pixel row (16-B vectors, fully coalesced), RPI = NT/TPR rows per iteration; every
// thread keeps its VEC channels' parameters in registers for the whole block (no per-element
// channel index arithmetic, no parameter reloads).
struct RowTile {
  int cg, tpr, rpi, lane_c, lane_r;
  DV_DEVICE RowTile(int C, int VEC) {
    cg = C / VEC; tpr = cg < NT ? cg : NT; rpi = NT / tpr;
    lane_c = threadIdx.x % tpr; lane_r = threadIdx.x / tpr;
  }
};

// ---- out = act(x*scale + shift (+res)) ----
// POST: out = act(x*scale + shift) + res -- a residual added after the activation (Darknet's
// x + leaky(bn(conv(.))), models/yolov3.py), replacing a separate add pass
template <int VEC, bool MB, bool RBN = false, int UNR = 2, bool POST = false, bool NTL = false>
__global__ __launch_bounds__(NT) void bn_apply_kernel(const u16* __restrict__ x, const u16* __restrict__ res,
                                                        u16* __restrict__ out, int64_t rows, int C, int64_t rows_per_block,
                                                        const float* __restrict__ scale, const float* __restrict__ shift,
                                                        int act, float slope, uint8_t* __restrict__ mask,
                                                        const float* __restrict__ rscale, const float* __restrict__ rshift) {
  RowTile t(C, VEC);
  if (t.lane_r >= t.rpi) return;
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  const bool pack4 = MB && (t.cg & 3) == 0;  // C % 32 == 0: whole 4-lane groups share a row
  for (int g = t.lane_c; g < t.cg; g += t.tpr) {
    float sc[VEC], sf[VEC], rs[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      sc[k] = scale[g * VEC + k]; sf[k] = shift[g * VEC + k];
      // residual BN: z = x*sc + res*rs + (sf + rshift): one shift per channel
      if constexpr (RBN) { rs[k] = rscale[g * VEC + k]; sf[k] += rshift[g * VEC + k]; }
    }
#pragma unroll UNR
    for (int64_t r = r0 + t.lane_r; r < r1; r += t.rpi) {
      const int64_t o = r * C + g * VEC;
      float v[VEC], rv[VEC];
      ldv<NTL, VEC>(x + o, v);
      if (res) ldv<NTL, VEC>(res + o, rv);
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        float z = fmaf(v[k], sc[k], sf[k]);
        if constexpr (RBN) z = fmaf(rv[k], rs[k], z);
        else if (res && !POST) z += rv[k];
        if constexpr (MB) bits |= (z > 0.f ? 1u : 0u) << k;
        v[k] = act_fwd(z, act, slope);
        if constexpr (POST) v[k] += rv[k];
      }
      VecIO<VEC>::store(out + o, v);
      if constexpr (MB) {  // activation mask, 1 bit per element (VEC == 8)
        if (pack4) {
          // 4 consecutive channel groups (one aligned 4-lane group: same row, all active or all
          // not) merge their bytes and one lane stores the 32-bit word: a quarter of the store
          // instructions of byte-wide stores, 4-B instead of 1-B pieces
          uint32_t w = bits << (8 * (t.lane_c & 3));
          w |= __shfl_xor(w, 1, 64);
          w |= __shfl_xor(w, 2, 64);
          if ((t.lane_c & 3) == 0) *reinterpret_cast<uint32_t*>(mask + (o >> 3)) = w;
        } else {
          mask[o >> 3] = (uint8_t)bits;
        }
      }
    }
  }
}

// ---- backward reduce: sum dz, sum dz*xhat (xhat = (x-mean)*invstd) ----
// The activation mask comes from the saved output `out` when present (residual blocks), else it
// is recomputed from the BN input: z = x*mscale + mshift (one tensor read less per pass).
enum { MM_NONE = 0, MM_OUT = 1, MM_X = 2, MM_BITS = 3 };  // activation-mask source (compile time: no branchy loads)
// MM_BITS: the forward apply stored the mask as bits (VEC == 8: one byte per 8 channels), 1/16 of
// the bytes of re-reading the bf16 output (residual blocks, where the mask cannot come from x)

template <int VEC, int MM, int UNR = 2>
__global__ __launch_bounds__(NT) void bn_bwd_reduce_kernel(const u16* __restrict__ dout, const u16* __restrict__ out,
                                                             const u16* __restrict__ x, int64_t rows, int C,
                                                             const float* __restrict__ mean, const float* __restrict__ invstd,
                                                             const float* __restrict__ mscale, const float* __restrict__ mshift,
                                                             int act, float slope, float* __restrict__ acc,
                                                             float* __restrict__ det) {
  SlabTile t(C, VEC, rows);
  const int g = t.g;
  float s[VEC], q[VEC], mu[VEC], is[VEC], ms[VEC], mh[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { s[i] = 0.f; q[i] = 0.f; }
  if (t.active()) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      mu[i] = mean[g * VEC + i]; is[i] = invstd[g * VEC + i];
      ms[i] = MM == MM_X ? mscale[g * VEC + i] : 0.f;
      mh[i] = MM == MM_X ? mshift[g * VEC + i] : 0.f;
    }
#pragma unroll UNR
    for (int64_t r = t.r0 + t.lane_r; r < t.r1; r += t.rpi) {
      float d[VEC], o[VEC], xv[VEC];
      VecIO<VEC>::load(dout + r * C + g * VEC, d);
      VecIO<VEC>::load(x + r * C + g * VEC, xv);
      if constexpr (MM == MM_OUT) VecIO<VEC>::load(out + r * C + g * VEC, o);
      uint32_t mb = 0;
      if constexpr (MM == MM_BITS) mb = reinterpret_cast<const uint8_t*>(out)[(r * C + g * VEC) >> 3];
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float dz = d[i];
        if constexpr (MM == MM_OUT) dz = act_bwd(d[i], o[i], act, slope);
        if constexpr (MM == MM_BITS) dz = ((mb >> i) & 1u) ? d[i] : (act == 2 ? d[i] * slope : 0.f);
        if constexpr (MM == MM_X) dz = act_bwd(d[i], fmaf(xv[i], ms[i], mh[i]), act, slope);
        s[i] += dz; q[i] += dz * (xv[i] - mu[i]) * is[i];
      }
    }
  }
  slab_commit<VEC>(t, s, q, acc, C, det);
}

// fold backward shards (and re-zero them): dbeta = sum dz, dgamma = sum dz*xhat (written, or
// added into the live gradient buffer when `accumulate`), and the per-channel affine form of
// the input gradient  dx = kA*dz + kB*x + kC  (kA = gamma*invstd,
// kB = -kA*invstd*mean(dz*xhat), kC = kA*(mean*invstd*mean(dz*xhat) - mean(dz)))
// xsum (optional): sum over the batch of dx = kA*dz + kB*x + kC -- the gradient of a bias added
// to x before this BatchNorm (the producing conv's bias), added into xsum. In exact arithmetic it
// is 0 (the training BN's input gradient sums to zero per channel); evaluated here in fp64 from
// the same per-channel sums (sum x = count * mean), it replaces a reduction pass over dx.
__global__ void bn_bwd_finalize_kernel(float* __restrict__ acc, int C, double count, const float* __restrict__ gamma,
                                       const float* __restrict__ mean, const float* __restrict__ invstd,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta, int accumulate,
                                       float* __restrict__ kA, float* __restrict__ kB, float* __restrict__ kC,
                                       float* __restrict__ xsum) {
  // per-channel operands fetched before the fold (see bn_finalize_kernel)
  const int c = blockIdx.x * 64 + threadIdx.x;
  const bool own = threadIdx.x < 64 && c < C;
  float gm = 1.f, mu = 0.f, isd = 0.f, db0 = 0.f, dg0 = 0.f, xs0 = 0.f;
  if (own) {
    if (gamma) gm = gamma[c];
    mu = mean[c]; isd = invstd[c];
    if (accumulate && dbeta) db0 = dbeta[c];
    if (accumulate && dgamma) dg0 = dgamma[c];
    if (xsum) xs0 = xsum[c];
  }
  double s, q;
  if (!fold_shards(acc, C, s, q)) return;
  if (dbeta) dbeta[c] = accumulate ? db0 + (float)s : (float)s;
  if (dgamma) dgamma[c] = accumulate ? dg0 + (float)q : (float)q;
  const double mdz = s / count, mdzx = q / count;
  const double is = isd, a = (double)gm * is;
  kA[c] = (float)a;
  kB[c] = (float)(-a * is * mdzx);
  kC[c] = (float)(a * ((double)mu * is * mdzx - mdz));
  if (xsum) {
    const double b = -a * is * mdzx, cc = a * ((double)mu * is * mdzx - mdz);
    xs0 += (float)(a * s + b * count * (double)mu + count * cc);
    xsum[c] = xs0;
  }
}

// dx = kA*dz + kB*x + kC (+ addend + addend2) ; optionally dres = dz. ``addend`` / ``addend2``:
// other gradients of the same input (a pre-activation block's residual path, an hourglass level's
// pooled branch -- models/hourglass.py) summed in this pass instead of separate adds; ``addend``
// may alias dx (each element is read before it is written by the same thread), hence no
// __restrict__ on the two. ``colsum``: per-channel sums of dx into a [SHARDS][2][C] accumulator --
// the bias gradient of the conv that produced x when dx is x's whole gradient (models/hourglass.py
// block outputs), instead of a separate reduction pass over it. Host: C / VEC <= NT.
template <int VEC, int MM, int UNR = 2, bool NTL = false>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(const u16* __restrict__ dout, const u16* __restrict__ out,
                                                            const u16* __restrict__ x, u16* dx, u16* __restrict__ dres,
                                                            int64_t rows, int C, int64_t rows_per_block, const float* __restrict__ kA,
                                                            const float* __restrict__ kB, const float* __restrict__ kC,
                                                            const float* __restrict__ mscale, const float* __restrict__ mshift,
                                                            int act, float slope, const u16* addend,
                                                            const u16* __restrict__ addend2, float* __restrict__ colsum) {
  RowTile t(C, VEC);
  const bool live = t.lane_r < t.rpi;
  if (!live && !colsum) return;
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  float cs[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) cs[k] = 0.f;
  for (int g = live ? t.lane_c : t.cg; g < t.cg; g += t.tpr) {
    float a[VEC], b[VEC], cc[VEC], ms[VEC], mh[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      a[k] = kA[g * VEC + k]; b[k] = kB[g * VEC + k]; cc[k] = kC[g * VEC + k];
      ms[k] = MM == MM_X ? mscale[g * VEC + k] : 0.f;
      mh[k] = MM == MM_X ? mshift[g * VEC + k] : 0.f;
    }
#pragma unroll UNR
    for (int64_t r = r0 + t.lane_r; r < r1; r += t.rpi) {
      const int64_t o = r * C + g * VEC;
      float d[VEC], ov[VEC], xv[VEC], rr[VEC], av[VEC], a2[VEC];
      ldv<NTL, VEC>(dout + o, d);
      ldv<NTL, VEC>(x + o, xv);
      if constexpr (MM == MM_OUT) ldv<NTL, VEC>(out + o, ov);
      if (addend) ldv<NTL, VEC>(addend + o, av);
      if (addend2) ldv<NTL, VEC>(addend2 + o, a2);
      uint32_t mb = 0;
      if constexpr (MM == MM_BITS) mb = reinterpret_cast<const uint8_t*>(out)[o >> 3];
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        float dz = d[k];
        if constexpr (MM == MM_OUT) dz = act_bwd(d[k], ov[k], act, slope);
        if constexpr (MM == MM_BITS) dz = ((mb >> k) & 1u) ? d[k] : (act == 2 ? d[k] * slope : 0.f);
        if constexpr (MM == MM_X) dz = act_bwd(d[k], fmaf(xv[k], ms[k], mh[k]), act, slope);
        rr[k] = dz;
        d[k] = fmaf(a[k], dz, fmaf(b[k], xv[k], cc[k]));
        if (addend) d[k] += av[k];
        if (addend2) d[k] += a2[k];
        cs[k] += bf2f(f2bf(d[k]));  // the stored value: the sum a reduction pass over dx would take
      }
      VecIO<VEC>::store(dx + o, d);
      if (dres) VecIO<VEC>::store(dres + o, rr);
    }
  }
  if (colsum) {  // [row lane][channel] partials -> one coalesced atomic row per block
    __shared__ float csh[NT * VEC];
    if (live) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) csh[t.lane_r * C + t.lane_c * VEC + k] = cs[k];
    }
    __syncthreads();
    float* a = stat_row(colsum, nullptr, blockIdx.x, C);
    for (int ch = threadIdx.x; ch < C; ch += NT) {
      float v = 0.f;
      for (int rr = 0; rr < t.rpi; ++rr) v += csh[rr * C + ch];
      atomicAdd(a + ch, v);
    }
  }
}

// The two BatchNorms of a residual block's output join out = act(bn(x) + bn2(x2)) (the projection
// BN folded into the block's last pass, bn_apply_kernel RBN) share dz = act'(z) * dout: one pass
// reads dout, the mask bits, x and x2 once and writes both input gradients (two separate apply
// passes read dout and the bits twice). k / k2: [3][C] = kA, kB, kC of each BN.
template <int UNR = 2, bool NTL = false>
__global__ __launch_bounds__(NT) void bn_bwd_apply_dual_kernel(const u16* __restrict__ dout, const uint8_t* __restrict__ bits,
                                                                 const u16* __restrict__ x, const u16* __restrict__ x2,
                                                                 u16* __restrict__ dx, u16* __restrict__ dx2, int64_t rows, int C,
                                                                 int64_t rows_per_block, const float* __restrict__ k,
                                                                 const float* __restrict__ k2, int act, float slope) {
  constexpr int VEC = 8;
  RowTile t(C, VEC);
  if (t.lane_r >= t.rpi) return;
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  for (int g = t.lane_c; g < t.cg; g += t.tpr) {
    float a[VEC], b[VEC], cc[VEC], a2[VEC], b2[VEC], c2[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const int c = g * VEC + e;
      a[e] = k[c]; b[e] = k[C + c]; cc[e] = k[2 * C + c];
      a2[e] = k2[c]; b2[e] = k2[C + c]; c2[e] = k2[2 * C + c];
    }
#pragma unroll UNR
    for (int64_t r = r0 + t.lane_r; r < r1; r += t.rpi) {
      const int64_t o = r * C + g * VEC;
      float d[VEC], xv[VEC], xv2[VEC];
      ldv<NTL, VEC>(dout + o, d);
      ldv<NTL, VEC>(x + o, xv);
      ldv<NTL, VEC>(x2 + o, xv2);
      const uint32_t mb = bits[o >> 3];
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float dz = ((mb >> e) & 1u) ? d[e] : (act == 2 ? d[e] * slope : 0.f);
        xv[e] = fmaf(a[e], dz, fmaf(b[e], xv[e], cc[e]));
        xv2[e] = fmaf(a2[e], dz, fmaf(b2[e], xv2[e], c2[e]));
      }
      VecIO<VEC>::store(dx + o, xv);
      VecIO<VEC>::store(dx2 + o, xv2);
    }
  }
}

// eval-mode / frozen-stat backward: dx = scale * dz
template <int VEC>
__global__ __launch_bounds__(NT) void bn_bwd_eval_kernel(const u16* __restrict__ dout, const u16* __restrict__ out,
                                                           u16* __restrict__ dx, u16* __restrict__ dres, int64_t rows, int C,
                                                           int64_t rows_per_block, const float* __restrict__ scale, int act,
                                                           float slope) {
  RowTile t(C, VEC);
  if (t.lane_r >= t.rpi) return;
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  for (int g = t.lane_c; g < t.cg; g += t.tpr) {
    float sc[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) sc[k] = scale[g * VEC + k];
#pragma unroll 2
    for (int64_t r = r0 + t.lane_r; r < r1; r += t.rpi) {
      const int64_t o = r * C + g * VEC;
      float d[VEC], ov[VEC], rr[VEC];
      VecIO<VEC>::load(dout + o, d);
      if (act) VecIO<VEC>::load(out + o, ov);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const float dz = act ? act_bwd(d[k], ov[k], act, slope) : d[k];
        rr[k] = dz; d[k] = dz * sc[k];
      }
      VecIO<VEC>::store(dx + o, d);
      if (dres) VecIO<VEC>::store(dres + o, rr);
    }
  }
}

inline int vec_for(int C) { return (C % 8 == 0) ? 8 : (C % 4 == 0) ? 4 : (C % 2 == 0) ? 2 : 1; }
int g_reduce_blocks = 1024;  // benchmarking override (dv_bn_tuning)
int g_reduce_unroll = 2;
// (row blocks, channel slabs): ~4 blocks per CU (8 with several slabs), >= 32 rows per block
inline dim3 reduce_grid(int64_t rows, int C) {
  const int v = vec_for(C), cg = C / v, tpr = cg < SLAB_TPR ? cg : SLAB_TPR;
  const int slabs = (cg + tpr - 1) / tpr;
  const int64_t target = (int64_t)g_reduce_blocks * (slabs > 1 ? 2 : 1) / slabs;
  const int64_t g = std::min<int64_t>(std::max<int64_t>(target, 1), std::max<int64_t>(1, rows / 32));
  return dim3((unsigned)g, (unsigned)slabs);
}
// rows per block for the row-tiled apply passes: ~16384 blocks for tensors of >= 40M elements,
// ~8192 below (tools/bn_apply_bench.py, profiles/bn_apply_bench.txt: 16384 is 3-10 % faster from
// 1024@14 up, 8192 wins at 2048@7), a multiple of rows/iteration; g_apply_blocks / g_apply_unroll:
// benchmarking overrides (dv_bn_apply_tuning; 0 = this heuristic)
int g_apply_blocks = 0;
int g_apply_unroll = 2;
inline int64_t apply_rows_per_block(int64_t rows, int C, int v) {
  const int cg = C / v, tpr = cg < NT ? cg : NT, rpi = NT / tpr;
  const int64_t blocks = g_apply_blocks > 0 ? g_apply_blocks : (rows * C >= (int64_t)40 << 20 ? 16384 : 8192);
  int64_t rpb = (rows + blocks - 1) / blocks;
  rpb = ((rpb + rpi - 1) / rpi) * rpi;
  return std::max<int64_t>(rpb, rpi);
}
}  // namespace

// ---- deterministic mode (kernels.h DetStats) ----
// Per-stream, zero-kept fp32 scratch for the per-block statistics rows of one producer launch.
// Grow-only like dv_slab_workspace: a captured graph keeps the pointer it recorded, so a buffer
// is never freed once handed out; it cannot grow while the stream is being captured.
namespace {
struct DetWs {
  float* ptr = nullptr;
  size_t elems = 0;
};
std::unordered_map<hipStream_t, DetWs> g_det_ws;
std::vector<float*> g_det_retired;

// slab rows [blocks][width] -> the 64 shard rows of acc (row stride `stride`): shard g gets the
// in-order sum of rows [g*rows/64, (g+1)*rows/64) (4 partial chains over r mod 4, combined in
// fixed order), then those slab rows are zeroed again. One atomic per (shard, column): at most
// two producers on concurrent streams meet in a shard, 0 + a + b == 0 + b + a.
__global__ __launch_bounds__(256) void det_fold_kernel(float* __restrict__ slab, int64_t rows, int64_t width,
                                                      float* __restrict__ acc, int64_t stride) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= width) return;
  const int g = blockIdx.y;
  const int64_t r0 = rows * g / SHARDS, r1 = rows * (g + 1) / SHARDS;
  float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
  int64_t r = r0;
  for (; r + 3 < r1; r += 4) {
    float* a = slab + r * width + j;
    p0 += a[0]; p1 += a[width]; p2 += a[2 * width]; p3 += a[3 * width];
    a[0] = 0.f; a[width] = 0.f; a[2 * width] = 0.f; a[3 * width] = 0.f;
  }
  for (; r < r1; ++r) { float* a = slab + r * width + j; p0 += a[0]; a[0] = 0.f; }
  const float t = (p0 + p1) + (p2 + p3);
  if (r1 > r0) atomicAdd(acc + (int64_t)g * stride + j, t);
}
}  // namespace

float* dv_det_workspace(size_t elems, hipStream_t st) {
  DetWs& w = g_det_ws[st];
  if (elems > w.elems) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      throw std::runtime_error("deterministic mode: statistics scratch must grow during a stream capture "
                               "(run an eager warm-up step with the same shapes first)");
    const size_t want = elems + elems / 2;
    float* fresh = nullptr;
    if (hipMalloc(&fresh, want * sizeof(float)) != hipSuccess)
      throw std::runtime_error("deterministic mode: out of memory for the statistics scratch");
    if (hipMemsetAsync(fresh, 0, want * sizeof(float), st) != hipSuccess)
      throw std::runtime_error("deterministic mode: scratch memset failed");
    if (w.ptr) g_det_retired.push_back(w.ptr);
    w.ptr = fresh;
    w.elems = want;
  }
  return w.ptr;
}

// dst[j] += sum over the slab rows of column j: one block per column, a fixed thread <- row
// assignment and a fixed tree (reproducible bits); the slab is zeroed again
__global__ __launch_bounds__(256) void det_sum_kernel(float* __restrict__ slab, int64_t rows, int64_t width,
                                                     float* __restrict__ dst) {
  __shared__ float sh[256];
  const int64_t j = blockIdx.x;
  float v = 0.f;
  for (int64_t r = threadIdx.x; r < rows; r += 256) {
    v += slab[r * width + j];
    slab[r * width + j] = 0.f;
  }
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) dst[j] += sh[0];
}

void dv_det_sum(float* slab, int64_t rows, int64_t width, float* dst, hipStream_t st) {
  det_sum_kernel<<<(unsigned)width, 256, 0, st>>>(slab, rows, width, dst);
}

void dv_det_fold(float* slab, int64_t rows, int64_t width, float* acc, int64_t stride, hipStream_t st) {
  const dim3 grid((unsigned)((width + 255) / 256), SHARDS);
  det_fold_kernel<<<grid, 256, 0, st>>>(slab, rows, width, acc, stride);
}

#define DISPATCH_VEC(C, KERNEL, ...)                                              \
  switch (vec_for(C)) {                                                          \
    case 8: KERNEL<8> __VA_ARGS__; break;                                          \
    case 4: KERNEL<4> __VA_ARGS__; break;                                          \
    case 2: KERNEL<2> __VA_ARGS__; break;                                          \
    default: KERNEL<1> __VA_ARGS__; break;                                         \
  }

void dv_bn_tuning(int reduce_blocks, int reduce_unroll) {
  g_reduce_blocks = reduce_blocks > 0 ? reduce_blocks : 1024;
  g_reduce_unroll = reduce_unroll == 4 ? 4 : 2;
}

void dv_bn_apply_tuning(int blocks, int unroll) {
  g_apply_blocks = blocks > 0 ? blocks : 0;
  g_apply_unroll = unroll == 4 ? 4 : 2;
}

void dv_bn_stats(const void* x, int64_t rows, int C, float* acc, hipStream_t st) {
  const dim3 g = reduce_grid(rows, C);
  DetStats d(g.x, C, st);
  DISPATCH_VEC(C, bn_stats_kernel, <<<g, NT, 0, st>>>((const u16*)x, rows, C, acc, d.slab))
  d.fold(acc);
}

// Per-channel sum of an NHWC tensor (conv / Linear bias gradient): the statistics reduction into
// the self-cleaning shard accumulator, then one fold that zeroes the shards again and writes (or
// adds into the live fp32 gradient buffer) the sums -- 2 launches, no memset, no fp32 copy of dy.
__global__ void channel_sum_finalize_kernel(float* __restrict__ acc, int ld, int C, float* __restrict__ out,
                                            int accumulate) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  const float o0 = (accumulate && threadIdx.x < 64 && c < C) ? out[c] : 0.f;  // before the fold's round trip
  double s, q;
  if (!fold_shards(acc, ld, s, q)) return;
  if (c < C) out[c] = accumulate ? o0 + (float)s : (float)s;
}

void dv_channel_sum(const void* x, int64_t rows, int ld, int C, float* acc, float* out, int accumulate, hipStream_t st) {
  dv_bn_stats(x, rows, ld, acc, st);
  channel_sum_finalize_kernel<<<(ld + 63) / 64, 256, 0, st>>>(acc, ld, C, out, accumulate);
}

void dv_channel_sum_finalize(float* acc, int ld, int C, float* out, int accumulate, hipStream_t st) {
  channel_sum_finalize_kernel<<<(ld + 63) / 64, 256, 0, st>>>(acc, ld, C, out, accumulate);
}

void dv_bn_finalize(float* acc, int C, double count, float eps, float momentum, const float* gamma,
                    const float* beta, float* rm, float* rv, float* save_mean, float* save_invstd, float* scale,
                    float* shift, hipStream_t st) {
  bn_finalize_kernel<<<(C + 63) / 64, 256, 0, st>>>(acc, C, count, eps, momentum, gamma, beta, rm, rv, save_mean,
                                                      save_invstd, scale, shift);
}

void dv_bn_eval_prep(int C, float eps, const float* gamma, const float* beta, const float* rm, const float* rv,
                     float* scale, float* shift, hipStream_t st) {
  bn_eval_prep_kernel<<<(C + 255) / 256, 256, 0, st>>>(C, eps, gamma, beta, rm, rv, scale, shift);
}

template <bool NTL>
static void bn_apply_dispatch(const void* x, const void* res, void* out, int64_t n, int C, const float* scale,
                              const float* shift, int act, float slope, void* mask, const float* rscale,
                              const float* rshift, hipStream_t st, int post) {
  const int v = vec_for(C);
  const int64_t rows = n / C;
  const int64_t rpb = apply_rows_per_block(rows, C, v);
  const int g = (int)((rows + rpb - 1) / rpb);
#define AP_ARGS <<<g, NT, 0, st>>>((const u16*)x, (const u16*)res, (u16*)out, rows, C, rpb, scale, shift, act, slope, (uint8_t*)mask, rscale, rshift)
  if (post && res) {  // post-activation residual: the mask comes from x in backward (no bits)
    switch (v) {
      case 8: bn_apply_kernel<8, false, false, 2, true, NTL> AP_ARGS; break;
      case 4: bn_apply_kernel<4, false, false, 2, true, NTL> AP_ARGS; break;
      case 2: bn_apply_kernel<2, false, false, 2, true, NTL> AP_ARGS; break;
      default: bn_apply_kernel<1, false, false, 2, true, NTL> AP_ARGS; break;
    }
    return;
  }
  if (g_apply_unroll == 4 && mask && v == 8) {
    if (res && rscale && rshift) bn_apply_kernel<8, true, true, 4, false, NTL> AP_ARGS;
    else bn_apply_kernel<8, true, false, 4, false, NTL> AP_ARGS;
    return;
  }
  if (res && rscale && rshift) {
    if (mask && v == 8) bn_apply_kernel<8, true, true, 2, false, NTL> AP_ARGS;
    else if (v == 8) bn_apply_kernel<8, false, true, 2, false, NTL> AP_ARGS;
    else if (v == 4) bn_apply_kernel<4, false, true, 2, false, NTL> AP_ARGS;
    else if (v == 2) bn_apply_kernel<2, false, true, 2, false, NTL> AP_ARGS;
    else bn_apply_kernel<1, false, true, 2, false, NTL> AP_ARGS;
    return;
  }
  if (mask && v == 8) { bn_apply_kernel<8, true, false, 2, false, NTL> AP_ARGS; return; }
  switch (v) {
    case 8: bn_apply_kernel<8, false, false, 2, false, NTL> AP_ARGS; break;
    case 4: bn_apply_kernel<4, false, false, 2, false, NTL> AP_ARGS; break;
    case 2: bn_apply_kernel<2, false, false, 2, false, NTL> AP_ARGS; break;
    default: bn_apply_kernel<1, false, false, 2, false, NTL> AP_ARGS; break;
  }
#undef AP_ARGS
}

void dv_bn_apply(const void* x, const void* res, void* out, int64_t n, int C, const float* scale, const float* shift,
                 int act, float slope, void* mask, const float* rscale, const float* rshift, hipStream_t st, int post) {
  if (n >= NT_LOAD_MIN_ELEMS) bn_apply_dispatch<true>(x, res, out, n, C, scale, shift, act, slope, mask, rscale, rshift, st, post);
  else bn_apply_dispatch<false>(x, res, out, n, C, scale, shift, act, slope, mask, rscale, rshift, st, post);
}

template <int MM>
static void bwd_reduce_launch(dim3 g, const void* dout, const void* out, const void* x, int64_t rows, int C, const float* mean,
                              const float* invstd, const float* mscale, const float* mshift, int act, float slope, float* acc,
                              float* det, hipStream_t st) {
  switch (vec_for(C)) {
    case 8: bn_bwd_reduce_kernel<8, MM><<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, rows, C, mean, invstd, mscale, mshift, act, slope, acc, det); break;
    case 4: bn_bwd_reduce_kernel<4, MM><<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, rows, C, mean, invstd, mscale, mshift, act, slope, acc, det); break;
    case 2: bn_bwd_reduce_kernel<2, MM><<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, rows, C, mean, invstd, mscale, mshift, act, slope, acc, det); break;
    default: bn_bwd_reduce_kernel<1, MM><<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, rows, C, mean, invstd, mscale, mshift, act, slope, acc, det); break;
  }
}

void dv_bn_bwd_reduce(const void* dout, const void* out, const void* x, int64_t rows, int C, const float* mean,
                      const float* invstd, const float* mscale, const float* mshift, int act, float slope, float* acc,
                      int mask_bits, hipStream_t st) {
  const dim3 g = reduce_grid(rows, C);
  DetStats d(g.x, C, st);
  float* det = d.slab;
  if (act && mask_bits && vec_for(C) == 8) {
    if (g_reduce_unroll == 4)
      bn_bwd_reduce_kernel<8, MM_BITS, 4><<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, rows, C, mean,
                                                              invstd, mscale, mshift, act, slope, acc, det);
    else
      bn_bwd_reduce_kernel<8, MM_BITS><<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, rows, C, mean,
                                                           invstd, mscale, mshift, act, slope, acc, det);
  } else if (act && !out && vec_for(C) == 8 && g_reduce_unroll == 4) {
    bn_bwd_reduce_kernel<8, MM_X, 4><<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, rows, C, mean,
                                                         invstd, mscale, mshift, act, slope, acc, det);
  } else if (!act) {
    bwd_reduce_launch<MM_NONE>(g, dout, out, x, rows, C, mean, invstd, mscale, mshift, act, slope, acc, det, st);
  } else if (out) {
    bwd_reduce_launch<MM_OUT>(g, dout, out, x, rows, C, mean, invstd, mscale, mshift, act, slope, acc, det, st);
  } else {
    bwd_reduce_launch<MM_X>(g, dout, out, x, rows, C, mean, invstd, mscale, mshift, act, slope, acc, det, st);
  }
  d.fold(acc);
}

void dv_bn_bwd_finalize(float* acc, int C, double count, const float* gamma, const float* mean, const float* invstd,
                        float* dgamma, float* dbeta, int accumulate, float* kA, float* kB, float* kC, hipStream_t st,
                        float* xsum) {
  bn_bwd_finalize_kernel<<<(C + 63) / 64, 256, 0, st>>>(acc, C, count, gamma, mean, invstd, dgamma, dbeta, accumulate,
                                                          kA, kB, kC, xsum);
}

template <int MM, bool NTL>
static void bwd_apply_launch(int g, const void* dout, const void* out, const void* x, void* dx, void* dres, int64_t rows,
                             int C, int64_t rpb, const float* kA, const float* kB, const float* kC, const float* mscale,
                             const float* mshift, int act, float slope, const void* addend, const void* addend2,
                             float* colsum, hipStream_t st) {
#define BA_ARGS <<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, (u16*)dx, (u16*)dres, rows, C, rpb, kA, kB, kC, mscale, mshift, act, slope, (const u16*)addend, (const u16*)addend2, colsum)
  switch (vec_for(C)) {
    case 8: bn_bwd_apply_kernel<8, MM, 2, NTL> BA_ARGS; break;
    case 4: bn_bwd_apply_kernel<4, MM, 2, NTL> BA_ARGS; break;
    case 2: bn_bwd_apply_kernel<2, MM, 2, NTL> BA_ARGS; break;
    default: bn_bwd_apply_kernel<1, MM, 2, NTL> BA_ARGS; break;
  }
#undef BA_ARGS
}

template <bool NTL>
static void bwd_apply_dispatch(const void* dout, const void* out, const void* x, void* dx, void* dres, int64_t n, int C,
                               const float* kA, const float* kB, const float* kC, const float* mscale,
                               const float* mshift, int act, float slope, int mask_bits, const void* addend,
                               const void* addend2, float* colsum, hipStream_t st) {
  const int v = vec_for(C);
  const int64_t rows = n / C;
  const int64_t rpb = apply_rows_per_block(rows, C, v);
  const int g = (int)((rows + rpb - 1) / rpb);
  if (act && mask_bits && v == 8 && g_apply_unroll == 4) {
    bn_bwd_apply_kernel<8, MM_BITS, 4, NTL><<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, (u16*)dx,
                                                           (u16*)dres, rows, C, rpb, kA, kB, kC, mscale, mshift, act, slope,
                                                           (const u16*)addend, (const u16*)addend2, colsum);
    return;
  }
  if (act && mask_bits && v == 8) {
    bn_bwd_apply_kernel<8, MM_BITS, 2, NTL><<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, (u16*)dx,
                                                        (u16*)dres, rows, C, rpb, kA, kB, kC, mscale, mshift, act, slope,
                                                        (const u16*)addend, (const u16*)addend2, colsum);
    return;
  }
  if (!act) bwd_apply_launch<MM_NONE, NTL>(g, dout, out, x, dx, dres, rows, C, rpb, kA, kB, kC, mscale, mshift, act, slope, addend, addend2, colsum, st);
  else if (out) bwd_apply_launch<MM_OUT, NTL>(g, dout, out, x, dx, dres, rows, C, rpb, kA, kB, kC, mscale, mshift, act, slope, addend, addend2, colsum, st);
  else bwd_apply_launch<MM_X, NTL>(g, dout, out, x, dx, dres, rows, C, rpb, kA, kB, kC, mscale, mshift, act, slope, addend, addend2, colsum, st);
}

void dv_bn_bwd_apply(const void* dout, const void* out, const void* x, void* dx, void* dres, int64_t n, int C,
                     const float* kA, const float* kB, const float* kC, const float* mscale, const float* mshift, int act,
                     float slope, int mask_bits, const void* addend, const void* addend2, float* colsum,
                     hipStream_t st) {
  if (colsum && C / vec_for(C) > NT) throw std::runtime_error("bn_bwd_apply colsum: C / VEC must be <= 256");
  if (n >= NT_LOAD_MIN_ELEMS)
    bwd_apply_dispatch<true>(dout, out, x, dx, dres, n, C, kA, kB, kC, mscale, mshift, act, slope, mask_bits, addend, addend2, colsum, st);
  else
    bwd_apply_dispatch<false>(dout, out, x, dx, dres, n, C, kA, kB, kC, mscale, mshift, act, slope, mask_bits, addend, addend2, colsum, st);
}

void dv_bn_bwd_apply_dual(const void* dout, const void* bits, const void* x, const void* x2, void* dx, void* dx2,
                          int64_t n, int C, const float* k, const float* k2, int act, float slope, hipStream_t st) {
  const int64_t rows = n / C;
  const int64_t rpb = apply_rows_per_block(rows, C, 8);
  const int g = (int)((rows + rpb - 1) / rpb);
  if (n >= NT_LOAD_MIN_ELEMS)
    bn_bwd_apply_dual_kernel<2, true><<<g, NT, 0, st>>>((const u16*)dout, (const uint8_t*)bits, (const u16*)x,
                                                         (const u16*)x2, (u16*)dx, (u16*)dx2, rows, C, rpb, k, k2, act, slope);
  else
    bn_bwd_apply_dual_kernel<2, false><<<g, NT, 0, st>>>((const u16*)dout, (const uint8_t*)bits, (const u16*)x,
                                                          (const u16*)x2, (u16*)dx, (u16*)dx2, rows, C, rpb, k, k2, act, slope);
}

void dv_bn_bwd_eval(const void* dout, const void* out, void* dx, void* dres, int64_t n, int C, const float* scale,
                    int act, float slope, hipStream_t st) {
  const int v = vec_for(C);
  const int64_t rows = n / C;
  const int64_t rpb = apply_rows_per_block(rows, C, v);
  const int g = (int)((rows + rpb - 1) / rpb);
  DISPATCH_VEC(C, bn_bwd_eval_kernel, <<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (u16*)dx, (u16*)dres, rows, C, rpb, scale, act, slope))
}

// ---------------------------------------------------------------------------------------------
// Small BatchNorms: the shard fold inside the apply pass (no finalize launch).
// Hourglass-104 / YOLOv3 carry hundreds of BatchNorms over a few thousand rows each (the 16x16 ..
// 4x4 hourglass levels at batch 32): there the separate finalize launch (~5 us of pure latency,
// 230 + 230 of them per Hourglass step, profiles/hourglass_step_census.txt) cost as much as the
// apply pass itself. These passes tile [row range] x [64-channel slab]: every block folds its
// slab's SHARDS x 64 partial sums (32 KB, L2-resident: the producer just wrote them) in its
// prologue, in the order of bn_finalize_kernel (same bits as the two-launch form), block (0, slab)
// publishes the per-channel results (running statistics, save_mean / invstd / scale / shift, or
// dgamma / dbeta / the producer's bias gradient), and the LAST block of the slab to finish (a
// ticket counter) re-zeroes the slab's shards -- and, forward, stores the batch mean as the next
// shift -- after every block of the slab has read them.
namespace {
constexpr int FIN_CH = 64;  // channels per slab
struct FwdFin {
  float* acc; double count; float eps, momentum;
  const float* gamma; const float* beta; float* rm; float* rv;
  float* prm;   // [4][C]: scale, shift, mean, invstd
  int* ticket;  // [C / 64], zero between uses
};
struct BwdFin {
  float* acc; double count;
  const float* gamma; const float* mean; const float* invstd;
  float* dgamma; float* dbeta; int accumulate; float* xsum;
  int* ticket;
};

// fold channels [c0, c0 + 64) of a [SHARDS][2][C] accumulator (fold_shards' order, no zeroing):
// every thread returns its channel's (c0 + tid % 64) totals
DV_DEVICE void fold64(const float* __restrict__ acc, int C, int c0, double& s, double& q) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  constexpr int PER = SHARDS / 4;
  float va[PER], vb[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const float* p = acc + (int64_t)(grp * PER + i) * 2 * C + c0 + cl;
    va[i] = p[0]; vb[i] = p[C];
  }
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int i = 0; i < PER; ++i) { a += va[i]; b += vb[i]; }
  red[0][grp][cl] = a; red[1][grp][cl] = b;
  __syncthreads();
  s = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
  q = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
}

// Ticket of the slab, taken by thread 0 after every thread of the block has drained its global
// loads (the shard values of fold64 AND the shift k read before it: the last block rewrites *shiftp
// and re-zeroes the shards at its end, so no block may still have one of those loads in flight when
// its ticket is counted). The ticket is a relaxed agent-scope atomic: an acq_rel one would emit an
// L2 write-back (buffer_wbl2) and invalidate per block. fin_last() broadcasts the answer.
DV_DEVICE void fin_ticket(int* ticket, int nblocks, int* last) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    *last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1;
}
DV_DEVICE bool fin_last(const int* last) {
  __syncthreads();
  return *last;
}
DV_DEVICE void fin_zero(float* __restrict__ acc, int C, int c0) {
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  constexpr int PER = SHARDS / 4;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    float* p = acc + (int64_t)(grp * PER + i) * 2 * C + c0 + cl;
    p[0] = 0.f; p[C] = 0.f;
  }
}

// 8 threads x 8 channels cover a row of the slab; 32 rows per iteration
template <bool MB, bool POST, bool NTL>
__global__ __launch_bounds__(NT) void bn_fin_apply_kernel(const u16* __restrict__ x, const u16* __restrict__ res,
                                                          u16* __restrict__ out, int64_t rows, int C, int64_t rpb,
                                                          int act, float slope, uint8_t* __restrict__ mask, FwdFin f) {
  __shared__ float ssc[FIN_CH], ssf[FIN_CH];
  const int c0 = (int)blockIdx.y * FIN_CH;
  const int cl = threadIdx.x & 63, c = c0 + cl;
  float* shiftp = stat_shift(f.acc, C) + c;
  // per-channel operands before the fold (one round trip for both)
  const float k = *shiftp;
  const float g = f.gamma ? f.gamma[c] : 1.f, b = f.beta ? f.beta[c] : 0.f;
  const bool pub = blockIdx.x == 0 && threadIdx.x < 64;
  float rm0 = 0.f, rv0 = 0.f;
  if (pub && f.rm) { rm0 = f.rm[c]; rv0 = f.rv[c]; }
  double s, q;
  fold64(f.acc, C, c0, s, q);
  __shared__ int last;
  fin_ticket(f.ticket + blockIdx.y, gridDim.x, &last);
  const double dm = s / f.count;
  const double mean = (double)k + dm;
  double var = q / f.count - dm * dm;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float scale = g * invstd, shift = b - (float)mean * g * invstd;
  if (threadIdx.x < 64) { ssc[cl] = scale; ssf[cl] = shift; }
  if (pub) {  // bn_finalize_kernel's outputs
    f.prm[c] = scale; f.prm[C + c] = shift; f.prm[2 * C + c] = (float)mean; f.prm[3 * C + c] = invstd;
    if (f.rm && isfinite(mean) && isfinite(var)) {
      const double unb = f.count > 1 ? var * f.count / (f.count - 1) : var;
      f.rm[c] = (1.f - f.momentum) * rm0 + f.momentum * (float)mean;
      f.rv[c] = (1.f - f.momentum) * rv0 + f.momentum * (float)unb;
    }
  }
  __syncthreads();
  const int lane_c = threadIdx.x & 7, lane_r = threadIdx.x >> 3;
  float sc[8], sf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sc[e] = ssc[lane_c * 8 + e]; sf[e] = ssf[lane_c * 8 + e]; }
  const int64_t r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
#pragma unroll 2
  for (int64_t r = r0 + lane_r; r < r1; r += NT / 8) {
    const int64_t o = r * C + c0 + lane_c * 8;
    float v[8], rv[8];
    ldv<NTL, 8>(x + o, v);
    if (res) ldv<NTL, 8>(res + o, rv);
    uint32_t bits = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float z = fmaf(v[e], sc[e], sf[e]);
      if (res && !POST) z += rv[e];
      if constexpr (MB) bits |= (z > 0.f ? 1u : 0u) << e;
      v[e] = act_fwd(z, act, slope);
      if constexpr (POST) v[e] += rv[e];
    }
    VecIO<8>::store(out + o, v);
    if constexpr (MB) {  // 4 lanes = 32 channels = one aligned 32-bit word of the mask (C % 64 == 0)
      uint32_t w = bits << (8 * (lane_c & 3));
      w |= __shfl_xor(w, 1, 64);
      w |= __shfl_xor(w, 2, 64);
      if ((lane_c & 3) == 0) *reinterpret_cast<uint32_t*>(mask + (o >> 3)) = w;
    }
  }
  if (fin_last(&last)) {
    fin_zero(f.acc, C, c0);
    if (threadIdx.x < 64) *shiftp = isfinite(mean) ? (float)mean : 0.f;  // the next batch's shift
    if (threadIdx.x == 0) f.ticket[blockIdx.y] = 0;
  }
}

template <int MM, bool NTL>
__global__ __launch_bounds__(NT) void bn_bwd_fin_apply_kernel(const u16* __restrict__ dout, const u16* __restrict__ out,
                                                              const u16* __restrict__ x, u16* dx, u16* __restrict__ dres,
                                                              int64_t rows, int C, int64_t rpb,
                                                              const float* __restrict__ mscale, const float* __restrict__ mshift,
                                                              int act, float slope, const u16* addend,
                                                              const u16* __restrict__ addend2, float* __restrict__ colsum,
                                                              BwdFin f) {
  __shared__ float sk[3][FIN_CH];
  const int c0 = (int)blockIdx.y * FIN_CH;
  const int cl = threadIdx.x & 63, c = c0 + cl;
  const bool pub = blockIdx.x == 0 && threadIdx.x < 64;
  const float gm = f.gamma ? f.gamma[c] : 1.f, mu = f.mean[c], isd = f.invstd[c];
  float db0 = 0.f, dg0 = 0.f, xs0 = 0.f;
  if (pub) {
    if (f.accumulate && f.dbeta) db0 = f.dbeta[c];
    if (f.accumulate && f.dgamma) dg0 = f.dgamma[c];
    if (f.xsum) xs0 = f.xsum[c];
  }
  double s, q;
  fold64(f.acc, C, c0, s, q);
  __shared__ int last;
  fin_ticket(f.ticket + blockIdx.y, gridDim.x, &last);
  // bn_bwd_finalize_kernel's coefficients of dx = kA*dz + kB*x + kC
  const double mdz = s / f.count, mdzx = q / f.count;
  const double is = isd, a = (double)gm * is;
  const double kb = -a * is * mdzx, kc = a * ((double)mu * is * mdzx - mdz);
  if (threadIdx.x < 64) { sk[0][cl] = (float)a; sk[1][cl] = (float)kb; sk[2][cl] = (float)kc; }
  if (pub) {
    if (f.dbeta) f.dbeta[c] = f.accumulate ? db0 + (float)s : (float)s;
    if (f.dgamma) f.dgamma[c] = f.accumulate ? dg0 + (float)q : (float)q;
    if (f.xsum) f.xsum[c] = xs0 + (float)(a * s + kb * f.count * (double)mu + f.count * kc);
  }
  __syncthreads();
  const int lane_c = threadIdx.x & 7, lane_r = threadIdx.x >> 3;
  float ka[8], kbv[8], kcv[8], ms[8], mh[8], cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int ch = lane_c * 8 + e;
    ka[e] = sk[0][ch]; kbv[e] = sk[1][ch]; kcv[e] = sk[2][ch];
    ms[e] = MM == MM_X ? mscale[c0 + ch] : 0.f;
    mh[e] = MM == MM_X ? mshift[c0 + ch] : 0.f;
    cs[e] = 0.f;
  }
  const int64_t r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
#pragma unroll 2
  for (int64_t r = r0 + lane_r; r < r1; r += NT / 8) {
    const int64_t o = r * C + c0 + lane_c * 8;
    float d[8], ov[8], xv[8], rr[8], av[8], a2[8];
    ldv<NTL, 8>(dout + o, d);
    ldv<NTL, 8>(x + o, xv);
    if constexpr (MM == MM_OUT) ldv<NTL, 8>(out + o, ov);
    if (addend) ldv<NTL, 8>(addend + o, av);
    if (addend2) ldv<NTL, 8>(addend2 + o, a2);
    uint32_t mb = 0;
    if constexpr (MM == MM_BITS) mb = reinterpret_cast<const uint8_t*>(out)[o >> 3];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float dz = d[e];
      if constexpr (MM == MM_OUT) dz = act_bwd(d[e], ov[e], act, slope);
      if constexpr (MM == MM_BITS) dz = ((mb >> e) & 1u) ? d[e] : (act == 2 ? d[e] * slope : 0.f);
      if constexpr (MM == MM_X) dz = act_bwd(d[e], fmaf(xv[e], ms[e], mh[e]), act, slope);
      rr[e] = dz;
      d[e] = fmaf(ka[e], dz, fmaf(kbv[e], xv[e], kcv[e]));
      if (addend) d[e] += av[e];
      if (addend2) d[e] += a2[e];
      cs[e] += bf2f(f2bf(d[e]));
    }
    VecIO<8>::store(dx + o, d);
    if (dres) VecIO<8>::store(dres + o, rr);
  }
  if (colsum) {  // [row lane][slab channel] -> one coalesced atomic row of 64 channels per block
    __shared__ float csh[NT / 8][FIN_CH];
#pragma unroll
    for (int e = 0; e < 8; ++e) csh[lane_r][lane_c * 8 + e] = cs[e];
    __syncthreads();
    if (threadIdx.x < FIN_CH) {
      float v = 0.f;
      for (int rr = 0; rr < NT / 8; ++rr) v += csh[rr][threadIdx.x];
      atomicAdd(stat_row(colsum, nullptr, blockIdx.x, C) + c0 + threadIdx.x, v);
    }
  }
  if (fin_last(&last)) {
    fin_zero(f.acc, C, c0);
    if (threadIdx.x == 0) f.ticket[blockIdx.y] = 0;
  }
}

// row blocks per 64-channel slab: 32 rows (one iteration) each up to ~1,024 blocks in all -- the
// pass is latency-bound at these sizes, each block's shard fold is one round trip of 32 loads
inline int fin_row_blocks(int64_t rows, int C, int64_t& rpb) {
  const int slabs = C / FIN_CH;
  int64_t nrb = std::max<int64_t>(1, std::min<int64_t>((rows + 31) / 32, std::max(1, 1024 / slabs)));
  rpb = (rows + nrb - 1) / nrb;
  rpb = (rpb + 31) / 32 * 32;
  return (int)((rows + rpb - 1) / rpb);
}
}  // namespace

bool dv_bn_fin_ok(int64_t n, int C) { return C % FIN_CH == 0 && C > 0 && n <= DV_BN_FIN_MAX_ELEMS; }

void dv_bn_fin_apply(float* acc, double count, float eps, float momentum, const float* gamma, const float* beta,
                     float* rm, float* rv, float* prm, int* ticket, const void* x, const void* res, void* out, int64_t n,
                     int C, int act, float slope, void* mask, int post, hipStream_t st) {
  const int64_t rows = n / C;
  int64_t rpb;
  const dim3 g((unsigned)fin_row_blocks(rows, C, rpb), (unsigned)(C / FIN_CH));
  const FwdFin f{acc, count, eps, momentum, gamma, beta, rm, rv, prm, ticket};
#define FA_ARGS <<<g, NT, 0, st>>>((const u16*)x, (const u16*)res, (u16*)out, rows, C, rpb, act, slope, (uint8_t*)mask, f)
  if (post && res) bn_fin_apply_kernel<false, true, false> FA_ARGS;
  else if (mask) bn_fin_apply_kernel<true, false, false> FA_ARGS;
  else bn_fin_apply_kernel<false, false, false> FA_ARGS;
#undef FA_ARGS
}

void dv_bn_bwd_fin_apply(float* acc, double count, const float* gamma, const float* mean, const float* invstd,
                         float* dgamma, float* dbeta, int accumulate, float* xsum, int* ticket, const void* dout,
                         const void* out, const void* x, void* dx, void* dres, int64_t n, int C, const float* mscale,
                         const float* mshift, int act, float slope, int mask_bits, const void* addend,
                         const void* addend2, float* colsum, hipStream_t st) {
  const int64_t rows = n / C;
  int64_t rpb;
  const dim3 g((unsigned)fin_row_blocks(rows, C, rpb), (unsigned)(C / FIN_CH));
  const BwdFin f{acc, count, gamma, mean, invstd, dgamma, dbeta, accumulate, xsum, ticket};
#define FB_ARGS <<<g, NT, 0, st>>>((const u16*)dout, (const u16*)out, (const u16*)x, (u16*)dx, (u16*)dres, rows, C, rpb, mscale, mshift, act, slope, (const u16*)addend, (const u16*)addend2, colsum, f)
  if (act && mask_bits) bn_bwd_fin_apply_kernel<MM_BITS, false> FB_ARGS;
  else if (!act) bn_bwd_fin_apply_kernel<MM_NONE, false> FB_ARGS;
  else if (out) bn_bwd_fin_apply_kernel<MM_OUT, false> FB_ARGS;
  else bn_bwd_fin_apply_kernel<MM_X, false> FB_ARGS;
#undef FB_ARGS
}
