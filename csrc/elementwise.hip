// Vectorized elementwise kernels and layout/cast preparation.
//   * activations fwd/bwd (relu / leaky / tanh / sigmoid) on bf16, 16-B vectors
//   * residual add, scale
//   * dropout with a counter-based hash RNG: the mask is regenerated in backward from
//     (seed, element index), so nothing but the seed is saved
//   * weight preparation: fp32 OIHW master weights -> bf16 MFMA operand layouts
//       mode 0: [G][Og][R][S][Ig_pad]   (forward: K-contiguous rows)
//       mode 1: [G][Ig][R][S][Og_pad]   (dgrad / ConvTranspose forward)
//   * fp32 / bf16 NCHW -> bf16 NHWC with channel padding (network input)
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

DV_DEVICE void ld8(const u16* p, float* v) {
  uint4 r = *reinterpret_cast<const uint4*>(p); uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = bf2f(w[i] & 0xffff); v[2 * i + 1] = bf2f(w[i] >> 16); }
}
DV_DEVICE void st8(u16* p, const float* v) {
  uint4 r; r.x = pack2bf(v[0], v[1]); r.y = pack2bf(v[2], v[3]); r.z = pack2bf(v[4], v[5]); r.w = pack2bf(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = r;
}

enum { A_RELU = 1, A_LEAKY = 2, A_TANH = 3, A_SIGMOID = 4 };

DV_DEVICE float actf(float x, int a, float s) {
  switch (a) {
    case A_RELU: return fmaxf(x, 0.f);
    case A_LEAKY: return x > 0.f ? x : x * s;
    case A_TANH: return tanhf(x);
    case A_SIGMOID: return 1.f / (1.f + __expf(-x));
    default: return x;
  }
}
// gradient from the OUTPUT y
DV_DEVICE float actb(float dy, float y, int a, float s) {
  switch (a) {
    case A_RELU: return y > 0.f ? dy : 0.f;
    case A_LEAKY: return y > 0.f ? dy : dy * s;
    case A_TANH: return dy * (1.f - y * y);
    case A_SIGMOID: return dy * y * (1.f - y);
    default: return dy;
  }
}

// n8 = number of 8-vectors, tail handled by the scalar kernel
__global__ __launch_bounds__(NT) void act_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y, int64_t n, int a, float s) {
  const int64_t n8 = n / 8;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n8; i += (int64_t)gridDim.x * NT) {
    float v[8]; ld8(x + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = actf(v[k], a, s);
    st8(y + i * 8, v);
  }
  const int64_t t = n8 * 8 + blockIdx.x * (int64_t)NT + threadIdx.x;
  if (t < n && blockIdx.x * (int64_t)NT + threadIdx.x < 8) y[t] = f2bf(actf(bf2f(x[t]), a, s));
}

__global__ __launch_bounds__(NT) void act_bwd_kernel(const u16* __restrict__ dy, const u16* __restrict__ y,
                                                       u16* __restrict__ dx, int64_t n, int a, float s) {
  const int64_t n8 = n / 8;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n8; i += (int64_t)gridDim.x * NT) {
    float d[8], v[8]; ld8(dy + i * 8, d); ld8(y + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = actb(d[k], v[k], a, s);
    st8(dx + i * 8, d);
  }
  const int64_t t = n8 * 8 + blockIdx.x * (int64_t)NT + threadIdx.x;
  if (t < n && blockIdx.x * (int64_t)NT + threadIdx.x < 8) dx[t] = f2bf(actb(bf2f(dy[t]), bf2f(y[t]), a, s));
}

// activation backward over rows x C (C % 8 == 0) of three NHWC tensors with their own pixel
// strides: a conv output written into a concat slice and its gradient (a slice of the concat
// gradient) are strided views, the result is dense
__global__ __launch_bounds__(NT) void act_bwd_rows_kernel(const u16* __restrict__ dy, int lddy, const u16* __restrict__ y,
                                                            int ldy, u16* __restrict__ dx, int lddx, int64_t rows, int C,
                                                            int a, float s) {
  const int cg = C / 8;
  const int64_t total = rows * cg;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int64_t r = t / cg;
    const int c = (int)(t - r * cg) * 8;
    float d[8], v[8];
    ld8(dy + r * lddy + c, d);
    ld8(y + r * ldy + c, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = actb(d[k], v[k], a, s);
    st8(dx + r * lddx + c, d);
  }
}

// y = alpha*a + beta*b, optional activation
__global__ __launch_bounds__(NT) void add_kernel(const u16* __restrict__ a, const u16* __restrict__ b, u16* __restrict__ y,
                                                   int64_t n, float alpha, float beta, int act, float s) {
  const int64_t n8 = n / 8;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n8; i += (int64_t)gridDim.x * NT) {
    float u[8], v[8]; ld8(a + i * 8, u); ld8(b + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = actf(alpha * u[k] + beta * v[k], act, s);
    st8(y + i * 8, u);
  }
  const int64_t t = n8 * 8 + blockIdx.x * (int64_t)NT + threadIdx.x;
  if (t < n && blockIdx.x * (int64_t)NT + threadIdx.x < 8) y[t] = f2bf(actf(alpha * bf2f(a[t]) + beta * bf2f(b[t]), act, s));
}

DV_DEVICE uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  // murmur3-style finalizer over a 96-bit key (counter-based, stateless)
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

// y = x * mask / (1-p);   mask_i = hash(seed, i) >= p*2^32. `step` (optional, device): a per-step
// counter mixed into the key -- a captured graph bakes the host seed into the launch, and the
// replayer advances the counter so every replay draws fresh masks (train/graph.py)
__global__ __launch_bounds__(NT) void dropout_kernel(const u16* __restrict__ x, u16* __restrict__ y, int64_t n, uint32_t thr,
                                                       float scale, uint32_t seed_lo, uint32_t seed_hi,
                                                       const uint32_t* __restrict__ step) {
  if (step) {
    const uint32_t k = step[0];
    seed_lo ^= k * 0x9E3779B9u;
    seed_hi += k;
  }
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const uint32_t h = hash3(seed_lo, seed_hi, (uint32_t)i ^ (uint32_t)(i >> 32) * 0x27D4EB2Fu);
    y[i] = (h >= thr) ? f2bf(bf2f(x[i]) * scale) : (u16)0;
  }
}

__global__ void wprep_kernel(const float* __restrict__ w, u16* __restrict__ out, int G, int Og, int Ig, int R, int S,
                             int pad, int mode, int Sp) {
  // mode 0: out[g][o][r][s][i], i padded to `pad` (>= Ig)
  // mode 1: out[g][i][r][s][o], o padded to `pad` (>= Og)
  // mode 2: mode 0 with the filter width padded to Sp (>= S): the tap-packed stem operand
  const int SS = mode == 2 ? Sp : S;
  const int64_t total = mode != 1 ? (int64_t)G * Og * pad * R * SS : (int64_t)G * Ig * pad * R * S;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t u = t;
    int g, o, i, r, s;
    bool ok;
    if (mode != 1) {
      i = (int)(u % pad); u /= pad;
      s = (int)(u % SS); u /= SS;
      r = (int)(u % R); u /= R;
      o = (int)(u % Og); g = (int)(u / Og);
      ok = i < Ig && s < S;
    } else {
      o = (int)(u % pad); u /= pad;
      s = (int)(u % S); u /= S;
      r = (int)(u % R); u /= R;
      i = (int)(u % Ig); g = (int)(u / Ig);
      ok = o < Og;
    }
    out[t] = ok ? f2bf(w[((((int64_t)(g * Og + o)) * Ig + i) * R + r) * S + s]) : (u16)0;
  }
}

// Batched weight prep: every conv / linear weight of the model re-laid-out in ONE launch after the
// optimizer step (one block per 4096-element chunk of one descriptor), instead of one launch per
// layer per call. Descriptors / chunk table live in device memory (built once on the host).
DV_DEVICE FastDiv fastdiv_dev(uint32_t d) {
  FastDiv f{0u, 0u, d};
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.shr = l;
  f.mul = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1ull);
  return f;
}

__global__ __launch_bounds__(256) void wprep_batched_kernel(const WprepDesc* __restrict__ descs,
                                                            const int2* __restrict__ chunks) {
  __shared__ float tile[64][65];
  const int2 ch = chunks[blockIdx.x];
  const WprepDesc d = descs[ch.x];
  if (d.mode == 1) {
    // dgrad layout = per-group transpose: out[g][k][o] (o padded to pad) <- w[g*Og + o][k], k = (i, r, s).
    // 64x64 tiles through LDS: coalesced reads along k and coalesced writes along o.
    const int K = d.Ig * d.R * d.S;
    const int tk = (K + 63) / 64, to = (d.pad + 63) / 64;
    const int tid = ch.y, g = tid / (tk * to), rem = tid - g * tk * to;
    const int k0 = (rem / to) * 64, o0 = (rem % to) * 64;
    const float* w = d.w + (int64_t)g * d.Og * K;
    for (int e = threadIdx.x; e < 4096; e += 256) {
      const int r = e >> 6, c = e & 63;  // r: o offset, c: k offset
      tile[r][c] = (o0 + r < d.Og && k0 + c < K) ? w[(int64_t)(o0 + r) * K + k0 + c] : 0.f;
    }
    __syncthreads();
    u16* out = d.out + (int64_t)g * K * d.pad;
    for (int e = threadIdx.x; e < 4096; e += 256) {
      const int r = e >> 6, c = e & 63;  // r: k offset, c: o offset
      if (k0 + r < K && o0 + c < d.pad) out[(int64_t)(k0 + r) * d.pad + o0 + c] = f2bf(tile[c][r]);
    }
    return;
  }
  // forward layout: out[g][o][r][s][i] (i padded; s padded to Sp in mode 2) -- reads stay inside
  // one filter row (cached)
  const int SS = d.mode == 2 ? d.Sp : d.S;
  const FastDiv fpad = fastdiv_dev(d.pad), fs = fastdiv_dev(SS), fr = fastdiv_dev(d.R);
  const FastDiv fo = fastdiv_dev(d.Og);
  const uint32_t t0 = (uint32_t)ch.y * WPREP_CHUNK;
  const uint32_t t1 = (uint32_t)min(d.total, (int64_t)t0 + WPREP_CHUNK);
  for (uint32_t t = t0 + threadIdx.x; t < t1; t += 256) {
    uint32_t u = t, q;
    q = fdiv(u, fpad); const int i = (int)(u - q * d.pad); u = q;
    q = fdiv(u, fs); const int s = (int)(u - q * SS); u = q;
    q = fdiv(u, fr); const int r = (int)(u - q * d.R); u = q;
    q = fdiv(u, fo); const int o = (int)(u - q * d.Og); const int g = (int)q;
    d.out[t] = (i < d.Ig && s < d.S) ? f2bf(d.w[((((int64_t)(g * d.Og + o)) * d.Ig + i) * d.R + r) * d.S + s]) : (u16)0;
  }
}

// fp32 [G][O][R][S][Ipad] gradient (kernel layout) -> fp32 OIHW param-grad layout (drop padding)
// [G][Og][R][S][Ipad] (GEMM layout) -> [G*Og][Ig][R][S]; walks the SOURCE (coalesced reads).
// With zero_src the source is re-zeroed as it is consumed: the wgrad workspace is persistent and
// self-cleaning, so the split-K atomics need no memset launch.
__global__ void wgrad_unprep_kernel(float* __restrict__ src, float* __restrict__ dst, int G, int Og, int Ig,
                                    int R, int S, int Ipad, float alpha, int accumulate, int zero_src) {
  const int64_t total = (int64_t)G * Og * R * S * Ipad;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % Ipad);
    const int64_t ors = t / Ipad;  // (o, r, s)
    const int rs = (int)(ors % (R * S));
    const int64_t o = ors / (R * S);  // o includes group
    const float v = src[t];
    if (zero_src) src[t] = 0.f;
    if (i < Ig) {
      const int64_t d = (o * Ig + i) * (R * S) + rs;
      dst[d] = accumulate ? dst[d] + alpha * v : alpha * v;
    }
  }
}

// The same transform through LDS, one block per output channel o: the [R*S][Ipad] source row is
// read (and re-zeroed) with coalesced accesses, the [Ig][R*S] destination row is written with
// coalesced accesses (the direct form above writes at a stride of R*S floats: ~R*S x the write
// transactions; 24 us -> a few us on a 3x3 x 512 layer).
__global__ __launch_bounds__(256) void wgrad_unprep_rows_kernel(float* __restrict__ src, float* __restrict__ dst, int Ig,
                                                                int RS, int Ipad, float alpha, int accumulate, int zero_src) {
  extern __shared__ float row[];
  const int64_t o = blockIdx.x;
  const int n = RS * Ipad;
  float* s = src + o * n;
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    row[t] = s[t];
    if (zero_src) s[t] = 0.f;
  }
  __syncthreads();
  float* d = dst + o * (int64_t)Ig * RS;
  for (int t = threadIdx.x; t < Ig * RS; t += blockDim.x) {
    const int i = t / RS, rs = t - i * RS;
    const float v = alpha * row[rs * Ipad + i];
    d[t] = accumulate ? d[t] + v : v;
  }
}

// NCHW (fp32 or bf16) -> NHWC bf16 with channel padding. One thread per pixel and group of 8
// output channels: reads are coalesced across threads (consecutive w), writes are 16-B vectors.
template <typename T>
__global__ void to_nhwc_kernel(const T* __restrict__ x, u16* __restrict__ y, int N, int C, int H, int W, int Cp) {
  const int64_t HW = (int64_t)H * W;
  const int cg = Cp / 8;
  const int64_t total = (int64_t)N * HW * cg;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = t % (N * HW);  // pixel fastest -> coalesced reads
    const int g = (int)(t / (N * HW));
    const int64_t n = pix / HW, hw = pix - n * HW;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = g * 8 + k;
      v[k] = 0.f;
      if (c < C) {
        const int64_t src = (n * C + c) * HW + hw;
        if constexpr (sizeof(T) == 4) v[k] = x[src]; else v[k] = bf2f(x[src]);
      }
    }
    uint4 r;
    r.x = pack2bf(v[0], v[1]); r.y = pack2bf(v[2], v[3]); r.z = pack2bf(v[4], v[5]); r.w = pack2bf(v[6], v[7]);
    *reinterpret_cast<uint4*>(y + pix * Cp + g * 8) = r;
  }
}

// Stem input for tap-packed convolution (conv_fwd.hip "packed" mode): NCHW (C <= 4, fp32 or
// bf16) -> bf16 [N][Hp][Wp][4], zero-padded by (pt, pl) at the top/left and to (Hp, Wp) at the
// bottom/right, channel 3 (and up) zero. Each pixel is 8 bytes, so the 16 bytes a K-chunk reads
// are two horizontally adjacent pixels = two filter taps of one row. One thread per pixel.
template <typename T>
__global__ void stem_pack_kernel(const T* __restrict__ x, u16* __restrict__ y, int N, int C, int H, int W, int Hp,
                                 int Wp, int pt, int pl, int reflect) {
  const int64_t total = (int64_t)N * Hp * Wp;
  const int64_t HW = (int64_t)H * W;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int wp = (int)(t % Wp);
    const int64_t nh = t / Wp;
    const int hp = (int)(nh % Hp);
    const int64_t n = nh / Hp;
    int h = hp - pt, w = wp - pl;
    if (reflect) {  // ReflectionPad2d; positions past the reflected border (tap-packing slack,
                    // multiplied by zero weights) are clamped so they stay finite
      h = h < 0 ? -h : (h >= H ? 2 * H - 2 - h : h);
      w = w < 0 ? -w : (w >= W ? 2 * W - 2 - w : w);
      h = h < 0 ? 0 : (h >= H ? H - 1 : h);
      w = w < 0 ? 0 : (w >= W ? W - 1 : w);
    }
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (h >= 0 && h < H && w >= 0 && w < W) {
      const int64_t src = n * C * HW + (int64_t)h * W + w;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < C) {
          if constexpr (sizeof(T) == 4) v[c] = x[src + c * HW]; else v[c] = bf2f(x[src + c * HW]);
        }
    }
    uint2 r;
    r.x = pack2bf(v[0], v[1]); r.y = pack2bf(v[2], v[3]);
    *reinterpret_cast<uint2*>(y + t * 4) = r;
  }
}

// Input pipeline, device side (data/device_input.py): uint8 HWC crops as the loader workers ship
// them (a quarter of the fp32 CHW bytes over PCIe) -> normalised bf16 NCHW network input:
// y[n][c][h][w] = (x[n][h][w'][c] * scale - mean[c]) / std[c], w' = W-1-w for flipped samples.
// One thread per output pixel quad (4 consecutive w of one (n, c, h)): 8-B stores.
__global__ void u8_normalize_kernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ flip,
                                    u16* __restrict__ y, int N, int C, int H, int W, float scale, float m0, float m1,
                                    float m2, float is0, float is1, float is2) {
  const int WQ = (W + 3) / 4;
  const int64_t total = (int64_t)N * C * H * WQ;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int wq = (int)(t % WQ);
    int64_t r = t / WQ;
    const int h = (int)(r % H); r /= H;
    const int c = (int)(r % C);
    const int64_t n = r / C;
    const bool f = flip && flip[n];
    const float m = c == 0 ? m0 : (c == 1 ? m1 : m2), is = c == 0 ? is0 : (c == 1 ? is1 : is2);
    const uint8_t* row = x + ((n * H + h) * (int64_t)W) * C + c;
    u16 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int w = wq * 4 + k;
      const int ws = f ? W - 1 - w : w;
      v[k] = w < W ? f2bf(((float)row[(int64_t)ws * C] * scale - m) * is) : (u16)0;
    }
    u16* out = y + ((n * C + c) * (int64_t)H + h) * W + wq * 4;
    if ((W & 3) == 0) {
      uint2 pk; pk.x = v[0] | ((uint32_t)v[1] << 16); pk.y = v[2] | ((uint32_t)v[3] << 16);
      *reinterpret_cast<uint2*>(out) = pk;
    } else {
      for (int k = 0; k < 4 && wq * 4 + k < W; ++k) out[k] = v[k];
    }
  }
}

// ColorJitter on the device (the trainer's uint8 crops, before u8_normalize): the arithmetic of
// csrc/host/io_core.h color_jitter, i.e. PIL's enhancers -- brightness / contrast / saturation in
// the drawn order, each Image.blend(degenerate, image, f) truncated to uint8, luma
// (19595 R + 38470 G + 7471 B + 0x8000) >> 16, the contrast gray = round(mean luma) -- so the
// bytes equal the worker-side jitter's. One block per image; an image that fits the LDS (a
// 224x224 crop is 147 KB of the 160 KB) is read once and written once, a larger one is worked in
// place in global memory. prm[n] = {f_bright, f_contrast, f_sat, op0, op1, op2}; a factor of
// exactly 1 is skipped, as on the host. No FMA contraction: the blends round like the host's
// separate multiply and add (SSE, no FMA).
DV_DEVICE uint8_t jit_clip(float v) { return (uint8_t)(int)fminf(255.f, fmaxf(0.f, v)); }
DV_DEVICE int jit_luma(const uint8_t* q) { return (q[0] * 19595 + q[1] * 38470 + q[2] * 7471 + 0x8000) >> 16; }
template <bool IN_LDS>
__global__ __launch_bounds__(256) void u8_jitter_kernel(uint8_t* __restrict__ x, const float* __restrict__ prm,
                                                        int64_t npix) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) uint8_t jbuf[];
  __shared__ long long red[4];
  const int64_t nb = npix * 3;
  uint8_t* gimg = x + (int64_t)blockIdx.x * nb;
  uint8_t* img = IN_LDS ? jbuf : gimg;
  const float* p = prm + (int64_t)blockIdx.x * 6;
  if constexpr (IN_LDS) {
    for (int64_t i = threadIdx.x; i < nb; i += 256) jbuf[i] = gimg[i];
    __syncthreads();
  }
  for (int k = 0; k < 3; ++k) {
    const int op = (int)p[3 + k];
    const float a = p[op];
    if (a == 1.f) continue;  // uniform over the block
    if (op == 0) {
      for (int64_t i = threadIdx.x; i < nb; i += 256) img[i] = jit_clip((float)img[i] * a);
    } else if (op == 1) {
      long long s = 0;
      for (int64_t i = threadIdx.x; i < npix; i += 256) s += jit_luma(img + 3 * i);
      for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
      __syncthreads();
      const long long tot = red[0] + red[1] + red[2] + red[3];
      const float m = (float)(long long)((double)tot / (double)npix + 0.5);
      for (int64_t i = threadIdx.x; i < nb; i += 256) img[i] = jit_clip(m + a * ((float)img[i] - m));
    } else {
      for (int64_t i = threadIdx.x; i < npix; i += 256) {
        uint8_t* q = img + 3 * i;
        const float g = (float)jit_luma(q);
        const uint8_t r = jit_clip(g + a * ((float)q[0] - g)), gg = jit_clip(g + a * ((float)q[1] - g)),
                      b = jit_clip(g + a * ((float)q[2] - g));
        q[0] = r; q[1] = gg; q[2] = b;
      }
    }
    __syncthreads();
  }
  if constexpr (IN_LDS) {
    for (int64_t i = threadIdx.x; i < nb; i += 256) gimg[i] = jbuf[i];
  }
}

// NHWC channel-slice copy / gather: dst[row][c] = src[row][idx ? idx[c] : c] for c < C.
// Contiguous copies (concat into a channel slice) move 16-B vectors; gathers (channel shuffle
// and its inverse) read 2-B elements through the index table.
__global__ void nhwc_copy_kernel(const u16* __restrict__ src, int lds, u16* __restrict__ dst, int ldd, int64_t rows,
                                 int C) {
  const int cg = C / 8;
  const int64_t total = rows * cg;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / cg;
    const int c = (int)(t - r * cg) * 8;
    *reinterpret_cast<uint4*>(dst + r * ldd + c) = *reinterpret_cast<const uint4*>(src + r * lds + c);
  }
}
__global__ void nhwc_gather_kernel(const u16* __restrict__ src, int lds, u16* __restrict__ dst, int ldd, int64_t rows,
                                   int C, const int* __restrict__ idx) {
  const int64_t total = rows * C;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / C;
    const int c = (int)(t - r * C);
    dst[r * ldd + c] = src[r * lds + idx[c]];
  }
}

// reflection-pad backward (NHWC bf16, 8 channels per thread): gather the interior position and
// the mirrored border positions that reflect onto (h, w); fp32 sum, one bf16 store
__global__ void reflect_pad_bwd_kernel(const u16* __restrict__ dxp, u16* __restrict__ dx, int N, int H, int W, int C,
                                       int ldp, int ld, int ph, int pw) {
  const int Hp = H + 2 * ph, Wp = W + 2 * pw, cg = C / 8;
  const int64_t total = (int64_t)N * H * W * cg;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(t % cg) * 8;
    int64_t r = t / cg;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const int64_t n = r / H;
    int hs[3], ws[3], nh = 1, nw = 1;
    hs[0] = h + ph; ws[0] = w + pw;
    if (h >= 1 && h <= ph) hs[nh++] = ph - h;                          // top border reflects onto h
    if (h >= H - 1 - ph && h <= H - 2) hs[nh++] = 2 * (H - 1) - h + ph;  // bottom border (both on tiny maps)
    if (w >= 1 && w <= pw) ws[nw++] = pw - w;
    if (w >= W - 1 - pw && w <= W - 2) ws[nw++] = 2 * (W - 1) - w + pw;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < nh; ++i)
      for (int j = 0; j < nw; ++j) {
        const uint4 v = *reinterpret_cast<const uint4*>(dxp + ((n * Hp + hs[i]) * (int64_t)Wp + ws[j]) * ldp + c);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) { acc[2 * e] += bf2f((u16)(u[e] & 0xffff)); acc[2 * e + 1] += bf2f((u16)(u[e] >> 16)); }
      }
    uint4 o;
    o.x = pack2bf(acc[0], acc[1]); o.y = pack2bf(acc[2], acc[3]); o.z = pack2bf(acc[4], acc[5]); o.w = pack2bf(acc[6], acc[7]);
    *reinterpret_cast<uint4*>(dx + ((n * H + h) * (int64_t)W + w) * ld + c) = o;
  }
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, u16* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) y[i] = f2bf(x[i]);
}

inline int grid_for(int64_t total, int per = 1) {
  int64_t g = (total / per + NT - 1) / NT;
  return (int)std::min<int64_t>(std::max<int64_t>(g, 1), 256 * 16);
}
}  // namespace

void dv_act_fwd(const void* x, void* y, int64_t n, int act, float slope, hipStream_t st) {
  act_fwd_kernel<<<grid_for(n, 8), NT, 0, st>>>((const u16*)x, (u16*)y, n, act, slope);
}
void dv_act_bwd(const void* dy, const void* y, void* dx, int64_t n, int act, float slope, hipStream_t st) {
  act_bwd_kernel<<<grid_for(n, 8), NT, 0, st>>>((const u16*)dy, (const u16*)y, (u16*)dx, n, act, slope);
}
int dv_act_bwd_rows(const void* dy, int lddy, const void* y, int ldy, void* dx, int lddx, int64_t rows, int C, int act,
                    float slope, hipStream_t st) {
  if (C % 8 || lddy % 8 || ldy % 8 || lddx % 8 || lddy < C || ldy < C || lddx < C) return -1;
  act_bwd_rows_kernel<<<grid_for(rows * (C / 8)), NT, 0, st>>>((const u16*)dy, lddy, (const u16*)y, ldy, (u16*)dx, lddx,
                                                              rows, C, act, slope);
  return 0;
}
void dv_add(const void* a, const void* b, void* y, int64_t n, float alpha, float beta, int act, float slope, hipStream_t st) {
  add_kernel<<<grid_for(n, 8), NT, 0, st>>>((const u16*)a, (const u16*)b, (u16*)y, n, alpha, beta, act, slope);
}
void dv_dropout(const void* x, void* y, int64_t n, float p, uint64_t seed, const uint32_t* step, hipStream_t st) {
  const double thr = (double)p * 4294967296.0;
  const uint32_t t = thr >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)thr;
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  dropout_kernel<<<grid_for(n), NT, 0, st>>>((const u16*)x, (u16*)y, n, t, scale, (uint32_t)seed, (uint32_t)(seed >> 32),
                                             step);
}
void dv_wprep(const float* w, void* out, int G, int Og, int Ig, int R, int S, int pad, int mode, int Sp, hipStream_t st) {
  const int64_t total = (int64_t)G * (mode != 1 ? Og : Ig) * pad * R * (mode == 2 ? Sp : S);
  wprep_kernel<<<grid_for(total), NT, 0, st>>>(w, (u16*)out, G, Og, Ig, R, S, pad, mode, Sp);
}
void dv_stem_pack(const void* x, int x_is_f32, void* y, int N, int C, int H, int W, int Hp, int Wp, int pt, int pl,
                  int reflect, hipStream_t st) {
  const int64_t total = (int64_t)N * Hp * Wp;
  if (x_is_f32) stem_pack_kernel<float><<<grid_for(total), NT, 0, st>>>((const float*)x, (u16*)y, N, C, H, W, Hp, Wp, pt, pl, reflect);
  else stem_pack_kernel<u16><<<grid_for(total), NT, 0, st>>>((const u16*)x, (u16*)y, N, C, H, W, Hp, Wp, pt, pl, reflect);
}
int dv_nhwc_copy(const void* src, int lds, void* dst, int ldd, int64_t rows, int C, const int* idx, hipStream_t st) {
  if (idx != nullptr) {
    nhwc_gather_kernel<<<grid_for(rows * C), NT, 0, st>>>((const u16*)src, lds, (u16*)dst, ldd, rows, C, idx);
    return 0;
  }
  if (C % 8 || lds % 8 || ldd % 8) return -1;  // plain copies move whole 16-B vectors
  nhwc_copy_kernel<<<grid_for(rows * (C / 8)), NT, 0, st>>>((const u16*)src, lds, (u16*)dst, ldd, rows, C);
  return 0;
}
void dv_reflect_pad_bwd(const void* dxp, void* dx, int N, int H, int W, int C, int ldp, int ld, int ph, int pw,
                        hipStream_t st) {
  const int64_t total = (int64_t)N * H * W * (C / 8);
  reflect_pad_bwd_kernel<<<grid_for(total), NT, 0, st>>>((const u16*)dxp, (u16*)dx, N, H, W, C, ldp, ld, ph, pw);
}
void dv_wprep_batched(const void* descs, const void* chunks, int nchunks, hipStream_t st) {
  if (nchunks > 0)
    wprep_batched_kernel<<<nchunks, 256, 0, st>>>((const WprepDesc*)descs, (const int2*)chunks);
}
void dv_wgrad_unprep(float* src, float* dst, int G, int Og, int Ig, int R, int S, int Ipad, float alpha,
                     int accumulate, int zero_src, hipStream_t st) {
  const int64_t total = (int64_t)G * Og * R * S * Ipad;
  const size_t row_bytes = (size_t)R * S * Ipad * sizeof(float);
  if (row_bytes <= 64 * 1024) {
    wgrad_unprep_rows_kernel<<<G * Og, 256, row_bytes, st>>>(src, dst, Ig, R * S, Ipad, alpha, accumulate, zero_src);
    return;
  }
  wgrad_unprep_kernel<<<grid_for(total), NT, 0, st>>>(src, dst, G, Og, Ig, R, S, Ipad, alpha, accumulate, zero_src);
}
void dv_u8_normalize(const void* x, const void* flip, void* y, int N, int C, int H, int W, float scale, const float* mean,
                     const float* std_, hipStream_t st) {
  const int64_t total = (int64_t)N * C * H * ((W + 3) / 4);
  u8_normalize_kernel<<<grid_for(total), NT, 0, st>>>((const uint8_t*)x, (const uint8_t*)flip, (u16*)y, N, C, H, W, scale,
                                                     mean[0], C > 1 ? mean[1] : 0.f, C > 2 ? mean[2] : 0.f, 1.f / std_[0],
                                                     C > 1 ? 1.f / std_[1] : 1.f, C > 2 ? 1.f / std_[2] : 1.f);
}

void dv_u8_jitter(void* x, const float* prm, int N, int64_t npix, hipStream_t st) {
  const int64_t nb = npix * 3;
  static const bool lds_ok = [] {
    return hipFuncSetAttribute((const void*)u8_jitter_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               150 * 1024) == hipSuccess;
  }();
  if (lds_ok && nb <= 150 * 1024)
    u8_jitter_kernel<true><<<N, 256, (size_t)((nb + 15) / 16 * 16), st>>>((uint8_t*)x, prm, npix);
  else
    u8_jitter_kernel<false><<<N, 256, 0, st>>>((uint8_t*)x, prm, npix);
}
void dv_to_nhwc(const void* x, int x_is_f32, void* y, int N, int C, int H, int W, int Cp, hipStream_t st) {
  const int64_t total = (int64_t)N * H * W * (Cp / 8);
  if (x_is_f32) to_nhwc_kernel<float><<<grid_for(total), NT, 0, st>>>((const float*)x, (u16*)y, N, C, H, W, Cp);
  else to_nhwc_kernel<u16><<<grid_for(total), NT, 0, st>>>((const u16*)x, (u16*)y, N, C, H, W, Cp);
}
void dv_f32_to_bf16(const float* x, void* y, int64_t n, hipStream_t st) {
  f32_to_bf16_kernel<<<grid_for(n), NT, 0, st>>>(x, (u16*)y, n);
}
