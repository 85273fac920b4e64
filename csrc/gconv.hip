// Grouped 1x1 convolution with small, unaligned per-group channel counts (ShuffleNet V1, g = 3:
// 20 / 40 / 80 channels per group) and the channel shuffle fused into the store (SURVEY §2.7 K7;
// the reference's R/ShuffleNet/pytorch/models/shufflenet_v1.py is empty, design from the paper).
//
//   y[m][pos_out(g*Og + j)] = sum_{k < Cg} x[m][pos_in(g*Cg + k)] * W[g*Og + j][k]
//
// pos(l) is the identity or the ShuffleNet permutation of C channels in `sg` groups (logical
// channel l = a*(C/sg) + b stored at b*sg + a). The forward of ShuffleNet's first grouped 1x1
// stores its output shuffled (pos_out); its dgrad reads that gradient back through the same map
// (pos_in) -- the shuffle never runs as a separate pass.
//
// Structure (one 256-thread block = BM pixel rows x ALL output channels):
//   1. the BM input rows are copied into LDS with 16-B loads (rows are 16-B aligned NHWC);
//   2. LDS "repack": per group, the Cg channels are gathered (through pos_in) into a logical
//      image [BM][G*Kp], each group zero-padded to Kp = round32(Cg) -- from here on every MFMA
//      fragment is one aligned ds_read_b128 whatever Cg, the group offset or the permutation;
//   3. each wave takes (16-row fragment, group, 4 output-column fragments) items:
//      v_mfma_f32_16x16x32_bf16 with the weights [G][Orows][Kp] (wcache layout) as the A operand;
//   4. the epilogue writes bf16 results into an LDS output tile at pos_out (the shuffle), folds
//      the shifted BatchNorm partial statistics (DPP row sums, LDS, one sharded atomic row per
//      block, csrc/kernels.h DV_STAT_ROWS) and stores whole rows with vector stores.
// The weight gradient (gconv_wgrad_kernel) reduces over pixels with 4x4 register blocks per
// thread (these layers are memory-bound: a few tens of MACs per loaded byte).
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

struct GcParams {
  const u16* x;
  int ldx, Cin, in_sg;
  const u16* w;  // [G][Orows][Kp] bf16 (rows >= Og are never used)
  int Orows;
  u16* y;
  int ldy, Cout, out_sg;
  int M, G, Cg, Og, Kp;
  float* stats;  // shifted BN statistics of y by stored channel position, or nullptr
};

DV_DEVICE int perm_pos(int l, int C, int sg) {
  if (sg <= 1) return l;
  const int cpg = C / sg;
  return (l % cpg) * sg + l / cpg;
}

struct GcLayout {
  int RP, PK, PP, YP;
  bool direct;  // the input rows already are the logical padded image (no repack)
};
inline __host__ __device__ int r8(int v) { return (v + 7) & ~7; }
inline __host__ __device__ GcLayout gc_layout(int Cin, int G, int Cg, int Kp, int in_sg, int Cout) {
  GcLayout L;
  L.direct = in_sg <= 1 && Cg == Kp && Cin == G * Cg;
  L.RP = r8(Cin) + 8;
  L.PK = G * Kp;
  L.PP = L.direct ? L.RP : L.PK + 8;
  L.YP = r8(Cout) + 8;
  return L;
}
inline __host__ __device__ size_t gc_lds_bytes(const GcLayout& L, int BM, int Cout, bool stats) {
  // [BM][RP] input rows | [BM][PP] logical image (unless direct) | [BM][YP] output tile | stats
  return (size_t)BM * (L.RP + (L.direct ? 0 : L.PP) + L.YP) * 2 + (stats ? (size_t)2 * Cout * 4 : 0);
}

template <int BM>
__global__ __launch_bounds__(NT) void gconv_kernel(GcParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const GcLayout L = gc_layout(p.Cin, p.G, p.Cg, p.Kp, p.in_sg, p.Cout);
  u16* raw = reinterpret_cast<u16*>(smem);
  u16* pk = L.direct ? raw : raw + BM * L.RP;
  u16* ys = pk + (L.direct ? BM * L.RP : BM * L.PP);
  float* st = reinterpret_cast<float*>(ys + BM * L.YP);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.x * BM;

  // 1. input rows -> LDS (whole 16-B chunks; the channel padding of the NHWC storage rides along)
  const int cpr = r8(p.Cin) / 8;
  for (int i = tid; i < BM * cpr; i += NT) {
    const int r = i / cpr, c = i - r * cpr;
    const int m = m0 + r;
    uint4 v = {0u, 0u, 0u, 0u};
    if (m < p.M) v = *reinterpret_cast<const uint4*>(p.x + (int64_t)m * p.ldx + c * 8);
    *reinterpret_cast<uint4*>(raw + r * L.RP + c * 8) = v;
  }
  if (p.stats)
    for (int i = tid; i < 2 * p.Cout; i += NT) st[i] = 0.f;
  __syncthreads();
  // 2. logical zero-padded image, 8 channels (one 16-B LDS write) per step
  if (!L.direct) {
    const int upr = L.PK / 8;
    for (int i = tid; i < BM * upr; i += NT) {
      const int r = i / upr, u = i - r * upr;
      const int g = (u * 8) / p.Kp, k0 = u * 8 - g * p.Kp;
      uint32_t w4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ka = k0 + 2 * e, kb = ka + 1;
        const uint32_t lo = ka < p.Cg ? raw[r * L.RP + perm_pos(g * p.Cg + ka, p.Cin, p.in_sg)] : 0u;
        const uint32_t hi = kb < p.Cg ? raw[r * L.RP + perm_pos(g * p.Cg + kb, p.Cin, p.in_sg)] : 0u;
        w4[e] = lo | (hi << 16);
      }
      *reinterpret_cast<uint4*>(pk + r * L.PP + u * 8) = uint4{w4[0], w4[1], w4[2], w4[3]};
    }
    __syncthreads();
  }
  // 3. MFMA items: (row fragment, group, chunk of 4 output-column fragments)
  const int nrf = BM / 16;
  const int ncf = (p.Og + 15) / 16;
  const int ncc = (ncf + 3) / 4;
  const int nitems = nrf * p.G * ncc;
  const int nkc = p.Kp / 32;
  const float* shift = p.stats ? stat_shift(p.stats, p.Cout) : nullptr;
  for (int it = wid; it < nitems; it += NT / 64) {
    const int rf = it % nrf;
    const int t = it / nrf;
    const int cc = t % ncc, g = t / ncc;
    f32x4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int row = rf * 16 + (lane & 15);
    for (int kc = 0; kc < nkc; ++kc) {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(pk + row * L.PP + g * p.Kp + kc * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cf = cc * 4 + q;
        if (cf < ncf) {  // wave-uniform
          const int j = min(cf * 16 + (lane & 15), p.Og - 1);  // rows >= Og: discarded results
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(p.w + ((int64_t)g * p.Orows + j) * p.Kp + kc * 32 +
                                                          8 * (lane >> 4));
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[q], 0, 0, 0);
        }
      }
    }
    // 4. acc[q][r] = y[pixel row][channel j = cf*16 + (lane>>4)*4 + r] of group g
    const bool mv = m0 + row < p.M;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cf = cc * 4 + q;
      if (cf >= ncf) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = cf * 16 + (lane >> 4) * 4 + r;
        const bool jv = j < p.Og;
        const int pos = jv ? perm_pos(g * p.Og + j, p.Cout, p.out_sg) : 0;
        const float v = acc[q][r];
        if (jv) ys[row * L.YP + pos] = f2bf(v);
        if (p.stats) {  // wave-uniform
          const float d = (jv && mv) ? v - shift[pos] : 0.f;
          const float s1 = row16_sum(d), s2 = row16_sum(d * d);
          if ((lane & 15) == 0 && jv) {
            atomicAdd(st + pos, s1);
            atomicAdd(st + p.Cout + pos, s2);
          }
        }
      }
    }
  }
  __syncthreads();
  if (p.stats) {
    float* a = p.stats + (int64_t)(blockIdx.x % DV_STAT_SHARDS) * 2 * p.Cout;
    for (int c = tid; c < p.Cout; c += NT) {
      atomicAdd(a + c, st[c]);
      atomicAdd(a + p.Cout + c, st[p.Cout + c]);
    }
  }
  // 5. output rows: 16-B / 8-B / 2-B pieces by alignment
  const int vw = (p.Cout % 8 == 0 && p.ldy % 8 == 0) ? 8 : (p.Cout % 4 == 0 && p.ldy % 4 == 0) ? 4 : 1;
  const int ppr = p.Cout / vw;
  for (int i = tid; i < BM * ppr; i += NT) {
    const int r = i / ppr, c = (i - r * ppr) * vw;
    const int m = m0 + r;
    if (m >= p.M) continue;
    u16* dst = p.y + (int64_t)m * p.ldy + c;
    const u16* src = ys + r * L.YP + c;
    if (vw == 8) *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    else if (vw == 4) *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(src);
    else *dst = *src;
  }
}

// ---- weight gradient: dW[g*Og + j][k] += sum_m dy[m][pos_out(g*Og+j)] * x[m][pos_in(g*Cg+k)] ----
// Block = a chunk of rows (in tiles of WB pixels) x a chunk of 256 (4 j x 4 k) output blocks; the
// tiles are repacked into logical (unpermuted, dense) order in LDS, each thread accumulates its
// 16 outputs in fp32 registers over all the chunk's rows and adds them into dW once.
struct GwParams {
  const u16* x;
  int ldx, Cin, in_sg;
  const u16* dy;
  int ldy, Cout, out_sg;
  float* dw;  // [G*Og][Cg] fp32, accumulated
  int M, G, Cg, Og, rows_per_block, WB;  // WB: rows per LDS tile (64 / 32 / 16, LDS budget)
};

__global__ __launch_bounds__(NT) void gconv_wgrad_kernel(GwParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int XL = p.G * p.Cg, YL = p.G * p.Og;  // logical row lengths (multiples of 4)
  const int XP = XL + 4, YPp = YL + 4;         // pitches (8-B aligned rows)
  const int XR = r8(p.Cin) + 8, YR = r8(p.Cout) + 8;
  const int WB = p.WB;
  u16* xraw = reinterpret_cast<u16*>(smem);
  u16* yraw = xraw + WB * XR;
  u16* xl = yraw + WB * YR;
  u16* yl = xl + WB * XP;
  const int tid = threadIdx.x;
  // this thread's 4x4 output block
  const int jb = p.Og / 4, kb = p.Cg / 4;
  const int item = blockIdx.y * NT + tid;
  const bool active = item < p.G * jb * kb;
  const int g = active ? item / (jb * kb) : 0;
  const int rem = active ? item - g * jb * kb : 0;
  const int j0 = (rem / kb) * 4, k0 = (rem % kb) * 4;
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
  const int rbeg = blockIdx.x * p.rows_per_block, rend = min(p.M, rbeg + p.rows_per_block);
  const int xc = r8(p.Cin) / 8, yc = r8(p.Cout) / 8;
  for (int t0 = rbeg; t0 < rend; t0 += WB) {
    __syncthreads();  // the previous tile's logical images are no longer read
    for (int i = tid; i < WB * (xc + yc); i += NT) {
      const bool isx = i < WB * xc;
      const int ii = isx ? i : i - WB * xc;
      const int cpr = isx ? xc : yc;
      const int r = ii / cpr, c = ii - r * cpr;
      const int m = t0 + r;
      uint4 v = {0u, 0u, 0u, 0u};
      if (m < rend) v = *reinterpret_cast<const uint4*>((isx ? p.x : p.dy) + (int64_t)m * (isx ? p.ldx : p.ldy) + c * 8);
      *reinterpret_cast<uint4*>((isx ? xraw + r * XR : yraw + r * YR) + c * 8) = v;
    }
    __syncthreads();
    for (int i = tid; i < WB * (XL + YL) / 2; i += NT) {  // logical images, 2 channels per step
      const bool isx = i < WB * XL / 2;
      const int ii = isx ? i : i - WB * XL / 2;
      const int half = (isx ? XL : YL) / 2;
      const int r = ii / half, l = (ii - r * half) * 2;
      const u16* src = isx ? xraw + r * XR : yraw + r * YR;
      const int C = isx ? p.Cin : p.Cout, sg = isx ? p.in_sg : p.out_sg;
      const uint32_t lo = src[perm_pos(l, C, sg)], hi = src[perm_pos(l + 1, C, sg)];
      *reinterpret_cast<uint32_t*>((isx ? xl + r * XP : yl + r * YPp) + l) = lo | (hi << 16);
    }
    __syncthreads();
    if (active) {
      const int nr = min(WB, rend - t0);
      for (int r = 0; r < nr; ++r) {
        const uint2 xv = *reinterpret_cast<const uint2*>(xl + r * XP + g * p.Cg + k0);
        const uint2 yv = *reinterpret_cast<const uint2*>(yl + r * YPp + g * p.Og + j0);
        const float xf[4] = {bf2f(xv.x & 0xffff), bf2f(xv.x >> 16), bf2f(xv.y & 0xffff), bf2f(xv.y >> 16)};
        const float yf[4] = {bf2f(yv.x & 0xffff), bf2f(yv.x >> 16), bf2f(yv.y & 0xffff), bf2f(yv.y >> 16)};
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = fmaf(yf[a], xf[b], acc[a][b]);
      }
    }
  }
  if (!active) return;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) atomicAdd(p.dw + (int64_t)(g * p.Og + j0 + a) * p.Cg + k0 + b, acc[a][b]);
}
}  // namespace

// fwd / dgrad; returns -1 for an unsupported shape (the caller falls back)
int dv_gconv(const void* x, int ldx, int Cin, int in_sg, const void* w, int Orows, void* y, int ldy, int Cout, int out_sg,
             int M, int G, int Cg, int Og, int Kp, float* stats, hipStream_t st) {
  if (Cin != G * Cg || Cout != G * Og || Kp % 32 || Kp < Cg || ldx % 8 || ldy % 4 || (uintptr_t)x % 16 ||
      (uintptr_t)w % 16 || r8(Cin) > ldx || (in_sg > 1 && Cin % in_sg) || (out_sg > 1 && Cout % out_sg) || Orows < Og)
    return -1;
  GcParams p{(const u16*)x, ldx, Cin, in_sg, (const u16*)w, Orows, (u16*)y, ldy, Cout, out_sg, M, G, Cg, Og, Kp, stats};
  const GcLayout L = gc_layout(Cin, G, Cg, Kp, in_sg, Cout);
  // 64 rows while two blocks fit a CU, else 32 / 16
  int BM = 64;
  while (BM > 16 && gc_lds_bytes(L, BM, Cout, stats) > 80 * 1024) BM /= 2;
  const size_t lds = gc_lds_bytes(L, BM, Cout, stats);
  if (lds > 160 * 1024) return -1;
  const unsigned grid = (unsigned)((M + BM - 1) / BM);
  static bool attr[3] = {false, false, false};
#define GC_LAUNCH(B, I)                                                                                        \
  do {                                                                                                         \
    if (!attr[I]) {                                                                                            \
      hipFuncSetAttribute((const void*)gconv_kernel<B>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      attr[I] = true;                                                                                          \
    }                                                                                                          \
    gconv_kernel<B><<<grid, NT, lds, st>>>(p);                                                                 \
  } while (0)
  if (BM == 64) GC_LAUNCH(64, 0);
  else if (BM == 32) GC_LAUNCH(32, 1);
  else GC_LAUNCH(16, 2);
#undef GC_LAUNCH
  return 0;
}

int dv_gconv_wgrad(const void* x, int ldx, int Cin, int in_sg, const void* dy, int ldy, int Cout, int out_sg, float* dw,
                   int M, int G, int Cg, int Og, hipStream_t st) {
  if (Cin != G * Cg || Cout != G * Og || Cg % 4 || Og % 4 || ldx % 8 || ldy % 8 || (uintptr_t)x % 16 ||
      (uintptr_t)dy % 16 || r8(Cin) > ldx || r8(Cout) > ldy)
    return -1;
  auto lds_of = [&](int wb) { return (size_t)wb * ((r8(Cin) + 8) + (r8(Cout) + 8) + (G * Cg + 4) + (G * Og + 4)) * 2; };
  int WB = 64;
  while (WB > 16 && lds_of(WB) > 80 * 1024) WB /= 2;
  const size_t lds = lds_of(WB);
  if (lds > 160 * 1024) return -1;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gconv_wgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int items = G * (Og / 4) * (Cg / 4);
  const int ichunks = (items + NT - 1) / NT;
  // ~1024 blocks in all, >= 4 row tiles per block (the 16 atomics per thread amortised)
  int64_t rchunks = std::max<int64_t>(1, 1024 / ichunks);
  int64_t rpb = (M + rchunks - 1) / rchunks;
  rpb = std::max<int64_t>(4 * WB, (rpb + WB - 1) / WB * WB);
  rchunks = (M + rpb - 1) / rpb;
  GwParams p{(const u16*)x, ldx, Cin, in_sg, (const u16*)dy, ldy, Cout, out_sg, dw, M, G, Cg, Og, (int)rpb, WB};
  gconv_wgrad_kernel<<<dim3((unsigned)rchunks, (unsigned)ichunks), NT, lds, st>>>(p);
  return 0;
}
