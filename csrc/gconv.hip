// Grouped 1x1 convolution with small, unaligned per-group channel counts (ShuffleNet V1, g = 3:
// 20 / 40 / 80 channels per group) and the channel shuffle fused into the store (SURVEY §2.7 K7;
// the reference's R/ShuffleNet/pytorch/models/shufflenet_v1.py is empty, design from the paper).
//
//   y[m][pos_out(g*Og + j)] = sum_{k < Cg} x[m][pos_in(g*Cg + k)] * W[g*Og + j][k]
//
// pos() is the identity or the ShuffleNet permutation (logical channel l = a*(C/sg) + b stored at
// b*sg + a), passed as a small int16 table (nullptr = identity): the forward of ShuffleNet's
// first grouped 1x1 stores its output shuffled, its dgrad and wgrad read that gradient back
// through the same table -- the shuffle never runs as a separate pass.
//
// Forward / dgrad (gconv_kernel, one 256-thread block = BM pixel rows x ALL output channels):
//   1. the rows are loaded straight into a logical LDS image [BM][G*Kp] (each group's Cg
//      channels zero-padded to Kp = round32(Cg)): aligned 8-channel pieces by one 16-B load,
//      unaligned / permuted ones element-wise -- every MFMA fragment is then one ds_read_b128;
//   2. each wave takes (16-row fragment, group, 4 output-column fragments) items:
//      v_mfma_f32_16x16x32_bf16, weights [G][Orows][Kp] (ops/wcache layouts) as the A operand;
//   3. the epilogue writes bf16 results into an LDS output tile at pos_out (the shuffle), folds
//      the shifted BatchNorm partial statistics (DPP row sums, LDS, one sharded atomic row per
//      block, csrc/kernels.h DV_STAT_ROWS) and stores whole rows with vector stores.
// Weight gradient (gconv_wgrad_kernel): per group dW_g = dY_g^T X_g, a GEMM whose reduction runs
// over the pixels. 64-pixel tiles of both operands are staged row-major with an XOR swizzle and
// read as MFMA fragments by the hardware-transposed ds_read_b64_tr_b16 (as conv_wgrad.hip);
// blocks split the pixels (split-K) and add their fp32 tiles into dW once.
#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;
inline __host__ __device__ int r8(int v) { return (v + 7) & ~7; }
// operand load modes (uniform per launch): 8 aligned channels per 16-B load / even offsets in
// 4-byte pairs / a permuted or odd layout gathered element-wise through an LDS position table
enum { GW_V16 = 0, GW_PAIR = 1, GW_GATHER = 2 };

struct GcParams {
  const u16* x;
  int ldx, Cin;
  const int16_t* tin;  // logical -> stored input channel, or nullptr (identity)
  const u16* w;        // [G][Orows][Kp] bf16 (rows >= Og are never used)
  int Orows;
  u16* y;
  int ldy, Cout;
  const int16_t* tout;  // logical -> stored output channel, or nullptr
  int M, G, Cg, Og, Kp;
  float* stats;  // shifted BN statistics of y by stored channel position, or nullptr
  FastDiv div_upr, div_kc;  // chunks per row (G*Kp/8), chunks per group (Kp/8)
  // deterministic mode (kernels.h DetStats): per-block slab rows; the 4 waves then keep separate
  // LDS statistics rows summed in wave order (LDS float atomics from several waves have no order)
  float* sdet;
};

// LDS statistics rows: one shared row, or one per wave in deterministic mode
inline __host__ __device__ int gc_stat_rows(bool det) { return det ? NT / 64 : 1; }
inline __host__ __device__ size_t gc_lds_bytes(int BM, int G, int Kp, int Cout, bool stats, bool det = false) {
  // [BM][G*Kp + 8] logical input image | [BM][r8(Cout) + 8] output tile | [Cout] table | stats
  return (size_t)BM * ((G * Kp + 8) + (r8(Cout) + 8)) * 2 + (size_t)Cout * 2 +
         (stats ? (size_t)2 * Cout * 4 * gc_stat_rows(det) : 0) + 16 + (size_t)G * Kp * 2;  // + the input position table
}

template <int BM, int MODE>
__global__ __launch_bounds__(NT) void gconv_kernel(GcParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int PK = p.G * p.Kp, PP = PK + 8, YP = r8(p.Cout) + 8;
  u16* pk = reinterpret_cast<u16*>(smem);
  u16* ys = pk + BM * PP;
  int16_t* tout = reinterpret_cast<int16_t*>(ys + BM * YP);
  float* st = reinterpret_cast<float*>(smem + (((size_t)BM * (PP + YP) * 2 + (size_t)p.Cout * 2 + 15) & ~(size_t)15));
  const int srows = gc_stat_rows(p.sdet != nullptr);
  int16_t* tin = reinterpret_cast<int16_t*>(st + (p.stats ? 2 * p.Cout * srows : 0));  // [G*Kp] (GATHER)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float* stw = st + (srows > 1 ? wid * 2 * p.Cout : 0);  // this wave's LDS statistics row
  const int m0 = blockIdx.x * BM;

  for (int c = tid; c < p.Cout; c += NT) tout[c] = p.tout ? p.tout[c] : (int16_t)c;
  if constexpr (MODE == GW_GATHER) {
    for (int u = tid; u < PK; u += NT) {  // logical padded channel -> stored channel (-1: padding)
      const int g = u / p.Kp, k = u - g * p.Kp;
      tin[u] = k < p.Cg ? (p.tin ? p.tin[g * p.Cg + k] : (int16_t)(g * p.Cg + k)) : (int16_t)-1;
    }
    __syncthreads();
  }
  if (p.stats)
    for (int i = tid; i < 2 * p.Cout * srows; i += NT) st[i] = 0.f;
  // 1. logical zero-padded input image, one 8-channel piece per step. The loads of 8 pieces are
  // issued before any LDS write and never sit behind a branch (hipcc waits for a load right at
  // a branch around it): padding / out-of-range pieces read the zero page instead.
  const int upr = PK / 8;
  const int total = BM * upr;
  const u16* zp = reinterpret_cast<const u16*>(dv_zero_page);
  for (int base = tid; base < total; base += 8 * NT) {
    uint4 v[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int i = min(base + b * NT, total - 1);
      const int r = (int)fdiv((uint32_t)i, p.div_upr), u = i - r * upr;
      const int g = (int)fdiv((uint32_t)u, p.div_kc), k0 = (u - g * (p.Kp / 8)) * 8;
      const int m = m0 + r;
      const int l0 = g * p.Cg + k0;
      const bool ok = m < p.M && k0 < p.Cg;
      const u16* row = p.x + (int64_t)(ok ? m : 0) * p.ldx;
      if constexpr (MODE == GW_V16) {
        v[b] = *reinterpret_cast<const uint4*>(ok ? row + l0 : zp);
      } else if constexpr (MODE == GW_PAIR) {
        uint32_t w4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool va = ok && k0 + 2 * e < p.Cg;
          const uint32_t x2 = *reinterpret_cast<const uint32_t*>(row + (va ? l0 + 2 * e : 0));
          w4[e] = va ? x2 : 0u;
        }
        v[b] = uint4{w4[0], w4[1], w4[2], w4[3]};
      } else {
        uint32_t w4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int pa = tin[u * 8 + 2 * e], pb = tin[u * 8 + 2 * e + 1];
          const uint32_t lo = row[(ok && pa >= 0) ? pa : 0], hi = row[(ok && pb >= 0) ? pb : 0];
          w4[e] = ((ok && pa >= 0) ? lo : 0u) | (((ok && pb >= 0) ? hi : 0u) << 16);
        }
        v[b] = uint4{w4[0], w4[1], w4[2], w4[3]};
      }
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int i = base + b * NT;
      if (i < total) {
        const int r = (int)fdiv((uint32_t)i, p.div_upr), u = i - r * upr;
        *reinterpret_cast<uint4*>(pk + r * PP + u * 8) = v[b];
      }
    }
  }
  __syncthreads();
  // 2. MFMA items: (row fragment, group, chunk of 4 output-column fragments)
  constexpr int NRF = BM / 16;
  const int ncf = (p.Og + 15) / 16;
  const int ncc = (ncf + 3) / 4;
  const int nitems = NRF * p.G * ncc;
  const int nkc = p.Kp / 32;
  const float* shift = p.stats ? stat_shift(p.stats, p.Cout) : nullptr;
  for (int it = wid; it < nitems; it += NT / 64) {
    const int rf = it % NRF;
    const int t = it / NRF;
    const int cc = t % ncc, g = t / ncc;
    f32x4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int row = rf * 16 + (lane & 15);
    // weight fragments come from L2: the next k-chunk's four are loaded while this chunk's MFMAs
    // run (unconditional loads from clamped rows: rows >= Og give discarded results)
    const u16* wq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      wq[q] = p.w + ((int64_t)g * p.Orows + min((cc * 4 + q) * 16 + (lane & 15), p.Og - 1)) * p.Kp + 8 * (lane >> 4);
    bf16x8 a[4], an[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = *reinterpret_cast<const bf16x8*>(wq[q]);
    for (int kc = 0; kc < nkc; ++kc) {
      const int kn = min(kc + 1, nkc - 1) * 32;
#pragma unroll
      for (int q = 0; q < 4; ++q) an[q] = *reinterpret_cast<const bf16x8*>(wq[q] + kn);
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(pk + row * PP + g * p.Kp + kc * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (cc * 4 + q < ncf) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[q], b, acc[q], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = an[q];
    }
    // 3. acc[q][r] = y[pixel row][channel j = cf*16 + (lane>>4)*4 + r] of group g
    const bool mv = m0 + row < p.M;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cf = cc * 4 + q;
      if (cf >= ncf) break;
      const int j4 = cf * 16 + (lane >> 4) * 4;  // Og % 4 == 0: the 4 channels are all valid or none
      if (!p.tout && j4 < p.Og)  // contiguous output channels: one 8-byte LDS write
        *reinterpret_cast<uint2*>(ys + row * YP + g * p.Og + j4) =
            uint2{pack2bf(acc[q][0], acc[q][1]), pack2bf(acc[q][2], acc[q][3])};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = j4 + r;
        const bool jv = j < p.Og;
        const int pos = jv ? tout[g * p.Og + j] : 0;
        const float v = acc[q][r];
        if (jv && p.tout) ys[row * YP + pos] = f2bf(v);
        if (p.stats) {  // wave-uniform
          const float d = (jv && mv) ? v - shift[pos] : 0.f;
          const float s1 = row16_sum(d), s2 = row16_sum(d * d);
          if ((lane & 15) == 0 && jv) {
            atomicAdd(stw + pos, s1);
            atomicAdd(stw + p.Cout + pos, s2);
          }
        }
      }
    }
  }
  __syncthreads();
  if (p.stats) {
    float* a = stat_row(p.stats, p.sdet, blockIdx.x, p.Cout);
    for (int c = tid; c < p.Cout; c += NT) {
      float s1 = st[c], s2 = st[p.Cout + c];
      for (int w = 1; w < srows; ++w) { s1 += st[w * 2 * p.Cout + c]; s2 += st[w * 2 * p.Cout + p.Cout + c]; }
      atomicAdd(a + c, s1);
      atomicAdd(a + p.Cout + c, s2);
    }
  }
  // 4. output rows: 16-B / 8-B / 2-B pieces by alignment
  const int vw = (p.Cout % 8 == 0 && p.ldy % 8 == 0) ? 8 : (p.Cout % 4 == 0 && p.ldy % 4 == 0) ? 4 : 1;
  const int ppr = p.Cout / vw;
  for (int i = tid; i < BM * ppr; i += NT) {
    const int r = i / ppr, c = (i - r * ppr) * vw;
    const int m = m0 + r;
    if (m >= p.M) continue;
    u16* dst = p.y + (int64_t)m * p.ldy + c;
    const u16* src = ys + r * YP + c;
    if (vw == 8) *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    else if (vw == 4) *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(src);
    else *dst = *src;
  }
}

// ---- weight gradient: dW[g*Og + j][k] += sum_m dy[m][tout(g*Og+j)] * x[m][tin(g*Cg+k)] ----
constexpr int FPW = 4;    // output fragments per wave; a block = 16 fragments, dealt round-robin

struct GwParams {
  const u16* x;
  int ldx;
  const int16_t* tin;
  const u16* dy;
  int ldy;
  const int16_t* tout;
  float* dw;  // [G*Og][Cg] fp32, accumulated
  int M, G, Cg, Og;
  int CJ, CK;        // image widths (columns): 64 or a multiple of 128
  int WT;            // pixels per tile: 64, or 32 for wide images (LDS / staging registers)
  int nkf, nfrag;    // fragments: ceil(Og/16) x ceil(Cg/16), row-major over (jf, kf)
  int fchunks;       // blockIdx.y = g * fchunks + fragment chunk (4 * FPW fragments)
  int tiles_per_block;
  float* slab;       // deterministic mode: block-row x's partial dW at slab + x * G*Og*Cg (plain stores)
};

// 16-byte-chunk XOR key of pixel row k (conv_wgrad.hip mn_swz): 8 keys for rows >= 256 B,
// 4 keys for 128-B rows; conflict-free transposed reads for rows that are multiples of 256 B
DV_DEVICE int gw_swz(int k, int cols) {
  if (cols >= 128) return ((k & 3) | ((k >> 1) & 4)) << 1;
  return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
}
DV_DEVICE bf16x8 gw_read(const char* img, int cols, int col0, int kbase, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k1 = kbase + 8 * g + q, k2 = k1 + 4;
  const int u = (col0 >> 2) + p;
  const char* a1 = img + k1 * (cols * 2) + ((u ^ (gw_swz(k1, cols) << 1)) << 3);
  const char* a2 = img + k2 * (cols * 2) + ((u ^ (gw_swz(k2, cols) << 1)) << 3);
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)LDS_PTR(a1));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)LDS_PTR(a2));
  i16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

// 8 logical channels [c0, c0 + 8) of group g of one pixel row (zeros past nch / when !ok);
// unconditional loads (the zero page or clamped indices), see gconv_kernel; MODE: GW_*
template <int MODE>
DV_DEVICE uint4 gw_piece(const u16* row, bool ok, const int16_t* pos, int base, int c0, int nch) {
  const int l0 = base + c0;
  if constexpr (MODE == GW_V16) {
    return *reinterpret_cast<const uint4*>(ok && c0 < nch ? row + l0 : reinterpret_cast<const u16*>(dv_zero_page));
  } else if constexpr (MODE == GW_PAIR) {
    uint32_t w4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool va = ok && c0 + 2 * e < nch;
      const uint32_t v = *reinterpret_cast<const uint32_t*>(row + (va ? l0 + 2 * e : 0));
      w4[e] = va ? v : 0u;
    }
    return uint4{w4[0], w4[1], w4[2], w4[3]};
  } else {
    uint32_t w4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ka = c0 + 2 * e, kb = ka + 1;
      const bool va = ok && ka < nch, vb = ok && kb < nch;
      const uint32_t lo = row[va ? pos[2 * e] : 0], hi = row[vb ? pos[2 * e + 1] : 0];
      w4[e] = (va ? lo : 0u) | ((vb ? hi : 0u) << 16);
    }
    return uint4{w4[0], w4[1], w4[2], w4[3]};
  }
}

template <int MY, int MX, int MAXP>
__global__ __launch_bounds__(NT) void gconv_wgrad_kernel(GwParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int WT = p.WT;
  char* yimg = smem;                  // [WT][CJ] dY of group g, swizzled 16-B chunks
  char* ximg = smem + WT * p.CJ * 2;  // [WT][CK] X of group g
  int16_t* posy = reinterpret_cast<int16_t*>(ximg + WT * p.CK * 2);  // [Og] stored dY channels of g
  int16_t* posx = posy + p.Og;                                        // [Cg] stored X channels of g
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = blockIdx.y / p.fchunks, fc = blockIdx.y - g * p.fchunks;
  if constexpr (MY == GW_GATHER)
    for (int j = tid; j < p.Og; j += NT) posy[j] = p.tout ? p.tout[g * p.Og + j] : (int16_t)(g * p.Og + j);
  if constexpr (MX == GW_GATHER)
    for (int k = tid; k < p.Cg; k += NT) posx[k] = p.tin ? p.tin[g * p.Cg + k] : (int16_t)(g * p.Cg + k);
  if constexpr (MY == GW_GATHER || MX == GW_GATHER) __syncthreads();
  f32x4 acc[FPW];
#pragma unroll
  for (int f = 0; f < FPW; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntiles = (p.M + WT - 1) / WT;
  const int t0 = blockIdx.x * p.tiles_per_block, t1 = min(ntiles, t0 + p.tiles_per_block);
  const int cj8 = p.CJ / 8, ck8 = p.CK / 8;
  const int total = WT * (cj8 + ck8);  // <= MAXP * NT (host check)
  uint4 v[MAXP];
  // the next tile's pieces are loaded into registers while the current tile's MFMAs run
  auto fetch = [&](int t) {
#pragma unroll
    for (int b = 0; b < MAXP; ++b) {
      const int i = min(tid + b * NT, total - 1);
      const bool isy = i < WT * cj8;
      const int ii = isy ? i : i - WT * cj8;
      const int c8 = isy ? cj8 : ck8;
      const int r = ii / c8, c = ii - r * c8;
      const int m = t * WT + r;
      const bool ok = m < p.M;
      const int mm = ok ? m : 0;
      v[b] = isy ? gw_piece<MY>(p.dy + (int64_t)mm * p.ldy, ok, posy + c * 8, g * p.Og, c * 8, p.Og)
                 : gw_piece<MX>(p.x + (int64_t)mm * p.ldx, ok, posx + c * 8, g * p.Cg, c * 8, p.Cg);
    }
  };
  if (t0 < t1) fetch(t0);
  for (int t = t0; t < t1; ++t) {
    __syncthreads();  // the previous tile's fragments are read
#pragma unroll
    for (int b = 0; b < MAXP; ++b) {
      const int i = tid + b * NT;
      if (i < total) {
        const bool isy = i < WT * cj8;
        const int ii = isy ? i : i - WT * cj8;
        const int c8 = isy ? cj8 : ck8;
        const int r = ii / c8, c = ii - r * c8;
        const int cols = isy ? p.CJ : p.CK;
        char* img = isy ? yimg : ximg;
        *reinterpret_cast<uint4*>(img + r * cols * 2 + ((c ^ gw_swz(r, cols)) << 4)) = v[b];
      }
    }
    __syncthreads();
    if (t + 1 < t1) fetch(t + 1);
#pragma unroll
    for (int f = 0; f < FPW; ++f) {
      const int fi = fc * 4 * FPW + f * 4 + wid;  // round-robin over the block's 4 waves
      if (fi < p.nfrag) {                          // wave-uniform
        const int jf = fi / p.nkf, kf = fi - jf * p.nkf;
        for (int ks = 0; ks < WT / 32; ++ks) {
          const bf16x8 a = gw_read(yimg, p.CJ, jf * 16, ks * 32, lane);
          const bf16x8 b = gw_read(ximg, p.CK, kf * 16, ks * 32, lane);
          acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[f], 0, 0, 0);
        }
      }
    }
  }
  // acc[f][r] = dW[j = jf*16 + (lane>>4)*4 + r][k = kf*16 + (lane&15)] of group g
#pragma unroll
  for (int f = 0; f < FPW; ++f) {
    const int fi = fc * 4 * FPW + f * 4 + wid;
    if (fi >= p.nfrag) break;
    const int jf = fi / p.nkf, kf = fi - jf * p.nkf;
    const int k = kf * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jf * 16 + (lane >> 4) * 4 + r;
      if (j < p.Og && k < p.Cg) {
        const int64_t o = (int64_t)(g * p.Og + j) * p.Cg + k;
        if (p.slab) p.slab[(int64_t)blockIdx.x * p.G * p.Og * p.Cg + o] = acc[f][r];
        else atomicAdd(p.dw + o, acc[f][r]);
      }
    }
  }
}
}  // namespace

// fwd / dgrad; returns -1 for an unsupported shape (the caller falls back)
int dv_gconv(const void* x, int ldx, int Cin, const int16_t* tin, const void* w, int Orows, void* y, int ldy, int Cout,
             const int16_t* tout, int M, int G, int Cg, int Og, int Kp, float* stats, hipStream_t st) {
  if (Cin != G * Cg || Cout != G * Og || Kp % 32 || Kp < Cg || ldx % 8 || ldy % 4 || (uintptr_t)x % 16 ||
      (uintptr_t)w % 16 || Orows < Og || Cout > 32767 || Cin > 32767)
    return -1;
  const bool detm = dv_deterministic() && stats;
  int BM = 64;  // two blocks per CU where the tiles allow
  while (BM > 16 && gc_lds_bytes(BM, G, Kp, Cout, stats, detm) > 80 * 1024) BM /= 2;
  const size_t lds = gc_lds_bytes(BM, G, Kp, Cout, stats, detm);
  if (lds > 160 * 1024) return -1;
  const unsigned grid = (unsigned)((M + BM - 1) / BM);
  const DetStats det(detm ? grid : 0, Cout, st);
  GcParams p{(const u16*)x, ldx, Cin, tin, (const u16*)w, Orows, (u16*)y, ldy, Cout, tout, M, G, Cg, Og, Kp, stats,
             make_fastdiv((uint32_t)(G * Kp / 8)), make_fastdiv((uint32_t)(Kp / 8)), det.slab};
  const int mode = tin ? GW_GATHER : (Cg % 8 == 0) ? GW_V16 : (Cg % 2 == 0) ? GW_PAIR : GW_GATHER;
  static bool attr[9] = {};
#define GC_LAUNCH(B, MD, I)                                                                                         \
  do {                                                                                                              \
    if (!attr[I]) {                                                                                                 \
      hipFuncSetAttribute((const void*)gconv_kernel<B, MD>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      attr[I] = true;                                                                                               \
    }                                                                                                               \
    gconv_kernel<B, MD><<<grid, NT, lds, st>>>(p);                                                                  \
  } while (0)
#define GC_BM(MD, I0)                  \
  if (BM == 64) GC_LAUNCH(64, MD, I0);  \
  else if (BM == 32) GC_LAUNCH(32, MD, I0 + 1); \
  else GC_LAUNCH(16, MD, I0 + 2);
  if (mode == GW_V16) { GC_BM(GW_V16, 0) }
  else if (mode == GW_PAIR) { GC_BM(GW_PAIR, 3) }
  else { GC_BM(GW_GATHER, 6) }
#undef GC_BM
#undef GC_LAUNCH
  det.fold(stats);
  return 0;
}

int dv_gconv_wgrad(const void* x, int ldx, const int16_t* tin, const void* dy, int ldy, const int16_t* tout, float* dw,
                   int M, int G, int Cg, int Og, hipStream_t st) {
  if ((uintptr_t)x % 16 || (uintptr_t)dy % 16 || ldx % 8 || ldy % 8) return -1;
  GwParams p{};
  p.x = (const u16*)x; p.ldx = ldx; p.tin = tin; p.dy = (const u16*)dy; p.ldy = ldy; p.tout = tout; p.dw = dw;
  p.M = M; p.G = G; p.Cg = Cg; p.Og = Og;
  // image widths: 64 columns, or a multiple of 128 (the XOR key stays inside 16-chunk blocks)
  auto width = [](int c) { return c <= 64 ? 64 : (c + 127) / 128 * 128; };
  p.CJ = width(Og); p.CK = width(Cg);
  p.nkf = (Cg + 15) / 16;
  p.nfrag = ((Og + 15) / 16) * p.nkf;
  p.fchunks = (p.nfrag + 4 * FPW - 1) / (4 * FPW);
  auto mode_of = [](const int16_t* tab, int nch, int G_) {
    if (tab) return (int)GW_GATHER;
    if ((nch & 7) == 0) return (int)GW_V16;  // base = g * nch stays 8-aligned
    if ((nch & 1) == 0) return (int)GW_PAIR;
    (void)G_;
    return (int)GW_GATHER;
  };
  const int my = mode_of(tout, Og, G), mx = mode_of(tin, Cg, G);
  const int maxp = 8;
  p.WT = 64;
  while (p.WT > 32 && p.WT * (p.CJ + p.CK) / 8 > maxp * NT) p.WT /= 2;
  if (p.WT * (p.CJ + p.CK) / 8 > maxp * NT) return -1;
  const size_t lds = (size_t)p.WT * (p.CJ + p.CK) * 2 + (size_t)(Og + Cg) * 2;
  // split the pixels so that ~1024 blocks run (each adds its tile into dW once: the atomic
  // traffic is blocks x outputs per block, 16 fragments = 16 KB)
  const int ntiles = (M + p.WT - 1) / p.WT;
  const int cols = G * p.fchunks;
  const int rchunks = std::max(1, std::min(ntiles, 1024 / cols));
  p.tiles_per_block = (ntiles + rchunks - 1) / rchunks;
  const int gx = (ntiles + p.tiles_per_block - 1) / p.tiles_per_block;
  const dim3 grid((unsigned)gx, (unsigned)cols);
  const int64_t nout = (int64_t)G * Og * Cg;
  p.slab = dv_deterministic() ? dv_slab_workspace((size_t)gx * nout, st) : nullptr;
  if (dv_deterministic() && !p.slab) return -1;
#define GW_CASE(A, B, P)                                                                                          \
  if (my == A && mx == B) {                                                                                       \
    gconv_wgrad_kernel<A, B, P><<<grid, NT, lds, st>>>(p);                                                        \
    if (p.slab) dv_slab_reduce(p.slab, dw, nout, gx, 1, st);                                                      \
    return 0;                                                                                                     \
  }
  GW_CASE(GW_V16, GW_V16, 8) GW_CASE(GW_V16, GW_PAIR, 8) GW_CASE(GW_PAIR, GW_V16, 8) GW_CASE(GW_PAIR, GW_PAIR, 8)
  GW_CASE(GW_GATHER, GW_V16, 8) GW_CASE(GW_GATHER, GW_PAIR, 8) GW_CASE(GW_V16, GW_GATHER, 8)
  GW_CASE(GW_PAIR, GW_GATHER, 8) GW_CASE(GW_GATHER, GW_GATHER, 8)
#undef GW_CASE
  return -1;
}
