#pragma once
// Shared core of the implicit-GEMM convolution (csrc/conv_fwd.hip): the parameter block, the
// main kernel template and its launchers.
// Implicit-GEMM convolution FORWARD on gfx950 MFMA (bf16 in, fp32 accumulate).
// Also serves conv dgrad, ConvTranspose forward and Linear forward/dgrad (SURVEY §2.7 K1-K4,
// K9, K13).
//
//   C[m = out pixel][n = out channel] = sum_k im2col(X)[m][k] * W[n][k],  k = (r, s, c)
//
// Structure (see /opt/skills/guides/cdna_hip_programming.md §5):
//   * block tile BM x BN x 64, 256 threads = 4 waves, each wave a 64x64 sub-tile of
//     4x4 v_mfma_f32_16x16x32_bf16. Tile variants: 128x128 (2x2 waves) and 256x64 (4x1 waves,
//     for 64-channel layers that would waste half of a 128-wide tile).
//   * operands staged global->LDS by LDS-DMA (global_load_lds_dwordx4); out-of-range /
//     padding lanes read a zero page, so the im2col halo costs no branches.
//   * K-contiguous LDS images, 128-B rows, XOR-swizzled on the SOURCE address (chunk ^
//     (row>>1)&7) and read back with ds_read_b128 conflict-free.
//   * 2-stage double buffer, one barrier per K-tile; a single stage (and so twice the
//     blocks per CU) when K fits one tile — the HBM-bound 1x1 layers.
//   * loader for C % 64 == 0 ("FASTC"): every K-tile is one filter tap (r, s) and a 64-channel
//     slice, so each lane keeps a per-row base pointer and a tap-validity bitmask; per K-tile
//     the address is base + a wave-uniform scalar offset (a few VALU per DMA instruction).
//   * epilogue: +bias, ReLU/LeakyReLU, per-channel BatchNorm partial statistics (DPP row
//     reductions + sharded atomics), then the tile is staged through LDS and written with
//     16-byte stores covering whole 128-B lines of the NHWC output (any channel slice).
//   * XCD-aware logical tile order: N-tiles of one M-panel run on one XCD (shared L2).
#include "common.h"
#include "kernels.h"


namespace dvconv {

struct FwdParams {
  const u16* x;
  const u16* w;
  u16* y;
  const float* bias;
  float* stats;
  const u16* res;  // optional: y = conv + res (same layout as y; may alias y -> in-place accumulate)
  int M, N, K, G;
  int Hin, Win, Cg, ldx;
  int P, Q;
  int R, S, sh, sw, ph, pw, dh, dw;
  int OH, OW, osh, osw, oph, opw, ldy;
  int act; float slope;
  int identity_map;
  FastDiv div_pq, div_q;
  // fused BatchNorm-backward statistics of y (see kernels.h ConvFwdArgs)
  const u16* bnx;
  const uint8_t* bnbits;
  const float* bnprm;
  float* bnacc;
  int bnmode, bnact; float bnslope;
  const uint8_t* resbits;  // RES only: res is masked by act'() bits before the add
  int resact; float resslope;
  int reflect;             // generic loader: reflected instead of zero-filled out-of-image taps
  int ksplit, kt_per;      // split-K: K-tiles [split*kt_per, +kt_per) per block (kernels.h)
  float* ypart;            // split-K fp32 slabs [ksplit][M][N] (single group)
  int zfill;               // strided scatter output: also zero the untouched sibling pixels (kernels.h)
  const u16* bnx2;         // BNR: second BatchNorm fed by the same dz (kernels.h ConvFwdArgs), or nullptr
  const float* bnprm2;
  float* bnacc2;
  int wld, wkr, wks;  // weight row / tap strides (kernels.h ConvFwdArgs w_ld, w_kr, w_ks)
  int ntl;            // epilogue reads of once-used tensors (residual, BN input) with the non-temporal policy
  // deterministic mode (kernels.h DetStats): per-row-tile slabs of stats / bnacc / bnacc2, or nullptr
  float* sdet;
  float* bdet;
  float* bdet2;
};

}  // namespace dvconv

extern int dv_g_last_ksplit;  // splits launched by the last split-K launch (finalize pass)
extern int dv_g_fwd_variant;  // benchmarking override of the tile / pipeline choice (0 = heuristic)

namespace {

using dvconv::FwdParams;

constexpr int EPI_PITCH = 72;                      // bf16 elements per staged row (64 + 8 pad)
constexpr int EPI_WAVE_BYTES = 64 * EPI_PITCH * 2;  // 9216
// every wave owns a WMT x 64 output sub-tile (WMT = 64 or 128 output pixels x 64 channels):
// a BM x BN tile runs on (BM/WMT)*(BN/64) waves. A 128-row wave tile reads 12 LDS fragments per
// 32 MFMAs instead of 8 per 16 and issues half the DMA instructions per MFMA.
template <int BM_, int BN_, int WMT = 64>
constexpr int n_waves() { return (BM_ / WMT) * (BN_ / 64); }
template <int BM_, int BN_, int WMT = 64>
constexpr int epi_bytes() { return n_waves<BM_, BN_, WMT>() * EPI_WAVE_BYTES; }
// statistics scratch behind the staged tile: [WM][BN][2] (fwd BN stats) or [waves][64][3] (BNR:
// sum dz, sum dz*xhat and the dual BN's sum dz*xhat2)
template <int BM_, int BN_, int WMT = 64>
constexpr int stat_bytes() { return n_waves<BM_, BN_, WMT>() * 64 * 3 * 4; }

enum { KM_FAST = 0, KM_GENERIC = 1, KM_TGATHER = 2 };
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_LEAKY = 2 };


// ReflectionPad2d index map (pad < n): -1 -> 1, n -> n - 2
DV_DEVICE int reflect_idx(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

// act'(z)*g for one element of a masked residual gradient (bit set: z > 0)
DV_DEVICE float masked_res(float g, uint32_t mb, int e, int act, float slope) {
  return ((mb >> e) & 1u) ? g : (act == 2 ? g * slope : 0.f);
}

// 16-B load of a tensor the epilogue reads once; `nt`: non-temporal policy (tensors far beyond the
// MALL, csrc/bn.hip NT_LOAD_MIN_ELEMS)
DV_DEVICE uint4 ld16_once(const u16* ptr, int nt) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  if (nt) {
    const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ptr));
    return uint4{r.x, r.y, r.z, r.w};
  }
  return *reinterpret_cast<const uint4*>(ptr);
}
DV_DEVICE void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(GLB_PTR(src), LDS_PTR(lds_wave_base), 16, 0, 0);
}
// K-contiguous LDS image, rows of BK bf16 (128 B for BK=64, 64 B for BK=32), XOR-swizzled on
// the 16-B chunk index; both swizzles are conflict-free for the ds_read_b128 lane groups.
template <int BK_>
DV_DEVICE int kc_swz(int row) {
  if constexpr (BK_ == 64) return (row >> 1) & 7;
  else return ((row >> 2) & 1) << 1;
}
template <int BK_>
DV_DEVICE bf16x8 read_kc(const char* img, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(img + row * (BK_ * 2) + ((chunk ^ kc_swz<BK_>(row)) << 4));
}

template <int BM_, int BN_, int BK_>
constexpr int stage_bytes() { return (BM_ + BN_) * BK_ * 2; }

// BatchNorm-backward reduction terms of 8 stored gradient values `o` (bf16, exactly what the
// unfused bn_bwd_reduce pass would read back) at element offset `off` of the BN input / mask:
// dz = act'(z) * dout, sum dz and sum dz * (x - mean) (csrc/bn.hip bn_bwd_reduce_kernel; the
// invstd factor is applied once per channel after the loop). Element pairs run as packed fp32
// (v_pk_add / v_pk_fma: half the VALU issue of the scalar form in an epilogue-bound kernel).
typedef float f32x2 __attribute__((ext_vector_type(2)));
DV_DEVICE f32x2 bf2x(uint32_t w) { return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)}; }
// DUAL: a second BatchNorm on the same dz (mode 3 only) adds its own sum dz*(x2 - mean2) into bq2
// (its sum dz is the first one's).
template <bool DUAL = false>
DV_DEVICE void bn_bwd_accum(const FwdParams& p, const uint4& o, const uint4& xr, uint32_t mb, f32x2* bs, f32x2* bq,
                            const f32x2* bmu, const f32x2* bms, const f32x2* bmh, const uint4* xr2 = nullptr,
                            f32x2* bq2 = nullptr, const f32x2* bmu2 = nullptr) {
  const uint32_t dw[4] = {o.x, o.y, o.z, o.w}, xw[4] = {xr.x, xr.y, xr.z, xr.w};
  uint32_t xw2[4] = {0u, 0u, 0u, 0u};
  if constexpr (DUAL) { xw2[0] = xr2->x; xw2[1] = xr2->y; xw2[2] = xr2->z; xw2[3] = xr2->w; }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const f32x2 d = bf2x(dw[e]), x = bf2x(xw[e]);
    f32x2 dz = d;
    if (p.bnmode == 3) {
      const f32x2 neg = p.bnact == 2 ? d * p.bnslope : f32x2{0.f, 0.f};
      dz.x = ((mb >> (2 * e)) & 1u) ? d.x : neg.x;
      dz.y = ((mb >> (2 * e + 1)) & 1u) ? d.y : neg.y;
    } else if (p.bnmode == 2) {
      const f32x2 z = x * bms[e] + bmh[e];
      const f32x2 neg = p.bnact == 2 ? d * p.bnslope : f32x2{0.f, 0.f};
      dz.x = z.x > 0.f ? d.x : neg.x;
      dz.y = z.y > 0.f ? d.y : neg.y;
    }
    bs[e] += dz;
    bq[e] = __builtin_elementwise_fma(dz, x - bmu[e], bq[e]);
    if constexpr (DUAL) bq2[e] = __builtin_elementwise_fma(dz, bf2x(xw2[e]) - bmu2[e], bq2[e]);
  }
}

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left at their maxima (gfx9 encoding: vmcnt bits
// [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8]).
template <int N>
DV_DEVICE void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

// EPI (compile-time epilogue): EPI_PLAIN = store only (dgrad, ConvTranspose), EPI_STATS = + BN
// partial statistics (the convs feeding a BatchNorm), EPI_FULL = runtime bias / activation /
// statistics. The plain forms drop ~8 VALU per output element (profiled: on the short-K 1x1
// layers the epilogue VALU outweighs the MFMA work).
enum { EPI_PLAIN = 0, EPI_STATS = 1, EPI_FULL = 2 };

// 256 threads (4 waves: one per SIMD, two blocks per CU) or 512 threads (8 waves: two per SIMD
// from one block, whose deep LDS ring then holds one CU); __launch_bounds__' second argument is
// waves per SIMD, so both forms get up to 256 VGPRs.
template <int BM_, int BN_, int BK_, int KMODE, bool RES, int STAGES, int BNR = 0, int EPI = EPI_FULL,
          int WMT = 64>
__global__ __launch_bounds__((64 * n_waves<BM_, BN_, WMT>()), 2) void conv_fwd_kernel(FwdParams p) {
  constexpr int WN = BN_ / 64, WM = BM_ / WMT;
  constexpr int NW = WN * WM;
  constexpr int FM = WMT / 16;         // M fragments per wave (4 or 8)
  constexpr int HM = WMT / 64;         // 64-row epilogue passes per wave
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(WMT == 64 || WMT == 128, "wave tile rows");
  constexpr int EPI_BYTES = epi_bytes<BM_, BN_, WMT>();
  constexpr int CH = BK_ / 8;          // 16-B chunks per LDS row
  constexpr int RPI = 64 / CH;         // rows written by one 1-KB DMA wave-instruction
  constexpr int MI = BM_ / RPI / NW;   // M-operand DMA instructions per wave per K-tile
  constexpr int NI = BN_ / RPI / NW;   // N-operand DMA instructions per wave per K-tile
  static_assert(MI * RPI * NW == BM_ && NI * RPI * NW == BN_, "loader rows must split evenly over the waves");
  constexpr int KK = BK_ / 32;         // 32-deep MFMA steps per K-tile
  constexpr int STAGE = stage_bytes<BM_, BN_, BK_>();
  constexpr int IPT = MI + NI;         // DMA instructions per wave per K-tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wave_m = wid / WN, wave_n = wid % WN;

  const int tiles_m = (p.M + BM_ - 1) / BM_, tiles_n = (p.N + BN_ - 1) / BN_;
  int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = logical % tiles_n; logical /= tiles_n;
  const int tm = logical % tiles_m; logical /= tiles_m;
  const int split = logical % p.ksplit;
  const int grp = logical / p.ksplit;
  const int m0 = tm * BM_, n0 = tn * BN_;
  const int nt_all = (p.K + BK_ - 1) / BK_;
  const int kt0 = split * p.kt_per;                     // first K-tile of this block
  const int nt = min(nt_all, kt0 + p.kt_per) - kt0;     // K-tiles of this block
  const char* zero = dv_zero_page;
  const int64_t goff_x = (int64_t)grp * p.Cg;

  // ---------------- per-lane load descriptors (fixed for the whole K loop) ----------------
  const u16* wrow[NI];
  bool wok[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int row = (wid * NI + j) * RPI + lane / CH;
    const int lc = (lane % CH) ^ kc_swz<BK_>(row);
    const int n = n0 + row;
    wok[j] = n < p.N;
    wrow[j] = p.w + ((int64_t)grp * p.N + (wok[j] ? n : 0)) * p.wld + lc * 8;
  }
  const u16* xrow[MI];      // KM_FAST: pointer at (pixel origin, channel lc*8)
  uint32_t tapmask[MI];     // KM_FAST: bit r (h valid) | bit 16+s (w valid); 0 for m >= M
  int64_t pixbase[MI];      // generic: img*Hin*Win
  int hb[MI], wb[MI];
  bool mok[MI];
#pragma unroll
  for (int j = 0; j < MI; ++j) {
    const int row = (wid * MI + j) * RPI + lane / CH;
    const int lc = (lane % CH) ^ kc_swz<BK_>(row);
    const int m = m0 + row;
    mok[j] = m < p.M;
    const int mm = mok[j] ? m : 0;
    const int img = (int)fdiv((uint32_t)mm, p.div_pq), rem = mm - img * (p.P * p.Q);
    const int pp = (int)fdiv((uint32_t)rem, p.div_q), qq = rem - pp * p.Q;
    pixbase[j] = (int64_t)img * p.Hin * p.Win;
    if (KMODE == KM_TGATHER) { hb[j] = pp + p.ph; wb[j] = qq + p.pw; }
    else { hb[j] = pp * p.sh - p.ph; wb[j] = qq * p.sw - p.pw; }
    if (KMODE == KM_FAST) {
      uint32_t mk = 0;
      for (int r = 0; r < p.R; ++r) { const int h = hb[j] + r * p.dh; mk |= (uint32_t)(h >= 0 && h < p.Hin) << r; }
      for (int s = 0; s < p.S; ++s) { const int w = wb[j] + s * p.dw; mk |= (uint32_t)(w >= 0 && w < p.Win) << (16 + s); }
      tapmask[j] = mok[j] ? mk : 0u;
      xrow[j] = p.x + (pixbase[j] + (int64_t)hb[j] * p.Win + wb[j]) * p.ldx + goff_x + lc * 8;
    }
  }

  // FASTC tap walker (wave-uniform), started at this block's first K-tile (every K-tile lies
  // inside one tap: Cg % 64 == 0)
  int t_r = 0, t_s = 0, t_c = 0;
  if (KMODE == KM_FAST && kt0 > 0) {
    const int k0 = kt0 * BK_, rs = k0 / p.Cg;
    t_c = k0 - rs * p.Cg; t_r = rs / p.S; t_s = rs - t_r * p.S;
  }
  // one 16-B piece per lane of wave-instruction `slot`, LDS-DMA straight into the image; the source
  // (operand or zero row) is chosen by integer select (v_cndmask), not a branch around the load
  auto sel = [](bool ok, const void* a, const void* z) {
    const uint64_t ia = reinterpret_cast<uint64_t>(a), iz = reinterpret_cast<uint64_t>(z);
    return reinterpret_cast<const void*>(ok ? ia : iz);
  };
  auto stage = [&](int kt, int buf) {
    char* img_n = smem + buf * STAGE;
    char* img_m = img_n + BN_ * BK_ * 2;
    const int k0 = kt * BK_;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = (wid * NI + j) * RPI + lane / CH;
      const int lc = (lane % CH) ^ kc_swz<BK_>(row);
      const bool ok = wok[j] && (KMODE == KM_FAST || k0 + lc * 8 < p.K);
      // fast loader: the weight offset of this K-tile's tap (equal to k0 for a whole filter)
      const int64_t wo = KMODE == KM_FAST ? (int64_t)t_r * p.wkr + t_s * p.wks + t_c : k0;
      const void* src = sel(ok, wrow[j] + wo, zero);
      glds16(src, img_n + (wid * NI + j) * 1024);
    }
    if (KMODE == KM_FAST) {
      const int64_t koff = ((int64_t)(t_r * p.dh) * p.Win + t_s * p.dw) * p.ldx + t_c;
      const int sh_r = t_r, sh_s = 16 + t_s;
#pragma unroll
      for (int j = 0; j < MI; ++j) {
        const bool ok = (tapmask[j] >> sh_r) & (tapmask[j] >> sh_s) & 1u;
        const void* src = sel(ok, xrow[j] + koff, zero);
        glds16(src, img_m + (wid * MI + j) * 1024);
      }
    } else {
#pragma unroll
      for (int j = 0; j < MI; ++j) {
        const int row = (wid * MI + j) * RPI + lane / CH;
        const int lc = (lane % CH) ^ kc_swz<BK_>(row);
        const int k = k0 + lc * 8;
        const int rs = k / p.Cg, c = k - rs * p.Cg;
        const int r = rs / p.S, s = rs - r * p.S;
        bool ok = mok[j] && k < p.K;
        int h, w;
        if (KMODE == KM_TGATHER) {
          const int hn = hb[j] - r * p.dh, wn = wb[j] - s * p.dw;
          ok = ok && hn >= 0 && wn >= 0 && (hn % p.sh) == 0 && (wn % p.sw) == 0;
          h = hn / p.sh; w = wn / p.sw;
        } else {
          h = hb[j] + r * p.dh; w = wb[j] + s * p.dw;
          if (p.reflect) { h = reflect_idx(h, p.Hin); w = reflect_idx(w, p.Win); }
        }
        ok = ok && h >= 0 && h < p.Hin && w >= 0 && w < p.Win;
        const void* src = zero;
        if (ok) src = p.x + (pixbase[j] + (int64_t)h * p.Win + w) * p.ldx + goff_x + c;
        glds16(src, img_m + (wid * MI + j) * 1024);
      }
    }
  };
  auto advance = [&]() {
    if (KMODE == KM_FAST) {
      t_c += BK_;
      if (t_c >= p.Cg) { t_c = 0; if (++t_s == p.S) { t_s = 0; ++t_r; } }
    }
  };

  f32x4 acc[4][FM];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < FM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf, int kt) {
    const char* img_n = smem + buf * STAGE;
    const char* img_m = img_n + BN_ * BK_ * 2;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8 fa[4], fb[FM];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fa[j] = read_kc<BK_>(img_n, wave_n * 64 + j * 16 + (lane & 15), kk * 4 + (lane >> 4));
#pragma unroll
      for (int i = 0; i < FM; ++i)
        fb[i] = read_kc<BK_>(img_m, wave_m * WMT + i * 16 + (lane & 15), kk * 4 + (lane >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[j], fb[i], acc[j][i], 0, 0, 0);
    }
  };
  if constexpr (STAGES == 2) {
    // double buffer, one barrier per K-tile: the DMA of tile t+1 overlaps the MFMAs of tile t
    stage(kt0, 0);
    advance();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      if (t + 1 < nt) { stage(kt0 + t + 1, cur ^ 1); advance(); }
      compute(cur, kt0 + t);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // STAGES-deep ring: STAGES-2 tiles stay in flight across each barrier. A counted vmcnt
    // retires only tile t's DMAs (IPT per wave per tile, issued in order) and the raw s_barrier
    // does not drain the younger ones (__syncthreads() would emit vmcnt(0)).
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nt) { stage(kt0 + s, s); advance(); }
    int cur = 0, nxt = STAGES - 1;
    for (int t = 0; t < nt; ++t) {
      const int ahead = min(nt - 1, t + STAGES - 2) - t;  // tiles issued after t
      if (ahead >= STAGES - 2) wait_vm<(STAGES - 2) * IPT>();
      else if (STAGES > 3 && ahead == 1) wait_vm<IPT>();
      else wait_vm<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + STAGES - 1 < nt) { stage(kt0 + t + STAGES - 1, nxt); advance(); }
      compute(cur, kt0 + t);
      cur = cur + 1 == STAGES ? 0 : cur + 1;
      nxt = nxt + 1 == STAGES ? 0 : nxt + 1;
    }
    __syncthreads();  // every DMA retired (vmcnt(0) on the last tile): smem is free for the epilogue
  }

  // ---------------- split-K epilogue: raw fp32 partial tile -> this split's slab ----------------
  if constexpr (EPI == EPI_FULL && !RES && !BNR) {
    if (p.ypart) {
      float* slab = p.ypart + (int64_t)split * p.M * p.N;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wave_n * 64 + j * 16 + (lane >> 4) * 4;  // N % 4 == 0: whole float4 or none
        if (n >= p.N) continue;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = m0 + wave_m * WMT + i * 16 + (lane & 15);
          if (m < p.M) *reinterpret_cast<f32x4*>(slab + (int64_t)m * p.N + n) = acc[j][i];
        }
      }
      return;
    }
  }
  // ---------------- epilogue ----------------
  // acc[j][i][r]: n_local = j*16 + (lane>>4)*4 + r, m_local = i*16 + (lane&15) within the wave
  // tile; a 128-row wave tile is written as two 64-row passes through the same staging rows.
  const int nw0 = n0 + wave_n * 64;  // first channel of this wave
  const int64_t goff_y = (int64_t)grp * p.N;
  const bool vec = ((p.N & 7) == 0) && ((p.ldy & 7) == 0) && ((goff_y & 7) == 0);
  constexpr bool PF = RES || BNR;
  float bsum[4][4], bsq[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { bsum[j][r] = 0.f; bsq[j][r] = 0.f; }
  // BNR: this lane's 8 channels are fixed over the store loop (rows it*8 + lane/8)
  // dual: a second BatchNorm on the same dz (kernels.h ConvFwdArgs bnx2): its sum dz*(x2 - mean2)
  f32x2 bs2[4], bq2[4], bmu2[4], bms2[4], bmh2[4], dq2[4], dmu2[4];
  constexpr bool dual = BNR == 2;  // compile-time: the single-BN forms keep their registers
  if constexpr (BNR) {
    const int nb = nw0 + (lane & 7) * 8;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bs2[e] = f32x2{0.f, 0.f}; bq2[e] = f32x2{0.f, 0.f}; dq2[e] = f32x2{0.f, 0.f};
      const bool ok0 = nb + 2 * e < p.N, ok1 = nb + 2 * e + 1 < p.N;
      dmu2[e] = f32x2{(dual && ok0) ? p.bnprm2[2 * p.N + nb + 2 * e] : 0.f,
                      (dual && ok1) ? p.bnprm2[2 * p.N + nb + 2 * e + 1] : 0.f};
      bms2[e] = f32x2{ok0 ? p.bnprm[nb + 2 * e] : 0.f, ok1 ? p.bnprm[nb + 2 * e + 1] : 0.f};
      bmh2[e] = f32x2{ok0 ? p.bnprm[p.N + nb + 2 * e] : 0.f, ok1 ? p.bnprm[p.N + nb + 2 * e + 1] : 0.f};
      bmu2[e] = f32x2{ok0 ? p.bnprm[2 * p.N + nb + 2 * e] : 0.f, ok1 ? p.bnprm[2 * p.N + nb + 2 * e + 1] : 0.f};
    }
  }
  // RES with statistics: the BatchNorm statistics are of the STORED output y = conv (+ bias) +
  // residual (a pre-activation block's output feeding the next block's BN; the split-K finalize
  // computes the same), accumulated per lane over its 8 fixed channels in the store loop (vector
  // stores only: the host rejects the combination otherwise)
  constexpr bool RST = RES && EPI != EPI_PLAIN;
  f32x2 rs1[RST ? 4 : 1], rs2[RST ? 4 : 1], rkq[RST ? 4 : 1];
  if constexpr (RST) {
    const int nb = nw0 + (lane & 7) * 8;
    const float* kp = p.stats ? stat_shift(p.stats, (int64_t)p.G * p.N) + grp * p.N : nullptr;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      rs1[e] = f32x2{0.f, 0.f}; rs2[e] = f32x2{0.f, 0.f};
      rkq[e] = f32x2{(kp && nb + 2 * e < p.N) ? kp[nb + 2 * e] : 0.f, (kp && nb + 2 * e + 1 < p.N) ? kp[nb + 2 * e + 1] : 0.f};
    }
  }
  u16* st = reinterpret_cast<u16*>(smem + wid * EPI_WAVE_BYTES);
#pragma unroll
  for (int h = 0; h < HM; ++h) {
    const int mw0 = m0 + wave_m * WMT + h * 64;  // first output row of this 64-row pass
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float bv[4], kq[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nw0 + j * 16 + (lane >> 4) * 4 + r;
        bv[r] = 0.f;
        kq[r] = 0.f;
        if constexpr (EPI == EPI_FULL) bv[r] = (p.bias && n < p.N) ? p.bias[grp * p.N + n] : 0.f;
        // shifted statistics: sums of (t - K), K = this BN's previous batch mean (stat_shift)
        if constexpr (EPI != EPI_PLAIN && !RES) kq[r] = (p.stats && n < p.N) ? stat_shift(p.stats, (int64_t)p.G * p.N)[grp * p.N + n] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ml = i * 16 + (lane & 15);
        const bool mv = mw0 + ml < p.M;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t = acc[j][h * 4 + i][r];
          if constexpr (EPI == EPI_FULL) {
            t += bv[r];
            if (p.act == ACT_RELU) t = fmaxf(t, 0.f);
            else if (p.act == ACT_LEAKY) t = t > 0.f ? t : t * p.slope;
          }
          v[r] = t;
          if constexpr (EPI != EPI_PLAIN && !RES) {
            if (mv) { const float d = t - kq[r]; bsum[j][r] += d; bsq[j][r] = fmaf(d, d, bsq[j][r]); }
          }
        }
        uint2 pk; pk.x = pack2bf(v[0], v[1]); pk.y = pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(st + ml * EPI_PITCH + j * 16 + (lane >> 4) * 4) = pk;
      }
    }
    // Prefetch what the store loop reads besides the staged tile (the residual gradient, the BN
    // input and mask) for all 8 row groups now: issued in the loop they would each wait behind the
    // previous iteration's stores (one vmcnt queue for loads and stores), 8 serial round trips.
    int64_t pf_off[PF ? 8 : 1];
    uint4 pf_res[RES ? 8 : 1], pf_x[BNR ? 8 : 1], pf_x2[dual ? 8 : 1];
    uint32_t pf_mb[BNR ? 8 : 1], pf_rmb[RES ? 8 : 1];
    if constexpr (PF) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int m = mw0 + it * 8 + (lane >> 3);
        const int n = nw0 + (lane & 7) * 8;
        int64_t off = -1;
        if (m < p.M && n < p.N) {
          int64_t opix;
          if (p.identity_map) opix = m;
          else {
            const int img = (int)fdiv((uint32_t)m, p.div_pq), rem = m - img * (p.P * p.Q);
            const int pp = (int)fdiv((uint32_t)rem, p.div_q), qq = rem - pp * p.Q;
            opix = ((int64_t)img * p.OH + pp * p.osh + p.oph) * p.OW + qq * p.osw + p.opw;
          }
          off = opix * p.ldy + goff_y + n;
        }
        pf_off[it] = off;
        const bool ld = off >= 0 && vec;
        if constexpr (RES) {
          pf_res[it] = ld ? ld16_once(p.res + off, p.ntl) : uint4{0u, 0u, 0u, 0u};
          pf_rmb[it] = (off >= 0 && p.resbits) ? (uint32_t)p.resbits[off >> 3] : 0xffu;
        }
        if constexpr (BNR) {
          pf_x[it] = ld ? ld16_once(p.bnx + off, p.ntl) : uint4{0u, 0u, 0u, 0u};
          pf_mb[it] = (ld && p.bnmode == 3) ? (uint32_t)p.bnbits[off >> 3] : 0u;
          if constexpr (dual) pf_x2[it] = ld ? ld16_once(p.bnx2 + off, p.ntl) : uint4{0u, 0u, 0u, 0u};
        }
      }
    }
    // staged rows -> global: each wave writes its 64 rows x 64 channels as 16-B pieces (the
    // wave reads back only its own staging rows: LDS order within a wave, no barrier)
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int rl = it * 8 + (lane >> 3), ch = (lane & 7) * 8;
      const int m = mw0 + rl;
      const int n = nw0 + ch;
      if (m >= p.M || n >= p.N) continue;
      int64_t yoff;
      if constexpr (PF) yoff = pf_off[it];
      else {
        int64_t opix;
        if (p.identity_map) opix = m;
        else {
          const int img = (int)fdiv((uint32_t)m, p.div_pq), rem = m - img * (p.P * p.Q);
          const int pp = (int)fdiv((uint32_t)rem, p.div_q), qq = rem - pp * p.Q;
          const int oh = pp * p.osh + p.oph, ow = qq * p.osw + p.opw;
          opix = ((int64_t)img * p.OH + oh) * p.OW + ow;
          if constexpr (!RES) {
            if (p.zfill && vec) {  // the (osh x osw) - 1 pixels no tap of this output row reaches
              for (int a = 0; a < p.osh; ++a)
                for (int b = 0; b < p.osw; ++b)
                  if ((a | b) && oh + a < p.OH && ow + b < p.OW)
                    *reinterpret_cast<uint4*>(p.y + (opix + (int64_t)a * p.OW + b) * p.ldy + goff_y + n) =
                        uint4{0u, 0u, 0u, 0u};
            }
          }
        }
        yoff = opix * p.ldy + goff_y + n;
      }
      u16* dst = p.y + yoff;
      const u16* src = st + rl * EPI_PITCH + ch;
      if constexpr (RES) {  // residual-gradient join: dX += stashed gradient (fused instead of an add pass)
        const u16* rp = p.res + yoff;
        if (vec) {
          const uint4 a = *reinterpret_cast<const uint4*>(src), b = pf_res[it];
          const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, bw[4] = {b.x, b.y, b.z, b.w};
          uint32_t ov[4];
          const uint32_t rmb = pf_rmb[it];
#pragma unroll
          for (int e = 0; e < 4; ++e) {  // packed fp32 pairs: act'(res) * res + conv result
            const f32x2 r = bf2x(bw[e]);
            const f32x2 neg = p.resact == 2 ? r * p.resslope : f32x2{0.f, 0.f};
            const f32x2 m = f32x2{((rmb >> (2 * e)) & 1u) ? r.x : neg.x, ((rmb >> (2 * e + 1)) & 1u) ? r.y : neg.y};
            const f32x2 t = bf2x(aw[e]) + m;
            ov[e] = pack2bf(t.x, t.y);
          }
          const uint4 o = uint4{ov[0], ov[1], ov[2], ov[3]};
          *reinterpret_cast<uint4*>(dst) = o;
          if constexpr (RST) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {  // of the stored bf16 values, as a separate stats pass would read them
              const f32x2 d = bf2x(ov[e]) - rkq[e];
              rs1[e] += d;
              rs2[e] = __builtin_elementwise_fma(d, d, rs2[e]);
            }
          }
          if constexpr (BNR) {
            if constexpr (dual) bn_bwd_accum<true>(p, o, pf_x[it], pf_mb[it], bs2, bq2, bmu2, bms2, bmh2, &pf_x2[it], dq2, dmu2);
            else bn_bwd_accum(p, o, pf_x[it], pf_mb[it], bs2, bq2, bmu2, bms2, bmh2);
          }
        } else {
          const uint32_t rmb = pf_rmb[it];
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (n + e < p.N) dst[e] = f2bf(bf2f(src[e]) + masked_res(bf2f(rp[e]), rmb, e, p.resact, p.resslope));
        }
      } else if (vec) {
        const uint4 o = *reinterpret_cast<const uint4*>(src);
        *reinterpret_cast<uint4*>(dst) = o;
        if constexpr (BNR) {
          if constexpr (dual) bn_bwd_accum<true>(p, o, pf_x[it], pf_mb[it], bs2, bq2, bmu2, bms2, bmh2, &pf_x2[it], dq2, dmu2);
          else bn_bwd_accum(p, o, pf_x[it], pf_mb[it], bs2, bq2, bmu2, bms2, bmh2);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) if (n + e < p.N) dst[e] = src[e];
      }
    }
  }
  if constexpr (RST) {
    if (p.stats) {
      // lanes sharing (lane & 7) hold the same 8 channels: butterfly over lane bits 3-5, then the
      // WM waves of one channel column meet in LDS; one coalesced atomic row per block
      float s1[8], s2[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) { s1[2 * e] = rs1[e].x; s1[2 * e + 1] = rs1[e].y; s2[2 * e] = rs2[e].x; s2[2 * e + 1] = rs2[e].y; }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int off = 8; off < 64; off <<= 1) {
          s1[e] += __shfl_xor(s1[e], off, 64);
          s2[e] += __shfl_xor(s2[e], off, 64);
        }
      }
      float* sh = reinterpret_cast<float*>(smem + EPI_BYTES);  // [waves][64 channels][2]
      if (lane < 8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          sh[(wid * 64 + lane * 8 + e) * 2 + 0] = s1[e];
          sh[(wid * 64 + lane * 8 + e) * 2 + 1] = s2[e];
        }
      }
      __syncthreads();
      if (threadIdx.x < BN_) {
        const int nl = threadIdx.x, n = n0 + nl;
        if (n < p.N) {
          float t1 = 0.f, t2 = 0.f;
#pragma unroll
          for (int wm = 0; wm < WM; ++wm) {
            const int w = wm * WN + nl / 64;
            t1 += sh[(w * 64 + (nl & 63)) * 2];
            t2 += sh[(w * 64 + (nl & 63)) * 2 + 1];
          }
          const int64_t ncols = (int64_t)p.G * p.N;
          float* a = stat_row(p.stats, p.sdet, tm, ncols);
          atomicAdd(a + grp * p.N + n, t1);
          atomicAdd(a + ncols + grp * p.N + n, t2);
        }
      }
    }
  }
  if (!RES && EPI != EPI_PLAIN && p.stats) {
    float* sh = reinterpret_cast<float*>(smem + EPI_BYTES);  // [WM][BN_][2]
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s1 = row16_sum(bsum[j][r]);
        const float s2 = row16_sum(bsq[j][r]);
        if ((lane & 15) == 0) {
          const int nl = wave_n * 64 + j * 16 + (lane >> 4) * 4 + r;
          sh[(wave_m * BN_ + nl) * 2 + 0] = s1;
          sh[(wave_m * BN_ + nl) * 2 + 1] = s2;
        }
      }
    __syncthreads();
    if (threadIdx.x < BN_) {
      const int n = n0 + threadIdx.x;
      if (n < p.N) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) { s1 += sh[(w * BN_ + threadIdx.x) * 2]; s2 += sh[(w * BN_ + threadIdx.x) * 2 + 1]; }
        const int64_t ncols = (int64_t)p.G * p.N;
        float* a = stat_row(p.stats, p.sdet, tm, ncols);
        atomicAdd(a + grp * p.N + n, s1);
        atomicAdd(a + ncols + grp * p.N + n, s2);
      }
    }
  }
  if constexpr (BNR) {
    // lanes sharing (lane & 7) hold partials of the same 8 channels: butterfly over lane bits 3-5,
    // then the WM waves of one channel column meet in LDS; one coalesced atomic row per block
    float bs[8], bq[8], bd[8];
    {
      const int nb = nw0 + (lane & 7) * 8;
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // sum dz*(x - mean) -> sum dz*xhat: one invstd per channel
        const float i0 = nb + 2 * e < p.N ? p.bnprm[3 * p.N + nb + 2 * e] : 0.f;
        const float i1 = nb + 2 * e + 1 < p.N ? p.bnprm[3 * p.N + nb + 2 * e + 1] : 0.f;
        const float j0 = (dual && nb + 2 * e < p.N) ? p.bnprm2[3 * p.N + nb + 2 * e] : 0.f;
        const float j1 = (dual && nb + 2 * e + 1 < p.N) ? p.bnprm2[3 * p.N + nb + 2 * e + 1] : 0.f;
        bs[2 * e] = bs2[e].x; bs[2 * e + 1] = bs2[e].y;
        bq[2 * e] = bq2[e].x * i0; bq[2 * e + 1] = bq2[e].y * i1;
        bd[2 * e] = dq2[e].x * j0; bd[2 * e + 1] = dq2[e].y * j1;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int off = 8; off < 64; off <<= 1) {
        bs[e] += __shfl_xor(bs[e], off, 64);
        bq[e] += __shfl_xor(bq[e], off, 64);
        if constexpr (dual) bd[e] += __shfl_xor(bd[e], off, 64);
      }
    }
    float* sh = reinterpret_cast<float*>(smem + EPI_BYTES);  // [waves][64 channels][3]
    if (lane < 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sh[(wid * 64 + lane * 8 + e) * 3 + 0] = bs[e];
        sh[(wid * 64 + lane * 8 + e) * 3 + 1] = bq[e];
        sh[(wid * 64 + lane * 8 + e) * 3 + 2] = bd[e];
      }
    }
    __syncthreads();
    if (threadIdx.x < BN_) {
      const int nl = threadIdx.x, n = n0 + nl;
      if (n < p.N) {
        float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
        for (int wm = 0; wm < WM; ++wm) {
          const int w = wm * WN + nl / 64;
          s1 += sh[(w * 64 + (nl & 63)) * 3];
          s2 += sh[(w * 64 + (nl & 63)) * 3 + 1];
          s3 += sh[(w * 64 + (nl & 63)) * 3 + 2];
        }
        float* a = stat_row(p.bnacc, p.bdet, tm, p.N);
        atomicAdd(a + n, s1);
        atomicAdd(a + p.N + n, s2);
        if constexpr (dual) {  // the same dz: the second BN's sum dz is s1
          float* a2 = stat_row(p.bnacc2, p.bdet2, tm, p.N);
          atomicAdd(a2 + n, s1);
          atomicAdd(a2 + p.N + n, s3);
        }
      }
    }
  }
}

// the epilogue staging tile and the statistics scratch reuse the (drained) operand stages
template <int BM_, int BN_, int BK_, int WMT = 64>
constexpr int lds_bytes(int stages) {
  constexpr int epi = epi_bytes<BM_, BN_, WMT>() + stat_bytes<BM_, BN_, WMT>();
  return stages * stage_bytes<BM_, BN_, BK_>() > epi ? stages * stage_bytes<BM_, BN_, BK_>() : epi;
}

constexpr size_t LDS_MAX = 160 * 1024;

template <int BM_, int BN_, int BK_, int KMODE, bool RES, int STAGES, int BNR = 0, int EPI = EPI_FULL,
          int WMT = 64>
void launch_fwd(const FwdParams& p, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_fwd_kernel<BM_, BN_, BK_, KMODE, RES, STAGES, BNR, EPI, WMT>,
                        hipFuncAttributeMaxDynamicSharedMemorySize,
                        lds_bytes<BM_, BN_, BK_, WMT>(STAGES));
    attr = true;
  }
  FwdParams q = p;
  const int nt_all = (p.K + BK_ - 1) / BK_;
  q.ksplit = p.ypart ? max(1, min(p.ksplit, nt_all)) : 1;
  q.kt_per = (nt_all + q.ksplit - 1) / q.ksplit;
  q.ksplit = (nt_all + q.kt_per - 1) / q.kt_per;  // no empty splits
  const int nt = q.kt_per;
  const size_t lds = lds_bytes<BM_, BN_, BK_, WMT>(nt < STAGES ? nt : STAGES);
  const int blocks = ((p.M + BM_ - 1) / BM_) * ((p.N + BN_ - 1) / BN_) * p.G * q.ksplit;
  conv_fwd_kernel<BM_, BN_, BK_, KMODE, RES, STAGES, BNR, EPI, WMT>
      <<<dim3(blocks), dim3(64 * n_waves<BM_, BN_, WMT>()), lds, st>>>(q);
  if (p.ypart) dv_g_last_ksplit = q.ksplit;
}

// Tile choice measured on the ResNet-50 layer set (tools/bench_conv.py, profiles/convbench_*):
//  * N <= 64: a 256x64 tile keeps every MFMA useful; short K (<= 256, HBM-bound 1x1 layers)
//    runs best with a 3-deep ring, long K with the plain double buffer;
//  * N > 64: 128x128. K <= 64 is one K-tile (single stage, most blocks per CU); up to K < 2048
//    BK=32 (32 KB of LDS: up to 4 blocks per CU) beats BK=64 by 5-25 %; long-K layers (3x3 x
//    256+ channels, 2048-deep 1x1) keep BK=64;
//  * N % 256 == 0, K >= 1024 and >= 192 tiles of 256x256: one 512-thread block per CU with
//    128x64 wave tiles (half the LDS fragment reads and DMA instructions per MFMA) is 8-12 %
//    faster (3x3x256 @14: 67 vs 76 us; 1x1 1024->256 @14: 38 vs 42 us); with fewer tiles
//    (the 7x7 stage: 98 tiles on 256 CUs) it loses to the 4-block-per-CU 128x128 tile.
//    (profiles/convbench_wave_tiles.txt)
template <int KMODE>
bool big_tile_ok(const FwdParams& p) {
  if (KMODE != KM_FAST || p.N % 256 != 0 || p.K < 1024) return false;
  const int64_t tiles = (int64_t)((p.M + 255) / 256) * (p.N / 256) * p.G;
  return tiles >= 192 || dv_g_fwd_variant == 100;  // 100: tests force it at small shapes
}

}  // namespace

