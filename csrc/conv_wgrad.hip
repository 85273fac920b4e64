// Implicit-GEMM convolution WEIGHT GRADIENT on gfx950 MFMA (also ConvTranspose
// and Linear wgrad).
//
//   dW[m = out channel][n = (r, s, c)] = sum_{pix} dY[pix][m] * im2col(X)[pix][n]
//
// The reduction runs over every output pixel of the batch (up to N*H*W = 802,816 for ResNet-50
// at batch 256), so the K dimension is split over blocks ("split-K") and each block adds its
// fp32 tile into dW with 256-B-row atomics staged through LDS (Guideline 12: the atomic traffic
// per FLOP is bounded by giving every split >= 2048 pixels).
//
// Both operands are MN-contiguous in NHWC (pixels are rows, channels contiguous), so they are
// staged by LDS-DMA as [64 pixels][cols] images and fed to MFMA through the hardware-transposed
// read ds_read_b64_tr_b16. The column XOR swizzle (on 8-byte units, keyed by the pixel row) makes
// those reads conflict-free for any row length that is a multiple of 256 B.
//
// Tile variants (4 waves of 64x64): 128x128, and 64x256 for 64-output-channel layers.
// A plain-row fast path serves 1x1 / stride-1 / pad-0 convs and Linear (no spatial decode).
#include <cstdlib>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BK = 64;  // pixels per K-tile of the split bookkeeping (kernels may use BKW = 32)
constexpr int NT = 256;
constexpr int F32_PAD = 4;

struct WgParams {
  const u16* x;   // im2col source (N operand)
  const u16* dy;  // M operand rows
  float* dw;      // [G][M][N]
  int M, N, K, G;
  int Hin, Win, Cg, ldx, ldm;
  int P, Q;
  int R, S, sh, sw, ph, pw, dh, dw_;
  int splits, ktiles_per_split, atomic_out, accumulate;
  int oirs_ig;  // > 0: write dW straight into the parameter layout [G*M][oirs_ig][R][S]
  int64_t slab;  // > 0: deterministic mode, split s writes its partial tile at dw + s * slab
  int reflect;   // reflected (ReflectionPad2d) instead of zero-filled out-of-image taps
  FastDiv div_pq, div_q, div_cg, div_s;
};

// LDS-DMA of one 1-KB wave piece, issued from inline asm (M0 written and restored in the same
// statement). The builtin form makes hipcc treat the transposed LDS reads (ds_read_b64_tr_b16,
// no alias scope) as possibly aliasing the in-flight DMA: it then put an s_waitcnt vmcnt(0) in
// front of every compute phase, draining the next tile's prefetch and serialising load and MFMA
// (measured: wgrad at 18-20 % MFMA busy). Asm DMAs are invisible to that bookkeeping; the
// explicit vmcnt waits before each barrier below are what order them.
DV_DEVICE void glds16(const void* src, uint32_t dst) {  // dst: wave-uniform LDS byte address
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}
// 16-byte-chunk XOR key of pixel row k (multiples of 2 chunks = 32-B blocks). Rows of >= 256 B
// take 8 keys; 128-B rows (64 columns) take 4 keys and rely on the row parity for the other
// half of the bank row. Both verified conflict-free for the tr-read lane groups.
template <int COLS>
DV_DEVICE int mn_swz(int k) {
  if constexpr (COLS >= 128) return ((k & 3) | ((k >> 1) & 4)) << 1;
  else return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
}

// 8-element MFMA fragment from an MN image [64 k][COLS] via two transposed reads.
template <int COLS>
DV_DEVICE bf16x8 read_mn(const char* img, int col0, int kbase, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k1 = kbase + 8 * g + q, k2 = k1 + 4;
  const int u = (col0 >> 2) + p;
  const char* a1 = img + k1 * (COLS * 2) + ((u ^ (mn_swz<COLS>(k1) << 1)) << 3);
  const char* a2 = img + k2 * (COLS * 2) + ((u ^ (mn_swz<COLS>(k2) << 1)) << 3);
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)LDS_PTR(a1));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)LDS_PTR(a2));
  i16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <int N>
DV_DEVICE void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

// Waves: (BM_ / WMT) x (BN_ / 64), each a WMT x 64 (M x N) sub-tile; WMT = 128 halves the LDS
// fragment reads and DMA instructions per MFMA (the 8-wave 256x256 tile, cf. conv_fwd.hip).
template <int BM_, int BN_, int WMT = 64>
constexpr int wg_waves() { return (BM_ / WMT) * (BN_ / 64); }
// epilogue rows staged per pass: the whole tile, or halves when BM_ x BN_ fp32 exceeds the LDS
template <int BM_, int BN_>
constexpr int wg_epi_rows() { return BM_ * (BN_ + F32_PAD) * 4 > 96 * 1024 ? BM_ / 2 : BM_; }

template <int BM_, int BN_, bool PLAIN, int BK = 64, int STAGES = 2, int WMT = 64>
__global__ __launch_bounds__((64 * wg_waves<BM_, BN_, WMT>()), 2) void conv_wgrad_kernel(WgParams p) {
  constexpr int WN = BN_ / 64, WM = BM_ / WMT;
  constexpr int NW = WN * WM;
  constexpr int FM = WMT / 16;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int MCH = BM_ / 8, NCH = BN_ / 8;        // 16-B chunks per image row
  constexpr int MRPI = 64 / MCH, NRPI = 64 / NCH;    // image rows per 1-KB DMA instruction
  constexpr int MI = (BK / MRPI) / NW, NI = (BK / NRPI) / NW;  // DMA instructions per wave per tile
  static_assert(MI * MRPI * NW == BK && NI * NRPI * NW == BK, "loader rows must split evenly over the waves");
  constexpr int MBYTES = BK * BM_ * 2, STAGE = BK * (BM_ + BN_) * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wave_m = wid / WN, wave_n = wid % WN;

  const int tiles_m = (p.M + BM_ - 1) / BM_, tiles_n = (p.N + BN_ - 1) / BN_;
  int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = logical % tiles_n; logical /= tiles_n;
  const int tm = logical % tiles_m; logical /= tiles_m;
  const int split = logical % p.splits, grp = logical / p.splits;
  const int m0 = tm * BM_, n0 = tn * BN_;
  const char* zero = dv_zero_page;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));  // LDS address of smem
  const int kt0 = split * p.ktiles_per_split;
  const int kt1 = min((p.K + BK - 1) / BK, kt0 + p.ktiles_per_split);
  const int nt = kt1 - kt0;
  const int64_t goff_x = (int64_t)grp * p.Cg;

  // ---- M operand (dY): per instruction a fixed 8-channel chunk; pixel row = k0 + row ----
  const u16* mrow[MI];
  bool mok[MI];
#pragma unroll
  for (int j = 0; j < MI; ++j) {
    const int row = (wid * MI + j) * MRPI + lane / MCH;
    const int lc = (lane % MCH) ^ mn_swz<BM_>(row);
    const int m = m0 + lc * 8;
    mok[j] = m < p.M;
    mrow[j] = p.dy + (int64_t)row * p.ldm + (int64_t)grp * p.M + (mok[j] ? m : 0);
  }
  // ---- N operand (im2col X): fixed column chunk (r, s, c) per lane, the pixel walked per tile ----
  // Multiply-free walk, 4 registers per DMA instruction: the tap pointer itself (x at the pixel's
  // window origin + the tap offset), hw = p*sh << 16 | q*sw and the tap's (r*dh - ph, s*dw - pw)
  // as two int16 (a column past N gets an always-out-of-image row offset). A tile step adds
  // wave-uniform deltas and carries q -> p -> image. (The per-tile decode with 64-bit multiplies
  // ran ~12 VALU per MFMA: the kernel was VALU-bound.)
  const u16* nptr[NI];   // PLAIN: pointer at (pixel row, channel); im2col: the tap pointer
  uint32_t w_hw[NI], n_tap[NI];
  bool nok[NI];          // PLAIN only
  const int64_t ldx = p.ldx, SWL = (int64_t)p.sw * ldx, SHL = (int64_t)p.sh * p.Win * ldx;
  const int64_t IMGL = (int64_t)p.Hin * p.Win * ldx;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int row = (wid * NI + j) * NRPI + lane / NCH;
    const int lc = (lane % NCH) ^ mn_swz<BN_>(row);
    const int n = n0 + lc * 8;
    nok[j] = n < p.N;
    const int nn = nok[j] ? n : 0;
    if (PLAIN) {
      nptr[j] = p.x + (int64_t)row * p.ldx + goff_x + nn;
    } else {
      const int rs = (int)fdiv((uint32_t)nn, p.div_cg);
      const int c = nn - rs * p.Cg;
      const int r = (int)fdiv((uint32_t)rs, p.div_s), sc = rs - r * p.S;
      const int hr = nok[j] ? r * p.dh - p.ph : -32768, wr = sc * p.dw_ - p.pw;
      n_tap[j] = ((uint32_t)hr << 16) | ((uint32_t)wr & 0xffffu);
      const int pix = kt0 * BK + row;
      const int img = (int)fdiv((uint32_t)pix, p.div_pq);
      const int rem = pix - img * p.P * p.Q;
      const int pp = (int)fdiv((uint32_t)rem, p.div_q);
      const int hb = pp * p.sh, wb = (rem - pp * p.Q) * p.sw;
      w_hw[j] = ((uint32_t)hb << 16) | (uint32_t)wb;
      nptr[j] = p.x + (int64_t)img * IMGL + ((int64_t)(hb + hr) * p.Win + (wb + wr)) * ldx + goff_x + c;
    }
  }
  // per-tile deltas (BK pixels) and the carries, all wave-uniform
  const int d_q = BK % p.Q, d_p = (BK / p.Q) % p.P, d_img = BK / (p.P * p.Q);
  const uint32_t dhw = ((uint32_t)(d_p * p.sh) << 16) + (uint32_t)(d_q * p.sw);
  const uint32_t Qsw = p.Q * p.sw, Psh = p.P * p.sh;
  const uint32_t cq_hw = ((uint32_t)p.sh << 16) - Qsw, cp_hw = Psh << 16;
  const int64_t dpo = (int64_t)d_q * SWL + (int64_t)d_p * SHL + (int64_t)d_img * IMGL;
  const int64_t cq = SHL - (int64_t)p.Q * SWL, cp = IMGL - (int64_t)p.P * SHL;

  auto stage = [&](int kt, int buf) {
    char* img_m = smem + buf * STAGE;
    char* img_n = img_m + MBYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int j = 0; j < MI; ++j) {
      const int row = (wid * MI + j) * MRPI + lane / MCH;
      const bool ok = mok[j] && (k0 + row < p.K);
      glds16(ok ? (const void*)(mrow[j] + (int64_t)k0 * p.ldm) : (const void*)zero,
             lds0 + buf * STAGE + (wid * MI + j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = (wid * NI + j) * NRPI + lane / NCH;
      const void* src = zero;
      if (PLAIN) {
        if (nok[j] && k0 + row < p.K) src = nptr[j] + (int64_t)k0 * p.ldx;
      } else {
        const int hr = (int)n_tap[j] >> 16, wr = (int)(n_tap[j] << 16) >> 16;
        int h = (int)(w_hw[j] >> 16) + hr, w = (int)(w_hw[j] & 0xffffu) + wr;
        const u16* a = nptr[j];
        if (p.reflect) {  // wave-uniform: ReflectionPad2d-fused layers re-aim out-of-image taps
          const int h2 = h < 0 ? -h : (h >= p.Hin ? 2 * p.Hin - 2 - h : h);
          const int w2 = w < 0 ? -w : (w >= p.Win ? 2 * p.Win - 2 - w : w);
          a += ((int64_t)(h2 - h) * p.Win + (w2 - w)) * ldx;
          h = hr == -32768 ? -1 : h2;
          w = w2;
        }
        const bool ok = k0 + row < p.K && (unsigned)h < (unsigned)p.Hin && (unsigned)w < (unsigned)p.Win;
        src = ok ? (const void*)a : src;
      }
      glds16(src, lds0 + buf * STAGE + MBYTES + (wid * NI + j) * 1024);
    }
  };
  auto advance = [&]() {
    if (!PLAIN) {
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        uint32_t hw = w_hw[j] + dhw;
        int64_t d = dpo;
        if ((hw & 0xffffu) >= Qsw) { hw += cq_hw; d += cq; }
        if ((hw >> 16) >= Psh) { hw -= cp_hw; d += cp; }
        w_hw[j] = hw;
        nptr[j] += d;
      }
    }
  };

  f32x4 acc[4][FM];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < FM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // every fragment of the tile is read before the first MFMA (sched_barrier): left to itself the
  // scheduler recycled one fragment register per 4 MFMAs and waited on each re-read, exposing
  // the LDS latency every 4 MFMAs; here it is exposed once per tile, the in-order LDS returns
  // release the MFMAs as they arrive
  // a wave whose 64 columns all lie past N (the last N tile of 3x3 x 64: N = 576 on 256-wide
  // tiles) skips its fragment reads and MFMAs: its SIMD time goes to the co-resident waves
  const bool live = n0 + wave_n * 64 < p.N;
  auto compute = [&](int buf) {
    if (!live) return;
    const char* img_m = smem + buf * STAGE;
    const char* img_n = img_m + MBYTES;
    constexpr int KK = BK / 32;
    bf16x8 fa[KK][4], fb[KK][FM];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[kk][j] = read_mn<BN_>(img_n, wave_n * 64 + j * 16, kk * 32, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) fb[kk][i] = read_mn<BM_>(img_m, wave_m * WMT + i * 16, kk * 32, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][j], fb[kk][i], acc[j][i], 0, 0, 0);
    // keep the MFMAs ahead of the caller's DMA wait + barrier (the scheduler may otherwise hoist
    // that wait above them and expose the next tile's load latency)
    __builtin_amdgcn_sched_barrier(0);
  };
  if constexpr (STAGES == 2) {
    if (nt > 0) {
      stage(kt0, 0);
      advance();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int t = 0; t < nt; ++t) {
        const int cur = t & 1;
        if (t + 1 < nt) { stage(kt0 + t + 1, cur ^ 1); advance(); }
        compute(cur);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else {
    // STAGES-deep ring (see conv_fwd.hip): counted vmcnt + raw barrier keep STAGES-2 tiles in flight
    constexpr int IPT = MI + NI;
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nt) { stage(kt0 + s, s); advance(); }
    int cur = 0, nxt = STAGES - 1;
    for (int t = 0; t < nt; ++t) {
      const int ahead = min(nt - 1, t + STAGES - 2) - t;
      if (ahead >= STAGES - 2) wait_vm<(STAGES - 2) * IPT>();
      else if (STAGES > 3 && ahead == 1) wait_vm<IPT>();
      else wait_vm<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + STAGES - 1 < nt) { stage(kt0 + t + STAGES - 1, nxt); advance(); }
      compute(cur);
      cur = cur + 1 == STAGES ? 0 : cur + 1;
      nxt = nxt + 1 == STAGES ? 0 : nxt + 1;
    }
    __syncthreads();
  }

  // ---- epilogue: fp32 tile through LDS, then 256-B row segments (atomic or plain) ----
  // acc[j][i][r]: n_local = wave_n*64 + j*16 + (lane>>4)*4 + r ; m_local = wave_m*WMT + i*16 + (lane&15)
  // A tile larger than the LDS budget goes out in ER-row passes.
  constexpr int LD = BN_ + F32_PAD;
  constexpr int ER = wg_epi_rows<BM_, BN_>();
  float* T = reinterpret_cast<float*>(smem);  // [ER][LD]
  // destination of column n: packed [G][M][N] row offset n, or the parameter's OIRS position
  // (n = (r, s, c) -> c*R*S + r*S + s; padded channels c >= oirs_ig are dropped)
  const int64_t row_stride = p.oirs_ig > 0 ? (int64_t)p.oirs_ig * p.R * p.S : p.N;
  float* dwp = p.dw + (int64_t)grp * p.M * row_stride + (int64_t)split * p.slab;
  int64_t coff[BN_ / 64];
#pragma unroll
  for (int h = 0; h < BN_ / 64; ++h) {
    const int n = n0 + h * 64 + lane;
    coff[h] = n < p.N ? n : -1;
    if (p.oirs_ig > 0 && n < p.N) {
      const int rs = (int)fdiv((uint32_t)n, p.div_cg), c = n - rs * p.Cg;
      coff[h] = c < p.oirs_ig ? (int64_t)c * p.R * p.S + rs : -1;
    }
  }
#pragma unroll
  for (int pass = 0; pass < BM_ / ER; ++pass) {
    if (pass) __syncthreads();  // the previous pass's rows have been read back
    if (wave_m * WMT / ER == pass) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int nl = wave_n * 64 + j * 16 + (lane >> 4) * 4;
          const int ml = wave_m * WMT + i * 16 + (lane & 15) - pass * ER;
          *reinterpret_cast<f32x4*>(&T[ml * LD + nl]) = acc[j][i];
        }
    }
    __syncthreads();
    for (int rr = wid; rr < ER; rr += NW) {
      const int m = m0 + pass * ER + rr;
      if (m >= p.M) break;
#pragma unroll
      for (int h = 0; h < BN_ / 64; ++h) {
        if (coff[h] >= 0) {
          const float v = T[rr * LD + h * 64 + lane];
          float* dst = dwp + (int64_t)m * row_stride + coff[h];
          if (p.atomic_out) atomicAdd(dst, v);
          else *dst = p.accumulate ? *dst + v : v;
        }
      }
    }
  }
}

template <int BM_, int BN_, int BKW, int STAGES>
constexpr int wg_lds_bytes() {
  constexpr int st = STAGES * BKW * (BM_ + BN_) * 2, ep = wg_epi_rows<BM_, BN_>() * (BN_ + F32_PAD) * 4;
  return st > ep ? st : ep;
}

// p.ktiles_per_split arrives in 64-pixel units; BKW = 32 kernels walk twice as many tiles
template <int BM_, int BN_, bool PLAIN, int BKW = 64, int STAGES = 2, int WMT = 64>
void launch_wg(WgParams p, int blocks, hipStream_t st) {
  static bool attr = false;
  constexpr int lds = wg_lds_bytes<BM_, BN_, BKW, STAGES>();
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_wgrad_kernel<BM_, BN_, PLAIN, BKW, STAGES, WMT>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  p.ktiles_per_split *= BK / BKW;
  conv_wgrad_kernel<BM_, BN_, PLAIN, BKW, STAGES, WMT>
      <<<dim3(blocks), dim3(64 * wg_waves<BM_, BN_, WMT>()), lds, st>>>(p);
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// 64x256 tiles only when the weight gradient is 64 rows by >= 256 columns (else 3/4 of the tile idles)
inline bool wg_narrow(int M, int N) { return M <= 64 && N >= 192; }

int g_wg_variant = 0;       // benchmarking override of tile / K-depth / pipeline (0 = heuristic)
int g_wg_split_pct = 100;
int g_wg_fill = 0;           // > 0: splits = floor(fill / tiles) (benchmarking)   // benchmarking scale of the split-K heuristic

template <bool PLAIN>
void dispatch_wg(const WgParams& p, int blocks_narrow, int blocks_wide, hipStream_t st) {
  const int blocks_big = cdiv(p.M, 256) * cdiv(p.N, 256) * p.G * p.splits;
  const int blocks_tall = cdiv(p.M, 256) * cdiv(p.N, 128) * p.G * p.splits;
  switch (g_wg_variant) {
    // 128-row wave tiles: 8 waves on 256x256 (one block per CU), 4 waves on 256x128
    case 8: return launch_wg<256, 256, PLAIN, 64, 2, 128>(p, blocks_big, st);
    case 9: return launch_wg<256, 128, PLAIN, 32, 2, 128>(p, blocks_tall, st);
    case 1: return launch_wg<128, 128, PLAIN, 64, 2>(p, blocks_wide, st);
    case 2: return launch_wg<64, 256, PLAIN, 64, 2>(p, blocks_narrow, st);
    case 3: return launch_wg<128, 128, PLAIN, 32, 2>(p, blocks_wide, st);
    case 4: return launch_wg<64, 256, PLAIN, 32, 2>(p, blocks_narrow, st);
    case 5: return launch_wg<128, 128, PLAIN, 32, 4>(p, blocks_wide, st);
    case 6: return launch_wg<64, 256, PLAIN, 32, 4>(p, blocks_narrow, st);
    case 7: return launch_wg<128, 128, PLAIN, 64, 3>(p, blocks_wide, st);
    default: break;
  }
  if (wg_narrow(p.M, p.N)) launch_wg<64, 256, PLAIN>(p, blocks_narrow, st);
  else launch_wg<128, 128, PLAIN>(p, blocks_wide, st);
}

// deterministic split-K: dst[i] (+)= sum over s of slab[s][i], in split order
__global__ void slab_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dst, int64_t n, int splits,
                                   int accumulate) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = accumulate ? dst[i] : 0.f;
    for (int s = 0; s < splits; ++s) v += ws[(int64_t)s * n + i];
    dst[i] = v;
  }
}

// the same sum over 16-B vectors, the splits spread over SG thread groups (each walks its
// splits s = g, g + SG, ... with four loads in flight, added in order) and the SG partials
// combined in fixed order: 4 x the memory parallelism of the per-element serial chain above,
// still reproducible bit for bit. n % 4 == 0, 16-B aligned ws / dst.
constexpr int SLAB_SG = 4;
__global__ __launch_bounds__(256) void slab_reduce4_kernel(const float4* __restrict__ ws, float4* __restrict__ dst,
                                                          int64_t n4, int splits, int accumulate) {
  __shared__ float4 part[SLAB_SG][64];
  const int tx = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + tx;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  auto add = [](float4& a, const float4& b) { a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w; };
  if (i < n4) {
    int sp = g;
    for (; sp + 3 * SLAB_SG < splits; sp += 4 * SLAB_SG) {
      const float4 v0 = ws[(int64_t)sp * n4 + i], v1 = ws[(int64_t)(sp + SLAB_SG) * n4 + i];
      const float4 v2 = ws[(int64_t)(sp + 2 * SLAB_SG) * n4 + i], v3 = ws[(int64_t)(sp + 3 * SLAB_SG) * n4 + i];
      add(acc, v0); add(acc, v1); add(acc, v2); add(acc, v3);
    }
    for (; sp < splits; sp += SLAB_SG) add(acc, ws[(int64_t)sp * n4 + i]);
  }
  part[g][tx] = acc;
  __syncthreads();
  if (g == 0 && i < n4) {
    float4 t = accumulate ? dst[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < SLAB_SG; ++q) add(t, part[q][tx]);
    dst[i] = t;
  }
}

int g_deterministic = [] {
  const char* v = std::getenv("DV_DETERMINISTIC");
  return (v && v[0] && v[0] != '0') ? 1 : 0;
}();
// per-stream slab workspaces: independent branches of a model may run their wgrads concurrently
// on different streams (models/hourglass.py), each needs its own
struct SlabWs {
  float* ptr = nullptr;
  size_t elems = 0;
};
std::unordered_map<hipStream_t, SlabWs> g_slab_ws;
}  // namespace

void dv_set_deterministic(int on) { g_deterministic = on; }
int dv_deterministic() { return g_deterministic; }

// Grow-only: a HIP graph captured earlier keeps the pointer it was recorded with, so a buffer
// is never freed once handed out -- a larger request retires it (kept alive for the process)
// and allocates 1.5x the request, so a model's warm-up converges in a few steps. During a
// stream capture the buffer cannot grow (hipMalloc / a retire would change what the graph
// holds mid-capture): nullptr, and the caller falls back to atomics (or fails in
// deterministic mode).
std::vector<float*> g_slab_retired;
float* dv_slab_workspace(size_t elems, hipStream_t st) {
  SlabWs& w = g_slab_ws[st];
  if (elems > w.elems) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return nullptr;
    const size_t want = elems + elems / 2;
    float* fresh = nullptr;
    if (hipMalloc(&fresh, want * sizeof(float)) != hipSuccess) return nullptr;
    if (w.ptr) g_slab_retired.push_back(w.ptr);
    w.ptr = fresh;
    w.elems = want;
  }
  return w.ptr;
}

// The ordered slab sum of a packed [rows][RS][Ipad] weight gradient written straight into the
// parameter's [rows][Ig][RS] (OIHW) layout: one thread per packed element sums its splits in a
// fixed order (four loads in flight) and stores to the element's OIHW position -- the separate
// wgrad_unprep pass (and its read + re-zero of a packed workspace) is gone. The scattered 4-B
// stores touch only the weight tensor once; the slab reads stay coalesced.
__global__ __launch_bounds__(256) void slab_reduce_oirs_kernel(const float* __restrict__ ws, float* __restrict__ dst,
                                                               int rs, int ipad, int ig, int splits, int64_t slab,
                                                               int accumulate) {
  const int n = rs * ipad;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < slab; t += (int64_t)gridDim.x * 256) {
    const int64_t o = t / n;
    const int e = (int)(t - o * n), r = e / ipad, i = e - r * ipad;
    if (i >= ig) continue;
    float v = 0.f;
    int sp = 0;
    for (; sp + 4 <= splits; sp += 4) {
      const float a0 = ws[(int64_t)sp * slab + t], a1 = ws[(int64_t)(sp + 1) * slab + t];
      const float a2 = ws[(int64_t)(sp + 2) * slab + t], a3 = ws[(int64_t)(sp + 3) * slab + t];
      v += a0; v += a1; v += a2; v += a3;
    }
    for (; sp < splits; ++sp) v += ws[(int64_t)sp * slab + t];
    float* d = dst + (o * ig + i) * rs + r;
    *d = accumulate ? *d + v : v;
  }
}

void dv_slab_reduce(const float* ws, float* dst, int64_t n, int splits, int accumulate, hipStream_t st) {
  if (n % 4 == 0 && ((uintptr_t)ws & 15) == 0 && ((uintptr_t)dst & 15) == 0) {
    const int64_t n4 = n / 4;
    slab_reduce4_kernel<<<(unsigned)((n4 + 63) / 64), 256, 0, st>>>((const float4*)ws, (float4*)dst, n4, splits,
                                                                     accumulate);
    return;
  }
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  slab_reduce_kernel<<<grid, 256, 0, st>>>(ws, dst, n, splits, accumulate);
}

// split-K partials through plain-stored fp32 slabs + one ordered reduce pass instead of float
// atomics into dw (atomic adds run at ~1.3 TB/s chip-wide and land at the end of the grid, where
// every block reaches its epilogue together). -1 (default): slabs up to SLAB_MAX_SPLITS splits --
// the slab bytes grow with the split count and the reduce pass reads them all: slabs won 5-10 %
// on the 6-56-split layers (1x1 at 14x14 / 7x7, 3x3 at 28x28 / 14x14) and lost 4-8 % on the
// 96-392-split 56x56 / 28x28 1x1 layers (profiles/wgbench_slab.txt); 1 / 0 (DV_WG_SLAB,
// conv_wgrad_slab): always slabs / always atomics
constexpr int SLAB_MAX_SPLITS = 64;
int g_wg_slab = [] {
  const char* v = std::getenv("DV_WG_SLAB");
  return (v && (v[0] == '0' || v[0] == '1')) ? v[0] - '0' : -1;
}();
void dv_conv_wgrad_slab(int on) { g_wg_slab = on; }

int dv_conv_wgrad_splits(const ConvWgradArgs& a) {
  const int M = a.Kout, N = a.R * a.S * a.Cg, K = a.Nb * a.P * a.Q;
  const bool narrow = g_wg_variant == 2 || g_wg_variant == 4 || g_wg_variant == 6 ||
                      (g_wg_variant == 0 && wg_narrow(M, N));
  // narrow 64x256 tiles (64-output-channel layers, few tiles): twice the blocks (s1 3x3x64 at
  // 56x56: 195 vs 214 us, profiles/archive/wgbench_asm_dma.txt; the 1x1 narrow layers are flat)
  int tm = narrow ? 64 : 128, tn = narrow ? 256 : 128, target = narrow ? 768 : 384;
  if (g_wg_variant == 8) { tm = 256; tn = 256; target = 256; }  // one 8-wave block per CU
  if (g_wg_variant == 9) { tm = 256; tn = 128; target = 384; }
  const int tiles = cdiv(M, tm) * cdiv(N, tn) * a.G;
  const int ktiles = cdiv(K, BK);
  // ~1.5 blocks per CU: measured 5-15 % faster than 3 per CU on the ResNet-50 3x3 / strided
  // layers (half the atomic epilogues), equal on the rest (profiles/archive/wgbench_variants.txt)
  int splits = cdiv(target * g_wg_split_pct / 100, tiles);
  // im2col layers (3x3, strided 1x1, stems): a grid of whole waves of the 512 block slots (2 per
  // CU for both tile shapes) instead of ~1.5 blocks per CU, which left a tail of half-empty CUs:
  // 3x3 layers 10-15 % faster (s1 3x3x64 198 -> 169 us, s3 3x3x256 111 -> 99 us); single-tile
  // layers (the 7x7 stem, 3.2M-pixel reduction) fill three waves (254 -> 242 us). The plain 1x1
  // layers keep the target form (a full wave there was 0-8 % slower). profiles/wgbench_fill.txt
  const bool plain = a.R == 1 && a.S == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 && a.pw == 0 && a.P == a.H &&
                     a.Q == a.W && !a.reflect;
  const bool tuned = g_wg_variant == 0 && g_wg_split_pct == 100;
  if (g_wg_fill > 0) splits = std::max(1, g_wg_fill / tiles);  // benchmarking: whole waves of `fill` block slots
  else if (tuned && !plain) splits = std::max(1, (tiles == 1 ? 3 * 512 : 512) / tiles);
  int cap = ktiles / 32;  // >= 2048 pixels per split (atomic budget)
  // few output tiles (small maps / few channels: the Hourglass 8x8-32x32 scales had 9-36 blocks
  // on 256 CUs): trade atomic traffic for parallelism down to 512 pixels per split, until the
  // grid covers the chip (profiles/hourglass_conv_bench.txt)
  if ((int64_t)tiles * cap < 256) cap = std::max(cap, std::min(ktiles / 8, cdiv(256, tiles)));
  splits = std::min(splits, std::max(1, cap));
  return std::max(1, std::min(splits, ktiles));
}

int dv_conv_stats_tiles(int Nb, int P, int Q) { return cdiv(Nb * P * Q, 128); }

void dv_conv_wgrad_tuning(int variant, int split_pct) {
  g_wg_variant = variant;
  g_wg_split_pct = split_pct > 0 ? split_pct : 100;
  g_wg_fill = split_pct < 0 ? -split_pct : 0;
}

int dv_conv_wgrad(const ConvWgradArgs& a, hipStream_t st) {
  WgParams p{};
  p.x = (const u16*)a.x; p.dy = (const u16*)a.dy; p.dw = a.dw;
  p.G = a.G; p.M = a.Kout; p.N = a.R * a.S * a.Cg; p.K = a.Nb * a.P * a.Q;
  p.Hin = a.H; p.Win = a.W; p.Cg = a.Cg; p.ldx = a.ldx; p.ldm = a.ldy;
  p.P = a.P; p.Q = a.Q; p.R = a.R; p.S = a.S;
  p.sh = a.sh; p.sw = a.sw; p.ph = a.ph; p.pw = a.pw; p.dh = a.dh; p.dw_ = a.dw_;
  // ldx == 4: tap-packed stem image (see conv_fwd.hip): chunks of 2 pixels x 4 channels that
  // start at even pixels (even horizontal stride, no padding) stay 16-B aligned
  const bool packed = p.ldx == 4 && p.Cg % 32 == 0 && p.S == 1 && (p.sw & 1) == 0 && p.pw == 0 && p.ph == 0;
  if (p.Cg % 8 != 0 || (p.ldx % 8 != 0 && !packed) || p.ldm % 8 != 0) return -1;
  p.div_pq = make_fastdiv((uint32_t)(a.P * a.Q));
  p.div_q = make_fastdiv((uint32_t)a.Q);
  p.div_cg = make_fastdiv((uint32_t)a.Cg);
  p.div_s = make_fastdiv((uint32_t)a.S);
  const int ktiles = cdiv(p.K, BK);
  const int splits = a.splits > 0 ? a.splits : dv_conv_wgrad_splits(a);
  p.ktiles_per_split = cdiv(ktiles, splits);
  p.splits = cdiv(ktiles, p.ktiles_per_split);
  p.atomic_out = p.splits > 1 ? 1 : 0;
  p.accumulate = a.accumulate;
  p.oirs_ig = a.oirs_ig;
  p.slab = 0;
  p.reflect = a.reflect;
  if (p.reflect && (p.ph >= p.Hin || p.pw >= p.Win || p.ph < 0 || p.pw < 0)) return -1;
  if (p.oirs_ig > p.Cg) return -1;
  const size_t out_elems = (size_t)p.G * p.M * (p.oirs_ig > 0 ? (size_t)p.oirs_ig * p.R * p.S : (size_t)p.N);
  // deterministic mode, and by default every split-K launch: each split stores its partial tile
  // into its own slab (every valid element of dW is written once per split: no memset), the
  // slabs are summed in a fixed order afterwards -- no atomics, reproducible bits
  // tiny accumulating launches (Hourglass 4x4 / 8x8 maps, < 4 GFLOP): the reduce pass's launch
  // costs more than the atomics it avoids, and accumulating into a zeroed buffer needs no memset
  static const bool tiny_on = [] {
    const char* v = std::getenv("DV_WG_TINY");
    return !(v && v[0] == '0');
  }();
  const bool tiny = tiny_on && a.accumulate && 2.0 * p.M * (double)p.N * p.K * p.G < 4e9;
  const bool slab = g_wg_slab == 1 || (g_wg_slab < 0 && p.splits <= SLAB_MAX_SPLITS && !tiny);
  bool det = (g_deterministic || slab) && p.splits > 1;
  float* slab_ws = det ? dv_slab_workspace((size_t)p.splits * out_elems, st) : nullptr;
  if (det && !slab_ws) {
    if (g_deterministic) return -1;
    det = false;  // no room for the slabs: atomics
  }
  if (det) {
    p.dw = slab_ws;
    p.slab = (int64_t)out_elems;
    p.atomic_out = 0;
    p.accumulate = 0;
  } else if (p.atomic_out && !a.accumulate) {
    (void)hipMemsetAsync(a.dw, 0, out_elems * sizeof(float), st);
  }
  // plain rows: the im2col of a 1x1 / stride-1 / pad-0 conv is X itself (pixel grid == input grid)
  const bool plain = a.R == 1 && a.S == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 && a.pw == 0 && a.P == a.H &&
                     a.Q == a.W && !a.reflect;
  const int bn = cdiv(p.M, 64) * cdiv(p.N, 256) * p.G * p.splits;
  const int bw = cdiv(p.M, 128) * cdiv(p.N, 128) * p.G * p.splits;
  if (plain) dispatch_wg<true>(p, bn, bw, st);
  else dispatch_wg<false>(p, bn, bw, st);
  if (det) {
    static const bool final_on = [] {
      const char* v = std::getenv("DV_WG_FINAL");
      return !(v && v[0] == '0');
    }();
    if (final_on && a.out && p.oirs_ig == 0 && a.out_ig > 0 && a.out_ig <= p.Cg) {
      const unsigned grid = (unsigned)std::min<int64_t>(((int64_t)out_elems + 255) / 256, 8192);
      slab_reduce_oirs_kernel<<<grid, 256, 0, st>>>(slab_ws, a.out, a.R * a.S, p.Cg, a.out_ig, p.splits,
                                                    (int64_t)out_elems, a.out_accumulate);
      return p.splits | DV_WGRAD_FINAL;
    }
    dv_slab_reduce(slab_ws, a.dw, (int64_t)out_elems, p.splits, a.accumulate, st);
  }
  return p.splits;
}
