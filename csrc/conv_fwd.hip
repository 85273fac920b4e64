// Implicit-GEMM convolution FORWARD on gfx950 MFMA: dispatch, the warp-specialised ring variant,
// the split-K finalize pass and the host entry point. The kernel itself is in conv_fwd_core.h.
#include <cstdlib>

#include "conv_fwd_core.h"

int dv_g_last_ksplit = 1;
int dv_g_fwd_variant = 0;

namespace {

// ---------------------------------------------------------------------------------------------
// Warp-specialised forward (benchmark variants 20-23): 4 loader waves keep an NS-slot LDS ring
// filled by LDS-DMA, NCW = 4 or 8 consumer waves (64x64 wave tiles) run the MFMAs. Slots change
// hands through LDS counters -- FULL[s]: loader waves whose pieces of the slot's current fill have
// landed, FREE[s]: consumer waves that hold the slot's fragments in registers -- so consumers
// never issue a DMA or wait at a block barrier, and each loader wave keeps RING_LAG fills in
// flight (counted vmcnt). The block is persistent over output tiles: the ring runs on across tile
// boundaries, the loaders prefetch the next tile while the consumers store the current one.
// Scope: KM_FAST loader, identity output map, G == 1, EPI_PLAIN / EPI_STATS.
constexpr int RING_LAG = 3, RING_BK = 32, RING_EROWS = 16;
template <int BM_, int BN_>
constexpr int ring_slot_bytes() { return (BM_ + BN_) * RING_BK * 2; }
template <int BM_, int BN_>
constexpr int ring_ncw() { return (BM_ / 64) * (BN_ / 64); }
template <int BM_, int BN_>
constexpr int ring_stage_bytes() { return ring_ncw<BM_, BN_>() * RING_EROWS * EPI_PITCH * 2; }
template <int BM_, int BN_>
constexpr int ring_ns() {
  const int n = (150 * 1024 - ring_stage_bytes<BM_, BN_>()) / ring_slot_bytes<BM_, BN_>();
  return n > 6 ? 6 : n;
}
template <int BM_, int BN_>
constexpr int ring_lds_bytes() { return ring_ns<BM_, BN_>() * ring_slot_bytes<BM_, BN_>() + ring_stage_bytes<BM_, BN_>(); }

// LDS-DMA of one 1-KB wave piece from inline asm (M0 set and restored in the statement): hipcc does
// not track it, so it neither waits for it before the FULL publish nor before unrelated LDS work
DV_DEVICE void glds16_asm(const void* src, uint32_t dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}
// wait until an LDS counter reaches `target`; a guard bounds the spin so a broken handshake ends
// the kernel with wrong numbers instead of hanging the GPU
DV_DEVICE void ring_wait(volatile int* c, int target) {
  for (int guard = 0; *c < target && guard < (1 << 24); ++guard) {
  }
}

template <int BM_, int BN_, int EPI>
__global__ __launch_bounds__(64 * (4 + ring_ncw<BM_, BN_>()), 1) void conv_ring_kernel(FwdParams p) {
  constexpr int WN = BN_ / 64, WM = BM_ / 64, NCW = WM * WN, NS = ring_ns<BM_, BN_>();
  static_assert(NCW == 4 || NCW == 8, "4 or 8 consumer waves of 64x64");
  static_assert(NS > RING_LAG, "ring deeper than the loader lag");
  constexpr int BK_ = RING_BK, CH = BK_ / 8, RPI = 64 / CH;  // 16 rows of 64 B per 1-KB DMA
  constexpr int MI = BM_ / RPI / 4, NI = BN_ / RPI / 4;        // DMAs per loader wave per fill
  constexpr int IPL = MI + NI;
  constexpr int SLOT = ring_slot_bytes<BM_, BN_>();
  __shared__ int ring_full[NS], ring_free[NS];
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x < NS) { ring_full[threadIdx.x] = 0; ring_free[threadIdx.x] = 0; }
  __syncthreads();
  const int tiles_m = (p.M + BM_ - 1) / BM_, tiles_n = (p.N + BN_ - 1) / BN_;
  const int ntiles = tiles_m * tiles_n;
  const int nt = (p.K + BK_ - 1) / BK_;  // K-tiles per output tile (Cg % 64 == 0: one tap each)

  if (wid >= NCW) {
    // ---------------------------------- loader waves ----------------------------------
    const int lw = wid - NCW;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
    const char* zero = dv_zero_page;
    int fill = 0;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      const int tn = tile % tiles_n, tm = tile / tiles_n;
      const int m0 = tm * BM_, n0 = tn * BN_;
      const u16* wrow[NI];
      bool wok[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = (lw * NI + j) * RPI + lane / CH;
        const int lc = (lane % CH) ^ kc_swz<BK_>(row);
        const int n = n0 + row;
        wok[j] = n < p.N;
        wrow[j] = p.w + (int64_t)(wok[j] ? n : 0) * p.K + lc * 8;
      }
      const u16* xrow[MI];
      uint32_t tapmask[MI];
#pragma unroll
      for (int j = 0; j < MI; ++j) {
        const int row = (lw * MI + j) * RPI + lane / CH;
        const int lc = (lane % CH) ^ kc_swz<BK_>(row);
        const int m = m0 + row;
        const bool ok = m < p.M;
        const int mm = ok ? m : 0;
        const int img = (int)fdiv((uint32_t)mm, p.div_pq), rem = mm - img * (p.P * p.Q);
        const int pp = (int)fdiv((uint32_t)rem, p.div_q), qq = rem - pp * p.Q;
        const int hb = pp * p.sh - p.ph, wb = qq * p.sw - p.pw;
        uint32_t mk = 0;
        for (int r = 0; r < p.R; ++r) { const int h = hb + r * p.dh; mk |= (uint32_t)(h >= 0 && h < p.Hin) << r; }
        for (int s2 = 0; s2 < p.S; ++s2) { const int w = wb + s2 * p.dw; mk |= (uint32_t)(w >= 0 && w < p.Win) << (16 + s2); }
        tapmask[j] = ok ? mk : 0u;
        xrow[j] = p.x + ((int64_t)img * p.Hin * p.Win + (int64_t)hb * p.Win + wb) * p.ldx + lc * 8;
      }
      int t_r = 0, t_s = 0, t_c = 0;
      for (int kt = 0; kt < nt; ++kt, ++fill) {
        const int s = fill % NS, k = fill / NS;
        if (k > 0) ring_wait(&ring_free[s], NCW * k);  // every consumer holds the slot's last fill in registers
        const uint32_t img_n = lds0 + s * SLOT, img_m = img_n + BN_ * BK_ * 2;
        const int k0 = kt * BK_;
#pragma unroll
        for (int j = 0; j < NI; ++j) glds16_asm(wok[j] ? (const void*)(wrow[j] + k0) : (const void*)zero, img_n + (lw * NI + j) * 1024);
        const int64_t koff = ((int64_t)(t_r * p.dh) * p.Win + t_s * p.dw) * p.ldx + t_c;
#pragma unroll
        for (int j = 0; j < MI; ++j) {
          const bool ok = (tapmask[j] >> t_r) & (tapmask[j] >> (16 + t_s)) & 1u;
          glds16_asm(ok ? (const void*)(xrow[j] + koff) : (const void*)zero, img_m + (lw * MI + j) * 1024);
        }
        t_c += BK_;
        if (t_c >= p.Cg) { t_c = 0; if (++t_s == p.S) { t_s = 0; ++t_r; } }
        if (fill >= RING_LAG) {  // fill - LAG has landed (this wave's part): publish it
          wait_vm<IPL * RING_LAG>();
          if (lane == 0) atomicAdd(&ring_full[(fill - RING_LAG) % NS], 1);
        }
      }
    }
    // drain: publish the last LAG fills in order
    const int last = fill;
#pragma unroll
    for (int d = RING_LAG; d >= 1; --d) {
      const int f = last - d;
      if (f < 0) continue;
      if (d == 3) wait_vm<IPL * 2>();
      else if (d == 2) wait_vm<IPL>();
      else wait_vm<0>();
      if (lane == 0) atomicAdd(&ring_full[f % NS], 1);
    }
    return;
  }

  // ---------------------------------- consumer waves ----------------------------------
  const int wave_m = wid / WN, wave_n = wid % WN;
  u16* st = reinterpret_cast<u16*>(smem + NS * SLOT + wid * RING_EROWS * EPI_PITCH * 2);
  int fill = 0;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int tn = tile % tiles_n, tm = tile / tiles_n;
    const int m0 = tm * BM_, n0 = tn * BN_;
    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    // software-pipelined: fill t+1's fragment reads are in flight during fill t's MFMAs
    bf16x8 fa[4], fb[4];
    auto rd = [&](int f, bf16x8* a_, bf16x8* b_) {
      const int s = f % NS, k = f / NS;
      ring_wait(&ring_full[s], 4 * (k + 1));
      const char* img_n = smem + s * SLOT;
      const char* img_m = img_n + BN_ * BK_ * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) a_[j] = read_kc<BK_>(img_n, wave_n * 64 + j * 16 + (lane & 15), lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) b_[i] = read_kc<BK_>(img_m, wave_m * 64 + i * 16 + (lane & 15), lane >> 4);
    };
    auto release = [&](int f) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) atomicAdd(&ring_free[f % NS], 1);  // fragments in registers: the slot may refill
    };
    rd(fill, fa, fb);
    release(fill);
    for (int kt = 0; kt < nt; ++kt, ++fill) {
      bf16x8 na[4], nb[4];
      if (kt + 1 < nt) rd(fill + 1, na, nb);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[j], fb[i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nt) {
        release(fill + 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) { fa[j] = na[j]; fb[j] = nb[j]; }
      }
    }
    // epilogue (identity map): statistics of the fp32 results; the bf16 tile goes out through this
    // wave's private 16-row LDS staging in 4 passes, as 16-B pieces of whole NHWC rows
    const int nw0 = n0 + wave_n * 64, mw0 = m0 + wave_m * 64;
    float bsum[4][4], bsq[4][4], kq[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nw0 + j * 16 + (lane >> 4) * 4 + r;
        kq[j][r] = (EPI == EPI_STATS && n < p.N) ? stat_shift(p.stats, p.N)[n] : 0.f;
        bsum[j][r] = 0.f; bsq[j][r] = 0.f;
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool mv = mw0 + i * 16 + (lane & 15) < p.M;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[j][i][r];
          if constexpr (EPI == EPI_STATS) {
            if (mv) { const float d = v[r] - kq[j][r]; bsum[j][r] += d; bsq[j][r] = fmaf(d, d, bsq[j][r]); }
          }
        }
        uint2 pk; pk.x = pack2bf(v[0], v[1]); pk.y = pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(st + (lane & 15) * EPI_PITCH + j * 16 + (lane >> 4) * 4) = pk;
      }
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int rl = it * 8 + (lane >> 3), ch = (lane & 7) * 8;
        const int m = mw0 + i * 16 + rl, n = nw0 + ch;
        const uint4 o = *reinterpret_cast<const uint4*>(st + rl * EPI_PITCH + ch);
        if (m < p.M && n < p.N) *reinterpret_cast<uint4*>(p.y + (int64_t)m * p.ldy + n) = o;
      }
    }
    if constexpr (EPI == EPI_STATS) {
      float* a = p.stats + (int64_t)(tm % DV_STAT_SHARDS) * 2 * p.N;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float s1 = row16_sum(bsum[j][r]), s2 = row16_sum(bsq[j][r]);
          const int n = nw0 + j * 16 + (lane >> 4) * 4 + r;
          if ((lane & 15) == 0 && n < p.N) { atomicAdd(a + n, s1); atomicAdd(a + p.N + n, s2); }
        }
    }
  }
}

template <int BM_, int BN_, int EPI>
void launch_ring(const FwdParams& p, hipStream_t st) {
  constexpr int lds = ring_lds_bytes<BM_, BN_>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_ring_kernel<BM_, BN_, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const int ntiles = ((p.M + BM_ - 1) / BM_) * ((p.N + BN_ - 1) / BN_);
  conv_ring_kernel<BM_, BN_, EPI><<<dim3(std::min(ntiles, 256)), dim3(64 * (4 + ring_ncw<BM_, BN_>())), lds, st>>>(p);
}

template <int KMODE, bool RES, int BNR, int EPI>
void launch_heuristic(const FwdParams& p, hipStream_t st) {
  if (KMODE == KM_FAST) {
    if (big_tile_ok<KMODE>(p)) { launch_fwd<256, 256, 64, KMODE, RES, 2, BNR, EPI, 128>(p, st); return; }
    if (p.N <= 64) {
      if (p.K <= 256) launch_fwd<256, 64, 32, KMODE, RES, 3, BNR, EPI>(p, st);
      else launch_fwd<256, 64, 32, KMODE, RES, 2, BNR, EPI>(p, st);
    } else {
      if (p.K > 64 && p.K < 2048) launch_fwd<128, 128, 32, KMODE, RES, 2, BNR, EPI>(p, st);
      else launch_fwd<128, 128, 64, KMODE, RES, 2, BNR, EPI>(p, st);
    }
    return;
  }
  if (p.N <= 64) launch_fwd<256, 64, 32, KMODE, RES, 2, BNR, EPI>(p, st);
  else launch_fwd<128, 128, 64, KMODE, RES, 2, BNR, EPI>(p, st);
}

template <int KMODE, bool RES, int BNR = 0>
void dispatch_res(const FwdParams& p, hipStream_t st) {
  if constexpr (BNR) {  // fused BN-backward statistics (dgrads, KM_FAST only): plain epilogue
    launch_heuristic<KMODE, RES, BNR, EPI_PLAIN>(p, st);
    return;
  }
  if constexpr (KMODE == KM_FAST) {
    switch (dv_g_fwd_variant) {
      case 1: return launch_fwd<128, 128, 64, KMODE, RES, 2>(p, st);
      case 2: return launch_fwd<256, 64, 32, KMODE, RES, 2>(p, st);
      case 3: return launch_fwd<256, 64, 64, KMODE, RES, 2>(p, st);
      case 4: return launch_fwd<128, 128, 64, KMODE, RES, 3>(p, st);
      case 5: return launch_fwd<256, 64, 32, KMODE, RES, 4>(p, st);
      case 6: return launch_fwd<256, 64, 64, KMODE, RES, 3>(p, st);
      case 7: return launch_fwd<128, 128, 32, KMODE, RES, 4>(p, st);
      case 8: return launch_fwd<128, 128, 32, KMODE, RES, 2>(p, st);
      case 9: return launch_fwd<256, 64, 32, KMODE, RES, 3>(p, st);
      // 8-wave tiles (one 512-thread block per CU, deep LDS-DMA ring)
      case 10: return launch_fwd<256, 128, 64, KMODE, RES, 3>(p, st);
      // 128-row wave tiles (a wave = 128 pixels x 64 channels)
      case 12: return launch_fwd<256, 128, 64, KMODE, RES, 2, 0, EPI_FULL, 128>(p, st);  // 4 waves
      case 14: return launch_fwd<256, 256, 64, KMODE, RES, 2, 0, EPI_FULL, 128>(p, st);  // 8 waves
      default: break;
    }
    const bool full = p.bias || p.act || p.ypart;  // split-K slabs are written by the FULL form
    if (!full && !p.stats) launch_heuristic<KMODE, RES, 0, EPI_PLAIN>(p, st);
    else if (!full) launch_heuristic<KMODE, RES, 0, EPI_STATS>(p, st);
    else launch_heuristic<KMODE, RES, 0, EPI_FULL>(p, st);
    return;
  }
  launch_heuristic<KMODE, RES, 0, EPI_FULL>(p, st);
}

template <int KMODE>
void dispatch_tile(const FwdParams& p, hipStream_t st) {
  // in-place gradient accumulation / fused BN statistics epilogues are compile-time: no cost
  // for the others
  if constexpr (KMODE == KM_FAST) {
    if (p.bnmode) {  // BNR 2: a second BatchNorm on the same dz (projection-block join, bnx2)
      if (p.bnx2) {
        if (p.res) dispatch_res<KMODE, true, 2>(p, st);
        else dispatch_res<KMODE, false, 2>(p, st);
      } else {
        if (p.res) dispatch_res<KMODE, true, 1>(p, st);
        else dispatch_res<KMODE, false, 1>(p, st);
      }
      return;
    }
  }
  if (p.res) dispatch_res<KMODE, true>(p, st);
  else dispatch_res<KMODE, false>(p, st);
}

// y[m][n] = act(sum_s ypart[s][m][n] + bias[n]) (+ res[m][n]) in bf16, plus the BatchNorm
// partial statistics of y when `stats` is set (the epilogue work the split blocks skipped). The
// slabs are summed in split order (bitwise reproducible). Block = 64 column lanes x 4 columns
// (256 channels) x 4 row lanes walking FR_ROWS rows; statistics meet in LDS, one coalesced atomic
// row per block into shard blockIdx.y % SHARDS.
constexpr int FR_ROWS = 64;  // rows per block on large grids; small ones shrink it (dv_conv_fwd)
// BatchNorm-backward sums of a split-K dgrad's output (the conv epilogue's BNR, modes 1 / 2: the
// split blocks only write fp32 slabs, so the pass that stores dX reduces it): x = the BN input at
// dX's offsets (dense, ld = N), prm = [scale, shift, mean, invstd][N], acc = [SHARDS][2][N]
struct FinBnr {
  const u16* x;
  const float* prm;
  float* acc;
  int mode, act;
  float slope;
  float* det;
};

__global__ __launch_bounds__(256) void splitk_finalize_kernel(const float* __restrict__ ypart, int ksplit, int M, int N,
                                                              const float* __restrict__ bias, int act, float slope,
                                                              const u16* __restrict__ res, float* __restrict__ stats,
                                                              u16* __restrict__ y, int ldy, int fr, float* __restrict__ det,
                                                              FinBnr bnr) {
  __shared__ float red[2][4][256];
  const int lc = threadIdx.x & 63, lr = threadIdx.x >> 6;
  const int n = blockIdx.x * 256 + lc * 4;
  const bool nv = n < N;  // N % 4 == 0: whole column quads
  const int64_t slab = (int64_t)M * N;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f}, bv[4], kq[4], bsc[4], bsh[4], bmu[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    bv[r] = (bias && nv) ? bias[n + r] : 0.f;
    kq[r] = (stats && nv) ? stat_shift(stats, N)[n + r] : 0.f;
    bsc[r] = (bnr.acc && nv) ? bnr.prm[n + r] : 0.f;
    bsh[r] = (bnr.acc && nv) ? bnr.prm[N + n + r] : 0.f;
    bmu[r] = (bnr.acc && nv) ? bnr.prm[2 * N + n + r] : 0.f;
  }
  const int m1 = min(M, (int)(blockIdx.y + 1) * fr);
  for (int m = blockIdx.y * fr + lr; nv && m < m1; m += 4) {
    f32x4 a = *reinterpret_cast<const f32x4*>(ypart + (int64_t)m * N + n);
    for (int sp = 1; sp < ksplit; ++sp) a += *reinterpret_cast<const f32x4*>(ypart + sp * slab + (int64_t)m * N + n);
    float rv[4] = {0.f, 0.f, 0.f, 0.f};
    if (res) {
      const uint2 rr = *reinterpret_cast<const uint2*>(res + (int64_t)m * ldy + n);
      rv[0] = bf2f(rr.x & 0xffff); rv[1] = bf2f(rr.x >> 16); rv[2] = bf2f(rr.y & 0xffff); rv[3] = bf2f(rr.y >> 16);
    }
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float t = a[r] + bv[r];
      if (act == ACT_RELU) t = fmaxf(t, 0.f);
      else if (act == ACT_LEAKY) t = t > 0.f ? t : t * slope;
      t += rv[r];
      v[r] = t;
      if (stats) {  // (the BN-backward sums below use the same accumulators)
        const float d = t - kq[r];
        s1[r] += d; s2[r] = fmaf(d, d, s2[r]);
      }
    }
    uint2 pk; pk.x = pack2bf(v[0], v[1]); pk.y = pack2bf(v[2], v[3]);
    *reinterpret_cast<uint2*>(y + (int64_t)m * ldy + n) = pk;
    if (bnr.acc) {  // of the stored bf16 gradient, as the unfused reduce pass would read it back
      const uint2 xr = *reinterpret_cast<const uint2*>(bnr.x + (int64_t)m * N + n);
      const float d[4] = {bf2f(pk.x & 0xffff), bf2f(pk.x >> 16), bf2f(pk.y & 0xffff), bf2f(pk.y >> 16)};
      const float xv[4] = {bf2f(xr.x & 0xffff), bf2f(xr.x >> 16), bf2f(xr.y & 0xffff), bf2f(xr.y >> 16)};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float dz = d[r];
        if (bnr.mode == 2 && !(xv[r] * bsc[r] + bsh[r] > 0.f)) dz = bnr.act == 2 ? d[r] * bnr.slope : 0.f;
        s1[r] += dz;
        s2[r] = fmaf(dz, xv[r] - bmu[r], s2[r]);
      }
    }
  }
  if (!stats && !bnr.acc) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) { red[0][lr][lc * 4 + r] = s1[r]; red[1][lr][lc * 4 + r] = s2[r]; }
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < N) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) { t1 += red[0][q][threadIdx.x]; t2 += red[1][q][threadIdx.x]; }
    if (bnr.acc) {  // sum dz*(x - mean) -> sum dz*xhat: one invstd per channel
      float* sh = stat_row(bnr.acc, bnr.det, blockIdx.y, N);
      atomicAdd(sh + c, t1);
      atomicAdd(sh + N + c, t2 * bnr.prm[3 * N + c]);
    } else {
      float* sh = stat_row(stats, det, blockIdx.y, N);
      atomicAdd(sh + c, t1);
      atomicAdd(sh + N + c, t2);
    }
  }
}

}  // namespace

void dv_conv_fwd_variant(int v) { dv_g_fwd_variant = v; }

int dv_conv_fwd(const ConvFwdArgs& a, hipStream_t st) {
  FwdParams p{};
  p.x = (const u16*)a.x; p.w = (const u16*)a.w; p.y = (u16*)a.y;
  p.bias = a.bias; p.stats = a.stats; p.res = (const u16*)a.res;
  p.G = a.G; p.M = a.Nb * a.P * a.Q; p.N = a.Kout; p.K = a.R * a.S * a.Cg;
  p.Hin = a.H; p.Win = a.W; p.Cg = a.Cg; p.ldx = a.ldx;
  p.P = a.P; p.Q = a.Q; p.R = a.R; p.S = a.S;
  p.sh = a.sh; p.sw = a.sw; p.ph = a.ph; p.pw = a.pw; p.dh = a.dh; p.dw = a.dw;
  p.OH = a.OH; p.OW = a.OW; p.osh = a.osh; p.osw = a.osw; p.oph = a.oph; p.opw = a.opw; p.ldy = a.ldy;
  p.act = a.act; p.slope = a.slope;
  p.identity_map = (a.OH == a.P && a.OW == a.Q && a.osh == 1 && a.osw == 1 && a.oph == 0 && a.opw == 0);
  p.bnx = (const u16*)a.bnx; p.bnbits = (const uint8_t*)a.bnbits; p.bnprm = a.bnprm; p.bnacc = a.bnacc;
  p.bnmode = a.bnmode; p.bnact = a.bnact; p.bnslope = a.bnslope;
  p.bnx2 = (const u16*)a.bnx2; p.bnprm2 = a.bnprm2; p.bnacc2 = a.bnacc2;
  p.resbits = (const uint8_t*)a.resbits; p.resact = a.resact; p.resslope = a.resslope;
  p.reflect = a.reflect;
  static const int64_t nt_min = [] {
    const char* v = std::getenv("DV_EPI_NT_MIN");  // benchmarking override (elements of the output)
    return v ? (int64_t)std::atoll(v) : (24ll << 20);
  }();
  p.ntl = (int64_t)a.P * a.Q * a.Nb * a.G * a.Kout >= nt_min;
  p.wld = a.w_ld ? a.w_ld : p.K;
  p.wkr = a.w_kr ? a.w_kr : a.S * a.Cg;
  p.wks = a.w_ks ? a.w_ks : a.Cg;
  p.ksplit = 1; p.kt_per = 1 << 30; p.ypart = nullptr;
  // zero-filling scatter: plain epilogue, no residual, a strided map with no offset whose
  // siblings tile the output grid (OH <= P*osh, OW <= Q*osw), vector stores
  p.zfill = a.zfill;
  if (p.zfill && (a.bias || a.act || a.stats || a.res || a.bnmode || a.tgather || a.oph || a.opw || a.ksplit > 1 ||
                  a.OH > a.P * a.osh || a.OW > a.Q * a.osw || (a.Kout % 8) || (a.ldy % 8)))
    return -1;
  const u16* fin_res = nullptr;
  float* fin_stats = nullptr;
  FinBnr fin_bnr{};
  if (a.ksplit > 1 && a.ypart) {
    // split-K: single group, identity output map; bias / activation / residual / BN statistics
    // and the BN-backward sums of a dgrad (modes 1 / 2: no mask bits, no second BN) are applied
    // by the finalize pass (no masked residual)
    const bool bn_ok = !a.bnmode || ((a.bnmode == 1 || a.bnmode == 2) && !a.bnx2 && a.bnx && a.bnprm && a.bnacc &&
                                     !a.res && !a.stats && a.ldy == a.Kout);
    const bool ok = a.G == 1 && !a.tgather && bn_ok && !a.resbits && !a.reflect && (a.Kout % 4) == 0 &&
                    (a.ldy % 4) == 0 && a.OH == a.P && a.OW == a.Q && a.osh == 1 && a.osw == 1 && !a.oph && !a.opw;
    if (!ok) return -1;
    p.ksplit = a.ksplit; p.ypart = a.ypart;
    fin_res = p.res; fin_stats = p.stats;  // applied by the finalize pass, not the split blocks
    p.res = nullptr; p.stats = nullptr;
    if (a.bnmode) {
      fin_bnr = FinBnr{(const u16*)a.bnx, a.bnprm, a.bnacc, a.bnmode, a.bnact, a.bnslope, nullptr};
      p.bnmode = 0;  // the split blocks store raw slabs
    }
  }
  // statistics of a residual output (y = conv + bias + residual) are accumulated from the 16-B
  // vector stores of a single-group tensor (conv_fwd_core.h RST)
  if (p.res && p.stats && ((p.N & 7) || (p.ldy & 7) || p.G != 1)) return -1;
  if (p.reflect && (a.tgather || p.ph >= p.Hin || p.pw >= p.Win || p.ph < 0 || p.pw < 0 || p.bnmode)) return -1;
  // the mask bits are indexed by the dense element offset of y: a single-group tensor whose
  // pixel stride is its channel count, written by the identity-mapped (stride-1) epilogue
  if (p.resbits && (!p.res || (p.N & 7) || p.ldy != p.N || p.G != 1 || a.tgather ||
                    !(a.OH == a.P && a.OW == a.Q && a.osh == 1 && a.osw == 1 && a.oph == 0 && a.opw == 0)))
    return -1;
  // fused BN statistics need every element of y written by this kernel as 16-B vectors of a dense
  // single-group tensor on the fast loader (the dgrads of stride-1 convs)
  int bn_status = 0;
  if (p.bnmode) {
    // identity map, or the strided scatter of a 1x1 stride-s dgrad (no offset): the pixels it does
    // not write hold zero gradient and add nothing to either sum. Not with zfill (its sibling
    // zeroing lives in the non-prefetching store path).
    // (a parity part of a sub-pixel dgrad: offset map, its own disjoint pixels)
    const bool map_ok = p.identity_map || !p.zfill;
    const bool ok = a.tgather == 0 && map_ok && p.G == 1 && (p.N & 7) == 0 && p.ldy == p.N &&
                    p.Cg % 64 == 0 && p.ldx % 8 == 0 && p.R <= 16 && p.S <= 16 && p.bnx && p.bnprm && p.bnacc &&
                    (p.bnmode != 3 || p.bnbits) && (!p.bnx2 || (p.bnmode == 3 && p.bnprm2 && p.bnacc2));
    if (!ok) { p.bnmode = 0; bn_status = 1; }
  }
  if (!p.bnmode) p.bnx2 = nullptr;
  p.div_pq = make_fastdiv((uint32_t)(a.P * a.Q));
  p.div_q = make_fastdiv((uint32_t)a.Q);
  // deterministic statistics (kernels.h DetStats): one slab row per 128-row tile (every tile
  // shape has >= 128 rows), regions: forward statistics, BN-backward sums, the dual BN's sums
  const bool want_s = p.stats != nullptr, want_b = p.bnmode != 0;
  const DetStats det((want_s || want_b) ? (p.M + 127) / 128 : 0, (int64_t)p.G * p.N, st, 3);
  p.sdet = want_s ? det.region(0) : nullptr;
  p.bdet = want_b ? det.region(1) : nullptr;
  p.bdet2 = (want_b && p.bnx2) ? det.region(2) : nullptr;
  auto det_fold = [&]() {
    if (p.sdet) det.fold(p.stats, 0);
    if (p.bdet) det.fold(p.bnacc, 1);
    if (p.bdet2) det.fold(p.bnacc2, 2);
  };
  if (a.tgather == 2) {
    p.bnmode = 0;
    // Tap-packed input (stem convs with <= 4 input channels, ops/conv.py _StemConvFn): a padded
    // [N][Hp][Wp][4] image read as Cg = 32 "channels" at a pixel stride of 4, i.e. one 16-B
    // chunk = 2 horizontally adjacent pixels = 2 filter taps; one K-tile (BK = 32) = one filter
    // row of 8 taps. Needs: no padding (the image is pre-padded), 16-B aligned chunks (even
    // horizontal stride: every chunk starts at an even pixel), and BK = 32 tiles.
    if (p.Cg % 32 != 0 || p.ldx != 4 || p.S != 1 || (p.sw & 1) || p.ph || p.pw || p.dh != 1 || p.res) return -1;
    if (dv_g_fwd_variant == 5) launch_fwd<256, 64, 32, KM_FAST, false, 4>(p, st);
    else if (dv_g_fwd_variant == 7) launch_fwd<128, 128, 32, KM_FAST, false, 4>(p, st);
    else if (dv_g_fwd_variant == 8) launch_fwd<128, 128, 32, KM_FAST, false, 2>(p, st);
    else {
      // compile-time epilogue as in dispatch_res: the ResNet / Inception stems feed a BatchNorm
      // (statistics, no bias / activation) -- the runtime-flag epilogue cost ~8 VALU per element
      // 256x64 for the 64-channel stems with the plain double buffer: 40 KB of LDS, 4 blocks per
      // CU (the 3-deep ring fit 2): the 7-tile K loop is latency-bound, more resident blocks hide
      // it (ResNet-50 stem incl. pack 292 -> 246 us, measured in round 3)
      const bool full = p.bias || p.act || p.ypart;
      if (p.N <= 64) {
        if (full) launch_fwd<256, 64, 32, KM_FAST, false, 2, false, EPI_FULL>(p, st);
        else if (p.stats) launch_fwd<256, 64, 32, KM_FAST, false, 2, false, EPI_STATS>(p, st);
        else launch_fwd<256, 64, 32, KM_FAST, false, 2, false, EPI_PLAIN>(p, st);
      } else {
        if (full) launch_fwd<128, 128, 32, KM_FAST, false, 2, false, EPI_FULL>(p, st);
        else if (p.stats) launch_fwd<128, 128, 32, KM_FAST, false, 2, false, EPI_STATS>(p, st);
        else launch_fwd<128, 128, 32, KM_FAST, false, 2, false, EPI_PLAIN>(p, st);
      }
    }
    det_fold();
    return bn_status;
  }
  if (p.Cg % 8 != 0 || p.ldx % 8 != 0) return -1;
  // warp-specialised ring (benchmark variants 20: 128x128, 21: 256x64, 22: 256x128, 23: 128x256)
  if (dv_g_fwd_variant >= 20 && dv_g_fwd_variant <= 23 && !det.slab && !a.tgather && p.Cg % 64 == 0 && p.R <= 16 && p.S <= 16 &&
      !p.reflect && p.G == 1 && p.identity_map && !p.bias && !p.act && !p.res && !p.bnmode && !p.ypart && !p.zfill &&
      (p.N % 8) == 0 && (p.ldy % 8) == 0) {
    const bool sts = p.stats != nullptr;
    switch (dv_g_fwd_variant) {
      case 20: if (sts) launch_ring<128, 128, EPI_STATS>(p, st); else launch_ring<128, 128, EPI_PLAIN>(p, st); break;
      case 21: if (sts) launch_ring<256, 64, EPI_STATS>(p, st); else launch_ring<256, 64, EPI_PLAIN>(p, st); break;
      case 22: if (sts) launch_ring<256, 128, EPI_STATS>(p, st); else launch_ring<256, 128, EPI_PLAIN>(p, st); break;
      default: if (sts) launch_ring<128, 256, EPI_STATS>(p, st); else launch_ring<128, 256, EPI_PLAIN>(p, st); break;
    }
    return 0;
  }
  // a strided / offset weight layout is read by the fast loader only
  const bool fast = !a.tgather && p.Cg % 64 == 0 && p.R <= 16 && p.S <= 16 && !p.reflect;
  if ((a.w_ld || a.w_kr || a.w_ks) && !fast) return -1;
  // the fast loader needs every K-tile inside one filter tap: Cg % 64 == 0 covers both BKs
  if (a.tgather) dispatch_tile<KM_TGATHER>(p, st);
  else if (p.Cg % 64 == 0 && p.R <= 16 && p.S <= 16 && !p.reflect) dispatch_tile<KM_FAST>(p, st);
  else dispatch_tile<KM_GENERIC>(p, st);
  det_fold();
  if (p.ypart) {
    // split-K serves small grids (Hourglass 4x4-16x16 maps): 64-row blocks left 8-32 blocks walking
    // up to 16 slabs serially (37 us median); shrink the row block until ~512 blocks
    // -- but no more row blocks than statistics shards while that is possible: one block per shard
    // adds onto a zero, so small launches keep bitwise-reproducible BatchNorm statistics
    const int ncb = (p.N + 255) / 256;
    int fr = (int)(((int64_t)p.M * ncb + 511) / 512);
    fr = std::max(fr, (p.M + DV_STAT_SHARDS - 1) / DV_STAT_SHARDS);
    fr = std::max(4, std::min(FR_ROWS, (fr + 3) / 4 * 4));
    const dim3 grid((unsigned)ncb, (unsigned)((p.M + fr - 1) / fr));
    const DetStats fdet(fin_stats ? grid.y : 0, p.N, st);
    const DetStats bdet(fin_bnr.acc ? grid.y : 0, p.N, st);
    fin_bnr.det = bdet.slab;
    splitk_finalize_kernel<<<grid, dim3(256), 0, st>>>(p.ypart, dv_g_last_ksplit, p.M, p.N, p.bias, p.act, p.slope,
                                                       fin_res, fin_stats, p.y, p.ldy, fr, fdet.slab, fin_bnr);
    fdet.fold(fin_stats);
    if (fin_bnr.acc) bdet.fold(fin_bnr.acc);
  }
  return bn_status;
}
