// Implicit-GEMM convolution / GEMM on gfx950 MFMA (bf16 in, fp32 accumulate).
//
// One templated kernel covers every GEMM-shaped op of the framework (SURVEY §2.7 K1-K5,
// K9, K13):
//   MODE_FWD   : C[m = out pixel][n = out channel] = sum_k im2col(X)[m][k] * W[n][k]
//                - conv forward (W = bf16 [Cout][R][S][Cin])
//                - conv dgrad / ConvTranspose forward (X = dY, W = transposed weights
//                  [Cin][R][S][Cout]; stride-1 via negative pad/dilation, stride>1 via the
//                  TGATHER divisibility gather, 1x1-strided via the scattered output map)
//                - Linear forward / dgrad (H = W = R = S = 1)
//                Epilogue: +bias, ReLU/LeakyReLU, per-channel BN statistics partials,
//                bf16 NHWC store into an arbitrary channel slice (concat-free).
//   MODE_WGRAD : dW[m = out channel][n = (r,s,c)] = sum_{pix} dY[pix][m] * im2col(X)[pix][n]
//                split-K over pixels, fp32 output (plain store or atomic accumulate).
//
// Design (see /opt/skills/guides/cdna_hip_programming.md):
//   * 128x128x64 block tile, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4
//     v_mfma_f32_16x16x32_bf16 tiles.
//   * Operands are staged global->LDS with LDS-DMA (global_load_lds_dwordx4); padded /
//     out-of-range lanes read a zero page, which makes the im2col halo free.
//   * LDS images are lane-linear (DMA constraint); bank-conflict freedom comes from
//     XOR-permuting the SOURCE address and applying the same XOR on the read (rule 21):
//       K-contiguous image  [rows][64 k]  (128 B rows) read by ds_read_b128,
//                           chunk' = chunk ^ ((row >> 1) & 7)
//       MN-contiguous image [64 k][128 cols] (256 B rows) read by ds_read_b64_tr_b16
//                           (hardware transpose), chunk' = chunk ^ (((k&3)|((k>>1)&4))<<1)
//   * 2 LDS stages, one barrier per K-tile (T3/T4 "minimum 2-phase" structure).
//   * Logical tile order is XCD-remapped so the N-tiles of one M-panel share an L2.
//
// The N-dim operand is fed to MFMA as "A" and the M-dim operand as "B" so that every lane
// ends up owning 4 consecutive output channels of one pixel: 8-byte NHWC stores and
// channel-wise statistics reduce across the 16 lanes of a DPP row.
#include "common.h"
#include "kernels.h"

__device__ __attribute__((aligned(16))) char dv_zero_page[256];

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int NTHREADS = 256;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;  // 32 KB
constexpr int LDS_BYTES = 2 * STAGE_BYTES + 4096;  // +epilogue scratch (stats)
constexpr int WG_F32_LD = BN + 4;                 // fp32 epilogue tile row stride

enum { MODE_FWD = 0, MODE_WGRAD = 1 };
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_LEAKY = 2 };

struct Params {
  const u16* x;      // FWD: gathered activation (im2col source). WGRAD: im2col source (N operand)
  const u16* w;      // FWD: N-operand rows [G][N][K]. WGRAD: dY (M operand, MN-contiguous)
  void* y;           // FWD: bf16 output. WGRAD: fp32 dW [G][M][N]
  const float* bias; // per output channel (FWD) or nullptr
  float* stats;      // FWD: sharded BN-stat accumulators [SHARDS][2][G*N] or nullptr
  int M, N, K;       // GEMM sizes per group
  int G;             // groups
  // gathered tensor geometry
  int Hin, Win, Cg, ldx;           // Cg = channels per group in the gathered tensor
  int P, Q;                        // pixel grid that m (FWD) / k (WGRAD) enumerates
  int R, S, sh, sw, ph, pw, dh, dw;
  // FWD output mapping: out pixel = ((img*OH) + p*osh + oph)*OW + q*osw + opw
  int OH, OW, osh, osw, oph, opw, ldy;
  int act; float slope;
  // WGRAD
  int ldm;           // channel stride of dY rows
  int splits, ktiles_per_split;
  int atomic_out;
};

DV_DEVICE void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(GLB_PTR(src), LDS_PTR(lds_wave_base), 16, 0, 0);
}

DV_DEVICE int kc_swz(int row) { return (row >> 1) & 7; }
DV_DEVICE int mn_swz(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }

// Read an 8-element bf16 MFMA fragment from a K-contiguous image (row = fragment row).
DV_DEVICE bf16x8 read_kc(const char* img, int row, int chunk) {
  const char* p = img + row * (BK * 2) + ((chunk ^ kc_swz(row)) << 4);
  return *reinterpret_cast<const bf16x8*>(p);
}

// Read an 8-element fragment from an MN-contiguous image [64 k][128 cols] with two
// hardware-transposed reads. `col0` = first column of the 16-column tile, kbase = kk*32.
DV_DEVICE bf16x8 read_mn(const char* img, int col0, int kbase, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k1 = kbase + 8 * g + q, k2 = k1 + 4;
  const int u = (col0 >> 2) + p;  // 8-byte unit
  const char* a1 = img + k1 * 256 + ((u ^ (mn_swz(k1) << 1)) << 3);
  const char* a2 = img + k2 * 256 + ((u ^ (mn_swz(k2) << 1)) << 3);
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)LDS_PTR(a1));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)LDS_PTR(a2));
  i16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <int MODE, bool FASTC, bool TGATHER>
__global__ __launch_bounds__(NTHREADS, 2) void igemm_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wave_n = wid & 1, wave_m = wid >> 1;

  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  int logical = xcd_remap(blockIdx.x, nwg);
  const int tn = logical % tiles_n; logical /= tiles_n;
  const int tm = logical % tiles_m; logical /= tiles_m;
  int split = 0, grp;
  if (MODE == MODE_WGRAD) { split = logical % p.splits; grp = logical / p.splits; }
  else grp = logical;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---------------- per-thread load descriptors ----------------
  // Each operand tile is 16 KB = 16 DMA wave-instructions; wave `wid` issues j = 0..3.
  const char* zero = dv_zero_page;
  int ktile_begin = 0, ktile_end = (p.K + BK - 1) / BK;
  if (MODE == MODE_WGRAD) {
    ktile_begin = split * p.ktiles_per_split;
    ktile_end = min(ktile_end, ktile_begin + p.ktiles_per_split);
  }

  // FWD: M operand = im2col rows (KC image), N operand = weight rows (KC image)
  // WGRAD: M operand = dY (MN image), N operand = im2col columns (MN image)
  int64_t a_pixbase[4];  // FWD: img*Hin*Win
  int a_h[4], a_w[4];    // FWD: base h/w (pre-tap);  WGRAD: unused
  bool a_ok[4];
  int b_r[4], b_s[4], b_c[4]; bool b_ok[4];  // WGRAD im2col column decode
  int w_img[4], w_p[4], w_q[4];              // WGRAD pixel (k-row) decode, incremental

  if (MODE == MODE_FWD) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = (wid * 4 + j) * 8 + (lane >> 3);
      const int m = m0 + row;
      a_ok[j] = m < p.M;
      const int mm = a_ok[j] ? m : 0;
      const int img = mm / (p.P * p.Q), rem = mm - img * (p.P * p.Q);
      const int pp = rem / p.Q, qq = rem - pp * p.Q;
      a_pixbase[j] = (int64_t)img * p.Hin * p.Win;
      if (TGATHER) { a_h[j] = pp + p.ph; a_w[j] = qq + p.pw; }
      else { a_h[j] = pp * p.sh - p.ph; a_w[j] = qq * p.sw - p.pw; }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = (wid * 4 + j) * 4 + (lane >> 4);  // k-row inside the tile
      const int lc = (lane & 15) ^ mn_swz(row);
      const int n = n0 + lc * 8;  // first (r,s,c) column of this 8-chunk
      b_ok[j] = n < p.N;
      const int nn = b_ok[j] ? n : 0;
      const int rs = nn / p.Cg;
      b_c[j] = nn - rs * p.Cg;
      b_r[j] = rs / p.S; b_s[j] = rs - b_r[j] * p.S;
      const int pix = ktile_begin * BK + row;
      const int pq = p.P * p.Q;
      w_img[j] = pix / pq; const int rem = pix - w_img[j] * pq;
      w_p[j] = rem / p.Q; w_q[j] = rem - w_p[j] * p.Q;
    }
  }
  // WGRAD incremental pixel advance per K-tile (BK pixels)
  const int d_q = BK % p.Q, d_p = (BK / p.Q) % p.P, d_img = BK / (p.P * p.Q);

  // FWD fast-path tap state (C % BK == 0 -> one (r,s) per K-tile)
  int t_r = 0, t_s = 0, t_c = 0;
  if (MODE == MODE_FWD && FASTC) {
    const int k = ktile_begin * BK;
    const int rs = k / p.Cg; t_c = k - rs * p.Cg; t_r = rs / p.S; t_s = rs - t_r * p.S;
  }

  const int64_t goff_x = (int64_t)grp * p.Cg;  // channel slice of the gathered tensor

  auto stage = [&](int kt, int buf) {
    char* sbase = smem + buf * STAGE_BYTES;
    char* img_n = sbase;            // N operand image (16 KB)
    char* img_m = sbase + BN * BK * 2;  // M operand image (16 KB)
    const int k0 = kt * BK;
    if (MODE == MODE_FWD) {
      // ---- N operand: plain rows [N][K] ----
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (wid * 4 + j) * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ kc_swz(row);
        const int n = n0 + row, k = k0 + lc * 8;
        const void* src = zero;
        if (n < p.N && k < p.K) src = p.w + ((int64_t)grp * p.N + n) * p.K + k;
        glds16(src, img_n + (wid * 4 + j) * 1024);
      }
      // ---- M operand: im2col gather ----
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (wid * 4 + j) * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ kc_swz(row);
        int r, s, c;
        const int k = k0 + lc * 8;
        if (FASTC) { r = t_r; s = t_s; c = t_c + lc * 8; }
        else { const int rs = k / p.Cg; c = k - rs * p.Cg; r = rs / p.S; s = rs - r * p.S; }
        const void* src = zero;
        bool ok = a_ok[j] && k < p.K;
        int h, w;
        if (TGATHER) {
          const int hn = a_h[j] - r * p.dh, wn = a_w[j] - s * p.dw;
          ok = ok && hn >= 0 && wn >= 0 && (hn % p.sh) == 0 && (wn % p.sw) == 0;
          h = hn / p.sh; w = wn / p.sw;
        } else {
          h = a_h[j] + r * p.dh; w = a_w[j] + s * p.dw;
        }
        ok = ok && h >= 0 && h < p.Hin && w >= 0 && w < p.Win;
        if (ok) src = p.x + (a_pixbase[j] + (int64_t)h * p.Win + w) * p.ldx + goff_x + c;
        glds16(src, img_m + (wid * 4 + j) * 1024);
      }
    } else {
      // ---- M operand: dY rows (pixels) x output channels, MN-contiguous ----
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (wid * 4 + j) * 4 + (lane >> 4);
        const int lc = (lane & 15) ^ mn_swz(row);
        const int pix = k0 + row, m = m0 + lc * 8;
        const void* src = zero;
        if (pix < p.K && m < p.M) src = p.w + (int64_t)pix * p.ldm + (int64_t)grp * p.M + m;
        glds16(src, img_m + (wid * 4 + j) * 1024);
      }
      // ---- N operand: im2col(X) rows (pixels) x (r,s,c) columns ----
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = (wid * 4 + j) * 4 + (lane >> 4);
        const int pix = k0 + row;
        const int h = w_p[j] * p.sh - p.ph + b_r[j] * p.dh;
        const int w = w_q[j] * p.sw - p.pw + b_s[j] * p.dw;
        const void* src = zero;
        if (b_ok[j] && pix < p.K && h >= 0 && h < p.Hin && w >= 0 && w < p.Win)
          src = p.x + (((int64_t)w_img[j] * p.Hin + h) * p.Win + w) * p.ldx + goff_x + b_c[j];
        glds16(src, img_n + (wid * 4 + j) * 1024);
      }
    }
  };

  auto advance = [&]() {
    if (MODE == MODE_FWD && FASTC) {
      t_c += BK;
      if (t_c >= p.Cg) { t_c = 0; if (++t_s == p.S) { t_s = 0; ++t_r; } }
    }
    if (MODE == MODE_WGRAD) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int q = w_q[j] + d_q, pp = w_p[j] + d_p, im = w_img[j] + d_img;
        if (q >= p.Q) { q -= p.Q; ++pp; }
        if (pp >= p.P) { pp -= p.P; ++im; }
        w_q[j] = q; w_p[j] = pp; w_img[j] = im;
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = ktile_end - ktile_begin;
  if (nt > 0) {
    stage(ktile_begin, 0);
    advance();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      if (t + 1 < nt) { stage(ktile_begin + t + 1, cur ^ 1); advance(); }
      const char* img_n = smem + cur * STAGE_BYTES;
      const char* img_m = img_n + BN * BK * 2;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int nrow = wave_n * 64 + j * 16;
          const int mrow = wave_m * 64 + j * 16;
          if (MODE == MODE_FWD) {
            fa[j] = read_kc(img_n, nrow + (lane & 15), kk * 4 + (lane >> 4));
            fb[j] = read_kc(img_m, mrow + (lane & 15), kk * 4 + (lane >> 4));
          } else {
            fa[j] = read_mn(img_n, nrow, kk * 32, lane);
            fb[j] = read_mn(img_m, mrow, kk * 32, lane);
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[j], fb[i], acc[j][i], 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // ---------------- epilogue ----------------
  // acc[j][i][r]: n = n0 + wave_n*64 + j*16 + (lane>>4)*4 + r ; m = m0 + wave_m*64 + i*16 + (lane&15)
  if (MODE == MODE_FWD) {
    u16* y = reinterpret_cast<u16*>(p.y);
    const int ncol_base = n0 + wave_n * 64 + (lane >> 4) * 4;
    const int64_t goff_y = (int64_t)grp * p.N;
    const bool vec_ok = ((p.N & 3) == 0) && ((p.ldy & 3) == 0) && ((goff_y & 3) == 0);
    float bsum[4][4], bsq[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { bsum[j][r] = 0.f; bsq[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wave_m * 64 + i * 16 + (lane & 15);
      if (m >= p.M) continue;
      const int img = m / (p.P * p.Q), rem = m - img * (p.P * p.Q);
      const int pp = rem / p.Q, qq = rem - pp * p.Q;
      const int64_t opix = ((int64_t)img * p.OH + pp * p.osh + p.oph) * p.OW + qq * p.osw + p.opw;
      u16* yrow = y + opix * p.ldy + goff_y;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = ncol_base + j * 16;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t = acc[j][i][r];
          if (p.bias && n + r < p.N) t += p.bias[grp * p.N + n + r];
          if (p.act == ACT_RELU) t = fmaxf(t, 0.f);
          else if (p.act == ACT_LEAKY) t = t > 0.f ? t : t * p.slope;
          v[r] = t;
          bsum[j][r] += t; bsq[j][r] += t * t;
        }
        if (n + 3 < p.N && vec_ok) {
          uint2 pk; pk.x = pack2bf(v[0], v[1]); pk.y = pack2bf(v[2], v[3]);
          *reinterpret_cast<uint2*>(yrow + n) = pk;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) if (n + r < p.N) yrow[n + r] = f2bf(v[r]);
        }
      }
    }
    if (p.stats) {
      // reduce over the 16 pixels held by a DPP row, then over the 4 rows of the wave
      float* sh = reinterpret_cast<float*>(smem + 2 * STAGE_BYTES);  // [2 wave_m][128 n][2]
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float s1 = row16_sum(bsum[j][r]);
          const float s2 = row16_sum(bsq[j][r]);
          if ((lane & 15) == 0) {
            const int nl = wave_n * 64 + j * 16 + (lane >> 4) * 4 + r;
            sh[(wave_m * 128 + nl) * 2 + 0] = s1;
            sh[(wave_m * 128 + nl) * 2 + 1] = s2;
          }
        }
      __syncthreads();
      if (tid < BN) {
        const int n = n0 + tid;
        if (n < p.N) {
          const float s1 = sh[tid * 2] + sh[(128 + tid) * 2];
          const float s2 = sh[tid * 2 + 1] + sh[(128 + tid) * 2 + 1];
          const int64_t ncols = (int64_t)p.G * p.N;
          float* a = p.stats + (int64_t)(tm % DV_STAT_SHARDS) * 2 * ncols;
          atomicAdd(a + grp * p.N + n, s1);
          atomicAdd(a + ncols + grp * p.N + n, s2);
        }
      }
    }
  } else {
    // WGRAD: stage the fp32 tile through LDS so global writes / atomics are 256-B rows.
    float* T = reinterpret_cast<float*>(smem);  // [128 m][WG_F32_LD]
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int nl = wave_n * 64 + j * 16 + (lane >> 4) * 4;
        const int ml = wave_m * 64 + i * 16 + (lane & 15);
        *reinterpret_cast<f32x4*>(&T[ml * WG_F32_LD + nl]) = acc[j][i];
      }
    __syncthreads();
    float* dwp = reinterpret_cast<float*>(p.y) + (int64_t)grp * p.M * p.N;
    for (int rr = wid; rr < BM; rr += 4) {
      const int m = m0 + rr;
      if (m >= p.M) break;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int nl = h * 64 + lane, n = n0 + nl;
        if (n < p.N) {
          const float v = T[rr * WG_F32_LD + nl];
          float* dst = dwp + (int64_t)m * p.N + n;
          if (p.atomic_out) atomicAdd(dst, v); else *dst = v;
        }
      }
    }
  }
}

}  // namespace

// ----------------------------------------------------------------------------------
// host launchers
// ----------------------------------------------------------------------------------

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

template <int MODE, bool FASTC, bool TGATHER>
static void launch(const Params& p, int nblocks, hipStream_t st) {
  static_assert(LDS_BYTES >= BM * WG_F32_LD * 4, "wgrad epilogue tile must fit");
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)igemm_kernel<MODE, FASTC, TGATHER>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr_set = true;
  }
  hipLaunchKernelGGL((igemm_kernel<MODE, FASTC, TGATHER>), dim3(nblocks), dim3(NTHREADS), LDS_BYTES, st, p);
}

int dv_conv_fwd(const ConvFwdArgs& a, hipStream_t st) {
  Params p{};
  p.x = (const u16*)a.x; p.w = (const u16*)a.w; p.y = a.y;
  p.bias = a.bias; p.stats = a.stats;
  p.G = a.G; p.M = a.Nb * a.P * a.Q; p.N = a.Kout; p.K = a.R * a.S * a.Cg;
  p.Hin = a.H; p.Win = a.W; p.Cg = a.Cg; p.ldx = a.ldx;
  p.P = a.P; p.Q = a.Q; p.R = a.R; p.S = a.S;
  p.sh = a.sh; p.sw = a.sw; p.ph = a.ph; p.pw = a.pw; p.dh = a.dh; p.dw = a.dw;
  p.OH = a.OH; p.OW = a.OW; p.osh = a.osh; p.osw = a.osw; p.oph = a.oph; p.opw = a.opw; p.ldy = a.ldy;
  p.act = a.act; p.slope = a.slope;
  if (p.Cg % 8 != 0 || p.ldx % 8 != 0) return -1;
  const int tiles = cdiv(p.M, BM) * cdiv(p.N, BN) * p.G;
  const bool fastc = (p.Cg % BK) == 0;
  if (a.tgather) {
    if (fastc) launch<MODE_FWD, true, true>(p, tiles, st); else launch<MODE_FWD, false, true>(p, tiles, st);
  } else {
    if (fastc) launch<MODE_FWD, true, false>(p, tiles, st); else launch<MODE_FWD, false, false>(p, tiles, st);
  }
  return 0;
}

int dv_conv_stats_tiles(int Nb, int P, int Q) { return cdiv(Nb * P * Q, BM); }

int dv_conv_wgrad_splits(const ConvWgradArgs& a) {
  const int M = a.Kout, N = a.R * a.S * a.Cg, K = a.Nb * a.P * a.Q;
  const int tiles = cdiv(M, BM) * cdiv(N, BN) * a.G;
  const int ktiles = cdiv(K, BK);
  int splits = cdiv(1024, tiles);                       // aim ~4 blocks per CU
  splits = std::min(splits, std::max(1, ktiles / 32));  // >=2048-deep K per split (atomic budget)
  splits = std::max(1, std::min(splits, ktiles));
  return splits;
}

int dv_conv_wgrad(const ConvWgradArgs& a, hipStream_t st) {
  Params p{};
  p.x = (const u16*)a.x; p.w = (const u16*)a.dy; p.y = a.dw;
  p.G = a.G; p.M = a.Kout; p.N = a.R * a.S * a.Cg; p.K = a.Nb * a.P * a.Q;
  p.Hin = a.H; p.Win = a.W; p.Cg = a.Cg; p.ldx = a.ldx; p.ldm = a.ldy;
  p.P = a.P; p.Q = a.Q; p.R = a.R; p.S = a.S;
  p.sh = a.sh; p.sw = a.sw; p.ph = a.ph; p.pw = a.pw; p.dh = a.dh; p.dw = a.dw_;
  if (p.Cg % 8 != 0 || p.ldx % 8 != 0 || p.ldm % 8 != 0) return -1;
  const int ktiles = cdiv(p.K, BK);
  int splits = a.splits > 0 ? a.splits : dv_conv_wgrad_splits(a);
  p.splits = splits;
  p.ktiles_per_split = cdiv(ktiles, splits);
  p.splits = cdiv(ktiles, p.ktiles_per_split);
  p.atomic_out = p.splits > 1 ? 1 : 0;
  if (p.atomic_out) hipMemsetAsync(a.dw, 0, (size_t)p.G * p.M * p.N * sizeof(float), st);
  const int tiles = cdiv(p.M, BM) * cdiv(p.N, BN) * p.G * p.splits;
  launch<MODE_WGRAD, false, false>(p, tiles, st);
  return p.splits;
}
