// Stem convolutions (first layer, <= 4 input channels, 7x7, 64 output channels: ResNet-50 /
// ResNet-152 / Inception V1 / Hourglass, R/ResNet/pytorch/models/resnet50.py:60-64) as
// row-walking MFMA kernels on a sliding LDS window of input rows.
//
// Input: the tap-packed image of ops/conv.py _StemConvFn, [N][Hp][Wp][4] bf16, pre-padded; a
// 16-B chunk = 2 adjacent pixels x 4 channels. K index k = r*32 + 4*t + c (filter row r, tap
// t < 8, channel c < 4); weights [64][R][8][4] bf16.
//
// Why not the generic implicit-GEMM kernel (conv_fwd.hip packed mode): its M x K tiles gather
// every pixel's 7 x 64-B filter-row slices through LDS-DMA, re-reading each input chunk ~14x and
// re-staging the 28 KB weight tile for every 256 pixels; the tile loop is 7 K-steps deep, so
// each block is latency-bound (13.7 % MFMA busy, 84 % LDS bank conflicts:
// profiles/pmc_stem_conv.txt). Here
//   * a block owns a run of output rows of one image and walks them; the input rows it needs
//     live in a ring of LDS row slots filled by LDS-DMA (each input row is fetched ONCE per
//     block: sh new rows per output row), one group ahead of the compute;
//   * forward: the whole weight matrix sits in VGPRs as 16x16x32 MFMA A-fragments (4 channel
//     fragments x 7 filter rows); the pixel operand is ONE conflict-free ds_read_b128 per filter
//     row straight out of the input-row slot (chunk (sw*q + 2*(lane>>4)) of pixel q), no im2col;
//     BatchNorm statistics accumulate in registers for the block's whole lifetime (one atomic row
//     per block instead of one per 256-pixel tile);
//   * weight gradient: the output-gradient row is staged once per output row (XOR-swizzled 128-B
//     rows); 32x32x16 MFMAs take dY^T and the input window through ds_read_b64_tr_b16 transposed
//     reads (the overlapping 64-B "rows" of the packed image are valid tr-read rows), each wave
//     owns two filter rows; per-block fp32 partials go to a slab and one reduce pass sums them into
//     the parameter's [O][C][R][S] gradient (no atomics on the hot path, no unprep pass).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int SR = 7;        // filter rows handled by these kernels (7x7 stems)
constexpr int RG = 4;        // output rows per forward group
constexpr int NR_W = 16;     // weight-gradient ring slots: R + 3*sh (three output rows ahead)
constexpr int NDY = 4;       // weight-gradient dY row buffers (three in flight behind the one in use)
constexpr int OC = 64;       // output channels

struct StemParams {
  const u16* x;      // packed image [N][Hp][Wp][4]
  const u16* w;      // forward: [64][R][8][4] bf16
  u16* y;            // forward output NHWC [N][P][Q][64]
  const u16* dy;     // weight gradient: NHWC [N][P][Q][64]
  float* slab;       // weight gradient partials [blocks][64][R][32]
  const float* bias;
  float* stats;      // [SHARDS][2][64] + shift row, or nullptr
  float* sdet;       // deterministic mode: per-block slab rows (kernels.h DetStats), or nullptr
  int act; float slope;
  int Hp, Wp, P, Q, sh, sw;
  int rowbytes;      // Wp * 8
  int rowb;          // LDS slot pitch (multiple of 1024)
  int ipr;           // 1-KB DMA pieces per row
  int chunks, rpb;   // blocks per image, output rows per block
};

// LDS-DMA of one 1-KB wave piece (M0 set and restored inside the statement, cf. conv_wgrad.hip:
// the asm form keeps hipcc from treating the in-flight DMA as aliasing the LDS reads)
DV_DEVICE void glds16(const void* src, uint32_t dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory");
}

// input rows [r0, r0 + cnt) of image `xim` into their ring slots (row % NR): piece t of the
// cnt * ipr 1-KB pieces goes to wave t % NW; returns this wave's DMA count
template <int NR, int NW>
DV_DEVICE int load_rows(const StemParams& p, const char* xim, uint32_t ring, int r0, int cnt, int wid, int lane) {
  const void* zpage = dv_zero_page;
  int t = 0, n = 0;
  for (int rr = 0; rr < cnt; ++rr) {
    const int row = r0 + rr;
    const uint32_t slot = ring + (uint32_t)(((unsigned)row % NR) * p.rowb);
    for (int pc = 0; pc < p.ipr; ++pc, ++t) {
      if (t % NW != wid) continue;
      const int off = pc * 1024 + lane * 16;
      const bool ok = row < p.Hp && off < p.rowbytes;
      const void* src = ok ? (const void*)(xim + (int64_t)row * p.rowbytes + off) : zpage;
      glds16(src, slot + pc * 1024);
      ++n;
    }
  }
  return n;
}

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left at their maxima (gfx9 encoding)
template <int N>
DV_DEVICE void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}
// exact vmcnt(n) for a wave-uniform runtime n (a jump table of immediates); n >= 63 waits to 62
DV_DEVICE void wait_vm_dyn(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    case 7: wait_vm<7>(); break;
    case 8: wait_vm<8>(); break;
    case 9: wait_vm<9>(); break;
    case 10: wait_vm<10>(); break;
    case 11: wait_vm<11>(); break;
    case 12: wait_vm<12>(); break;
    case 13: wait_vm<13>(); break;
    case 14: wait_vm<14>(); break;
    case 15: wait_vm<15>(); break;
    case 16: wait_vm<16>(); break;
    case 17: wait_vm<17>(); break;
    case 18: wait_vm<18>(); break;
    case 19: wait_vm<19>(); break;
    case 20: wait_vm<20>(); break;
    case 21: wait_vm<21>(); break;
    case 22: wait_vm<22>(); break;
    case 23: wait_vm<23>(); break;
    case 24: wait_vm<24>(); break;
    case 25: wait_vm<25>(); break;
    case 26: wait_vm<26>(); break;
    case 27: wait_vm<27>(); break;
    case 28: wait_vm<28>(); break;
    case 29: wait_vm<29>(); break;
    case 30: wait_vm<30>(); break;
    case 31: wait_vm<31>(); break;
    case 32: wait_vm<32>(); break;
    case 33: wait_vm<33>(); break;
    case 34: wait_vm<34>(); break;
    case 35: wait_vm<35>(); break;
    case 36: wait_vm<36>(); break;
    case 37: wait_vm<37>(); break;
    case 38: wait_vm<38>(); break;
    case 39: wait_vm<39>(); break;
    case 40: wait_vm<40>(); break;
    case 41: wait_vm<41>(); break;
    case 42: wait_vm<42>(); break;
    case 43: wait_vm<43>(); break;
    case 44: wait_vm<44>(); break;
    case 45: wait_vm<45>(); break;
    case 46: wait_vm<46>(); break;
    case 47: wait_vm<47>(); break;
    case 48: wait_vm<48>(); break;
    case 49: wait_vm<49>(); break;
    case 50: wait_vm<50>(); break;
    case 51: wait_vm<51>(); break;
    case 52: wait_vm<52>(); break;
    case 53: wait_vm<53>(); break;
    case 54: wait_vm<54>(); break;
    case 55: wait_vm<55>(); break;
    case 56: wait_vm<56>(); break;
    case 57: wait_vm<57>(); break;
    case 58: wait_vm<58>(); break;
    case 59: wait_vm<59>(); break;
    case 60: wait_vm<60>(); break;
    case 61: wait_vm<61>(); break;
    case 62: wait_vm<62>(); break;
    default: wait_vm<62>(); break;
  }
}

enum { SE_STATS = 0, SE_FULL = 1 };

// ---------------------------------------------------------------- forward
// Stride-2 stems (ResNet / Inception / Hourglass). A group of RG output rows reads a window of
// FWIN = 2*(RG-1) + 7 input rows; each group's window is loaded whole into one of NWB buffers
// (two groups ahead of the compute) at a compile-time row pitch ROWB, so a fragment's 7
// filter-row reads are one VGPR base + immediate offsets. FULLQ: Q % 16 == 0 (no lane masking).
constexpr int FWIN = 2 * (RG - 1) + SR;
constexpr int NWB = 3;
template <int EPI, bool FULLQ, int ROWB>
__global__ __launch_bounds__(256, 2) void stem_fwd_kernel(StemParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int SW = 2, FSTRIDE = 128 * SW, WBYTES = FWIN * ROWB;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int img = blockIdx.x / p.chunks, chunk = blockIdx.x - img * p.chunks;
  const int p0 = chunk * p.rpb, p1 = min(p.P, p0 + p.rpb);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
  const char* xim = reinterpret_cast<const char*>(p.x) + (int64_t)img * p.Hp * p.rowbytes;
  const void* zpage = dv_zero_page;

  // weights as A-fragments: lane holds W[n = 16j + (lane&15)][k = 32r + 8(lane>>4) .. +7]
  bf16x8 wf[4][SR];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < SR; ++r)
      wf[j][r] = *reinterpret_cast<const bf16x8*>(p.w + (16 * j + (lane & 15)) * (SR * 32) + r * 32 + 8 * (lane >> 4));
  // this lane's 16 channels: n = 16j + 4(lane>>4) + e
  float kq[4][4], bv[4][4], s1[4][4], s2[4][4];
  const bool st = p.stats != nullptr;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = 16 * j + 4 * (lane >> 4) + e;
      kq[j][e] = st ? stat_shift(p.stats, OC)[n] : 0.f;
      bv[j][e] = (EPI == SE_FULL && p.bias) ? p.bias[n] : 0.f;
      s1[j][e] = 0.f; s2[j][e] = 0.f;
    }

  // window of the group starting at output row pg -> buffer gi % NWB (piece t to wave t % 4)
  auto load_win = [&](int pg, int gi) {
    const uint32_t base = lds0 + (uint32_t)((gi % NWB) * WBYTES);
    int t = 0, n = 0;
    for (int rr = 0; rr < FWIN; ++rr) {
      const int row = 2 * pg + rr;
      for (int pc = 0; pc < p.ipr; ++pc, ++t) {
        if ((t & 3) != wid) continue;
        const int off = pc * 1024 + lane * 16;
        const bool ok = row < p.Hp && off < p.rowbytes;
        glds16(ok ? (const void*)(xim + (int64_t)row * p.rowbytes + off) : zpage, base + rr * ROWB + pc * 1024);
        ++n;
      }
    }
    return n;
  };

  const int QF = (p.Q + 15) >> 4;
  const int colb0 = 8 * SW * (lane & 15) + 16 * (lane >> 4);  // pixel (lane&15), chunk 2*(lane>>4)
  const int yoff = (lane & 15) * OC + 4 * (lane >> 4);       // channel group 4*(lane>>4) of that pixel
  // pipeline: group g+2's window is issued while group g computes; before group g every
  // vector-memory op this wave issued in the previous iteration (group g+1's window, group g-1's
  // output stores) may stay in flight -- the exact counted vmcnt retires group g's window
  load_win(p0, 0);
  if (p0 + RG < p1) load_win(p0 + RG, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int pend = 0;
  for (int pg = p0, gi = 0; pg < p1; pg += RG, ++gi) {
    wait_vm_dyn(pend);
    __syncthreads();
    pend = 0;
    if (pg + 2 * RG < p1) pend = load_win(pg + 2 * RG, gi + 2);
    const int nf = min(RG, p1 - pg) * QF;
    const int myf = wid < nf ? (nf - wid + 3) / 4 : 0;  // fragments wid, wid+4, ...
    pend += 4 * myf;                                    // 4 output stores per fragment
    const char* win = smem + (gi % NWB) * WBYTES + colb0;
    int pl = 0, qf = wid;
    while (qf >= QF) { qf -= QF; ++pl; }
    // the 7 filter-row operands of fragment (pl, qf)
    auto rd = [&](int pl_, int qf_, bf16x8* xf) {
      int cb = 2 * pl_ * ROWB + qf_ * FSTRIDE;
      if constexpr (!FULLQ) cb = min(cb, 2 * pl_ * ROWB + 8 * SW * (p.Q - 1 - (lane & 15)));
      const char* xr = win + cb;
#pragma unroll
      for (int r = 0; r < SR; ++r) xf[r] = *reinterpret_cast<const bf16x8*>(xr + r * ROWB);
    };
    // software-pipelined: the next fragment's LDS reads are issued before this one's epilogue
    bf16x8 xf[SR];
    if (myf > 0) rd(pl, qf, xf);
    for (int i = 0; i < myf; ++i) {
      f32x4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][0], xf[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
      for (int r = 1; r < SR; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][r], xf[r], acc[j], 0, 0, 0);
      const int cpl = pl, cqf = qf;
      qf += 4;
      while (qf >= QF) { qf -= QF; ++pl; }
      if (i + 1 < myf) rd(pl, qf, xf);
      // D[n][q]: lane holds channels 16j + 4(lane>>4) + e of pixel q
      const bool valid = FULLQ || cqf * 16 + (lane & 15) < p.Q;
      u16* dst = p.y + (((int64_t)img * p.P + pg + cpl) * p.Q + cqf * 16) * OC + yoff;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = acc[j][e];
          if constexpr (EPI == SE_FULL) {
            t += bv[j][e];
            if (p.act == 1) t = fmaxf(t, 0.f);
            else if (p.act == 2) t = t > 0.f ? t : t * p.slope;
          }
          v[e] = t;
          const float d = valid ? t - kq[j][e] : 0.f;
          s1[j][e] += d; s2[j][e] = fmaf(d, d, s2[j][e]);
        }
        uint2 pk; pk.x = pack2bf(v[0], v[1]); pk.y = pack2bf(v[2], v[3]);
        if (valid) *reinterpret_cast<uint2*>(dst + 16 * j) = pk;
      }
    }
  }
  if (!st) return;
  __syncthreads();
  // lanes of one 16-lane row share channels: DPP row sums, then the 4 waves meet in LDS
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][64][2]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = row16_sum(s1[j][e]), b = row16_sum(s2[j][e]);
      if ((lane & 15) == 0) {
        const int n = 16 * j + 4 * (lane >> 4) + e;
        red[(wid * OC + n) * 2 + 0] = a;
        red[(wid * OC + n) * 2 + 1] = b;
      }
    }
  __syncthreads();
  if (threadIdx.x < OC) {
    const int n = threadIdx.x;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { a += red[(w * OC + n) * 2]; b += red[(w * OC + n) * 2 + 1]; }
    float* sh = stat_row(p.stats, p.sdet, blockIdx.x, OC);
    atomicAdd(sh + n, a);
    atomicAdd(sh + OC + n, b);
  }
}

// ---------------------------------------------------------------- weight gradient
typedef float f32x16 __attribute__((ext_vector_type(16)));

DV_DEVICE int dy_swz(int px) { return ((px >> 1) & 1) << 2; }  // 16-B chunk XOR of dY row px

DV_DEVICE bf16x8 tr_pair(const char* a1, const char* a2) {
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)LDS_PTR(a1));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)LDS_PTR(a2));
  i16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

// 8 waves: wave w owns filter rows {2(w&3), 2(w&3)+1} and the 16-pixel steps of parity w>>2 (two
// waves per SIMD hide each other's LDS latency); the two parities meet in LDS at the end
constexpr int WG_NW = 8;
template <bool FULLQ>
__global__ __launch_bounds__(512, 1) void stem_wgrad_kernel(StemParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int img = blockIdx.x / p.chunks, chunk = blockIdx.x - img * p.chunks;
  const int p0 = chunk * p.rpb, p1 = min(p.P, p0 + p.rpb);
  if (p0 >= p1) {  // never launched so (stem_blocks_ok); keep the slab row defined regardless
    for (int e = threadIdx.x; e < OC * SR * 32; e += blockDim.x) p.slab[(int64_t)blockIdx.x * OC * SR * 32 + e] = 0.f;
    return;
  }
  const int QS = (p.Q + 15) >> 4;           // 16-pixel MFMA k-steps per output row
  const int dyb = QS * 16 * 128;             // bytes of one staged dY row
  const uint32_t ring = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
  const uint32_t dyl = ring + NR_W * p.rowb;  // NDY dY row buffers behind the ring
  const char* xim = reinterpret_cast<const char*>(p.x) + (int64_t)img * p.Hp * p.rowbytes;

  // stage of output row pr: its dY row (8 pixel rows of 128 B per 1-KB piece, chunk XOR-swizzled
  // by pixel) into buffer pr % NDY, and the sh input rows its window adds (the first row's stage
  // loads the whole window). Pieces are dealt round-robin over the waves; returns this wave's DMA
  // count (the same for every row but the first, which the prologue waits out fully).
  auto stage = [&](int pr) {
    const u16* src_row = p.dy + ((int64_t)img * p.P + pr) * p.Q * OC;
    const uint32_t buf = dyl + (uint32_t)((pr % NDY) * dyb);
    int n = 0;
    for (int pc = wid; pc < QS * 2; pc += WG_NW, ++n) {
      const int px = pc * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ dy_swz(px);
      const void* src = (FULLQ || px < p.Q) ? (const void*)(src_row + px * OC + ch * 8) : (const void*)dv_zero_page;
      glds16(src, buf + pc * 1024);
    }
    if (pr == p0) return n + load_rows<NR_W, WG_NW>(p, xim, ring, p.sh * pr, SR, wid, lane);
    return n + load_rows<NR_W, WG_NW>(p, xim, ring, p.sh * pr + SR - p.sh, p.sh, wid, lane);
  };

  // tr-read lane roles: group g = lane>>4, q4 = (lane&15)>>2 (row in the 4-row block), pp = lane&3
  const int g = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3, hh = g >> 1;
  const int wr = wid & 3, par = wid >> 2;
  const int r_a = 2 * wr, r_b = 2 * wr + 1;  // this wave's filter rows
  const bool has_b = r_b < SR;
  // lane-constant byte offsets of the first tr-read of step 0 (pixel row 8hh + q4); step s adds
  // 16 pixel rows (2048 B of dY, 128*sw B of input), the second read 4 pixel rows
  const int px0 = 8 * hh + q4;
  int dya[2];
#pragma unroll
  for (int nh = 0; nh < 2; ++nh) {
    const int col = nh * 32 + 16 * (g & 1) + 4 * pp;  // channel of this lane's 8-B read
    dya[nh] = px0 * 128 + (((col >> 3) ^ dy_swz(px0)) << 4) + (col & 7) * 2;  // swz is the same for px0 + 4 + 16s
  }
  const int xo = 8 * p.sw * px0 + 2 * (16 * (g & 1) + 4 * pp);
  const int xstep = 128 * p.sw, xhalf = 32 * p.sw;
  f32x16 acc[2][2];  // [filter row][channel half]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  // pipeline: rows pr+1 .. pr+NDY-2 stay in flight while row pr computes; the counted vmcnt before
  // each row retires exactly that row's stage (every later stage issues `per` DMAs per wave)
  stage(p0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int per = 0;
  for (int k = 1; k < NDY - 1 && p0 + k < p1; ++k) per = stage(p0 + k);
  for (int pr = p0; pr < p1; ++pr) {
    wait_vm_dyn(per * min(NDY - 2, p1 - 1 - pr));
    __syncthreads();  // row pr landed for every wave; row pr-1's buffers are free
    if (pr + NDY - 1 < p1) stage(pr + NDY - 1);
    const char* dimg = smem + NR_W * p.rowb + (pr % NDY) * dyb;
    const char* xa = smem + ((p.sh * pr + r_a) % NR_W) * p.rowb + xo;
    const char* xb = smem + ((p.sh * pr + (has_b ? r_b : r_a)) % NR_W) * p.rowb + xo;
    for (int s = par; s < QS; s += 2) {
      bf16x8 fa[2], fxa, fxb;
#pragma unroll
      for (int nh = 0; nh < 2; ++nh) fa[nh] = tr_pair(dimg + dya[nh] + s * 2048, dimg + dya[nh] + s * 2048 + 512);
      int o1 = s * xstep, o2 = o1 + xhalf;
      if constexpr (!FULLQ) {  // pixels past Q (zero dY rows) read a valid pixel of the row
        const int lim = 8 * p.sw * (p.Q - 1 - px0);
        o1 = min(o1, lim); o2 = min(o2, lim);
      }
      fxa = tr_pair(xa + o1, xa + o2);
      fxb = tr_pair(xb + o1, xb + o2);
#pragma unroll
      for (int nh = 0; nh < 2; ++nh) {
        acc[0][nh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[nh], fxa, acc[0][nh], 0, 0, 0);
        if (has_b) acc[1][nh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[nh], fxb, acc[1][nh], 0, 0, 0);
      }
    }
  }
  // the two step parities meet in LDS (the staging area is free after the loop), then
  // D[n][kcol] -> slab: lane holds kcol = lane&31, n = nh*32 + (e&3) + 8(e>>2) + 4(lane>>5)
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [4 row pairs][2][2][16][64]
  if (par) {
#pragma unroll
    for (int ri = 0; ri < 2; ++ri)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int e = 0; e < 16; ++e) red[(((wr * 2 + ri) * 2 + nh) * 16 + e) * 64 + lane] = acc[ri][nh][e];
  }
  __syncthreads();
  if (par) return;
  float* sl = p.slab + (int64_t)blockIdx.x * OC * SR * 32;
#pragma unroll
  for (int ri = 0; ri < 2; ++ri) {
    const int r = ri ? r_b : r_a;
    if (r >= SR) continue;
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = nh * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        sl[(n * SR + r) * 32 + (lane & 31)] = acc[ri][nh][e] + red[(((wr * 2 + ri) * 2 + nh) * 16 + e) * 64 + lane];
      }
  }
}

// dw[n][c][r][t] (+)= sum over blocks of slab[b][n][r][4t + c]: blockIdx.y splits the blocks,
// each thread one slab element over its share, atomically added (dw zeroed or accumulating)
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ slab, int nblk, int per,
                                                                float* __restrict__ dw, int C, int S) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // (n, r, kcol)
  if (i >= OC * SR * 32) return;
  const int kc = i & 31, t = kc >> 2, c = kc & 3;
  if (t >= S || c >= C) return;
  const int nr = i >> 5, n = nr / SR, r = nr - n * SR;
  const int b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  float v = 0.f;
  for (int b = b0; b < b1; ++b) v += slab[(int64_t)b * OC * SR * 32 + i];
  atomicAdd(dw + ((n * C + c) * SR + r) * S + t, v);
}

int g_stem_blocks = 512;     // forward target grid (2 blocks per CU); tuning override
int g_stem_wg_blocks = 256;  // weight-gradient target grid (1 block per CU: 88 KB of LDS)

bool stem_setup(StemParams& p, int N, int Hp, int Wp, int P, int Q, int sh, int sw, int target) {
  p.Hp = Hp; p.Wp = Wp; p.P = P; p.Q = Q; p.sh = sh; p.sw = sw;
  p.rowbytes = Wp * 8;
  p.ipr = (p.rowbytes + 1023) / 1024;
  p.rowb = p.ipr * 1024;
  // window fits the rings; pixels read stay inside a row slot (sw*(Q-1) + 8 taps <= Wp)
  if (sh < 1 || sh > 4 || (sw & 1) || sw * (Q - 1) + 8 > Wp || Hp < (P - 1) * sh + SR) return false;
  p.chunks = std::max(1, std::min(P, (target + N - 1) / N));
  p.rpb = (P + p.chunks - 1) / p.chunks;
  p.chunks = (P + p.rpb - 1) / p.rpb;  // every block owns >= 1 output row (chunks * rpb may not overshoot P by a row)
  return true;
}
// block b of image b / chunks owns output rows [c * rpb, min(P, (c + 1) * rpb)): non-empty for every c
inline bool stem_blocks_ok(const StemParams& p) { return p.rpb >= 1 && (p.chunks - 1) * p.rpb < p.P; }

template <int EPI, bool FULLQ, int ROWB>
void launch_fwd(const StemParams& p, dim3 grid, hipStream_t st) {
  constexpr int lds = NWB * FWIN * ROWB;  // 78 KB at ROWB 2048: two blocks per CU
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)stem_fwd_kernel<EPI, FULLQ, ROWB>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  stem_fwd_kernel<EPI, FULLQ, ROWB><<<grid, 256, lds, st>>>(p);
}

template <bool FULLQ>
void launch_wg(const StemParams& p, int nblk, size_t lds, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)stem_wgrad_kernel<FULLQ>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    attr = true;
  }
  stem_wgrad_kernel<FULLQ><<<dim3(nblk), 64 * WG_NW, lds, st>>>(p);
}

}  // namespace

void dv_stem_tuning(int blocks, int wg_blocks) {
  g_stem_blocks = blocks > 0 ? blocks : 512;
  g_stem_wg_blocks = wg_blocks > 0 ? wg_blocks : 256;
}

int dv_stem_fwd(const void* xp, const void* w, void* y, const float* bias, float* stats, int act, float slope, int N,
                int Hp, int Wp, int P, int Q, int R, int Sp, int K, int sh, int sw, hipStream_t st) {
  if (R != SR || Sp != 8 || K != OC || sh != 2 || sw != 2) return -1;
  StemParams p{};
  if (!stem_setup(p, N, Hp, Wp, P, Q, sh, sw, g_stem_blocks)) return -1;
  if (p.rowbytes > 3072) return -1;
  p.rpb = (p.rpb + RG - 1) / RG * RG;  // whole groups
  p.chunks = (P + p.rpb - 1) / p.rpb;
  if (!stem_blocks_ok(p)) return -1;
  p.x = (const u16*)xp; p.w = (const u16*)w; p.y = (u16*)y; p.bias = bias; p.stats = stats;
  p.act = act; p.slope = slope;
  const bool full = bias || act, fq = Q % 16 == 0;
  const dim3 grid(N * p.chunks);
  const DetStats det(stats ? grid.x : 0, OC, st);
  p.sdet = det.slab;
  if (p.rowbytes <= 2048) {
    if (full) { if (fq) launch_fwd<SE_FULL, true, 2048>(p, grid, st); else launch_fwd<SE_FULL, false, 2048>(p, grid, st); }
    else { if (fq) launch_fwd<SE_STATS, true, 2048>(p, grid, st); else launch_fwd<SE_STATS, false, 2048>(p, grid, st); }
  } else {
    if (full) { if (fq) launch_fwd<SE_FULL, true, 3072>(p, grid, st); else launch_fwd<SE_FULL, false, 3072>(p, grid, st); }
    else { if (fq) launch_fwd<SE_STATS, true, 3072>(p, grid, st); else launch_fwd<SE_STATS, false, 3072>(p, grid, st); }
  }
  det.fold(stats);
  return 0;
}

int dv_stem_wgrad(const void* xp, const void* dy, int ldy, float* dw, int N, int C, int S, int Hp, int Wp, int P, int Q,
                  int R, int Sp, int K, int sh, int sw, hipStream_t st) {
  if (R != SR || Sp != 8 || K != OC || ldy != OC || C > 4 || S > 8) return -1;
  StemParams p{};
  if (!stem_setup(p, N, Hp, Wp, P, Q, sh, sw, g_stem_wg_blocks)) return -1;
  if (!stem_blocks_ok(p)) return -1;
  p.x = (const u16*)xp; p.dy = (const u16*)dy;
  const int QS = (Q + 15) / 16;
  // staging (input ring + dY buffers), at least the end-of-kernel parity reduction [4][2][2][16][64] f32
  const size_t lds = std::max((size_t)NR_W * p.rowb + NDY * (size_t)QS * 16 * 128, (size_t)4 * 2 * 2 * 16 * 64 * 4);
  if (lds > 150 * 1024) return -1;
  const int nblk = N * p.chunks;
  const size_t slab_elems = (size_t)nblk * OC * SR * 32;
  p.slab = dv_slab_workspace(slab_elems, st);
  if (!p.slab) return -1;
  if (Q % 16 == 0) launch_wg<true>(p, nblk, lds, st);
  else launch_wg<false>(p, nblk, lds, st);
  // deterministic mode: one y-block sums every block's slab in order (one atomic per element)
  const int per = dv_deterministic() ? nblk : 16;
  const dim3 rg((OC * SR * 32 + 255) / 256, (nblk + per - 1) / per);
  stem_wgrad_reduce_kernel<<<rg, 256, 0, st>>>(p.slab, nblk, per, dw, C, S);
  return 0;
}
