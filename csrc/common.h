// Shared device helpers for the deep_vision_amd gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in csrc/:
//   * Activations are bf16, physically NHWC ("channels_last"), logically NCHW in PyTorch.
//   * Weights handed to MFMA kernels are bf16 [Cout][R][S][Cin] (K-contiguous rows).
//   * Statistics / optimizer state / master weights are fp32.
//   * Wave size is 64 (hard-coded, never warpSize arithmetic on 32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DV_DEVICE __device__ __forceinline__

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))
#define GLB_PTR(p) ((const __attribute__((address_space(1))) void*)(p))

// ---- bf16 <-> fp32 (round-to-nearest-even; NaN preserved by the hardware cvt path) ----
DV_DEVICE float bf2f(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }
DV_DEVICE u16 f2bf(float f) {
  __bf16 b = (__bf16)f;  // hipcc emits v_cvt_pk_bf16_f32 at -O3 (RNE, NaN-safe)
  return __builtin_bit_cast(u16, b);
}
// one v_cvt_pk_bf16_f32 (the scalar-pair form f2bf(a) | f2bf(b) << 16 was sometimes emitted as
// two packed converts plus and/or/sdwa re-shuffles)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
DV_DEVICE uint32_t pack2bf(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}

// ---- wave / block reductions (wave64) ----
DV_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DV_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Sum within each 16-lane row via DPP (all 16 lanes receive the row sum).
DV_DEVICE float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false)); // row_ror:4
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false)); // row_ror:8
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `sh` needs NT/64 floats.
template <int NT>
DV_DEVICE float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += sh[i];
  return t;
}

// ---- XCD-aware bijective block remap (MI355X: 8 XCDs, blocks dealt round-robin) ----
// Consecutive *logical* tiles land on the same XCD so that tiles sharing an operand
// panel hit the same L2. Bijective for any nwg (see cdna_hip_programming.md §5).
DV_DEVICE int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + loc;
}

// Magic-number unsigned division for 0 <= n < 2^31 (Granlund-Montgomery): q = (umulhi(n,m)+n) >> s.
// Replaces the ~40-instruction integer division in index decodes (pixel -> (img, p, q)).
struct FastDiv {
  uint32_t mul, shr, d;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f{0u, 0u, d};
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.shr = l;
  f.mul = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1ull);
  return f;
}
DV_DEVICE uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.mul) + n) >> f.shr; }

// 16-byte aligned zero page used as the source address of padded / out-of-range
// LDS-DMA lanes (global_load_lds cannot predicate a lane to "write zeros"). One copy per
// translation unit: device code is not relocatable across TUs (no -fgpu-rdc).
static __device__ __attribute__((aligned(16))) char dv_zero_page[256];

#define DV_CHECK_LAUNCH() (void)hipGetLastError()

// Per-channel shift row of a forward BatchNorm statistics accumulator of `ncols` channels
// (layout: kernels.h DV_STAT_ROWS; 64 = DV_STAT_SHARDS, asserted there).
DV_DEVICE float* stat_shift(float* acc, int64_t ncols) { return acc + (int64_t)2 * 64 * ncols; }
// The [2][ncols] partial-sum row a block with reduction index `blk` adds into: shard blk % 64 of
// the accumulator, or -- deterministic mode (kernels.h DetStats) -- its own row of the launch's
// zeroed slab (one contribution per element, folded in a fixed order afterwards).
DV_DEVICE float* stat_row(float* acc, float* det, int64_t blk, int64_t ncols) {
  return det ? det + blk * 2 * ncols : acc + (blk % 64) * 2 * ncols;
}
