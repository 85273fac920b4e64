// MFMA shape micro-benchmark ("add v_mfma_f32_32x32x16_bf16 wave tiles ... halves
// the LDS fragment reads per FLOP"). Measures, on one MI355X, a 64x64 wave tile's K loop built
// from each bf16 MFMA shape with every operand fragment re-read from LDS (ds_read_b128) as the conv
// kernels do:
//   16x16x32: per K=32 step, 4 A + 4 B fragments (8 x 16 B per lane), 16 MFMAs
//   32x32x16: per K=32 step, 2 x (2 A + 2 B) fragments (8 x 16 B per lane), 8 MFMAs
// Both read the same 8 KB of LDS per wave per K=32 (the operand bytes of a 64x64 tile do not depend
// on the instruction shape), so the comparison is the instructions' own throughput.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/mfma_shape_bench.hip -o /tmp/mfma_shape_bench
// run:   /tmp/mfma_shape_bench            (prints TFLOP/s per shape at 1 and 2 waves per SIMD)
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((__vector_size__(8 * sizeof(short)))) short bf16x8;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;

constexpr int KSTEPS = 2048;  // K = 32 * KSTEPS per wave

// 64x64 wave tile from 16x16x32: acc[4][4] of f32x4
__global__ __launch_bounds__(256) void tile16(float* out, int salt) {
  __shared__ __attribute__((aligned(16))) char lds[64 * 1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 64 * 1024 / 4; i += 256) reinterpret_cast<int*>(lds)[i] = (i * 2654435761u + salt) & 0x3f7f3f7f;
  __syncthreads();
  f32x4 acc[4][4] = {};
  const char* base = lds + wid * 16384;
  for (int k = 0; k < KSTEPS; ++k) {
    const int o = ((k * salt) & 3) * 2048;  // runtime pattern: no fragment reuse across steps
    bf16x8 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(base + o + ((i * 64 + lane) * 16 & 2047));
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(base + 1024 + o + ((j * 64 + lane) * 16 & 2047));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// 64x64 wave tile from 32x32x16: acc[2][2] of f32x16, two K=16 halves per K=32 step
__global__ __launch_bounds__(256) void tile32(float* out, int salt) {
  __shared__ __attribute__((aligned(16))) char lds[64 * 1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 64 * 1024 / 4; i += 256) reinterpret_cast<int*>(lds)[i] = (i * 2654435761u + salt) & 0x3f7f3f7f;
  __syncthreads();
  f32x16 acc[2][2] = {};
  const char* base = lds + wid * 16384;
  for (int k = 0; k < KSTEPS; ++k) {
    const int o = ((k * salt) & 3) * 2048;  // runtime pattern: no fragment reuse across steps
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const bf16x8*>(base + o + (((h * 2 + i) * 64 + lane) * 16 & 2047));
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const bf16x8*>(base + 1024 + o + (((h * 2 + j) * 64 + lane) * 16 & 2047));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) s += acc[i][j][0] + acc[i][j][15];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K>
static double run(K kern, int blocks, float* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  kern<<<blocks, 256>>>(out, 1);
  (void)hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) kern<<<blocks, 256>>>(out, 2 * r + 1);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double flop = 2.0 * 64 * 64 * 32.0 * KSTEPS * 4 /*waves*/ * blocks * reps;
  return flop / (ms * 1e-3) / 1e12;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  float* out = nullptr;
  (void)hipMalloc(&out, (size_t)cus * 4 * 256 * sizeof(float));
  printf("# 64x64 wave tile, operands re-read from LDS per K step; %d CUs; TFLOP/s (dense bf16)\n", cus);
  for (int per_cu = 1; per_cu <= 2; ++per_cu) {
    const int blocks = cus * per_cu;  // 4 waves per block: per_cu waves per SIMD
    const double t16 = run(tile16, blocks, out), t32 = run(tile32, blocks, out);
    printf("waves/SIMD %d   16x16x32: %7.1f TF/s   32x32x16: %7.1f TF/s   ratio %.3f\n", per_cu, t16, t32, t16 / t32);
  }
  (void)hipFree(out);
  return 0;
}
