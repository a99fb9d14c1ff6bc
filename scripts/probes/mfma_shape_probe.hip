// MFMA shape probe (verdict item 2): can v_mfma_f32_32x32x16_bf16 beat v_mfma_f32_16x16x32_bf16 for
// the ping-pong GEMM's 128x64 wave tile on gfx950?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/mfma_shape_probe.hip -o /tmp/mfma_shape_probe
// Two kernels per shape, 8 waves (2 per SIMD) per workgroup, one workgroup per CU x REP rounds:
//   reg: the MFMAs of a 128x64 x K=32 step from registers, back to back (matrix-pipe throughput and
//        the clock the chip holds under it);
//   lds: the same step fed from LDS like the ping-pong's phase: 12 ds_read_b128 per wave (the same
//        bytes for both shapes: the wave tile sets them), lgkmcnt(0), barrier, MFMAs at priority 1,
//        barrier; the two wave groups a barrier apart (group 1 starts one barrier late).
// Prints TFLOP/s (dense bf16 MACs x 2 / wall time) and the mean core clock from s_memtime.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

__device__ __forceinline__ v4f m16(v8s a, v8s b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}
__device__ __forceinline__ v16f m32(v8s a, v8s b, v16f c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}

// 128x64 wave tile, K = 32 per step. SH 0: acc[8][4] of 16x16 (32 MFMAs of K 32);
// SH 1: acc[4][2] of 32x32 (16 MFMAs: 8 blocks x 2 k16 halves). 128 accumulator VGPRs either way.
template <int SH, bool LDS>
__global__ void __launch_bounds__(512, 1) probe(int iters, float* sink, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) char smem[65536];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, grp = wave >> 2;
  for (int i = threadIdx.x; i < 65536 / 4; i += 512) ((float*)smem)[i] = 0.001f * (i & 255);
  __syncthreads();
  v8s a[8], b[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = *(const v8s*)(smem + (i * 1024 + lane * 16));
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = *(const v8s*)(smem + 8192 + (j * 1024 + lane * 16));
  v4f c16[8][4];
  v16f c32[4][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) c16[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) c32[i][j][r] = 0.f;
  __syncthreads();
  if (LDS && grp == 1) __builtin_amdgcn_s_barrier();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (LDS) {
      // this step's fragments: 12 x 16 B per lane from a rotating 24 KiB window (conflict-free rows)
      const int base = (it & 1) * 24576 + wave * 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = *(const __attribute__((address_space(3))) v8s*)(smem + base + i * 1024 + lane * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *(const __attribute__((address_space(3))) v8s*)(smem + base + 8192 + j * 1024 + lane * 16);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_setprio(1);
    }
    if constexpr (SH == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c16[i][j] = m16(a[i], b[j], c16[i][j]);
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h)  // the two k16 halves of the K-32 step
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) c32[i][j] = m32(a[2 * i + h], b[2 * j + h], c32[i][j]);
    }
    if constexpr (LDS) {
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (LDS && grp == 0) __builtin_amdgcn_s_barrier();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += c16[i][j][0] + c16[i][j][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) s += c32[i][j][0] + c32[i][j][15];
  if (s == 12345.f) sink[threadIdx.x] = s;  // keeps the MFMAs (never true for these inputs)
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int SH, bool LDS>
int run(const char* name, int cus, int iters, float* sink, unsigned long long* cyc) {
  const int grid = cus;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((probe<SH, LDS>), dim3(grid), dim3(512), 0, 0, 4, sink, cyc);  // warm-up
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  double clk = 0.0;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((probe<SH, LDS>), dim3(grid), dim3(512), 0, 0, iters, sink, cyc);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) {
      best = ms;
      std::vector<unsigned long long> c(grid);
      CHECK(hipMemcpy(c.data(), cyc, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      double m = 0.0;
      for (auto v : c) m += (double)v;
      clk = m / grid / (best * 1e-3) / 1e9;  // s_memtime cycles over the wall time: GHz (upper bound)
    }
  }
  const double flops = 2.0 * 128 * 64 * 32 * 8.0 * iters * grid;  // 8 waves x 128x64x32 MACs per step
  std::printf("%-28s %8.3f ms  %7.1f TFLOP/s  %5.2f GHz (s_memtime / wall)\n", name, best, flops / best / 1e9, clk);
  return 0;
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, dev));
  cus = prop.multiProcessorCount;
  float* sink;
  unsigned long long* cyc;
  CHECK(hipMalloc(&sink, 512 * sizeof(float)));
  CHECK(hipMalloc(&cyc, cus * sizeof(unsigned long long)));
  std::printf("# %s, %d CUs; 8 waves / CU, 128x64 wave tile, K 32 per step\n", prop.gcnArchName, cus);
  const int iters = 20000;
  for (int rep = 0; rep < 2; ++rep) {
    if (run<0, false>("reg 16x16x32", cus, iters, sink, cyc)) return 1;
    if (run<1, false>("reg 32x32x16", cus, iters, sink, cyc)) return 1;
    if (run<0, true>("lds+barrier 16x16x32", cus, iters, sink, cyc)) return 1;
    if (run<1, true>("lds+barrier 32x32x16", cus, iters, sink, cyc)) return 1;
  }
  CHECK(hipFree(sink));
  CHECK(hipFree(cyc));
  return 0;
}
