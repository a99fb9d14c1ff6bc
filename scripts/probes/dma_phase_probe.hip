// Ping-pong phase probe with the LDS-DMA operand stream (GEMM main-loop headroom): what does the
// global -> LDS DMA traffic of the 256x256 ping-pong GEMM cost its phase loop?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/dma_phase_probe.hip -o /tmp/dma_phase_probe
// One workgroup per CU, 8 waves (two groups a barrier apart, as csrc/gemm.hip's gemm_pp_kernel).
// A phase per wave: 6 ds_read_b128 fragment reads (the K loop's average), DMA issue, counted vmcnt,
// lgkmcnt(0), barrier, 16 v_mfma_f32_16x16x32_bf16 at priority 1, barrier. Modes:
//   0: no DMA (the LDS-fed phase alone);
//   1: 2 x 16 B/lane LDS-DMAs per wave per phase (the GEMM's 16 KiB per CU per phase), into a
//      3-slot LDS ring that the fragment reads never touch, source streamed through a 256 MiB
//      buffer (HBM / MALL), 2 phases in flight (vmcnt 4);
//   2: the same DMAs, source a 2 MiB window per workgroup (L2-resident reuse, like the B operand);
//   3: mode 1 with the DMAs issued in the MFMA segment (after the first barrier) instead of before it;
//   4: mode 1 issued by the 4 waves of group 0 only (4 DMAs each), group 1 none;
//   5: mode 1 with every workgroup reading the same 64 KiB (cache-hot: the issue / TA cost alone);
//   6: mode 1 with 4 phases in flight (vmcnt 8, 5-slot ring);
//   7: mode 1 with each workgroup streaming its own contiguous range (sequential 16 KiB per phase);
//   8: the GEMM's own operand pattern: per K-tile (4 phases) 256 A rows then 256 B rows of 128 B
//      (K = 768: 1536-B row stride), A tile = the workgroup's 256-row block of a 50432 x 768 matrix,
//      B tile = one of 3 256-row blocks of a 768 x 768 matrix, every workgroup at the same K-tile;
//   9: mode 8 with each workgroup starting its K loop at K-tile (id mod 12) (rotated start);
//  10: mode 8 with the ping-pong's uneven fragment reads: 12 / 4 / 8 / 0 per phase (A0 + B0, B1,
//      A1, none) instead of 6 each.
// Prints TFLOP/s of the MFMAs and the DMA bandwidth.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

__device__ __forceinline__ v4f m16(v8s a, v8s b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}

constexpr int FRAG = 0, RING = 49152, SLOT = 16384;  // LDS: fragment region | 5 x 16 KiB DMA ring

template <int MODE>
__global__ void __launch_bounds__(512, 1) probe(const uint16_t* src, unsigned src_bytes, int iters, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), grp = wave >> 2;
  for (int i = threadIdx.x; i < RING / 4; i += 512) ((float*)smem)[i] = 0.001f * (i & 255);
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(src), (short)0, (int)src_bytes, 0x00020000);
  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s a[4], b[2];
  if (grp == 1) __builtin_amdgcn_s_barrier();
  const unsigned wnd = MODE == 2 ? (2u << 20) : MODE == 5 ? 65536u : src_bytes;  // bytes this workgroup streams through
  const unsigned wbase = MODE == 2 ? (blockIdx.x * (2u << 20)) % (src_bytes - wnd + 1) : 0u;
  constexpr int NDMA = MODE == 0 ? 0 : MODE == 4 ? 4 : 2;
  constexpr int NSLOT = MODE == 6 ? 5 : 3, DEPTH = MODE == 6 ? 4 : 2;
  const bool issuer = MODE != 4 || grp == 0;
  auto issue = [&](int it) {
    if (!issuer) return;
    if constexpr (MODE == 8 || MODE == 9 || MODE == 10) {  // GEMM operand pattern (see the header)
      const int kt = ((it >> 2) + (MODE == 9 ? (int)blockIdx.x : 0)) % 12, ph = it & 3;
      const unsigned rowb = ph < 2 ? (unsigned)(blockIdx.x % 197) * 256u + (unsigned)ph * 128u
                                   : (unsigned)(blockIdx.x % 3) * 256u + (unsigned)(ph - 2) * 128u;
      const unsigned base = ph < 2 ? 0u : (96u << 20);
#pragma unroll
      for (int i = 0; i < NDMA; ++i) {
        const unsigned row = rowb + (unsigned)(2 * wave + i) * 8u + (unsigned)(lane >> 3);
        const unsigned off = base + row * 1536u + (unsigned)kt * 128u + (unsigned)(lane & 7) * 16u;
        char* dst = smem + RING + (it % NSLOT) * SLOT + (2 * wave + i) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, off, 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const unsigned piece = (unsigned)(it * 16 + (MODE == 4 ? 4 * wave + i : 2 * wave + i));  // 1 KiB pieces, 16 per phase
      const unsigned start = MODE == 7 ? (unsigned)blockIdx.x * (src_bytes / 256u) : (unsigned)blockIdx.x * 16384u * 7u;
      const unsigned off = wbase + (start + piece * 1024u) % wnd + (unsigned)lane * 16;
      char* dst = smem + RING + (it % NSLOT) * SLOT + (MODE == 4 ? 4 * wave + i : 2 * wave + i) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, off, 0, 0, 0);
    }
  };
  for (int it = 0; it < iters; ++it) {
    const char* fr = smem + FRAG + (it & 3) * 12288;  // 4 x 12 KiB: [0, 48 KiB)
    if constexpr (MODE == 10) {  // 12 / 4 / 8 / 0 reads (a: 4 x 2 k-steps, b: 2 x 2 in phase 0)
      const int ph = it & 3;
      if (ph == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = *(const __attribute__((address_space(3))) v8s*)(fr + i * 1024 + lane * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] ^= *(const __attribute__((address_space(3))) v8s*)(fr + 6144 + i * 1024 + lane * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = *(const __attribute__((address_space(3))) v8s*)(fr + 4096 + j * 1024 + lane * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] ^= *(const __attribute__((address_space(3))) v8s*)(fr + 10240 + j * 1024 + lane * 16);
      } else if (ph == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = *(const __attribute__((address_space(3))) v8s*)(fr + 4096 + j * 1024 + lane * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] ^= *(const __attribute__((address_space(3))) v8s*)(fr + 10240 + j * 1024 + lane * 16);
      } else if (ph == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = *(const __attribute__((address_space(3))) v8s*)(fr + i * 1024 + lane * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] ^= *(const __attribute__((address_space(3))) v8s*)(fr + 6144 + i * 1024 + lane * 16);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *(const __attribute__((address_space(3))) v8s*)(fr + i * 1024 + lane * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *(const __attribute__((address_space(3))) v8s*)(fr + 4096 + j * 1024 + lane * 16);
    }
    if constexpr (MODE != 0 && MODE != 3) issue(it);
    if constexpr (MODE != 0) {
      if (issuer) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH * NDMA) : "memory");  // the group DEPTH phases ago landed
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (MODE == 3) issue(it);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = m16(a[i], b[j & 1], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (grp == 0) __builtin_amdgcn_s_barrier();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][0];
  if (s == 12345.f) sink[threadIdx.x] = s;
}

template <int MODE>
int run(const char* name, int cus, const uint16_t* src, unsigned bytes, int iters, float* sink) {
  constexpr int SMEM = RING + 5 * SLOT;
  CHECK(hipFuncSetAttribute((const void*)probe<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(probe<MODE>, dim3(cus), dim3(512), SMEM, 0, src, bytes, 8, sink);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(probe<MODE>, dim3(cus), dim3(512), SMEM, 0, src, bytes, iters, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const double flops = 2.0 * 16 * 8192 * 8.0 * iters * cus;
  const double dma = MODE == 0 ? 0.0 : 16384.0 * iters * cus;
  std::printf("%-44s %8.3f ms  %7.1f TFLOP/s  DMA %6.2f TB/s  %5.0f cycles/phase @2.1 GHz\n", name, best, flops / best / 1e9,
              dma / best / 1e9, best * 1e-3 * 2.1e9 / iters);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const unsigned bytes = 256u << 20;
  uint16_t* src;
  float* sink;
  CHECK(hipMalloc(&src, bytes));
  CHECK(hipMemset(src, 0, bytes));
  CHECK(hipMalloc(&sink, 512 * sizeof(float)));
  std::printf("# %s, %d CUs; one 8-wave workgroup per CU; phase = 6 fragment reads + DMA + 16 MFMAs, 2 barriers\n",
              prop.gcnArchName, cus);
  const int iters = 40000;
  for (int rep = 0; rep < 2; ++rep) {
    if (run<0>("0 no DMA", cus, src, bytes, iters, sink)) return 1;
    if (run<1>("1 DMA 2/wave, streamed 256 MiB", cus, src, bytes, iters, sink)) return 1;
    if (run<2>("2 DMA 2/wave, 2 MiB window (L2)", cus, src, bytes, iters, sink)) return 1;
    if (run<3>("3 DMA 2/wave in the MFMA segment", cus, src, bytes, iters, sink)) return 1;
    if (run<4>("4 DMA 4/wave, group 0 only", cus, src, bytes, iters, sink)) return 1;
    if (run<5>("5 DMA 2/wave, one shared 64 KiB (hot)", cus, src, bytes, iters, sink)) return 1;
    if (run<6>("6 DMA 2/wave, 4 phases in flight", cus, src, bytes, iters, sink)) return 1;
    if (run<7>("7 DMA 2/wave, sequential per workgroup", cus, src, bytes, iters, sink)) return 1;
    if (run<8>("8 GEMM operand pattern (K 768)", cus, src, bytes, iters, sink)) return 1;
    if (run<9>("9 GEMM operand pattern, rotated K start", cus, src, bytes, iters, sink)) return 1;
    if (run<10>("10 GEMM pattern, reads 12/4/8/0 per phase", cus, src, bytes, iters, sink)) return 1;
  }
  CHECK(hipFree(src));
  CHECK(hipFree(sink));
  return 0;
}
