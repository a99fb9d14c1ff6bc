// Probe of ds_read_b64_tr_b8 lane semantics on gfx950: LDS byte at (row r, col c), row stride 128 B,
// holds (r * 16 + c) & 0xFF; each lane supplies the address of row 8g + (i >> 1), columns 8 (i & 1) .. +7
// (g = lane / 16, i = lane % 16) and prints the 8 bytes it receives.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 128];
  for (int k = threadIdx.x; k < 64 * 128; k += 64) lds[k] = (uint8_t)(((k / 128) * 16 + (k % 128)) & 0xFF);
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, i = l & 15;
  const uint32_t addr = (uint32_t)(uintptr_t)(lds) + (uint32_t)((8 * g + (i >> 1)) * 128 + 8 * (i & 1));
  typedef uint32_t v2u __attribute__((ext_vector_type(2)));
  v2u r;
  asm volatile("ds_read_b64_tr_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
  out[2 * l] = r.x;
  out[2 * l + 1] = r.y;
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 128 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[128];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int b = 0; b < 8; ++b) printf(" %3u", (h[2 * l + b / 4] >> (8 * (b % 4))) & 0xFF);
    printf("\n");
  }
  return 0;
}
