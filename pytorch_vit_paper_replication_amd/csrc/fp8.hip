// fp8 quantization for the ViT-H/14 fp8 training config (BASELINE.json config 5, SURVEY.md §7.2
// step 9): bf16 activations / weights -> OCP fp8 (e4m3 forward operands, e5m2 gradients) with
// per-tensor scales, and the delayed-scaling bookkeeping (amax history -> scale) kept entirely on
// the device so a training step never synchronises with the host.
//
//   quant:  y = sat(x * qscale) in fp8,  amax = max(amax, max|x|)   (one pass; qscale == null:
//           amax only, used to calibrate a tensor the first time it is seen / for weights)
//   update: per tensor slot, push amax into a history ring, qscale = fmax / max(history) / 2^margin,
//           dscale = 1 / qscale (the GEMM epilogue's dequant factor), reset amax; a non-finite
//           amax is dropped (scales unchanged), so one overflowing step cannot poison the history
#include "common.h"

#include <cstdlib>

namespace pvr {
namespace {

// 16 elements (two 16-B bf16 loads, one 16-B fp8 store) per thread and grid-stride step.
template <int FMT>
__global__ void __launch_bounds__(256) quant_kernel(const uint16_t* __restrict__ x, int64_t ldx, uint8_t* __restrict__ y, int64_t ldy,
                                                    int64_t rows, int cols, const float* __restrict__ qscale,
                                                    unsigned* __restrict__ amax) {
  const int per_row = cols >> 4;
  const int64_t n = rows * per_row;
  const float qs = qscale ? *qscale : 1.f;
  // dense tensors (the usual case): flat offsets, no 64-bit division per 16 elements
  const bool dense = ldx == cols && (!y || ldy == cols);
  float m = 0.f;
  // U grid-stride steps per trip with all their loads issued first (clamped, so unconditional):
  // the grid is capped at 256 blocks for the amax atomics, so memory-level parallelism has to come
  // from each thread keeping several 32-B loads in flight
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i0 = blockIdx.x * 256ll + threadIdx.x; i0 < n; i0 += U * stride) {
    uint4 ua[U], ub[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = min(i0 + u * stride, n - 1);
      const uint16_t* src = dense ? x + i * 16 : x + (i / per_row) * ldx + (int)(i % per_row) * 16;
      ua[u] = *(const uint4*)src;
      ub[u] = *(const uint4*)(src + 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n) break;
      const uint32_t w[8] = {ua[u].x, ua[u].y, ua[u].z, ua[u].w, ub[u].x, ub[u].y, ub[u].z, ub[u].w};
      float v[16];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[2 * j] = bf2f(w[j] & 0xFFFF);
        v[2 * j + 1] = bf2f(w[j] >> 16);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        // NaN-propagating max (fmaxf drops NaN): a NaN or Inf element makes this tensor's amax
        // non-finite, which scale_update_kernel then keeps out of the history
        const float a = fabsf(v[j]);
        m = (a > m || a != a) ? a : m;
      }
      if (y) {
        int o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int t = pack2_fp8<FMT, false>(v[4 * q] * qs, v[4 * q + 1] * qs, 0);
          o[q] = pack2_fp8<FMT, true>(v[4 * q + 2] * qs, v[4 * q + 3] * qs, t);
        }
        uint8_t* dst = dense ? y + i * 16 : y + (i / per_row) * ldy + (int)(i % per_row) * 16;
        *(int4*)dst = make_int4(o[0], o[1], o[2], o[3]);
      }
    }
  }
  // one same-address atomic per BLOCK: those serialise at L2 (~12 ns each), so the grid is capped
  // at 256 blocks and the 4 waves reduce through LDS first
  __shared__ float wm[4];
  m = wave_max_nan(m);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float b = nan_max(nan_max(wm[0], wm[1]), nan_max(wm[2], wm[3]));
    // |x| bits order like uints; Inf (0x7f800000) and NaN (> 0x7f800000) sort above every finite
    if (!(b <= 0.f)) atomicMax(amax, __float_as_uint(b));
  }
}

// Multi-tensor form for the per-step weight refresh (current scaling): one launch covers every
// weight. Segment table rows (int64): {src bf16 ptr, dst fp8 ptr, elements (multiple of 16), slot,
// first chunk}; a workgroup handles chunks of QM_CHUNK elements of one segment. AMAX: record
// max|x| per slot (NaN-propagating, one atomic per workgroup); else quantize with qscale[slot].
constexpr int QM_CHUNK = 256 * 16 * 4;
template <int FMT, bool AMAX>
__global__ void __launch_bounds__(256) quant_multi_kernel(const int64_t* __restrict__ segs, int nseg, int64_t nchunks,
                                                          const float* __restrict__ qscale, unsigned* __restrict__ amax) {
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    int lo = 0, hi = nseg - 1;  // last segment whose first chunk <= ch
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (segs[mid * 5 + 4] <= ch) lo = mid; else hi = mid - 1;
    }
    const int64_t* sg = segs + lo * 5;
    const uint16_t* x = reinterpret_cast<const uint16_t*>(sg[0]);
    uint8_t* y = reinterpret_cast<uint8_t*>(sg[1]);
    const int64_t n16 = sg[2] >> 4;
    const int slot = (int)sg[3];
    const int64_t g0 = (ch - sg[4]) * (QM_CHUNK / 16);
    const float qs = AMAX ? 1.f : qscale[slot];
    float m = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = g0 + u * 256 + threadIdx.x;
      if (i >= n16) break;
      const uint4 ua = *(const uint4*)(x + i * 16), ub = *(const uint4*)(x + i * 16 + 8);
      const uint32_t w[8] = {ua.x, ua.y, ua.z, ua.w, ub.x, ub.y, ub.z, ub.w};
      float v[16];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[2 * j] = bf2f(w[j] & 0xFFFF);
        v[2 * j + 1] = bf2f(w[j] >> 16);
      }
      if constexpr (AMAX) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const float a = fabsf(v[j]);
          m = (a > m || a != a) ? a : m;
        }
      } else {
        int o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int t = pack2_fp8<FMT, false>(v[4 * q] * qs, v[4 * q + 1] * qs, 0);
          o[q] = pack2_fp8<FMT, true>(v[4 * q + 2] * qs, v[4 * q + 3] * qs, t);
        }
        *(int4*)(y + i * 16) = make_int4(o[0], o[1], o[2], o[3]);
      }
    }
    if constexpr (AMAX) {
      __shared__ float wm[4];
      m = wave_max_nan(m);
      if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
      __syncthreads();
      if (threadIdx.x == 0) {
        const float b = nan_max(nan_max(wm[0], wm[1]), nan_max(wm[2], wm[3]));
        if (!(b <= 0.f)) atomicMax(amax + slot, __float_as_uint(b));
      }
      __syncthreads();
    }
  }
}

// Transposing quantize for the fp8 weight-gradient GEMM: x bf16 [T][C] (row stride ldx) ->
// y fp8 [C][ldy] with y[c][t] = sat(x[t][c] * qscale) for t < T and 0 for T <= t < ldy (the GEMM's
// reduction dim padded to a multiple of 128). 64 x 64 tiles through LDS; reads and writes are
// 16-B per thread. No amax: the tensor's amax is recorded by its non-transposed quantize pass.
template <int FMT>
__global__ void __launch_bounds__(256) quant_t_kernel(const uint16_t* __restrict__ x, int64_t ldx, uint8_t* __restrict__ y, int64_t ldy,
                                                      int T, int C, const float* __restrict__ qscale) {
  __shared__ uint16_t tile[64][64 + 8];
  const int t0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
  const float qs = *qscale;
  {  // load: row t0 + tid/4, cols c0 + 16 (tid%4) .. +15
    const int r = tid >> 2, cc = (tid & 3) * 16;
    const int t = t0 + r;
    uint4 a = make_uint4(0u, 0u, 0u, 0u), b = a;
    if (t < T && c0 + cc < C) {  // C % 16 == 0 (host check)
      const uint16_t* src = x + (int64_t)t * ldx + c0 + cc;
      a = *(const uint4*)src;
      b = *(const uint4*)(src + 8);
    }
    *(uint4*)&tile[r][cc] = a;
    *(uint4*)&tile[r][cc + 8] = b;
  }
  __syncthreads();
  // store: output row c0 + tid/4, t range t0 + 16 (tid%4) .. +15 (16 fp8 bytes)
  const int c = tid >> 2, tt = (tid & 3) * 16;
  if (c0 + c >= C || t0 + tt >= ldy) return;
  float v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = bf2f(tile[tt + j][c]) * qs;
  int o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int w = pack2_fp8<FMT, false>(v[4 * q], v[4 * q + 1], 0);
    o[q] = pack2_fp8<FMT, true>(v[4 * q + 2], v[4 * q + 3], w);
  }
  *(int4*)(y + (int64_t)(c0 + c) * ldy + t0 + tt) = make_int4(o[0], o[1], o[2], o[3]);
}

// Byte transpose of an fp8 tensor: x8 [T][C] (row stride ldx bytes) -> y [C][ldy], zero for
// T <= t < ldy. The weight-gradient GEMM's transposed operands from the row-major fp8 copies the
// forward / dgrad GEMMs already use (same slot, same scale: the bytes are exactly the transposing
// quantize pass's), so the pass reads 1 byte per element instead of 2. 64 x 64 tiles through LDS.
__global__ void __launch_bounds__(256) transpose8_kernel(const uint8_t* __restrict__ x, int64_t ldx, uint8_t* __restrict__ y,
                                                         int64_t ldy, int T, int C) {
  __shared__ uint8_t tile[64][64 + 4];
  const int t0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
  {  // load: row t0 + tid/4, cols c0 + 16 (tid%4) .. +15
    const int r = tid >> 2, cc = (tid & 3) * 16;
    const int t = t0 + r;
    uint4 a = make_uint4(0u, 0u, 0u, 0u);
    if (t < T && c0 + cc < C) a = *(const uint4*)(x + (int64_t)t * ldx + c0 + cc);  // C % 16 == 0 (host check)
    uint32_t* d = (uint32_t*)&tile[r][cc];
    d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
  }
  __syncthreads();
  // store: output row c0 + tid/4, t range t0 + 16 (tid%4) .. +15
  const int c = tid >> 2, tt = (tid & 3) * 16;
  if (c0 + c >= C || t0 + tt >= ldy) return;
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    o[q] = (uint32_t)tile[tt + 4 * q][c] | ((uint32_t)tile[tt + 4 * q + 1][c] << 8) | ((uint32_t)tile[tt + 4 * q + 2][c] << 16) |
           ((uint32_t)tile[tt + 4 * q + 3][c] << 24);
  *(uint4*)(y + (int64_t)(c0 + c) * ldy + t0 + tt) = make_uint4(o[0], o[1], o[2], o[3]);
}

// fp8 -> f32 (tests / debugging): y[i] = dscale * x[i]
template <int FMT>
__global__ void dequant_kernel(const uint8_t* __restrict__ x, float* __restrict__ y, int64_t n, const float* __restrict__ dscale) {
  const float ds = dscale ? *dscale : 1.f;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int word = x[i];
    float f;
    if constexpr (FMT == 0)
      f = __builtin_amdgcn_cvt_f32_fp8(word, 0);
    else
      f = __builtin_amdgcn_cvt_f32_bf8(word, 0);
    y[i] = f * ds;
  }
}

__global__ void scale_update_kernel(float* __restrict__ hist, int H, unsigned* __restrict__ amax, float* __restrict__ qscale,
                                    float* __restrict__ dscale, const float* __restrict__ fmax, int s0, int s1, float margin_mul) {
  const int i = s0 + blockIdx.x * 64 + threadIdx.x;
  if (i >= s1) return;
  float* h = hist + (int64_t)i * H;
  const float cur = __uint_as_float(amax[i]);
  amax[i] = 0u;
  // A non-finite amax (an overflowing step: Inf/NaN in the tensor) is not pushed into the history:
  // it would make qscale 0 and dscale Inf, i.e. NaN GEMM outputs for the next H steps. The previous
  // scales stay; the step itself is skipped by the optimizer's non-finite gradient check.
  if (!isfinite(cur)) return;
  float m = cur;
  for (int k = H - 1; k > 0; --k) {
    h[k] = h[k - 1];
    m = fmaxf(m, h[k]);
  }
  h[0] = cur;
  const float q = m > 0.f ? fmax[i] / m * margin_mul : 1.f;
  qscale[i] = q;
  dscale[i] = 1.f / q;
}

}  // namespace
}  // namespace pvr

extern "C" hipError_t pvr_fp8_quant(const uint16_t* x, int64_t ldx, uint8_t* y, int64_t ldy, int64_t rows, int cols, const float* qscale,
                                    unsigned* amax, int fmt, hipStream_t s) {
  using namespace pvr;
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (cols % 16) return hipErrorInvalidValue;
  // grid cap 512 (two blocks per CU) keeps enough loads in flight: 4.1 -> 5.0 TB/s at ViT-H/14
  // activation shapes, H/14 fp8 step 925 -> 938 img/s (profiles/fp8_quant_blocks_ab.log); more
  // blocks add same-address amax atomics without more bandwidth
  constexpr int cap = 512;
  int64_t blocks = (rows * (cols / 16) + 255) / 256;
  if (blocks > cap) blocks = cap;  // grid-stride over the tensor
  if (fmt == 0)
    hipLaunchKernelGGL(quant_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, s, x, ldx, y, ldy, rows, cols, qscale, amax);
  else
    hipLaunchKernelGGL(quant_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, s, x, ldx, y, ldy, rows, cols, qscale, amax);
  return hipGetLastError();
}

extern "C" hipError_t pvr_fp8_quant_multi(const int64_t* segs, int nseg, int64_t nchunks, const float* qscale, unsigned* amax,
                                          int fmt, int amax_only, hipStream_t s) {
  using namespace pvr;
  if (nseg <= 0 || nchunks <= 0) return hipSuccess;
  const unsigned grid = (unsigned)(nchunks < 8192 ? nchunks : 8192);
  if (amax_only)
    hipLaunchKernelGGL((quant_multi_kernel<0, true>), dim3(grid), dim3(256), 0, s, segs, nseg, nchunks, qscale, amax);
  else if (fmt == 0)
    hipLaunchKernelGGL((quant_multi_kernel<0, false>), dim3(grid), dim3(256), 0, s, segs, nseg, nchunks, qscale, amax);
  else
    hipLaunchKernelGGL((quant_multi_kernel<1, false>), dim3(grid), dim3(256), 0, s, segs, nseg, nchunks, qscale, amax);
  return hipGetLastError();
}

extern "C" hipError_t pvr_fp8_quant_t(const uint16_t* x, int64_t ldx, uint8_t* y, int64_t ldy, int T, int C, const float* qscale, int fmt,
                                      hipStream_t s) {
  using namespace pvr;
  if (T <= 0 || C <= 0) return hipSuccess;
  if (C % 16 || ldy % 64 || ldy < T) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(ldy / 64), (unsigned)((C + 63) / 64));
  if (fmt == 0)
    hipLaunchKernelGGL(quant_t_kernel<0>, grid, dim3(256), 0, s, x, ldx, y, ldy, T, C, qscale);
  else
    hipLaunchKernelGGL(quant_t_kernel<1>, grid, dim3(256), 0, s, x, ldx, y, ldy, T, C, qscale);
  return hipGetLastError();
}

extern "C" hipError_t pvr_fp8_transpose(const uint8_t* x, int64_t ldx, uint8_t* y, int64_t ldy, int T, int C, hipStream_t s) {
  using namespace pvr;
  if (T <= 0 || C <= 0) return hipSuccess;
  if (C % 16 || ldx % 16 || ldy % 64 || ldy < T) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(ldy / 64), (unsigned)((C + 63) / 64));
  hipLaunchKernelGGL(transpose8_kernel, grid, dim3(256), 0, s, x, ldx, y, ldy, T, C);
  return hipGetLastError();
}

extern "C" hipError_t pvr_fp8_dequant(const uint8_t* x, float* y, int64_t n, const float* dscale, int fmt, hipStream_t s) {
  using namespace pvr;
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (fmt == 0)
    hipLaunchKernelGGL(dequant_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, s, x, y, n, dscale);
  else
    hipLaunchKernelGGL(dequant_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, s, x, y, n, dscale);
  return hipGetLastError();
}

extern "C" hipError_t pvr_fp8_scale_update(float* hist, int H, unsigned* amax, float* qscale, float* dscale, const float* fmax, int s0,
                                           int s1, float margin_mul, hipStream_t s) {
  using namespace pvr;
  if (s1 <= s0) return hipSuccess;
  hipLaunchKernelGGL(scale_update_kernel, dim3((s1 - s0 + 63) / 64), dim3(64), 0, s, hist, H, amax, qscale, dscale, fmax, s0, s1,
                     margin_mul);
  return hipGetLastError();
}
