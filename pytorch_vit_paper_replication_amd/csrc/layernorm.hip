// LayerNorm forward/backward for the pre-LN ViT blocks (reference models/vit.py:83, :115, :216;
// SURVEY.md K5). One wave per token row, bf16 I/O with 16-B vector accesses, fp32 statistics.
// The backward fuses the residual-branch gradient add (dx = dres + LN'(dy)) and reduces
// d(gamma)/d(beta) per block in LDS before one f32 atomic per column per block. It can also emit
// the dropout backward of the layer that PRODUCED x's residual stream (dz = mask * scale * dx, the
// previous encoder block's fc2 dropout, mask recomputed from the same counter hash) together with
// that layer's bias gradient (column sums of dz), so no separate pass re-reads dx for them.
#include "common.h"

namespace pvr {
namespace {

template <int MAXCH>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const uint16_t* __restrict__ x, int64_t x_stride,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      uint16_t* __restrict__ y, int64_t y_stride,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = D >> 3;
  PVR_ASSERT((D & 7) == 0 && nch <= 64 * MAXCH);
  const uint16_t* xr = x + (int64_t)row * x_stride;
  float v[MAXCH][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      const uint4 q = *(const uint4*)(xr + c * 8);
      const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[i][2 * j] = bf2f(u[j] & 0xFFFF);
        v[i][2 * j + 1] = bf2f(u[j] >> 16);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  const float mean = wave_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / D + eps);
  uint16_t* yr = y + (int64_t)row * y_stride;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      const float4 w0 = *(const float4*)(w + c * 8), w1 = *(const float4*)(w + c * 8 + 4);
      const float4 b0 = *(const float4*)(b + c * 8), b1 = *(const float4*)(b + c * 8 + 4);
      const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * ww[j] + bb[j];
      uint4 q;
      q.x = pack2bf(o[0], o[1]); q.y = pack2bf(o[2], o[3]);
      q.z = pack2bf(o[4], o[5]); q.w = pack2bf(o[6], o[7]);
      *(uint4*)(yr + c * 8) = q;
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// The same forward plus the output's e4m3 copy for an fp8 GEMM (producer-side quantization of the
// delayed-scaling recipe): yq = fp8(y * qscale), *amax = max(*amax, max|y|). Rows are grid-strided
// over a capped grid so the workgroups' same-address amax atomics (one each) stay few.
template <int MAXCH>
__global__ void __launch_bounds__(256) ln_fwd_q8_kernel(const uint16_t* __restrict__ x, int64_t x_stride,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        uint16_t* __restrict__ y, int64_t y_stride, uint8_t* __restrict__ yq,
                                                        int64_t q_stride, const float* __restrict__ qscale,
                                                        unsigned* __restrict__ amax, float* __restrict__ mean_out,
                                                        float* __restrict__ rstd_out, int rows, int D, float eps) {
  __shared__ float wm[4];
  const int lane = threadIdx.x & 63;
  const int nch = D >> 3;
  const float qs = *qscale;
  float am = 0.f;
  for (int row = blockIdx.x * 4 + (int)(threadIdx.x >> 6); row < rows; row += gridDim.x * 4) {
    const uint16_t* xr = x + (int64_t)row * x_stride;
    float v[MAXCH][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        const uint4 q = *(const uint4*)(xr + c * 8);
        const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[i][2 * j] = bf2f(u[j] & 0xFFFF);
          v[i][2 * j + 1] = bf2f(u[j] >> 16);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[i][j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
      }
    }
    const float mean = wave_sum(s) / D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[i][j] - mean;
          ss += d * d;
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(ss) / D + eps);
    uint16_t* yr = y ? y + (int64_t)row * y_stride : nullptr;  // null: only the e4m3 copy is consumed
    uint8_t* qr = yq + (int64_t)row * q_stride;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        const float4 w0 = *(const float4*)(w + c * 8), w1 = *(const float4*)(w + c * 8 + 4);
        const float4 b0 = *(const float4*)(b + c * 8), b1 = *(const float4*)(b + c * 8 + 4);
        const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        float o[8];
        float vm = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o[j] = (v[i][j] - mean) * rstd * ww[j] + bb[j];
          vm = nan_max(vm, fabsf(o[j]));
        }
        am = nan_max(am, vm);
        uint4 q;
        q.x = pack2bf(o[0], o[1]); q.y = pack2bf(o[2], o[3]);
        q.z = pack2bf(o[4], o[5]); q.w = pack2bf(o[6], o[7]);
        if (yr) *(uint4*)(yr + c * 8) = q;
        *(uint2*)(qr + c * 8) = pack8_fp8_fast<0>(o, qs, vm);
      }
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
  am = wave_max_nan(am);
  if (lane == 0) wm[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = nan_max(nan_max(wm[0], wm[1]), nan_max(wm[2], wm[3]));
    if (!(m <= 0.f)) atomicMax(amax, __float_as_uint(m));
  }
}

PVR_DEV void load8(const uint16_t* p, float* o) {
  const uint4 q = *(const uint4*)p;
  const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[2 * j] = bf2f(u[j] & 0xFFFF);
    o[2 * j + 1] = bf2f(u[j] >> 16);
  }
}

// W consecutive bf16 of a row (W = 8: one 16-B access, W = 4: one 8-B access)
template <int W>
struct RowVec;
template <>
struct RowVec<8> {
  uint32_t u[4];
  PVR_DEV void load(const uint16_t* p) { const uint4 q = *(const uint4*)p; u[0] = q.x; u[1] = q.y; u[2] = q.z; u[3] = q.w; }
  PVR_DEV void store(uint16_t* p) const { *(uint4*)p = make_uint4(u[0], u[1], u[2], u[3]); }
  PVR_DEV void zero() { u[0] = u[1] = u[2] = u[3] = 0u; }
};
template <>
struct RowVec<4> {
  uint32_t u[2];
  PVR_DEV void load(const uint16_t* p) { const uint2 q = *(const uint2*)p; u[0] = q.x; u[1] = q.y; }
  PVR_DEV void store(uint16_t* p) const { *(uint2*)p = make_uint2(u[0], u[1]); }
  PVR_DEV void zero() { u[0] = u[1] = 0u; }
};

// Grid-stride over rows: each wave keeps its lanes' dgamma/dbeta partials in registers. A lane owns
// MAXCH chunks of W columns (chunk c = lane + 64 i). W = 4 where D / 8 is not a multiple of 64 but
// D / 4 is (D = 768: 3 chunks of 4 per lane instead of 1.5 of 8, so no lane idles on the last chunk
// and the smaller register footprint doubles the waves in flight: 4 per SIMD instead of 2).
// Q8: the fp8-copy variant (qout / dz_nostore used); the bf16 instantiation carries none of it.
template <int MAXCH, int W, bool Q8>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const uint16_t* __restrict__ dy, int64_t dy_stride,
                                                      const uint16_t* __restrict__ x, int64_t x_stride,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      const float* __restrict__ w,
                                                      const uint16_t* __restrict__ dres, int64_t dres_stride,
                                                      uint16_t* __restrict__ dx, int64_t dx_stride,
                                                      float* __restrict__ dw, float* __restrict__ db, float* __restrict__ dsum,
                                                      float* __restrict__ part,
                                                      uint16_t* __restrict__ dz, int64_t dz_stride,
                                                      const uint64_t* __restrict__ seed_ptr, uint64_t seed_off, uint32_t thr,
                                                      float dscale, int dz_nostore, uint8_t* __restrict__ qout, int64_t q_stride,
                                                      const float* __restrict__ qscale, unsigned* __restrict__ amax, int qfmt,
                                                      int rows, int D) {
  __shared__ float red[4][MAXCH * 64 * W > 1280 ? 1280 : MAXCH * 64 * W];  // one partial at a time
  __shared__ float qred[4];
  const float qs = Q8 ? *qscale : 1.f;
  float qam = 0.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = D / W;
  float gw[MAXCH][W], gb[MAXCH][W], gs[MAXCH][W];
#pragma unroll
  for (int i = 0; i < MAXCH; ++i)
#pragma unroll
    for (int j = 0; j < W; ++j) gw[i][j] = gb[i][j] = gs[i][j] = 0.f;

  // Rows are software-pipelined: the x / dy / dres vectors of the wave's next row are loaded
  // before the current row's two wave reductions, so HBM latency overlaps the shuffles.
  const int stride = gridDim.x * 4;
  RowVec<W> cx[MAXCH], cdy[MAXCH], cr[MAXCH];
  // unconditional (clamped) loads: the compiler can then count them instead of waiting vmcnt(0)
  auto load_row = [&](int row, RowVec<W> (&qx)[MAXCH], RowVec<W> (&qd)[MAXCH], RowVec<W> (&qr)[MAXCH]) {
    const int rr = min(row, rows - 1);
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = min(lane + 64 * i, nch - 1);
      qx[i].load(x + (int64_t)rr * x_stride + c * W);
      qd[i].load(dy + (int64_t)rr * dy_stride + c * W);
      if (dres)
        qr[i].load(dres + (int64_t)rr * dres_stride + c * W);
      else
        qr[i].zero();
    }
  };
  // gamma is loop-invariant: keep this lane's columns in registers (a per-row reload would be
  // waited with vmcnt(0), which also drains the next row's prefetch)
  float wreg[MAXCH][W];
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = min(lane + 64 * i, nch - 1);
#pragma unroll
    for (int j = 0; j < W; j += 4) {
      const float4 w4 = *(const float4*)(w + c * W + j);
      wreg[i][j] = w4.x; wreg[i][j + 1] = w4.y; wreg[i][j + 2] = w4.z; wreg[i][j + 3] = w4.w;
    }
  }
  const uint64_t seed = dz ? *seed_ptr + seed_off : 0ull;
  int row = blockIdx.x * 4 + wave;
  load_row(row, cx, cdy, cr);
  float cmu = row < rows ? mean[row] : 0.f, crs = row < rows ? rstd[row] : 0.f;
  for (; row < rows; row += stride) {
    RowVec<W> nx[MAXCH], ndy[MAXCH], nr[MAXCH];
    load_row(row + stride, nx, ndy, nr);
    const int rn = min(row + stride, rows - 1);
    const float nmu = mean[rn], nrs = rstd[rn];
    const float mu = cmu, rs = crs;
    // xhat and g = dy * gamma are recomputed from the packed row in the second pass instead of kept
    // in registers between the two wave reductions (fewer VGPRs: more waves, more bytes in flight)
    auto xhat = [&](int i, int j) { return (bf2f(j & 1 ? cx[i].u[j >> 1] >> 16 : cx[i].u[j >> 1] & 0xFFFF) - mu) * rs; };
    auto dyv = [&](int i, int j) { return bf2f(j & 1 ? cdy[i].u[j >> 1] >> 16 : cdy[i].u[j >> 1] & 0xFFFF); };
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const float xh = xhat(i, j), dv = dyv(i, j);
          const float g = dv * wreg[i][j];
          s1 += g;
          s2 += g * xh;
          gw[i][j] += dv * xh;
          gb[i][j] += dv;
        }
      }
    }
    const float c1 = wave_sum(s1) / D, c2 = wave_sum(s2) / D;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float o[W];
#pragma unroll
        for (int j = 0; j < W; ++j) o[j] = (dyv(i, j) * wreg[i][j] - c1 - xhat(i, j) * c2) * rs;
        if (dres) {
#pragma unroll
          for (int j = 0; j < W; ++j) o[j] += bf2f(j & 1 ? cr[i].u[j >> 1] >> 16 : cr[i].u[j >> 1] & 0xFFFF);
        }
        RowVec<W> q;
#pragma unroll
        for (int j = 0; j < W; j += 2) q.u[j >> 1] = pack2bf(o[j], o[j + 1]);
        q.store(dx + (int64_t)row * dx_stride + c * W);
        if (dz) {  // uniform: dropout backward of the producing layer
#pragma unroll
          for (int j = 0; j < W; j += 2) {
            bool k0, k1;
            rng_keep2(seed, (uint64_t)row * D + c * W + j, thr, k0, k1);
            o[j] = k0 ? o[j] * dscale : 0.f;
            o[j + 1] = k1 ? o[j + 1] * dscale : 0.f;
          }
          if (!Q8 || !dz_nostore) {  // uniform; dz_nostore: only dz's e5m2 copy (qout) is consumed
#pragma unroll
            for (int j = 0; j < W; j += 2) q.u[j >> 1] = pack2bf(o[j], o[j + 1]);
            q.store(dz + (int64_t)row * dz_stride + c * W);
          }
        }
        if constexpr (Q8) {  // fp8 copy (qfmt 1 e5m2, 0 e4m3) of the gradient written last (dz, else dx) for the next fp8 dgrad GEMM
          uint32_t b4[W / 4];
          float vm = 0.f;
#pragma unroll
          for (int j = 0; j < W; ++j) vm = nan_max(vm, fabsf(o[j]));
          qam = nan_max(qam, vm);
          if (qfmt ? fp8_direct_ok<1>(vm, qs) : fp8_direct_ok<0>(vm, qs)) {  // no saturation / NaN handling needed in this wave
#pragma unroll
            for (int j = 0; j < W; j += 4)
              b4[j >> 2] = qfmt ? pack4_fp8_direct<1>(o[j] * qs, o[j + 1] * qs, o[j + 2] * qs, o[j + 3] * qs)
                                : pack4_fp8_direct<0>(o[j] * qs, o[j + 1] * qs, o[j + 2] * qs, o[j + 3] * qs);
          } else {
#pragma unroll
            for (int j = 0; j < W; j += 4) b4[j >> 2] = pack4_fp8_rt(qfmt, o[j] * qs, o[j + 1] * qs, o[j + 2] * qs, o[j + 3] * qs);
          }
          uint8_t* qp = qout + (int64_t)row * q_stride + c * W;
          if constexpr (W == 8)
            *(uint2*)qp = make_uint2(b4[0], b4[1]);
          else
            *(uint32_t*)qp = b4[0];
        }
#pragma unroll
        for (int j = 0; j < W; ++j) gs[i][j] += o[j];  // column sums of dx (or dz): a fused bias gradient
      }
    }
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      cx[i] = nx[i];
      cdy[i] = ndy[i];
      cr[i] = nr[i];
    }
    cmu = nmu;
    crs = nrs;
  }
  // block reduction of the dgamma / dbeta / dsum partials, one quantity at a time through a
  // [4][D] LDS buffer (keeps LDS at 4*D*4 bytes so occupancy is register-, not LDS-, bound),
  // then one atomic per column per block (deterministic mode: one partial row per block)
  float* outs[3] = {dw, db, dsum};
#pragma unroll
  for (int qn = 0; qn < 3; ++qn) {
    if (!outs[qn]) continue;  // uniform
    if (qn) __syncthreads();
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
#pragma unroll
        for (int j = 0; j < W; ++j) red[wave][c * W + j] = qn == 0 ? gw[i][j] : (qn == 1 ? gb[i][j] : gs[i][j]);
      }
    }
    __syncthreads();
    if (part) {  // deterministic mode: the block's partial row [block][quantity][D] (rows_reduce sums them)
      float* pr = part + ((int64_t)blockIdx.x * 3 + qn) * D;
      for (int col = threadIdx.x; col < D; col += 256) pr[col] = red[0][col] + red[1][col] + red[2][col] + red[3][col];
    } else {
      for (int col = threadIdx.x; col < D; col += 256)
        atomicAdd(outs[qn] + col, red[0][col] + red[1][col] + red[2][col] + red[3][col]);
    }
  }
  if constexpr (Q8) {  // max |gradient| of the block's rows: one atomic per workgroup (delayed-scaling amax record)
    qam = wave_max_nan(qam);
    if (lane == 0) qred[wave] = qam;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float m = nan_max(nan_max(qred[0], qred[1]), nan_max(qred[2], qred[3]));
      if (!(m <= 0.f)) atomicMax(amax, __float_as_uint(m));
    }
  }
}

}  // namespace
}  // namespace pvr

static int device_cus() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    return cus;
  }();
  return n;
}

extern "C" hipError_t pvr_layernorm_fwd(const uint16_t* x, int64_t x_stride, const float* w, const float* b,
                                        uint16_t* y, int64_t y_stride, float* mean, float* rstd, int rows, int D,
                                        float eps, hipStream_t s) {
  using namespace pvr;
  if (rows <= 0) return hipSuccess;
  if (D % 8 != 0 || D > 2048) return hipErrorInvalidValue;
  const dim3 grid((rows + 3) / 4), block(256);
  const int maxch = (D / 8 + 63) / 64;
  switch (maxch) {
    case 1: hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, block, 0, s, x, x_stride, w, b, y, y_stride, mean, rstd, rows, D, eps); break;
    case 2: hipLaunchKernelGGL(ln_fwd_kernel<2>, grid, block, 0, s, x, x_stride, w, b, y, y_stride, mean, rstd, rows, D, eps); break;
    case 3: hipLaunchKernelGGL(ln_fwd_kernel<3>, grid, block, 0, s, x, x_stride, w, b, y, y_stride, mean, rstd, rows, D, eps); break;
    default: hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, block, 0, s, x, x_stride, w, b, y, y_stride, mean, rstd, rows, D, eps); break;
  }
  return hipGetLastError();
}

// grid cap of ln_fwd_q8_kernel, in workgroups per CU (A/B: pvr_set_ln_fwd_q8_grid)
static int g_ln_q8_blocks_per_cu = 4;
extern "C" void pvr_set_ln_fwd_q8_grid(int per_cu) { g_ln_q8_blocks_per_cu = per_cu < 1 ? 1 : per_cu > 64 ? 64 : per_cu; }

// pvr_layernorm_fwd plus the e4m3 copy yq (row stride q_stride bytes) with scale *qscale and the
// amax record (see ln_fwd_q8_kernel)
extern "C" hipError_t pvr_layernorm_fwd_q8(const uint16_t* x, int64_t x_stride, const float* w, const float* b, uint16_t* y,
                                           int64_t y_stride, uint8_t* yq, int64_t q_stride, const float* qscale, unsigned* amax,
                                           float* mean, float* rstd, int rows, int D, float eps, hipStream_t s) {
  using namespace pvr;
  if (rows <= 0) return hipSuccess;
  if (D % 8 != 0 || D > 2048 || q_stride % 8 != 0) return hipErrorInvalidValue;
  int nblk = (rows + 3) / 4;
  const int cap = g_ln_q8_blocks_per_cu * device_cus();
  if (nblk > cap) nblk = cap;
  const dim3 grid(nblk), block(256);
  switch ((D / 8 + 63) / 64) {
    case 1: hipLaunchKernelGGL(ln_fwd_q8_kernel<1>, grid, block, 0, s, x, x_stride, w, b, y, y_stride, yq, q_stride, qscale, amax, mean, rstd, rows, D, eps); break;
    case 2: hipLaunchKernelGGL(ln_fwd_q8_kernel<2>, grid, block, 0, s, x, x_stride, w, b, y, y_stride, yq, q_stride, qscale, amax, mean, rstd, rows, D, eps); break;
    case 3: hipLaunchKernelGGL(ln_fwd_q8_kernel<3>, grid, block, 0, s, x, x_stride, w, b, y, y_stride, yq, q_stride, qscale, amax, mean, rstd, rows, D, eps); break;
    default: hipLaunchKernelGGL(ln_fwd_q8_kernel<4>, grid, block, 0, s, x, x_stride, w, b, y, y_stride, yq, q_stride, qscale, amax, mean, rstd, rows, D, eps); break;
  }
  return hipGetLastError();
}

extern "C" hipError_t pvr_rows_reduce(const float* part, int R, int C, int seg, float* d0, float* d1, float* d2, hipStream_t s);

// grid of the LayerNorm backward (= the partial rows [blocks][3][D] of its deterministic mode)
extern "C" int pvr_layernorm_bwd_blocks(int rows, int D) {
  const bool use_w4 = (D / 4) % 64 == 0 && (D / 8) % 64 != 0 && D / 4 <= 64 * 5;
  // D = 768 on 4-column chunks (146 VGPRs, 3 blocks per CU): one grid of exactly the resident blocks,
  // so no block starts late; otherwise 1024
  const int cap = use_w4 && D == 768 ? device_cus() * 3 : 1024;
  const int nblk = (rows + 3) / 4;
  return nblk > cap ? cap : nblk;
}

extern "C" hipError_t pvr_layernorm_bwd(const uint16_t* dy, int64_t dy_stride, const uint16_t* x, int64_t x_stride,
                                        const float* mean, const float* rstd, const float* w, const uint16_t* dres,
                                        int64_t dres_stride, uint16_t* dx, int64_t dx_stride, float* dw, float* db,
                                        float* dsum, uint16_t* dz, int64_t dz_stride, const uint64_t* seed_ptr,
                                        uint64_t seed_off, uint32_t thr, float dscale, int dz_nostore, uint8_t* q, int64_t q_stride,
                                        const float* qscale, unsigned* amax, int qfmt, int rows, int D, float* part,
                                        hipStream_t s) {
  using namespace pvr;
  if (rows <= 0) return hipSuccess;
  if (qfmt != 0 && qfmt != 1) return hipErrorInvalidValue;
  if (D % 8 != 0 || D > 1280 || (dz && (!seed_ptr || !thr))) return hipErrorInvalidValue;
  if (q && (!qscale || !amax || q_stride % 8 != 0 || reinterpret_cast<uintptr_t>(q) % 8 != 0)) return hipErrorInvalidValue;
  if (dz_nostore && (!dz || !q)) return hipErrorInvalidValue;  // skipping dz needs dz's fp8 copy
  // 4-column chunks (D = 768, profiles/r2s/ln_bwd_w4_ab.log): 79 -> 64 us per call (91 -> 79 with the
  // linked dropout backward); forcing 4 waves/SIMD (<= 128 VGPRs) spilled 18 VGPRs and took 114 us.
  // 4-column chunks when they tile the row over the 64 lanes exactly and 8-column ones do not
  const bool use_w4 = (D / 4) % 64 == 0 && (D / 8) % 64 != 0 && D / 4 <= 64 * 5;
  // 1024 blocks (4 per CU, ~12 pipelined rows per wave): in-step 0.2 % ahead of 512 and 768
  // (profiles/ln_bwd_grid_step_ab_r2.log); 2048 was 22 % slower in isolation, its 2048 x 3 x D column
  // atomics contending on the same addresses (profiles/kbench_ln_grid.log)
  const int nblk = pvr_layernorm_bwd_blocks(rows, D);
  if (!dw && !db && !dsum) part = nullptr;
  const dim3 grid(nblk), block(256);
#define PVR_LN_BWD(MC, W)                                                                                                   \
  hipLaunchKernelGGL(q ? (ln_bwd_kernel<MC, W, true>) : (ln_bwd_kernel<MC, W, false>), grid, block, 0, s, dy, dy_stride, x, x_stride, mean, rstd, w, dres, dres_stride, dx, \
                     dx_stride, dw, db, dsum, part, dz, dz_stride, seed_ptr, seed_off, thr, dscale, dz_nostore, q, q_stride, qscale, amax, \
                     qfmt, rows, D)
  if (use_w4) {
    switch (D / 256) {
      case 3: PVR_LN_BWD(3, 4); break;  // D = 768
      case 5: PVR_LN_BWD(5, 4); break;  // D = 1280
      default: PVR_LN_BWD(1, 4); break;  // D = 256
    }
  } else {
    const int maxch = (D / 8 + 63) / 64;
    switch (maxch) {
      case 1: PVR_LN_BWD(1, 8); break;
      case 2: PVR_LN_BWD(2, 8); break;
      default: PVR_LN_BWD(3, 8); break;
    }
  }
#undef PVR_LN_BWD
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess || !part) return e;
  return pvr_rows_reduce(part, nblk, 3 * D, D, dw, db, dsum, s);
}
