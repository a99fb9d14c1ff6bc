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

PVR_DEV void load8(const uint16_t* p, float* o) {
  const uint4 q = *(const uint4*)p;
  const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[2 * j] = bf2f(u[j] & 0xFFFF);
    o[2 * j + 1] = bf2f(u[j] >> 16);
  }
}

// Grid-stride over rows: each wave keeps its lanes' dgamma/dbeta partials in registers.
template <int MAXCH>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const uint16_t* __restrict__ dy, int64_t dy_stride,
                                                      const uint16_t* __restrict__ x, int64_t x_stride,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      const float* __restrict__ w,
                                                      const uint16_t* __restrict__ dres, int64_t dres_stride,
                                                      uint16_t* __restrict__ dx, int64_t dx_stride,
                                                      float* __restrict__ dw, float* __restrict__ db, float* __restrict__ dsum,
                                                      uint16_t* __restrict__ dz, int64_t dz_stride,
                                                      const uint64_t* __restrict__ seed_ptr, uint64_t seed_off, uint32_t thr,
                                                      float dscale, int rows, int D) {
  __shared__ float red[4][MAXCH * 64 * 8 > 1280 ? 1280 : MAXCH * 64 * 8];  // one partial at a time
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = D >> 3;
  float gw[MAXCH][8], gb[MAXCH][8], gs[MAXCH][8];
#pragma unroll
  for (int i = 0; i < MAXCH; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) gw[i][j] = gb[i][j] = gs[i][j] = 0.f;

  // Rows are software-pipelined: the x / dy / dres vectors of the wave's next row are loaded
  // before the current row's two wave reductions, so HBM latency overlaps the shuffles.
  const int stride = gridDim.x * 4;
  uint4 cx[MAXCH], cdy[MAXCH], cr[MAXCH];
  // unconditional (clamped) loads: the compiler can then count them instead of waiting vmcnt(0)
  auto load_row = [&](int row, uint4 (&qx)[MAXCH], uint4 (&qd)[MAXCH], uint4 (&qr)[MAXCH]) {
    const int rr = min(row, rows - 1);
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = min(lane + 64 * i, nch - 1);
      qx[i] = *(const uint4*)(x + (int64_t)rr * x_stride + c * 8);
      qd[i] = *(const uint4*)(dy + (int64_t)rr * dy_stride + c * 8);
      qr[i] = dres ? *(const uint4*)(dres + (int64_t)rr * dres_stride + c * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  // gamma is loop-invariant: keep this lane's columns in registers (a per-row reload would be
  // waited with vmcnt(0), which also drains the next row's prefetch)
  float wreg[MAXCH][8];
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = min(lane + 64 * i, nch - 1);
    const float4 w0 = *(const float4*)(w + c * 8), w1 = *(const float4*)(w + c * 8 + 4);
    wreg[i][0] = w0.x; wreg[i][1] = w0.y; wreg[i][2] = w0.z; wreg[i][3] = w0.w;
    wreg[i][4] = w1.x; wreg[i][5] = w1.y; wreg[i][6] = w1.z; wreg[i][7] = w1.w;
  }
  const uint64_t seed = dz ? *seed_ptr + seed_off : 0ull;
  int row = blockIdx.x * 4 + wave;
  load_row(row, cx, cdy, cr);
  float cmu = row < rows ? mean[row] : 0.f, crs = row < rows ? rstd[row] : 0.f;
  for (; row < rows; row += stride) {
    uint4 nx[MAXCH], ndy[MAXCH], nr[MAXCH];
    load_row(row + stride, nx, ndy, nr);
    const int rn = min(row + stride, rows - 1);
    const float nmu = mean[rn], nrs = rstd[rn];
    const float mu = cmu, rs = crs;
    float xh[MAXCH][8], g[MAXCH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        const uint32_t ux[4] = {cx[i].x, cx[i].y, cx[i].z, cx[i].w};
        const uint32_t ud[4] = {cdy[i].x, cdy[i].y, cdy[i].z, cdy[i].w};
        const float* ww = wreg[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xv = bf2f(j & 1 ? ux[j >> 1] >> 16 : ux[j >> 1] & 0xFFFF);
          const float dv = bf2f(j & 1 ? ud[j >> 1] >> 16 : ud[j >> 1] & 0xFFFF);
          xh[i][j] = (xv - mu) * rs;
          g[i][j] = dv * ww[j];
          s1 += g[i][j];
          s2 += g[i][j] * xh[i][j];
          gw[i][j] += dv * xh[i][j];
          gb[i][j] += dv;
        }
      }
    }
    const float c1 = wave_sum(s1) / D, c2 = wave_sum(s2) / D;
#pragma unroll
    for (int i = 0; i < MAXCH; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (g[i][j] - c1 - xh[i][j] * c2) * rs;
        if (dres) {
          const uint32_t ur[4] = {cr[i].x, cr[i].y, cr[i].z, cr[i].w};
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += bf2f(j & 1 ? ur[j >> 1] >> 16 : ur[j >> 1] & 0xFFFF);
        }
        uint4 q;
        q.x = pack2bf(o[0], o[1]); q.y = pack2bf(o[2], o[3]);
        q.z = pack2bf(o[4], o[5]); q.w = pack2bf(o[6], o[7]);
        *(uint4*)(dx + (int64_t)row * dx_stride + c * 8) = q;
        if (dz) {  // uniform: dropout backward of the producing layer
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            bool k0, k1;
            rng_keep2(seed, (uint64_t)row * D + c * 8 + j, thr, k0, k1);
            o[j] = k0 ? o[j] * dscale : 0.f;
            o[j + 1] = k1 ? o[j + 1] * dscale : 0.f;
          }
          q.x = pack2bf(o[0], o[1]); q.y = pack2bf(o[2], o[3]);
          q.z = pack2bf(o[4], o[5]); q.w = pack2bf(o[6], o[7]);
          *(uint4*)(dz + (int64_t)row * dz_stride + c * 8) = q;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) gs[i][j] += o[j];  // column sums of dx (or dz): a fused bias gradient
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
  // then one atomic per column per block
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
        for (int j = 0; j < 8; ++j) red[wave][c * 8 + j] = qn == 0 ? gw[i][j] : (qn == 1 ? gb[i][j] : gs[i][j]);
      }
    }
    __syncthreads();
    for (int col = threadIdx.x; col < D; col += 256)
      atomicAdd(outs[qn] + col, red[0][col] + red[1][col] + red[2][col] + red[3][col]);
  }
}

}  // namespace
}  // namespace pvr

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

extern "C" hipError_t pvr_layernorm_bwd(const uint16_t* dy, int64_t dy_stride, const uint16_t* x, int64_t x_stride,
                                        const float* mean, const float* rstd, const float* w, const uint16_t* dres,
                                        int64_t dres_stride, uint16_t* dx, int64_t dx_stride, float* dw, float* db,
                                        float* dsum, uint16_t* dz, int64_t dz_stride, const uint64_t* seed_ptr,
                                        uint64_t seed_off, uint32_t thr, float dscale, int rows, int D, hipStream_t s) {
  using namespace pvr;
  if (rows <= 0) return hipSuccess;
  if (D % 8 != 0 || D > 1280 || (dz && (!seed_ptr || !thr))) return hipErrorInvalidValue;
  static const int cap = [] {  // PVR_LN_BWD_BLOCKS: grid cap (A/B of row pipelining vs atomics per column)
    const char* e = getenv("PVR_LN_BWD_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 1024;
  }();
  int nblk = (rows + 3) / 4;
  // 1024 blocks (4 per CU, ~12 pipelined rows per wave): in-step 0.2 % ahead of 512 and 768
  // (profiles/ln_bwd_grid_step_ab_r2.log); 2048 was 22 % slower in isolation, its 2048 x 3 x D column
  // atomics contending on the same addresses (profiles/kbench_ln_grid.log)
  if (nblk > cap) nblk = cap;
  const dim3 grid(nblk), block(256);
  const int maxch = (D / 8 + 63) / 64;
  switch (maxch) {
    case 1: hipLaunchKernelGGL(ln_bwd_kernel<1>, grid, block, 0, s, dy, dy_stride, x, x_stride, mean, rstd, w, dres, dres_stride, dx, dx_stride, dw, db, dsum, dz, dz_stride, seed_ptr, seed_off, thr, dscale, rows, D); break;
    case 2: hipLaunchKernelGGL(ln_bwd_kernel<2>, grid, block, 0, s, dy, dy_stride, x, x_stride, mean, rstd, w, dres, dres_stride, dx, dx_stride, dw, db, dsum, dz, dz_stride, seed_ptr, seed_off, thr, dscale, rows, D); break;
    default: hipLaunchKernelGGL(ln_bwd_kernel<3>, grid, block, 0, s, dy, dy_stride, x, x_stride, mean, rstd, w, dres, dres_stride, dx, dx_stride, dw, db, dsum, dz, dz_stride, seed_ptr, seed_off, thr, dscale, rows, D); break;
  }
  return hipGetLastError();
}
