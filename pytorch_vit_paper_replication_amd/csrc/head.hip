// Classifier head of the ViT on the hand-written path (reference models/vit.py:216-222, :232-235;
// SURVEY.md K5 (final LayerNorm), K12):
//   forward   xhat = (x_cls - mean) * rstd,  logits = (xhat * gamma + beta) . W^T + bias      (fp32)
//   backward  dW += dlogits^T . xc,  db += colsum(dlogits),  dy = dlogits . W,
//             dgamma += sum_b dy * xhat,  dbeta += sum_b dy,  dx_cls = LN'(dy),  other token rows 0
// Only the CLS token is normalised (LayerNorm is per token, the classifier reads token 0 only).
// Sizes are small (B x C x D = 256 x 1000 x 768 at ViT-B/16 b256): the products run on the exact
// fp32 MFMA, one 16 x 16 output tile per workgroup with k split over its 4 waves, operands streamed
// from L2 (LDS only for the split-k reduction). They replace
// torch's F.linear / addmm / sum / copy launches (hipBLASLt Cijk kernels + ATen elementwise).
#include "common.h"

namespace pvr {
namespace {

// exact-fp32 MFMA (v_mfma_f32_16x16x4_f32, bit-for-bit a k-ordered fmaf chain): lane l holds
// A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15]; D[(l >> 4) * 4 + r][l & 15] in register r.
// A wave accumulates a 16 x 16 tile over its share of k; a lane loads 4 consecutive k of its operands (16 B where
// the layout allows) and issues 4 MFMAs with element j as that step's operand, so one 16-deep k
// slab costs 2 vector loads + 4 MFMAs (the k order within a slab is permuted: rounding only).
PVR_DEV v4f mfma_f32(float a, float b, v4f c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// ---------------------------------------------------------------------------------- forward
// LayerNorm of the CLS rows: one wave per image, 4 bf16 per lane-chunk (8-B loads, all issued up
// front), two-pass mean / variance in fp32. Writes xhat [B][D] and rstd [B].
__global__ void __launch_bounds__(256) head_ln_fwd_kernel(const uint16_t* __restrict__ tok, int64_t ld_tok, int B, int D, float eps,
                                                           float* __restrict__ xhat, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const uint16_t* x = tok + (int64_t)b * ld_tok;
  constexpr int MAXC = 6;  // D <= 6 * 256 = 1536 (host check), D % 4 == 0
  float v[MAXC * 4];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    v[4 * c] = v[4 * c + 1] = v[4 * c + 2] = v[4 * c + 3] = 0.f;
    if (c * 256 + lane * 4 < D) {
      const uint2 w = *(const uint2*)(x + c * 256 + lane * 4);
      v[4 * c] = bf2f(w.x & 0xFFFF); v[4 * c + 1] = bf2f(w.x >> 16);
      v[4 * c + 2] = bf2f(w.y & 0xFFFF); v[4 * c + 3] = bf2f(w.y >> 16);
      s += (v[4 * c] + v[4 * c + 1]) + (v[4 * c + 2] + v[4 * c + 3]);
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
    if (c * 256 + lane * 4 < D)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t = v[4 * c + j] - mean;
        q += t * t;
      }
  const float rs = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
    if (c * 256 + lane * 4 < D)
      *(float4*)(xhat + (int64_t)b * D + c * 256 + lane * 4) =
          make_float4((v[4 * c] - mean) * rs, (v[4 * c + 1] - mean) * rs, (v[4 * c + 2] - mean) * rs, (v[4 * c + 3] - mean) * rs);
  if (lane == 0) rstd_out[b] = rs;
}

// Split-K reduction of a 16 x 16 MFMA tile over the workgroup's 4 waves (each summed a quarter of
// k): waves 1..3 park their accumulators (and one extra per-lane float) in LDS, wave 0 adds them.
// Returns true in wave 0 only. Call from all 4 waves (uniform: one tile per workgroup).
PVR_DEV bool splitk_reduce(v4f& acc, float& extra, int wave, int lane) {
  __shared__ float red[3][5][64];
  if (wave) {
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave - 1][q][lane] = acc[q];
    red[wave - 1][4][lane] = extra;
  }
  __syncthreads();
  if (wave) return false;
#pragma unroll
  for (int w = 0; w < 3; ++w) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += red[w][q][lane];
    extra += red[w][4][lane];
  }
  return true;
}

// logits[b][c] = sum_k (xhat[b][k] * gamma[k] + beta[k]) * W[c][k] + bias[c]. One 16 x 16 (images x
// classes) tile per workgroup, k split over its 4 waves (short MFMA chains, 4x the loads in flight).
__global__ void __launch_bounds__(256) head_logits_kernel(const float* __restrict__ xhat, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, const float* __restrict__ W,
                                                           const float* __restrict__ bias, int B, int C, int D,
                                                           float* __restrict__ logits) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = blockIdx.x;
  const int ntc = (C + 15) / 16;
  const int b0 = (tile / ntc) * 16, c0 = (tile % ntc) * 16;
  const int r = lane & 15, kq = (lane >> 4) * 4;
  const int ba = min(b0 + r, B - 1), cb = min(c0 + r, C - 1);  // clamped rows: results discarded
  const float* xa = xhat + (int64_t)ba * D + kq;
  const float* wb = W + (int64_t)cb * D + kq;
  v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k = wave * 16; k < D; k += 64) {
    const float4 x = *(const float4*)(xa + k);
    const float4 w = *(const float4*)(wb + k);
    const float4 g = *(const float4*)(gamma + k + kq);
    const float4 be = *(const float4*)(beta + k + kq);
    acc = mfma_f32(fmaf(x.x, g.x, be.x), w.x, acc);
    acc = mfma_f32(fmaf(x.y, g.y, be.y), w.y, acc);
    acc = mfma_f32(fmaf(x.z, g.z, be.z), w.z, acc);
    acc = mfma_f32(fmaf(x.w, g.w, be.w), w.w, acc);
  }
  float unused = 0.f;
  if (!splitk_reduce(acc, unused, wave, lane)) return;
  const int c = c0 + (lane & 15);
  if (c < C) {
    const float bv = bias ? bias[c] : 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int b = b0 + (lane >> 4) * 4 + q;
      if (b < B) logits[(int64_t)b * C + c] = acc[q] + bv;
    }
  }
}

// ---------------------------------------------------------------------------------- backward GEMMs
// One launch, one 16 x 16 tile per workgroup (k split over its 4 waves, reduced in LDS):
//  tiles [0, nA): dW[c][d] += sum_b dl[b][c] * xc[b][d] (xc = xhat * gamma + beta; each (c, d) owned
//    by one lane: plain read-modify-write), and for the tiles of the first 16 dims db[c] += sum_b dl[b][c];
//  tiles [nA, nA + nB): dy[b][d] = sum_c dl[b][c] * W[c][d], plus dgamma[d] += sum_b dy * xhat,
//    dbeta[d] += sum_b dy over the tile's 16 images (f32 atomics, B / 16 adds per dim; deterministic
//    mode: partial rows summed in order by rows_reduce).
__global__ void __launch_bounds__(256) head_bwd_gemm_kernel(const float* __restrict__ dl, const float* __restrict__ xhat,
                                                             const float* __restrict__ gamma, const float* __restrict__ beta,
                                                             const float* __restrict__ W, int B, int C, int D, int nA, int nB,
                                                             float* __restrict__ dW, float* __restrict__ db,
                                                             float* __restrict__ dy, float* __restrict__ dgamma,
                                                             float* __restrict__ dbeta, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = blockIdx.x;
  const int r = lane & 15, kq = (lane >> 4) * 4;
  const int ntd = D / 16;
  if (tile < nA) {
    // dW tiles (c-block, d-block); with dW null (frozen weight, trainable bias) only the d-block-0
    // tile of each c-block runs, for db
    const int c0 = dW ? (tile / ntd) * 16 : tile * 16, d0 = dW ? (tile % ntd) * 16 : 0;
    const int ca = min(c0 + r, C - 1);  // A[m = c][k = b] = dl[b][c]; B[k = b][n = d] = xc[b][d]
    const float gd = gamma[d0 + r], bd = beta[d0 + r];
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    float bs = 0.f;
    for (int k = wave * 16; k < B; k += 64) {
      float a[4], x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = k + kq + j;
        const bool ok = b < B;
        a[j] = ok ? dl[(int64_t)b * C + ca] : 0.f;
        x[j] = ok ? fmaf(xhat[(int64_t)b * D + d0 + r], gd, bd) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc = mfma_f32(a[j], x[j], acc);
        bs += a[j];
      }
    }
    if (!splitk_reduce(acc, bs, wave, lane)) return;
    const int d = d0 + r;
    if (dW) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = c0 + (lane >> 4) * 4 + q;
        if (c < C) dW[(int64_t)c * D + d] += acc[q];
      }
    }
    if (d0 == 0 && db) {
      // bs: this lane's share (b = kq + j mod 16) of sum_b dl[b][c0 + r]; add the 4 lane groups
      bs += __shfl_xor(bs, 16, 64);
      bs += __shfl_xor(bs, 32, 64);
      if (lane < 16 && c0 + r < C) db[c0 + r] += bs;
    }
    return;
  }
  const int t2 = tile - nA;
  if (t2 >= nB) return;
  const int b0 = (t2 / ntd) * 16, d0 = (t2 % ntd) * 16;
  const int ba = min(b0 + r, B - 1);
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  const float* dla = dl + (int64_t)ba * C;
  for (int k = wave * 16; k < C; k += 64) {
    const int c = k + kq;
    float a[4], w[4];
    if (c + 3 < C && (C & 3) == 0) {
      const float4 av = *(const float4*)(dla + c);
      a[0] = av.x; a[1] = av.y; a[2] = av.z; a[3] = av.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = c + j < C ? dla[c + j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = c + j < C ? W[(int64_t)(c + j) * D + d0 + r] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = mfma_f32(a[j], w[j], acc);
  }
  float unused = 0.f;
  if (!splitk_reduce(acc, unused, wave, lane)) return;
  const int d = d0 + r;
  float pg = 0.f, pb = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int b = b0 + (lane >> 4) * 4 + q;
    if (b < B) {
      dy[(int64_t)b * D + d] = acc[q];
      pg += acc[q] * xhat[(int64_t)b * D + d];
      pb += acc[q];
    }
  }
  pg += __shfl_xor(pg, 16, 64);
  pg += __shfl_xor(pg, 32, 64);
  pb += __shfl_xor(pb, 16, 64);
  pb += __shfl_xor(pb, 32, 64);
  if (lane < 16) {
    if (part) {  // deterministic mode: this image block's partial row [b-block][dgamma | dbeta]
      part[(int64_t)(b0 / 16) * 2 * D + d] = pg;
      part[(int64_t)(b0 / 16) * 2 * D + D + d] = pb;
    } else {
      if (dgamma) atomicAdd(dgamma + d, pg);
      if (dbeta) atomicAdd(dbeta + d, pb);
    }
  }
}

// ---------------------------------------------------------------------------------- backward LN rows
// Blocks [0, ceil(B / 4)): one wave per image, dx_cls = rstd * (dxh - mean(dxh) - xhat * mean(dxh * xhat)),
// dxh = dy * gamma, written as the image's token-0 row of dtok (bf16). Blocks past that: zero the
// other token rows of dtok (16 B per lane, grid-stride), so dtok needs no separate fill.
__global__ void __launch_bounds__(256) head_ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ xhat,
                                                           const float* __restrict__ rstd, const float* __restrict__ gamma, int B,
                                                           int D, int ntok, uint16_t* __restrict__ dtok, int nrow_blocks) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if ((int)blockIdx.x < nrow_blocks) {
    const int b = blockIdx.x * 4 + wave;
    if (b >= B) return;
    const float* y = dy + (int64_t)b * D;
    const float* xh = xhat + (int64_t)b * D;
    float s1 = 0.f, s2 = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float g = y[d] * gamma[d];
      s1 += g;
      s2 += g * xh[d];
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
    const float r = rstd[b];
    uint16_t* out = dtok + (int64_t)b * ntok * D;
    for (int d = lane; d < D; d += 64) out[d] = f2bf(r * (y[d] * gamma[d] - s1 - xh[d] * s2));
    return;
  }
  // zero rows 1 .. ntok-1 of every image: D / 8 chunks of 16 B per row
  // (the host guarantees B * (ntok - 1) * D / 8 < 2^31: 32-bit index arithmetic)
  const uint32_t per_img = (uint32_t)(ntok - 1) * (uint32_t)(D / 8), total = (uint32_t)B * per_img;
  const uint32_t nblk = gridDim.x - (uint32_t)nrow_blocks;
  for (uint32_t e = (blockIdx.x - (uint32_t)nrow_blocks) * 256u + tid; e < total; e += nblk * 256u) {
    const uint32_t b = e / per_img, r = e - b * per_img;
    *(uint4*)(dtok + ((int64_t)b * ntok + 1) * D + (int64_t)r * 8) = make_uint4(0u, 0u, 0u, 0u);
  }
}

__global__ void __launch_bounds__(256) scale_by_kernel(const float* __restrict__ x, const float* __restrict__ s, float* __restrict__ y,
                                                        int64_t n) {
  const float c = *s;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] = x[i] * c;
}

// mean of n floats (one workgroup): the cross-entropy's batch mean
__global__ void __launch_bounds__(256) mean_kernel(const float* __restrict__ x, int n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = ((red[0] + red[1]) + (red[2] + red[3])) / (float)n;
}

// sums[0] += loss, sums[1] += (number of correct rows) / B: the engine's per-batch metric
// accumulation on the device (correct: xent's per-row argmax == label flags)
__global__ void __launch_bounds__(256) metrics_accum_kernel(float* __restrict__ sums, const float* __restrict__ loss,
                                                             const int* __restrict__ correct, int B) {
  __shared__ int red[4];
  int c = 0;
  for (int i = threadIdx.x; i < B; i += 256) c += correct[i];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    sums[0] += loss[0];
    sums[1] += (float)(red[0] + red[1] + red[2] + red[3]) / (float)B;
  }
}

// seed = rng; rng += 1 (the per-forward dropout seed snapshot; stays on the device so captured
// hipGraphs advance it on every replay)
__global__ void rng_next_kernel(int64_t* __restrict__ rng, int64_t* __restrict__ seed) {
  if (threadIdx.x == 0) {
    const int64_t r = *rng;
    *seed = r;
    *rng = r + 1;
  }
}

// x[0 .. n) = 0, 16-B stores (n % 4 == 0 and 16-B alignment checked by the host), grid-stride
__global__ void __launch_bounds__(256) zero_f32_kernel(float4* __restrict__ x, int64_t n4) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    x[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

}  // namespace
}  // namespace pvr

extern "C" hipError_t pvr_head_fwd(const uint16_t* tok, int64_t ld_tok, int B, int D, const float* gamma, const float* beta, float eps,
                                   const float* W, const float* bias, int C, float* xhat, float* rstd, float* logits, hipStream_t s) {
  using namespace pvr;
  if (B <= 0) return hipSuccess;
  if (D % 16 != 0 || D > 1536 || C <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(head_ln_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, s, tok, ld_tok, B, D, eps, xhat, rstd);
  const int tiles = ((B + 15) / 16) * ((C + 15) / 16);
  hipLaunchKernelGGL(head_logits_kernel, dim3(tiles), dim3(256), 0, s, xhat, gamma, beta, W, bias, B, C, D, logits);
  return hipGetLastError();
}

extern "C" hipError_t pvr_rows_reduce(const float* part, int R, int C, int seg, float* d0, float* d1, float* d2, hipStream_t s);

extern "C" hipError_t pvr_head_bwd(const float* dl, const float* xhat, const float* rstd, const float* gamma, const float* beta,
                                   const float* W, int B, int C, int D, int ntok, float* dW, float* db, float* dgamma, float* dbeta,
                                   float* dy, uint16_t* dtok, float* part, hipStream_t s) {
  using namespace pvr;
  if (B <= 0) return hipSuccess;
  if (!dgamma && !dbeta) part = nullptr;
  if (D % 16 != 0 || C <= 0) return hipErrorInvalidValue;
  const int ntd = D / 16;
  // dW tiles; without dW but with db (classifier weight frozen, bias trainable): one tile per
  // 16 classes for the bias gradient alone
  const int nA = dW ? ((C + 15) / 16) * ntd : db ? (C + 15) / 16 : 0;
  const int nB = ((B + 15) / 16) * ntd;
  hipLaunchKernelGGL(head_bwd_gemm_kernel, dim3(nA + nB), dim3(256), 0, s, dl, xhat, gamma, beta, W, B, C, D, nA, nB, dW, db,
                     dy, dgamma, dbeta, part);
  if (part) {  // part: f32 [ceil(B / 16)][2 D] (deterministic mode)
    const hipError_t e = pvr_rows_reduce(part, (B + 15) / 16, 2 * D, D, dgamma, dbeta, nullptr, s);
    if (e != hipSuccess) return e;
  }
  const int nrow = (B + 3) / 4;
  const int64_t zero_chunks = (int64_t)B * (ntok - 1) * (D / 8);
  if (zero_chunks >= (1ll << 31)) return hipErrorInvalidValue;
  int64_t nz = (zero_chunks + 255) / 256;
  if (nz > 2048) nz = 2048;
  hipLaunchKernelGGL(head_ln_bwd_kernel, dim3((unsigned)(nrow + nz)), dim3(256), 0, s, dy, xhat, rstd, gamma, B, D, ntok, dtok, nrow);
  return hipGetLastError();
}

extern "C" hipError_t pvr_scale_by(const float* x, const float* sc, float* y, int64_t n, hipStream_t s) {
  using namespace pvr;
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(scale_by_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, sc, y, n);
  return hipGetLastError();
}

extern "C" hipError_t pvr_mean(const float* x, int n, float* out, hipStream_t s) {
  using namespace pvr;
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, s, x, n, out);
  return hipGetLastError();
}

extern "C" hipError_t pvr_metrics_accum(float* sums, const float* loss, const int* correct, int B, hipStream_t s) {
  using namespace pvr;
  hipLaunchKernelGGL(metrics_accum_kernel, dim3(1), dim3(256), 0, s, sums, loss, correct, B);
  return hipGetLastError();
}

extern "C" hipError_t pvr_rng_next(int64_t* rng, int64_t* seed, hipStream_t s) {
  using namespace pvr;
  hipLaunchKernelGGL(rng_next_kernel, dim3(1), dim3(64), 0, s, rng, seed);
  return hipGetLastError();
}

extern "C" hipError_t pvr_zero_f32(float* x, int64_t n, hipStream_t s) {
  using namespace pvr;
  if (n <= 0) return hipSuccess;
  if ((n & 3) || (reinterpret_cast<uintptr_t>(x) & 15)) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  int64_t blocks = (n4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(zero_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, reinterpret_cast<float4*>(x), n4);
  return hipGetLastError();
}
