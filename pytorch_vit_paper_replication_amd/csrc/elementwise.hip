// Memory-bound helper kernels (16-B vector accesses throughout, SURVEY.md K1-K4, K11 bias-grad):
//   * flat fp32 -> bf16 shadow cast of the parameter store
//   * bias-gradient column sums, optionally fused with the dropout-mask backward
//   * patch embedding: im2col gather (fp32 image -> bf16 patch rows), CLS rows, and the backward
//     reduction of the embedding-dropout / position-embedding / CLS gradients.
#include "common.h"

namespace pvr {
namespace {

__global__ void __launch_bounds__(256) cast_f32_bf16_kernel(const float* __restrict__ in, uint16_t* __restrict__ out, int64_t n) {
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = ((const float4*)in)[i];
    uint2 o;
    o.x = pack2bf(v.x, v.y);
    o.y = pack2bf(v.z, v.w);
    ((uint2*)out)[i] = o;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    out[i] = f2bf(in[i]);
  }
}

// dY [rows][N] (row stride ld) -> db[N] += column sums of (mask * dY); if dz != null also writes
// the masked gradient dz (= dropout backward) with row stride ld_dz.
// Q8: also the fp8 copy (qfmt 1 e5m2, 0 e4m3) of the (masked) gradient, q[r][n] = fp8(v * *qscale), and its amax record
// (the fp8 dgrad operand of the same tensor whose column sums are the bias gradient: one read, two uses)
template <bool Q8>
__global__ void __launch_bounds__(256) colsum_kernel(const uint16_t* __restrict__ dy, int64_t ld, int rows, int N,
                                                      float* __restrict__ db, uint16_t* __restrict__ dz, int64_t ld_dz,
                                                      const uint64_t* seed_ptr, uint64_t seed_off, uint32_t thr, float scale,
                                                      uint8_t* __restrict__ qout, int64_t ld_q, const float* __restrict__ qscale,
                                                      unsigned* __restrict__ amax, int qfmt, float* __restrict__ part) {
  __shared__ float red[4][64 * 8];
  const float qs = Q8 ? *qscale : 1.f;
  float qam = 0.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;  // 8-column chunk
  const bool act = c * 8 < N;
  const uint64_t seed = thr ? (*seed_ptr + seed_off) : 0ull;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (act) {
    // 4 rows per trip with their loads issued together (clamped rows, so the loads are
    // unconditional and the compiler counts them instead of draining vmcnt per row)
    constexpr int U = 4;
    const int stride = gridDim.y * 4;
    for (int r0 = blockIdx.y * 4 + wave; r0 < rows; r0 += U * stride) {
      uint4 q[U];
#pragma unroll
      for (int u = 0; u < U; ++u) q[u] = *(const uint4*)(dy + (int64_t)min(r0 + u * stride, rows - 1) * ld + c * 8);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + u * stride;
        if (r >= rows) break;
        const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
        float v[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[2 * j] = bf2f(w[j] & 0xFFFF);
          v[2 * j + 1] = bf2f(w[j] >> 16);
        }
        if (thr) {
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            bool k0, k1;
            rng_keep2(seed, (uint64_t)r * N + c * 8 + j, thr, k0, k1);
            v[j] = k0 ? v[j] * scale : 0.f;
            v[j + 1] = k1 ? v[j + 1] * scale : 0.f;
          }
        }
        if (dz) {
          uint4 o;
          o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
          o.z = pack2bf(v[4], v[5]); o.w = pack2bf(v[6], v[7]);
          *(uint4*)(dz + (int64_t)r * ld_dz + c * 8) = o;
        }
        if constexpr (Q8) {
          float vm = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) vm = nan_max(vm, fabsf(v[j]));
          qam = nan_max(qam, vm);
          *(uint2*)(qout + (int64_t)r * ld_q + c * 8) = pack8_fp8_fast_rt(qfmt, v, qs, vm);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 8; i += 256) {
    const int col = blockIdx.x * 64 * 8 + i;
    if (col < N && part)  // deterministic mode: this row group's partial (rows_reduce sums them in order)
      part[(int64_t)blockIdx.y * N + col] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    else if (col < N && db)
      atomicAdd(db + col, red[0][i] + red[1][i] + red[2][i] + red[3][i]);
  }
  if constexpr (Q8) {  // one amax atomic per workgroup
    qam = wave_max_nan(qam);
    __syncthreads();  // red[] reads above are done: reuse red[0][0..3]
    if (lane == 0) red[0][wave] = qam;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float m = nan_max(nan_max(red[0][0], red[0][1]), nan_max(red[0][2], red[0][3]));
      if (!(m <= 0.f)) atomicMax(amax, __float_as_uint(m));
    }
  }
}

// img [B][C][H][W] fp32 -> patches [B*np][Kp] bf16, k = (c*P + ph)*P + pw, zero padded to Kp.
// One thread per 8 consecutive k of a patch row: with P % 8 == 0 they are 8 consecutive pixels of
// one image row (two float4 loads, one 16-B store); the zero padding past C*P*P and other patch
// sizes (P = 14) take the per-element path.
__global__ void __launch_bounds__(256) im2col_kernel(const float* __restrict__ img, uint16_t* __restrict__ out,
                                                      int B, int C, int H, int W, int P, int Kp) {
  const int gw = W / P, np = (H / P) * gw;
  const int kc = C * P * P, k8 = Kp / 8;
  const bool vec = (P % 8 == 0) && (W % 4 == 0);
  const int64_t total = (int64_t)B * np * k8;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int k0 = (int)(i % k8) * 8;
    const int64_t rowi = i / k8;
    const int pidx = (int)(rowi % np);
    const int b = (int)(rowi / np);
    const int y0 = (pidx / gw) * P, x0 = (pidx % gw) * P;
    float v[8];
    if (vec && k0 + 8 <= kc) {
      const int c = k0 / (P * P), rem = k0 % (P * P), ph = rem / P, pw = rem % P;
      const float* src = img + (((int64_t)b * C + c) * H + y0 + ph) * W + x0 + pw;
      const float4 a = *(const float4*)src, bq = *(const float4*)(src + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = bq.x; v[5] = bq.y; v[6] = bq.z; v[7] = bq.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = k0 + j;
        v[j] = 0.f;
        if (k < kc) {
          const int c = k / (P * P), rem = k % (P * P), ph = rem / P, pw = rem % P;
          v[j] = img[(((int64_t)b * C + c) * H + y0 + ph) * W + x0 + pw];
        }
      }
    }
    uint4 o;
    o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]); o.z = pack2bf(v[4], v[5]); o.w = pack2bf(v[6], v[7]);
    *(uint4*)(out + rowi * Kp + k0) = o;
  }
}

// out[b][0][:] = dropout(cls + pos[0])   (row b*(np+1) of the token tensor)
__global__ void __launch_bounds__(256) cls_rows_kernel(const float* __restrict__ cls, const float* __restrict__ pos,
                                                        uint16_t* __restrict__ out, int B, int D, int64_t row_stride,
                                                        const uint64_t* seed_ptr, uint64_t seed_off, uint32_t thr, float scale,
                                                        int64_t ncols_total) {
  const uint64_t seed = thr ? (*seed_ptr + seed_off) : 0ull;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < B * D; i += gridDim.x * 256) {
    const int b = i / D, d = i % D;
    float v = cls[d] + pos[d];
    // dropout index uses the logical [B*(np+1), D] element index (row b*(np+1))
    if (thr) v = rng_keep(seed, (uint64_t)(b * (row_stride / D)) * D + d, thr) ? v * scale : 0.f;
    out[(int64_t)b * row_stride + d] = f2bf(v);
  }
}

// Backward of  E = dropout(concat(cls, conv) + pos):  dE [B][np+1][D] bf16 ->
//   dpre = dE * mask;  dpos[n][d] += sum_b dpre;  dcls[d] += sum_b dpre[b][0][d];
//   dconv[b*np + n-1][d] = dpre (bf16, n >= 1);  dbias[d] += sum_{b, n>=1} dpre.
// Two passes and (almost) no atomics: device-scope f32 atomics that pile onto a few KB of addresses
// (dbias: 768 columns) serialise. At ViT-B/16 b256 this is 33 us; the one-pass kernel that added
// per-block partials with atomics took 250 us, one adding per-thread partials ~450 us
// (scripts/atomics_probe.py, profiles/atomics_probe.log).
//  pass 1: thread = one (token, 8-column chunk) pair of the flattened [ntok][D/8] grid (every lane
//          busy; D/8 = 96 does not fill power-of-two blocks), block.y = a group of PB_BAT images;
//          8 independent 16-B loads in flight per thread; writes the masked gradient (dconv) and
//          the group's per-(token, column) sums to ws[group][ntok][D] with plain stores;
//  pass 2: thread = (8-column chunk, token) sums the groups, owns dpos[n] (and dcls for n = 0), and
//          the block reduces its tokens' dbias partials in LDS into one partial row per token block;
//  pass 3: the conv-bias gradient sums those rows in block order (deterministic, no atomics).
constexpr int PB_BAT = 32, PB_UNROLL = 8;
__global__ void __launch_bounds__(256) patch_bwd_kernel(const uint16_t* __restrict__ dE, int B, int ntok, int D,
                                                         float* __restrict__ ws, uint16_t* __restrict__ dconv,
                                                         const uint64_t* seed_ptr, uint64_t seed_off, uint32_t thr, float scale) {
  const uint64_t seed = thr ? (*seed_ptr + seed_off) : 0ull;
  const int nch = D >> 3;
  const int flat = blockIdx.x * 256 + threadIdx.x;
  if (flat >= ntok * nch) return;
  const int n = flat / nch, c = flat - n * nch;
  const int b0 = blockIdx.y * PB_BAT, b1 = min(B, b0 + PB_BAT);
  const int64_t img_stride = (int64_t)ntok * D;  // elements between consecutive images
  const uint16_t* src = dE + (int64_t)n * D + c * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int bb = b0; bb < b1; bb += PB_UNROLL) {
    uint4 q[PB_UNROLL];
#pragma unroll
    for (int u = 0; u < PB_UNROLL; ++u) q[u] = *(const uint4*)(src + (int64_t)min(bb + u, b1 - 1) * img_stride);
#pragma unroll
    for (int u = 0; u < PB_UNROLL; ++u) {
      const int b = bb + u;
      if (b >= b1) break;
      const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[2 * j] = bf2f(w[j] & 0xFFFF);
        v[2 * j + 1] = bf2f(w[j] >> 16);
      }
      if (thr) {
        const uint64_t e0 = ((uint64_t)b * ntok + n) * D + c * 8;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          bool k0, k1;
          rng_keep2(seed, e0 + j, thr, k0, k1);
          v[j] = k0 ? v[j] * scale : 0.f;
          v[j + 1] = k1 ? v[j + 1] * scale : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += v[j];
      if (n > 0 && dconv) {
        uint4 o;
        o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]); o.z = pack2bf(v[4], v[5]); o.w = pack2bf(v[6], v[7]);
        *(uint4*)(dconv + ((int64_t)b * (ntok - 1) + n - 1) * D + c * 8) = o;
      }
    }
  }
  float* o = ws + ((int64_t)blockIdx.y * ntok + n) * D + c * 8;
  *(float4*)o = make_float4(s[0], s[1], s[2], s[3]);
  *(float4*)(o + 4) = make_float4(s[4], s[5], s[6], s[7]);
}

constexpr int PR_CH = 32, PR_TOK = 8;  // pass-2 block: 32 column chunks x 8 tokens
__global__ void __launch_bounds__(256) patch_bwd_reduce_kernel(const float* __restrict__ ws, int G, int ntok, int D,
                                                                float* __restrict__ dpos, float* __restrict__ dcls,
                                                                float* __restrict__ dbias_part) {
  __shared__ float red[PR_TOK][PR_CH * 8];
  const int nch = D >> 3;
  const int cl = threadIdx.x % PR_CH, tl = threadIdx.x / PR_CH;
  const int c = blockIdx.x * PR_CH + cl;
  const int n = blockIdx.y * PR_TOK + tl;
  float t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool ok = c < nch && n < ntok;
  if (ok) {
    const float* src = ws + (int64_t)n * D + c * 8;
    const int64_t gs = (int64_t)ntok * D;
    int g = 0;
    for (; g + 4 <= G; g += 4) {
      float4 a[8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[2 * u] = *(const float4*)(src + (g + u) * gs);
        a[2 * u + 1] = *(const float4*)(src + (g + u) * gs + 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        t[0] += a[2 * u].x; t[1] += a[2 * u].y; t[2] += a[2 * u].z; t[3] += a[2 * u].w;
        t[4] += a[2 * u + 1].x; t[5] += a[2 * u + 1].y; t[6] += a[2 * u + 1].z; t[7] += a[2 * u + 1].w;
      }
    }
    for (; g < G; ++g) {
      const float4 a0 = *(const float4*)(src + g * gs), a1 = *(const float4*)(src + g * gs + 4);
      t[0] += a0.x; t[1] += a0.y; t[2] += a0.z; t[3] += a0.w;
      t[4] += a1.x; t[5] += a1.y; t[6] += a1.z; t[7] += a1.w;
    }
    if (dpos) {  // this thread owns dpos[n][c*8 .. +8]
      float* d = dpos + (int64_t)n * D + c * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] += t[j];
    }
    if (n == 0 && dcls) {
#pragma unroll
      for (int j = 0; j < 8; ++j) dcls[c * 8 + j] += t[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tl][cl * 8 + j] = (ok && n > 0) ? t[j] : 0.f;
  __syncthreads();
  if (dbias_part) {  // this token block's partial column sums (summed in block order below: deterministic)
    const int col = blockIdx.x * PR_CH * 8 + threadIdx.x;  // 256 columns per block, one per thread
    if (col < D) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < PR_TOK; ++k) a += red[k][threadIdx.x];
      dbias_part[(int64_t)blockIdx.y * D + col] = a;
    }
  }
}

// Deterministic column reduction of partial rows: dst[c] += sum_r part[r][c] in row order, the C
// columns split into segments of `seg` going to d0 / d1 / d2 (null: dropped). Block = 8 row lanes x
// 32 columns; lane rl sums rows rl, rl + 8, ... and the 8 lane sums are added in lane order: the same
// bits on every run (the float-atomic reductions it replaces are order-dependent).
__global__ void __launch_bounds__(256) rows_reduce_kernel(const float* __restrict__ part, int R, int C, int seg,
                                                           float* __restrict__ d0, float* __restrict__ d1, float* __restrict__ d2) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float a = 0.f;
  if (c < C) {
    int r = rl;
    for (; r + 24 < R; r += 32) {  // four independent loads in flight
      const float x0 = part[(int64_t)r * C + c], x1 = part[(int64_t)(r + 8) * C + c];
      const float x2 = part[(int64_t)(r + 16) * C + c], x3 = part[(int64_t)(r + 24) * C + c];
      a += x0; a += x1; a += x2; a += x3;
    }
    for (; r < R; r += 8) a += part[(int64_t)r * C + c];
  }
  red[rl][cl] = a;
  __syncthreads();
  if (rl == 0 && c < C) {
    float t = red[0][cl];
#pragma unroll
    for (int k = 1; k < 8; ++k) t += red[k][cl];
    float* d = c < seg ? d0 : (c < 2 * seg ? d1 : d2);
    if (d) d[c % seg] += t;
  }
}

// Batched bf16 transpose: matrix t (rows R_t, cols C_t) at src + soff[t] -> dst + doff[t] as [C_t][R_t].
// 64x64 tiles through LDS held as bf16 pairs (u32, 33-word rows: conflict-free column reads);
// 16-B loads and stores, 8 lanes per 128-B row. tile_start[t] = prefix tile count (binary search).
__global__ void __launch_bounds__(256) transpose_batched_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                                 const int64_t* __restrict__ meta, int nmat) {
  __shared__ uint32_t tile[64][33];
  const int blk = blockIdx.x;
  int lo = 0, hi = nmat - 1;  // last t with tile_start[t] <= blk
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (meta[mid * 5 + 4] <= blk) lo = mid; else hi = mid - 1;
  }
  const int t = lo;
  const int64_t soff = meta[t * 5 + 0], doff = meta[t * 5 + 1];
  const int R = (int)meta[t * 5 + 2], C = (int)meta[t * 5 + 3];
  const int local = blk - (int)meta[t * 5 + 4];
  const int tc = (C + 63) / 64;
  const int r0 = (local / tc) * 64, c0 = (local % tc) * 64;
  const bool full = r0 + 64 <= R && c0 + 64 <= C && (C % 8) == 0 && (R % 8) == 0 && (soff % 8) == 0 && (doff % 8) == 0;
  const int tid = threadIdx.x;
  if (full) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int row = tid / 8 + 32 * it, ch = tid % 8;
      const uint4 q = *(const uint4*)(src + soff + (int64_t)(r0 + row) * C + c0 + ch * 8);
      tile[row][ch * 4 + 0] = q.x; tile[row][ch * 4 + 1] = q.y;
      tile[row][ch * 4 + 2] = q.z; tile[row][ch * 4 + 3] = q.w;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int idx = tid + 256 * it;
      const int cc = idx / 8, rch = idx % 8;  // output row (input column) cc, input rows rch*8 .. +7
      uint32_t h[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) h[j] = (tile[rch * 8 + j][cc >> 1] >> ((cc & 1) * 16)) & 0xFFFFu;
      uint4 o;
      o.x = h[0] | (h[1] << 16); o.y = h[2] | (h[3] << 16); o.z = h[4] | (h[5] << 16); o.w = h[6] | (h[7] << 16);
      *(uint4*)(dst + doff + (int64_t)(c0 + cc) * R + r0 + rch * 8) = o;
    }
    return;
  }
  uint16_t* t16 = (uint16_t*)&tile[0][0];  // edge tiles: element-wise through [64][66] bf16
  for (int i = tid; i < 64 * 64; i += 256) {
    const int rr = i / 64, cc = i % 64;
    if (r0 + rr < R && c0 + cc < C) t16[rr * 66 + cc] = src[soff + (int64_t)(r0 + rr) * C + c0 + cc];
  }
  __syncthreads();
  for (int i = tid; i < 64 * 64; i += 256) {
    const int cc = i / 64, rr = i % 64;
    if (r0 + rr < R && c0 + cc < C) dst[doff + (int64_t)(c0 + cc) * R + r0 + rr] = t16[rr * 66 + cc];
  }
}

// out (+)= sum over S split-K partial slices ws[s] (the second half of the store-then-reduce wgrad,
// tile 14); fixed slice order, so the result is deterministic. ws rows hold wcols floats, out rows
// the first ocols of them (ocols <= wcols, both % 4 == 0): a GEMM over a K padded to the tile width
// reduces straight into the unpadded weight gradient.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ ws, int S, int64_t stride,
                                                            float* __restrict__ out, int64_t n4, int ocols, int wcols,
                                                            int accumulate) {
  const int oc4 = ocols / 4;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 a = accumulate ? ((const float4*)out)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t row = i / oc4;
    const float* src = ws + row * wcols + 4 * (i - row * oc4);
    int s = 0;
    for (; s + 4 <= S; s += 4) {  // 4 independent loads in flight per trip
      const float4 b0 = *(const float4*)(src + (int64_t)s * stride);
      const float4 b1 = *(const float4*)(src + (int64_t)(s + 1) * stride);
      const float4 b2 = *(const float4*)(src + (int64_t)(s + 2) * stride);
      const float4 b3 = *(const float4*)(src + (int64_t)(s + 3) * stride);
      a.x += (b0.x + b1.x) + (b2.x + b3.x);
      a.y += (b0.y + b1.y) + (b2.y + b3.y);
      a.z += (b0.z + b1.z) + (b2.z + b3.z);
      a.w += (b0.w + b1.w) + (b2.w + b3.w);
    }
    for (; s < S; ++s) {
      const float4 b = *(const float4*)(src + (int64_t)s * stride);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    ((float4*)out)[i] = a;
  }
}

// dst[r][c] = c < cols ? src[r][c] : 0 for c < ld_dst (bf16; cols, ld_dst % 4 == 0): the patch
// embedding's conv weight [D][C*P*P] zero-padded to the GEMM's K tile
__global__ void __launch_bounds__(256) pad_cols_bf16_kernel(const uint16_t* __restrict__ src, int rows, int cols,
                                                            uint16_t* __restrict__ dst, int ld_dst) {
  const int q = ld_dst / 4;
  const int64_t n4 = (int64_t)rows * q;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / q;
    const int c = 4 * (int)(i - r * q);
    uint2 v = make_uint2(0u, 0u);
    if (c < cols) v = *(const uint2*)(src + r * cols + c);
    *(uint2*)(dst + r * ld_dst + c) = v;
  }
}

}  // namespace
}  // namespace pvr

extern "C" hipError_t pvr_splitk_reduce(const float* ws, int S, int64_t stride, float* out, int64_t n, int ocols, int wcols,
                                        int accumulate, hipStream_t s) {
  using namespace pvr;
  if (n <= 0) return hipSuccess;
  if (n % 4 || stride % 4 || ocols <= 0 || ocols % 4 || wcols % 4 || ocols > wcols || n % ocols) return hipErrorInvalidValue;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws, S, stride, out, n / 4, ocols, wcols,
                     accumulate);
  return hipGetLastError();
}

extern "C" hipError_t pvr_pad_cols_bf16(const uint16_t* src, int rows, int cols, uint16_t* dst, int ld_dst, hipStream_t s) {
  using namespace pvr;
  if (rows <= 0) return hipSuccess;
  if (cols % 4 || ld_dst % 4 || cols > ld_dst) return hipErrorInvalidValue;
  int64_t blocks = ((int64_t)rows * (ld_dst / 4) + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(pad_cols_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, rows, cols, dst, ld_dst);
  return hipGetLastError();
}

// meta: int64 [nmat][5] = {src_off, dst_off, rows, cols, tile_prefix}; total_tiles = sum of tiles
extern "C" hipError_t pvr_transpose_batched(const uint16_t* src, uint16_t* dst, const int64_t* meta, int nmat, int total_tiles,
                                            hipStream_t s) {
  using namespace pvr;
  if (total_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(transpose_batched_kernel, dim3(total_tiles), dim3(256), 0, s, src, dst, meta, nmat);
  return hipGetLastError();
}

extern "C" hipError_t pvr_cast_f32_bf16(const float* in, uint16_t* out, int64_t n, hipStream_t s) {
  using namespace pvr;
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, out, n);
  return hipGetLastError();
}

// row groups of the column-sum kernel's grid (= the partial rows of its deterministic mode)
extern "C" int pvr_colsum_part_rows(int rows) {
  const int gy = (rows + 63) / 64;
  return gy > 256 ? 256 : gy;
}
extern "C" hipError_t pvr_rows_reduce(const float* part, int R, int C, int seg, float* d0, float* d1, float* d2, hipStream_t s);

extern "C" hipError_t pvr_colsum(const uint16_t* dy, int64_t ld, int rows, int N, float* db, uint16_t* dz, int64_t ld_dz,
                                 const uint64_t* seed_ptr, uint64_t seed_off, uint32_t thr, float scale, uint8_t* q, int64_t ld_q,
                                 const float* qscale, unsigned* amax, int qfmt, float* part, hipStream_t s) {
  using namespace pvr;
  if (rows <= 0) return hipSuccess;
  if (N % 8 != 0 || (qfmt != 0 && qfmt != 1)) return hipErrorInvalidValue;
  if (q && (!qscale || !amax || ld_q % 8 != 0 || reinterpret_cast<uintptr_t>(q) % 8 != 0)) return hipErrorInvalidValue;
  const int gx = (N / 8 + 63) / 64;
  const int gy = pvr_colsum_part_rows(rows);
  if (!db) part = nullptr;
  hipLaunchKernelGGL(q ? colsum_kernel<true> : colsum_kernel<false>, dim3(gx, gy), dim3(256), 0, s, dy, ld, rows, N, db, dz, ld_dz,
                     seed_ptr, seed_off, thr, scale, q, ld_q, qscale, amax, qfmt, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !part) return e;
  return pvr_rows_reduce(part, gy, N, N, db, nullptr, nullptr, s);
}

extern "C" hipError_t pvr_im2col(const float* img, uint16_t* out, int B, int C, int H, int W, int P, int Kp, hipStream_t s) {
  using namespace pvr;
  if (Kp % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)B * (H / P) * (W / P) * (Kp / 8);
  if (total <= 0) return hipSuccess;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)blocks), dim3(256), 0, s, img, out, B, C, H, W, P, Kp);
  return hipGetLastError();
}

extern "C" hipError_t pvr_cls_rows(const float* cls, const float* pos, uint16_t* out, int B, int D, int64_t row_stride,
                                   const uint64_t* seed_ptr, uint64_t seed_off, uint32_t thr, float scale, hipStream_t s) {
  using namespace pvr;
  if (B * D <= 0) return hipSuccess;
  int blocks = (B * D + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(cls_rows_kernel, dim3(blocks), dim3(256), 0, s, cls, pos, out, B, D, row_stride, seed_ptr, seed_off, thr, scale, (int64_t)0);
  return hipGetLastError();
}

extern "C" hipError_t pvr_patch_bwd(const uint16_t* dE, int B, int ntok, int D, float* ws, float* dpos, float* dcls,
                                    uint16_t* dconv, float* dbias, const uint64_t* seed_ptr, uint64_t seed_off, uint32_t thr,
                                    float scale, hipStream_t s) {
  using namespace pvr;
  if (ntok * D <= 0 || B <= 0) return hipSuccess;
  if (D % 8) return hipErrorInvalidValue;
  const int G = (B + PB_BAT - 1) / PB_BAT;  // ws holds G * ntok * D floats (host-checked)
  hipLaunchKernelGGL(patch_bwd_kernel, dim3((ntok * (D / 8) + 255) / 256, G), dim3(256), 0, s, dE, B, ntok, D, ws, dconv,
                     seed_ptr, seed_off, thr, scale);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // ws also holds the conv-bias partials of the reduction's token blocks, after the group sums
  const int RB = (ntok + PR_TOK - 1) / PR_TOK;
  float* part = dbias ? ws + (int64_t)G * ntok * D : nullptr;
  hipLaunchKernelGGL(patch_bwd_reduce_kernel, dim3((D / 8 + PR_CH - 1) / PR_CH, RB), dim3(256), 0, s,
                     ws, G, ntok, D, dpos, dcls, part);
  e = hipGetLastError();
  if (e != hipSuccess || !dbias) return e;
  hipLaunchKernelGGL(rows_reduce_kernel, dim3((D + 31) / 32), dim3(256), 0, s, part, RB, D, D, dbias, (float*)nullptr, (float*)nullptr);
  return hipGetLastError();
}

extern "C" int pvr_patch_bwd_groups(int B) { return (B + pvr::PB_BAT - 1) / pvr::PB_BAT; }

// d0/d1/d2[c % seg] += sum over the R rows of part[R][C] (row order: deterministic)
extern "C" hipError_t pvr_rows_reduce(const float* part, int R, int C, int seg, float* d0, float* d1, float* d2, hipStream_t s) {
  if (R <= 0 || C <= 0) return hipSuccess;
  if (seg <= 0 || C > 3 * seg) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pvr::rows_reduce_kernel, dim3((C + 31) / 32), dim3(256), 0, s, part, R, C, seg, d0, d1, d2);
  return hipGetLastError();
}
// floats of the scratch pvr_patch_bwd needs: the group sums and the conv-bias partials
extern "C" int64_t pvr_patch_bwd_ws_floats(int B, int ntok, int D) {
  return ((int64_t)pvr_patch_bwd_groups(B) * ntok + (ntok + pvr::PR_TOK - 1) / pvr::PR_TOK) * D;
}

// Second half of the small-M split-K forward GEMM (few output tiles: serving-size batches): sum the
// S fp32 partial products ws[s][m][n] in a fixed order (deterministic) and apply the forward
// epilogue: + bias, exact-erf GELU (no derivative saved: inference), + residual, bf16 store.
// One thread per 4 consecutive columns of a row (N % 4 == 0).
namespace pvr {
namespace {
__global__ void __launch_bounds__(256) splitk_epilogue_kernel(const float* __restrict__ ws, int S, int64_t stride, int M, int N,
                                                              const float* __restrict__ bias, const uint16_t* __restrict__ resid,
                                                              int64_t ld_resid, int gelu, uint16_t* __restrict__ out, int64_t ldc) {
  const int n4 = N / 4;
  const int64_t total = (int64_t)M * n4;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int m = (int)(i / n4), n = (int)(i % n4) * 4;
    const float* src = ws + (int64_t)m * N + n;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = 0;
    for (; s + 4 <= S; s += 4) {  // 4 independent loads in flight per trip
      const float4 b0 = *(const float4*)(src + (int64_t)s * stride);
      const float4 b1 = *(const float4*)(src + (int64_t)(s + 1) * stride);
      const float4 b2 = *(const float4*)(src + (int64_t)(s + 2) * stride);
      const float4 b3 = *(const float4*)(src + (int64_t)(s + 3) * stride);
      a.x += (b0.x + b1.x) + (b2.x + b3.x);
      a.y += (b0.y + b1.y) + (b2.y + b3.y);
      a.z += (b0.z + b1.z) + (b2.z + b3.z);
      a.w += (b0.w + b1.w) + (b2.w + b3.w);
    }
    for (; s < S; ++s) {
      const float4 b = *(const float4*)(src + (int64_t)s * stride);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float v[4] = {a.x, a.y, a.z, a.w};
    if (bias) {
      const float4 b = *(const float4*)(bias + n);
      v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
    }
    if (gelu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float g, gp;
        gelu_and_grad(v[r], g, gp);
        v[r] = g;
      }
    }
    if (resid) {
      const uint2 rr = *(const uint2*)(resid + (int64_t)m * ld_resid + n);
      v[0] += bf2f(rr.x & 0xFFFF); v[1] += bf2f(rr.x >> 16);
      v[2] += bf2f(rr.y & 0xFFFF); v[3] += bf2f(rr.y >> 16);
    }
    uint2 o; o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
    *(uint2*)(out + (int64_t)m * ldc + n) = o;
  }
}
}  // namespace
}  // namespace pvr

extern "C" hipError_t pvr_splitk_epilogue(const float* ws, int S, int64_t stride, int M, int N, const float* bias,
                                          const uint16_t* resid, int64_t ld_resid, int gelu, uint16_t* out, int64_t ldc,
                                          hipStream_t s) {
  using namespace pvr;
  if (M <= 0 || N <= 0) return hipSuccess;
  if (N % 4 || S < 1) return hipErrorInvalidValue;
  int64_t blocks = ((int64_t)M * (N / 4) + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws, S, stride, M, N, bias, resid, ld_resid,
                     gelu, out, ldc);
  return hipGetLastError();
}
