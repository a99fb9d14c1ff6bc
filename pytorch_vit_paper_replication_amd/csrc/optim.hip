// Optimizer path over the flat parameter store:
//   * deterministic two-stage global L2 norm of the flat fp32 gradient buffer, finalised on the
//     device into {norm, clip coefficient, non-finite flag} (no host sync, identical on every DP rank)
//   * one fused Adam/AdamW pass: clip scale folded into the gradient read, coupled L2 (torch.optim.Adam
//     weight_decay) or decoupled decay, bias correction, fp32 master update, and the bf16 shadow copy
//     the next forward's GEMMs read, all in the same sweep over memory.
// Replaces clip_grad_norm_'s foreach kernels and torch.optim.Adam's ~7 ops per tensor
// (reference GM/engine.py:63-66; MAIN.ipynb:2818-2824).
#include "common.h"

namespace pvr {

struct AdamGroup {
  float lr, beta1, beta2, eps, weight_decay;
  float bc1, bc2_sqrt;  // 1 - beta1^t, sqrt(1 - beta2^t)
  int decoupled;
};

// Group table passed by value in the kernel arguments (eager stepping: no per-step host-to-device
// copy); graph-captured steps pass a device table instead (kernel arguments are frozen at capture).
constexpr int MAX_ARG_GROUPS = 8;
struct AdamGroupArgs {
  AdamGroup g[MAX_ARG_GROUPS];
};

namespace {

constexpr int NORM_BLOCKS = 1024;

__global__ void __launch_bounds__(256) sumsq_partial_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = ((const float4*)g)[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const float v = g[n4 * 4 + threadIdx.x];
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out[0] = ||g||, out[1] = min(1, max_norm / (||g|| + 1e-6)), out[2] = 1 if non-finite
__global__ void __launch_bounds__(256) norm_finalize_kernel(const float* __restrict__ partial, int np, float max_norm, float* __restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) s += (double)partial[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = (float)sqrt((red[0] + red[1]) + (red[2] + red[3]));
    const bool bad = !isfinite(norm);
    float coef = max_norm > 0.f ? max_norm / (norm + 1e-6f) : 1.f;
    if (coef > 1.f) coef = 1.f;
    out[0] = norm;
    out[1] = coef;
    out[2] = bad ? 1.f : 0.f;
  }
}

// seg_start[i] = first flat index of segment i (sorted), seg_group[i] = its param group.
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, uint16_t* __restrict__ shadow, int64_t n,
                                                    const int64_t* __restrict__ seg_start, const int* __restrict__ seg_group, int nseg,
                                                    const AdamGroup* __restrict__ groups, AdamGroupArgs garg,
                                                    const float* __restrict__ clip, int skip_nonfinite) {
  const float gscale = clip ? clip[1] : 1.f;
  if (clip && skip_nonfinite && clip[2] != 0.f) return;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 4;
    // binary search the segment containing e (segments are 4-element aligned by construction)
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (seg_start[mid] <= e) lo = mid; else hi = mid - 1;
    }
    const int gi = seg_group[lo];
    if (gi < 0) continue;  // frozen / padding
    const AdamGroup G = groups ? groups[gi] : garg.g[gi];
    float4 pp = ((float4*)p)[i];
    const float4 gg4 = ((const float4*)g)[i];
    float4 mm = ((float4*)m)[i];
    float4 vv = ((float4*)v)[i];
    float* pa = &pp.x; const float* ga = &gg4.x; float* ma = &mm.x; float* va = &vv.x;
    const float step = G.lr / G.bc1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gr = ga[j] * gscale;
      if (G.decoupled) {
        pa[j] *= 1.f - G.lr * G.weight_decay;
      } else if (G.weight_decay != 0.f) {
        gr += G.weight_decay * pa[j];
      }
      ma[j] = G.beta1 * ma[j] + (1.f - G.beta1) * gr;
      va[j] = G.beta2 * va[j] + (1.f - G.beta2) * gr * gr;
      const float denom = sqrtf(va[j]) / G.bc2_sqrt + G.eps;
      pa[j] -= step * ma[j] / denom;
    }
    ((float4*)p)[i] = pp;
    ((float4*)m)[i] = mm;
    ((float4*)v)[i] = vv;
    if (shadow) {
      uint2 o;
      o.x = pack2bf(pp.x, pp.y);
      o.y = pack2bf(pp.z, pp.w);
      ((uint2*)shadow)[i] = o;
    }
  }
}

// Adam + bf16 shadow + bf16 TRANSPOSED shadow in one pass (the dgrad GEMMs' k-contiguous W^T, which
// otherwise takes a separate transpose pass over every weight after each step).
// Blocks [0, ntiles): one 64x64 fp32 tile of a registered 2-D weight W [R][C] (R, C multiples of 64):
//   tmeta row {flat offset, W^T offset in shadow_t, R, C, first tile, param group}; the tile's p / g /
//   m / v are read and written row-major (16 lanes x 16 B per 256-B row), the bf16 values go to the
//   shadow and, through a [64][33] x 2-bf16 LDS image, to W^T [C][R] as 16-B column-row pieces.
// Blocks [ntiles, grid): grid-stride over every other parameter: fmeta row {flat start, elements
//   (multiple of 4), param group, first float4 of the range in the concatenation}.
__device__ __forceinline__ void adam4(float4& pp, const float4& gg4, float4& mm, float4& vv, const AdamGroup& G, float gscale) {
  float* pa = &pp.x; const float* ga = &gg4.x; float* ma = &mm.x; float* va = &vv.x;
  const float step = G.lr / G.bc1;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float gr = ga[j] * gscale;
    if (G.decoupled) {
      pa[j] *= 1.f - G.lr * G.weight_decay;
    } else if (G.weight_decay != 0.f) {
      gr += G.weight_decay * pa[j];
    }
    ma[j] = G.beta1 * ma[j] + (1.f - G.beta1) * gr;
    va[j] = G.beta2 * va[j] + (1.f - G.beta2) * gr * gr;
    const float denom = sqrtf(va[j]) / G.bc2_sqrt + G.eps;
    pa[j] -= step * ma[j] / denom;
  }
}

__global__ void __launch_bounds__(256) adam_t_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                                      float* __restrict__ v, uint16_t* __restrict__ shadow, uint16_t* __restrict__ shadow_t,
                                                      const int64_t* __restrict__ tmeta, int nmat, int ntiles,
                                                      const int64_t* __restrict__ fmeta, int nflat, int64_t flat4,
                                                      const AdamGroup* __restrict__ groups, AdamGroupArgs garg,
                                                      const float* __restrict__ clip, int skip_nonfinite) {
  const float gscale = clip ? clip[1] : 1.f;
  if (clip && skip_nonfinite && clip[2] != 0.f) return;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x < ntiles) {
    __shared__ uint32_t tile[64][33];
    const int blk = blockIdx.x;
    int lo = 0, hi = nmat - 1;  // last weight whose first tile <= blk
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tmeta[mid * 6 + 4] <= blk) lo = mid; else hi = mid - 1;
    }
    const int64_t soff = tmeta[lo * 6 + 0], doff = tmeta[lo * 6 + 1];
    const int R = (int)tmeta[lo * 6 + 2], C = (int)tmeta[lo * 6 + 3];
    const int gi = (int)tmeta[lo * 6 + 5];
    const int local = blk - (int)tmeta[lo * 6 + 4];
    const int tc = C / 64;
    const int r0 = (local / tc) * 64, c0 = (local % tc) * 64;
    if (gi < 0) return;  // frozen: master, shadow and W^T unchanged
    const AdamGroup G = groups ? groups[gi] : garg.g[gi];
    const int cq = (tid & 15) * 4;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = (tid >> 4) + 16 * it;
      const int64_t e = soff + (int64_t)(r0 + row) * C + c0 + cq;
      float4 pp = *(float4*)(p + e);
      const float4 gg4 = *(const float4*)(g + e);
      float4 mm = *(float4*)(m + e);
      float4 vv = *(float4*)(v + e);
      adam4(pp, gg4, mm, vv, G, gscale);
      *(float4*)(p + e) = pp;
      *(float4*)(m + e) = mm;
      *(float4*)(v + e) = vv;
      const uint32_t lo2 = pack2bf(pp.x, pp.y), hi2 = pack2bf(pp.z, pp.w);
      *(uint2*)(shadow + e) = make_uint2(lo2, hi2);
      tile[row][cq >> 1] = lo2;
      tile[row][(cq >> 1) + 1] = hi2;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int idx = tid + 256 * it;
      const int cc = idx / 8, rch = idx % 8;  // W^T row c0 + cc, W rows r0 + 8 rch .. + 7
      uint32_t h[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) h[j] = (tile[rch * 8 + j][cc >> 1] >> ((cc & 1) * 16)) & 0xFFFFu;
      uint4 o;
      o.x = h[0] | (h[1] << 16); o.y = h[2] | (h[3] << 16); o.z = h[4] | (h[5] << 16); o.w = h[6] | (h[7] << 16);
      *(uint4*)(shadow_t + doff + (int64_t)(c0 + cc) * R + r0 + rch * 8) = o;
    }
    return;
  }
  const int64_t nblk = (int64_t)gridDim.x - ntiles;
  for (int64_t i = ((int64_t)blockIdx.x - ntiles) * 256 + tid; i < flat4; i += nblk * 256) {
    int lo = 0, hi = nflat - 1;  // range holding float4 i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (fmeta[mid * 4 + 3] <= i) lo = mid; else hi = mid - 1;
    }
    const int gi = (int)fmeta[lo * 4 + 2];
    if (gi < 0) continue;
    const int64_t e = fmeta[lo * 4 + 0] + (i - fmeta[lo * 4 + 3]) * 4;
    const AdamGroup G = groups ? groups[gi] : garg.g[gi];
    float4 pp = *(float4*)(p + e);
    const float4 gg4 = *(const float4*)(g + e);
    float4 mm = *(float4*)(m + e);
    float4 vv = *(float4*)(v + e);
    adam4(pp, gg4, mm, vv, G, gscale);
    *(float4*)(p + e) = pp;
    *(float4*)(m + e) = mm;
    *(float4*)(v + e) = vv;
    *(uint2*)(shadow + e) = make_uint2(pack2bf(pp.x, pp.y), pack2bf(pp.z, pp.w));
  }
}

__global__ void __launch_bounds__(256) scale_kernel(float* __restrict__ g, int64_t n, const float* __restrict__ clip) {
  const float c = clip[1];
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) g[i] *= c;
}

// host: copy a [ngroups] table into the by-value kernel argument (false: too many groups)
bool adam_group_args(const AdamGroup* host, int ngroups, AdamGroupArgs& out) {
  if (!host || ngroups <= 0 || ngroups > MAX_ARG_GROUPS) return false;
  for (int i = 0; i < ngroups; ++i) out.g[i] = host[i];
  return true;
}

}  // namespace
}  // namespace pvr

extern "C" int pvr_norm_partial_blocks() { return pvr::NORM_BLOCKS; }

// workspace: NORM_BLOCKS floats. out: 3 floats.
extern "C" hipError_t pvr_grad_norm(const float* g, int64_t n, float max_norm, float* workspace, float* out, hipStream_t s) {
  using namespace pvr;
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(NORM_BLOCKS), dim3(256), 0, s, g, n, workspace);
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(256), 0, s, workspace, NORM_BLOCKS, max_norm, out);
  return hipGetLastError();
}

extern "C" hipError_t pvr_adam(float* p, const float* g, float* m, float* v, uint16_t* shadow, int64_t n,
                               const int64_t* seg_start, const int* seg_group, int nseg, const pvr::AdamGroup* groups,
                               const pvr::AdamGroup* host_groups, int ngroups, const float* clip, int skip_nonfinite,
                               hipStream_t s) {
  using namespace pvr;
  if (n <= 0) return hipSuccess;
  if (n % 4 != 0) return hipErrorInvalidValue;
  AdamGroupArgs ga{};
  if (!groups && !adam_group_args(host_groups, ngroups, ga)) return hipErrorInvalidValue;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, g, m, v, shadow, n, seg_start, seg_group, nseg,
                     groups, ga, clip, skip_nonfinite);
  return hipGetLastError();
}

extern "C" hipError_t pvr_scale_by_clip(float* g, int64_t n, const float* clip, hipStream_t s) {
  using namespace pvr;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) return hipSuccess;
  hipLaunchKernelGGL(scale_kernel, dim3((unsigned)blocks), dim3(256), 0, s, g, n, clip);
  return hipGetLastError();
}

// Adam with the transposed bf16 shadow (adam_t_kernel): tmeta int64 [nmat][6], fmeta int64 [nflat][4]
// (see the kernel), flat4 = float4s covered by fmeta.
extern "C" hipError_t pvr_adam_t(float* p, const float* g, float* m, float* v, uint16_t* shadow, uint16_t* shadow_t,
                                 const int64_t* tmeta, int nmat, int ntiles, const int64_t* fmeta, int nflat, int64_t flat4,
                                 const pvr::AdamGroup* groups, const pvr::AdamGroup* host_groups, int ngroups,
                                 const float* clip, int skip_nonfinite, hipStream_t s) {
  using namespace pvr;
  if (nmat <= 0 || ntiles <= 0 || nflat <= 0) return hipErrorInvalidValue;
  AdamGroupArgs ga{};
  if (!groups && !adam_group_args(host_groups, ngroups, ga)) return hipErrorInvalidValue;
  int64_t fb = (flat4 + 255) / 256;
  if (fb > 1024) fb = 1024;
  if (fb < 1) fb = 1;
  hipLaunchKernelGGL(adam_t_kernel, dim3((unsigned)(ntiles + fb)), dim3(256), 0, s, p, g, m, v, shadow, shadow_t, tmeta, nmat,
                     ntiles, fmeta, nflat, flat4, groups, ga, clip, skip_nonfinite);
  return hipGetLastError();
}
