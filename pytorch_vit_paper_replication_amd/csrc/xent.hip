// Fused softmax cross-entropy for the classifier logits (reference GM/engine.py:53, :73-74;
// SURVEY.md K13 + K16): one pass produces the per-row loss, d(loss)/d(logits) for the mean
// reduction, and the argmax==label flag per row for the accuracy metric, so the engine does not
// need a separate softmax/argmax/eq/sum chain or a host sync per batch.
#include "common.h"

namespace pvr {
namespace {

__global__ void __launch_bounds__(256) xent_kernel(const float* __restrict__ logits, int64_t ld, const int64_t* __restrict__ labels,
                                                    int B, int C, float* __restrict__ loss_rows, float* __restrict__ dlogits,
                                                    int* __restrict__ correct, float grad_scale) {
  __shared__ float smax[4], ssum[4];
  __shared__ int sidx[4];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* x = logits + (int64_t)b * ld;
  // max and first argmax
  float m = -INFINITY;
  int mi = 0x7FFFFFFF;
  for (int c = tid; c < C; c += 256) {
    const float v = x[c];
    if (v > m || (v == m && c < mi)) { m = v; mi = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    if (om > m || (om == m && oi < mi)) { m = om; mi = oi; }
  }
  if (lane == 0) { smax[wave] = m; sidx[wave] = mi; }
  __syncthreads();
  m = smax[0]; mi = sidx[0];
  for (int w = 1; w < 4; ++w)
    if (smax[w] > m || (smax[w] == m && sidx[w] < mi)) { m = smax[w]; mi = sidx[w]; }
  float s = 0.f;
  for (int c = tid; c < C; c += 256) s += __expf(x[c] - m);
  s = wave_sum(s);
  if (lane == 0) ssum[wave] = s;
  __syncthreads();
  s = ssum[0] + ssum[1] + ssum[2] + ssum[3];
  const float lse = m + __logf(s);
  const int64_t y = labels[b];
  const bool valid = y >= 0 && y < C;  // out-of-range labels (e.g. ignore_index) contribute nothing
  if (tid == 0) {
    loss_rows[b] = valid ? lse - x[y] : 0.f;
    if (correct) correct[b] = mi == (int)y ? 1 : 0;  // per-row flag: no zeroed counter needed
  }
  if (dlogits) {
    const float inv = 1.f / s;
    for (int c = tid; c < C; c += 256) {
      float p = __expf(x[c] - m) * inv;
      if (c == y) p -= 1.f;
      dlogits[(int64_t)b * C + c] = valid ? p * grad_scale : 0.f;
    }
  }
}

}  // namespace
}  // namespace pvr

extern "C" hipError_t pvr_xent(const float* logits, int64_t ld, const int64_t* labels, int B, int C, float* loss_rows,
                               float* dlogits, int* correct, float grad_scale, hipStream_t s) {
  using namespace pvr;
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(xent_kernel, dim3(B), dim3(256), 0, s, logits, ld, labels, B, C, loss_rows, dlogits, correct, grad_scale);
  return hipGetLastError();
}
