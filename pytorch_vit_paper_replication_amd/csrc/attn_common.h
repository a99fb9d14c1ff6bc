// Attention helpers shared by the attention kernels (attention.hip): head-row
// LDS images (128-B swizzled rows), MFMA operand fragments, LDS-DMA row staging, dropout hash.
#pragma once
#include "common.h"
#include <type_traits>

namespace pvr {
namespace {

template <int DH>
struct Hd {
  static_assert(DH % 16 == 0 && DH <= 128, "head dim must be a multiple of 16, at most 128");
  static constexpr int NH = (DH + 63) / 64;  // 128-B row images per head row
  static constexpr int KS = (DH + 31) / 32;  // MFMA k-steps over the head dim
  static constexpr int NE = DH / 16;         // 16-wide output fragments over the head dim
};
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// XOR on the 16-B chunk index of 128-B rows: conflict-free for row reads (ds_read_b128, 16 rows x
// one chunk), and for transposed reads of rows {4g+q, 16+4g+q} and {8g+q, 8g+4+q}.
PVR_DEV int swz_a(int r) { return (((r >> 1) & 1) << 1) ^ (((r >> 2) & 1) << 2) ^ (((r >> 3) & 1) * 5); }

// Byte offset of 16-B chunk `chunk` (0 .. 8*NH-1) of row `row` in an image of `rows` rows: the head
// row is split into 64-dim halves, each its own [rows][128 B] swizzled image.
PVR_DEV int lds_off(int rows, int row, int chunk) {
  return (chunk >> 3) * rows * 128 + row * 128 + (((chunk & 7) ^ swz_a(row)) << 4);
}

// DMA `rows` rows (multiple of 8) of a [row][NH*64] bf16 operand into NH swizzled 128-B-row images.
// Row r of the image comes from element offset (r * ld) of the buffer resource; bytes past the
// resource's extent (last row's tail past dh) read as zero.
template <int NH>
PVR_DEV void dma_rows(__amdgpu_buffer_rsrc_t rs, char* lds, int rows, int64_t ld, int row_base, int wave, int nwaves, int lane) {
#pragma unroll
  for (int hh = 0; hh < NH; ++hh)
    for (int s = wave; s < rows / 8; s += nwaves) {
      const int row = s * 8 + (lane >> 3);
      const int c = (lane & 7) ^ swz_a(row);
      const uint32_t voff = (uint32_t)((int64_t)(row_base + row) * ld * 2 + hh * 128 + c * 16);
      dma16(rs, to_lds(lds + hh * rows * 128 + s * 1024), voff);
    }
}

// 16x32 operand fragment from a swizzled image, rows r0 + (l&15), k = 32ks + 8(l>>4) + j.
PVR_DEV v8s frag_rows(const char* img, int rows, int r0, int ks, int lane) {
  return ds_read_b128(img + lds_off(rows, r0 + (lane & 15), ks * 4 + (lane >> 4)));
}

// Transposed fragment: lane i (of group g) gets img[row_of(g, j)][c0 + i] for j = 0..7 where rows are
// rowA + q (j = q) and rowB + q (j = 4 + q); cols c0..c0+15 (c0 multiple of 16).
PVR_DEV v8s frag_tr(const char* img, int rows, int rowA, int rowB, int c0, int lane) {
  const int q = (lane >> 2) & 3, p = lane & 3;
  const int chunk = (c0 >> 3) + (p >> 1);
  const v4s lo = ds_read_tr(img + lds_off(rows, rowA + q, chunk) + 8 * (p & 1));
  const v4s hi = ds_read_tr(img + lds_off(rows, rowB + q, chunk) + 8 * (p & 1));
  return cat44(lo, hi);
}

// frag_tr through ds_read_tr_async (no compiler drain of in-flight LDS-DMA in front of it); the
// caller combines the halves with cat44 after lds_wait().
PVR_DEV void frag_tr_async(const char* img, int rows, int rowA, int rowB, int c0, int lane, v4s& lo, v4s& hi) {
  const int q = (lane >> 2) & 3, p = lane & 3;
  const int chunk = (c0 >> 3) + (p >> 1);
  lo = ds_read_tr_async(img + lds_off(rows, rowA + q, chunk) + 8 * (p & 1));
  hi = ds_read_tr_async(img + lds_off(rows, rowB + q, chunk) + 8 * (p & 1));
}

// Global 8-element fragment at head-dim offset d0, zero past the head dim.
template <int DH>
PVR_DEV v8s load_frag(const uint16_t* p, int d0) {
  if (d0 >= DH) return v8s{0, 0, 0, 0, 0, 0, 0, 0};
  return *(const v8s*)(p + d0);
}

PVR_DEV v8s pack_p(const v4f& a, const v4f& b) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u w = {pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(b[0], b[1]), pack2bf(b[2], b[3])};
  return __builtin_bit_cast(v8s, w);
}

// c + sum_j a[j] * b[j] over 8 bf16 pairs (v_dot2c_f32_bf16, fp32 accumulation)
PVR_DEV float dot8_bf16(const v8s& a, const v8s& b, float c) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  const v8bf x = __builtin_bit_cast(v8bf, a), y = __builtin_bit_cast(v8bf, b);
#pragma unroll
  for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_fdot2_f32_bf16(bf2{x[2 * j], x[2 * j + 1]}, bf2{y[2 * j], y[2 * j + 1]}, c, false);
  return c;
}

template <int I, int N, class F>
PVR_DEV void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

PVR_DEV uint32_t clamp_bytes(int64_t b) { return b < 0 ? 0u : (b > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)b); }

// Attention-probability dropout (nn.MultiheadAttention(dropout=p), reference models/vit.py:86-90):
// element (query q, key k) of pair bh is kept iff the 16-bit half (k even: low, odd: high) of
// rng_mix32((idx >> 1) ^ key(bh)) >= thr16, idx = q * Npad + k (Npad = N rounded up to 4, so a row's
// 4-key groups start at a multiple of 4). The forward draws 4 consecutive keys per 2 hashes
// (rng_keep4_32), the backward one element at a time: the same bits, no stored mask. Kept
// probabilities scale by 65536 / (65536 - thr16); the softmax normaliser uses the undropped P.
struct AttnDrop {
  const uint64_t* seed;  // device seed (the step's snapshot); null: no dropout
  uint64_t off;          // per-layer site offset
  uint32_t thr;          // round(p * 65536)
  float scale;           // 1 / keep probability
};
// Optional e4m3 copy of the attention output for an fp8 out-proj GEMM (producer-side quantization):
// out[row][col] = fp8(o * (*qs)), *amax = max(*amax, max|o|); out == null: none
struct AttnQ8 {
  uint8_t* out;
  int64_t ld;
  const float* qs;
  unsigned* amax;
  int only;  // backward: store only the fp8 copy, not the bf16 gradient (every reader takes the copy)
  int fmt;   // backward copies: 1 e5m2 (default), 0 e4m3 (enable_fp8(grad_fmt="e4m3")); forward: 0
};
// max|x| record with few same-address atomics: most waves find the running amax already larger
PVR_DEV void amax_record(unsigned* amax, float m) {
  if (!(m <= 0.f) && !(m <= __uint_as_float(__builtin_nontemporal_load(amax)))) atomicMax(amax, __float_as_uint(m));
}
PVR_DEV uint32_t attn_drop_key(const AttnDrop& d, int bh) {
  return rng_mix32(rng_key(*d.seed + d.off) ^ (0x9E3779B9u * (uint32_t)(bh + 1)));
}
PVR_DEV bool attn_keep1(uint32_t key, uint32_t idx, uint32_t thr) {
  const uint32_t h = rng_mix32((idx >> 1) ^ key);
  return ((idx & 1u) ? (h >> 16) : (h & 0xFFFFu)) >= thr;
}

}  // namespace
}  // namespace pvr
