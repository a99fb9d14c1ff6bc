// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of this package.
//
// Everything here is written for 64-lane wavefronts, MFMA bf16 16x16x32 fragments and
// LDS-DMA (buffer_load ... lds) staging. No CUDA/HIP dual paths: this is CDNA4 code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tile_plan.h"

#define PVR_DEV __device__ __forceinline__

typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

typedef __attribute__((address_space(3))) void lds_void;

// Debug builds (build_extension(debug=True) -> _C_debug, loaded with PVR_DEBUG_KERNELS=1) check
// kernel invariants on the device: a violated one prints its location and traps, so the failing
// launch is reported by the HIP runtime instead of corrupting memory silently.
#ifdef PVR_DEBUG
#define PVR_ASSERT(cond)                                                                     \
  do {                                                                                       \
    if (!(cond)) {                                                                           \
      printf("PVR_ASSERT failed %s:%d (block %d thread %d): %s\n", __FILE__, __LINE__,        \
             (int)blockIdx.x, (int)threadIdx.x, #cond);                                      \
      __builtin_trap();                                                                      \
    }                                                                                        \
  } while (0)
#else
#define PVR_ASSERT(cond) \
  do {                   \
  } while (0)
#endif

namespace pvr {

PVR_DEV float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
// Round-to-nearest-even f32->bf16 (NaN stays NaN through the plain cast path).
PVR_DEV uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
// Two f32 -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (the scalar-cast form costs two conversions,
// a shift and an SDWA or: 4 VALU per pair in every epilogue).
PVR_DEV uint32_t pack2bf(float a, float b) {
  typedef float v2f __attribute__((ext_vector_type(2)));
  typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((v2f){a, b}, v2bf));
}

// 16x16x32 bf16 MFMA: D = A(16x32) * B(32x16) + C.
// lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15], D[row 4(l>>4)+r][col l&15].
PVR_DEV v4f mfma16(v8s a, v8s b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a),
                                                  __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}

// Buffer resource: hardware range check returns 0 for every byte past `bytes`.
PVR_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// LDS-DMA: 16 bytes per lane, LDS destination = lds_base (wave-uniform) + lane*16.
PVR_DEV void dma16(__amdgpu_buffer_rsrc_t r, lds_void* lds_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds_base, 16, voff, 0, 0, 0);
}

PVR_DEV lds_void* to_lds(void* p) { return (lds_void*)p; }

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, cols 4p..4p+3 of a 4x16
// block; lane i receives column i of the 4 rows (row q in element q).
PVR_DEV v4s ds_read_tr(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)lds_ptr);
}

// The same read as inline asm. hipcc models the ds_read_tr builtin as possibly writing LDS, so it
// drains every in-flight LDS-DMA (s_waitcnt vmcnt(0)) in front of it, which defeats a prefetch of
// the next tile into the other buffer. The asm form is invisible to the compiler's wait insertion:
// the caller waits for it with lds_wait() before the first use of the result.
PVR_DEV v4s ds_read_tr_async(const void* lds_ptr) {
  v4s r;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_ptr;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
// ds_read_tr_async at a compile-time byte offset from `lds_ptr` (one address VGPR for a whole
// unrolled sweep of reads OFF apart).
template <int OFF>
PVR_DEV v4s ds_read_tr_async_at(const void* lds_ptr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16 bits");
  v4s r;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_ptr;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
// Lane id recomputed where it is used (volatile: not hoisted out of loops and kept live, which at
// high register pressure gets it spilled and reloaded behind an s_waitcnt vmcnt(0))
PVR_DEV int lane_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
// Cross-lane sums on DPP (register-to-register lane moves inside a 16-lane row): a constant-offset
// __shfl_xor lowers to ds_bpermute, an LDS round trip per step. dpp_mov<CTRL>: the lane value
// selected by the DPP control (quad_perm 0x00-0xFF, row_ror:n 0x120+n, row_half_mirror 0x141).
template <int CTRL>
PVR_DEV float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// sum over the 16 lanes of each row (every lane of the row receives it)
PVR_DEV float row16_sum(float v) {
  v += dpp_mov<0x128>(v);  // row_ror:8
  v += dpp_mov<0x124>(v);  // row_ror:4
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  return v;
}
// sum over each aligned group of 8 lanes (every lane of the group receives it)
PVR_DEV float oct_sum(float v) {
  v += dpp_mov<0x141>(v);  // row_half_mirror: lane i + lane 7 - i within each 8
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0xB1>(v);
  return v;
}
// Wait for every outstanding LDS read (including ds_read_tr_async) and keep the compiler from
// scheduling their consumers above the wait (an MFMA has no memory operand, so the asm's "memory"
// clobber alone does not order it).
PVR_DEV void lds_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Wait until at most N of this wave's vector-memory ops (LDS-DMA, loads, stores) are outstanding,
// then barrier. The asm "memory" clobbers keep the compiler from moving LDS accesses across it.
template <int N>
PVR_DEV void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// Same, and also retire this wave's outstanding LDS reads/writes (their slot is refilled, or their
// data read by other waves, after the barrier).
template <int N>
PVR_DEV void wait_barrier_lds() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

PVR_DEV v8s ds_read_b128(const void* lds_ptr) {
  return *(const __attribute__((address_space(3))) v8s*)lds_ptr;
}

PVR_DEV v8s cat44(v4s a, v4s b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7); }

// Counter-based dropout RNG over (seed, element index). Shared by every kernel that recomputes a
// mask in backward, so forward and backward agree bit for bit without storing the mask.
// The seed is folded into one 32-bit key (wave-uniform, hoisted out of element loops); the element
// index then goes through Wellons' "lowbias32" finaliser: two 32-bit multiplies per hash (a
// quarter-rate instruction on CDNA, as costly as a v_exp) instead of four. Indices below 2^32 (every
// tensor of these models) make the high word a no-op.
PVR_DEV uint32_t rng_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
PVR_DEV uint32_t rng_key(uint64_t seed) { return rng_mix32((uint32_t)seed ^ rng_mix32((uint32_t)(seed >> 32) + 0x9E3779B9u)); }
PVR_DEV uint32_t rng_hash(uint64_t seed, uint64_t idx) {
  const uint32_t hi = (uint32_t)(idx >> 32);
  return rng_mix32((uint32_t)idx ^ rng_key(seed) ^ ((hi << 16) | (hi >> 16)));
}
// Element idx is kept iff its 16-bit half of hash(seed, idx >> 1) is >= thr16 = round(p * 65536):
// one hash serves two neighbouring elements.
PVR_DEV bool rng_keep(uint64_t seed, uint64_t idx, uint32_t thr16) {
  return ((rng_hash(seed, idx >> 1) >> ((idx & 1) * 16)) & 0xFFFFu) >= thr16;
}
// Keep decisions of 4 consecutive elements from an even idx with idx + 3 < 2^32 (key = rng_key(seed)):
// the same hashes as two rng_keep2 calls (high word 0), in 32-bit index arithmetic.
PVR_DEV void rng_keep4_32(uint32_t key, uint32_t idx_even, uint32_t thr16, bool (&k)[4]) {
  const uint32_t i = idx_even >> 1;
  const uint32_t h0 = rng_mix32(i ^ key), h1 = rng_mix32((i + 1) ^ key);
  k[0] = (h0 & 0xFFFFu) >= thr16;
  k[1] = (h0 >> 16) >= thr16;
  k[2] = (h1 & 0xFFFFu) >= thr16;
  k[3] = (h1 >> 16) >= thr16;
}
// Pair form for an even idx: keep decisions of idx and idx + 1 from one hash.
PVR_DEV void rng_keep2(uint64_t seed, uint64_t idx_even, uint32_t thr16, bool& k0, bool& k1) {
  const uint32_t h = rng_hash(seed, idx_even >> 1);
  k0 = (h & 0xFFFFu) >= thr16;
  k1 = (h >> 16) >= thr16;
}

PVR_DEV float gelu_erf(float u) { return 0.5f * u * (1.0f + erff(u * 0.70710678118654752f)); }

// Exact-erf GELU and its derivative from ONE exponential: Phi(u) = 1 - erfc(u/sqrt2)/2 with the
// Abramowitz-Stegun 7.1.26 erfc (|error| <= 1.5e-7, far below bf16 resolution), whose exp(-u^2/2)
// is exactly the normal pdf's exponential. ~15 VALU ops incl. one v_exp / one v_rcp instead of
// ocml erff + expf (the fc1 epilogue runs it 155M times per ViT-B/16 step).
PVR_DEV void gelu_and_grad(float u, float& g, float& gp) {
  const float au = fabsf(u);
  const float e = __builtin_amdgcn_exp2f(-0.72134752044448170f * u * u);  // exp(-u^2/2)
  const float t = __builtin_amdgcn_rcpf(fmaf(0.23164190f, au, 1.0f));     // 1/(1 + p*|u|/sqrt2)
  float poly = fmaf(t, 1.061405429f, -1.453152027f);
  poly = fmaf(t, poly, 1.421413741f);
  poly = fmaf(t, poly, -0.284496736f);
  poly = fmaf(t, poly, 0.254829592f);
  const float half_erfc = 0.5f * t * poly * e;  // erfc(|u|/sqrt2) / 2
  const float cdf = u >= 0.f ? 1.0f - half_erfc : half_erfc;
  g = u * cdf;
  gp = fmaf(u * 0.39894228040143268f, e, cdf);
}
// Two-lane form of gelu_and_grad: the polynomial and products as packed fp32 (v_pk_fma_f32 /
// v_pk_mul_f32 do two lanes' work per instruction), the exp / rcp per element. The 1/2 of the
// erfc is folded into the polynomial, and the sign select Phi = u >= 0 ? 1 - he : he is
// fma(s, he, (1 - s) / 2) with s = -1 / +1 made from u's sign bit by one bit operation (no
// compare / select pairs): ~21 issue slots per pair instead of ~27.
typedef float v2f __attribute__((ext_vector_type(2)));
PVR_DEV void gelu_and_grad2(v2f u, v2f& g, v2f& gp) {
  const v2f w = u * (u * (v2f){-0.72134752044448170f, -0.72134752044448170f});  // -u^2/2 * log2(e)
  v2f e, t;
  e.x = __builtin_amdgcn_exp2f(w.x);  // exp(-u^2/2)
  e.y = __builtin_amdgcn_exp2f(w.y);
  t.x = __builtin_amdgcn_rcpf(fmaf(0.23164190f, fabsf(u.x), 1.0f));  // 1/(1 + p*|u|/sqrt2)
  t.y = __builtin_amdgcn_rcpf(fmaf(0.23164190f, fabsf(u.y), 1.0f));
  v2f hp = __builtin_elementwise_fma(t, (v2f){0.5307027145f, 0.5307027145f}, (v2f){-0.7265760135f, -0.7265760135f});
  hp = __builtin_elementwise_fma(t, hp, (v2f){0.7107068705f, 0.7107068705f});
  hp = __builtin_elementwise_fma(t, hp, (v2f){-0.142248368f, -0.142248368f});
  hp = __builtin_elementwise_fma(t, hp, (v2f){0.127414796f, 0.127414796f});
  const v2f he = t * hp * e;  // erfc(|u|/sqrt2) / 2
  // s = -1 for u >= +0, +1 for u < 0 (and -0: Phi(0) = he = 1/2 either way)
  // (sign(u) & 0x80000000) ^ bits(-1.0): one v_bitop3_b32 (truth table 0x6A = (S0 & S1) ^ S2)
  const v2f s = {__uint_as_float(__builtin_amdgcn_bitop3_b32(__float_as_uint(u.x), 0x80000000u, 0xBF800000u, 0x6A)),
                 __uint_as_float(__builtin_amdgcn_bitop3_b32(__float_as_uint(u.y), 0x80000000u, 0xBF800000u, 0x6A))};
  const v2f cdf = __builtin_elementwise_fma(s, he, __builtin_elementwise_fma(s, (v2f){-0.5f, -0.5f}, (v2f){0.5f, 0.5f}));
  g = u * cdf;
  gp = __builtin_elementwise_fma(u * (v2f){0.39894228040143268f, 0.39894228040143268f}, e, cdf);
}
PVR_DEV float gelu_erf_grad(float u) {
  const float cdf = 0.5f * (1.0f + erff(u * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * u * u);
  return cdf + u * pdf;
}

// Whole-wave reductions without LDS round trips: DPP within each 16-lane row, then the gfx950 row
// swaps (v_permlane16_swap: rows 0<->1, 2<->3; v_permlane32_swap: rows 0,1 <-> 2,3). Every lane
// receives the result.
template <class Op>
PVR_DEV float wave_reduce(float v, Op op) {
  v = op(v, dpp_mov<0x128>(v));  // row_ror:8
  v = op(v, dpp_mov<0x124>(v));  // row_ror:4
  v = op(v, dpp_mov<0x4E>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_mov<0xB1>(v));   // quad_perm [1,0,3,2]
  // (inline asm: the builtins' results for swap(x, x) are folded to one value by this compiler)
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  v = op(a, b);
  a = v;
  b = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return op(a, b);
}
PVR_DEV float wave_sum(float v) {
  return wave_reduce(v, [](float a, float b) { return a + b; });
}
PVR_DEV float wave_max(float v) {
  return wave_reduce(v, [](float a, float b) { return fmaxf(a, b); });
}
// NaN-propagating max (fmaxf returns the non-NaN operand): a NaN on either side wins
// NaN-propagating max (IEEE 754-2019 maximum): one v_maximum3_f32 on gfx950, and chains of
// nan_max fold three operands per instruction (|x| operands as source modifiers)
PVR_DEV float nan_max(float a, float b) { return __builtin_elementwise_maximum(a, b); }
PVR_DEV float wave_max_nan(float v) { return wave_reduce(v, nan_max); }

// Bijective XCD-aware remap: blocks dealt round-robin over 8 XCDs (b, b+8 share one) are given
// contiguous logical tile ranges so neighbouring tiles share the XCD's L2 (csrc/tile_plan.h).
PVR_DEV int xcd_remap(int bid, int nblocks) { return xcd_remap_c(bid, nblocks); }

// Two f32 -> OCP fp8 (FMT 0 e4m3fn, 1 e5m2) into byte pair HI of `old` (v_cvt_pk_fp8 / bf8_f32):
// finite overflow saturates; a NaN stays a NaN (fminf/fmaxf would turn it into -FMAX and hide it)
template <int FMT, bool HI>
PVR_DEV int pack2_fp8(float a, float b, int old) {
  constexpr float FMAX = FMT == 0 ? 448.f : 57344.f;  // OCP e4m3fn / e5m2 largest finite
  a = a != a ? a : fminf(fmaxf(a, -FMAX), FMAX);
  b = b != b ? b : fminf(fmaxf(b, -FMAX), FMAX);
  if constexpr (FMT == 0)
    return __builtin_amdgcn_cvt_pk_fp8_f32(a, b, old, HI);
  else
    return __builtin_amdgcn_cvt_pk_bf8_f32(a, b, old, HI);
}
// 8 f32 -> 8 fp8 bytes (little-endian order) of format fmt
template <int FMT>
PVR_DEV uint2 pack8_fp8(const float (&v)[8], float qs) {
  uint2 r;
  r.x = (uint32_t)pack2_fp8<FMT, true>(v[2] * qs, v[3] * qs, pack2_fp8<FMT, false>(v[0] * qs, v[1] * qs, 0));
  r.y = (uint32_t)pack2_fp8<FMT, true>(v[6] * qs, v[7] * qs, pack2_fp8<FMT, false>(v[4] * qs, v[5] * qs, 0));
  return r;
}
// pack8_fp8 that pays the saturation / NaN handling (4 VALU per value) only when some lane of the
// wave needs it: with vmax = max |v| of the lane's 8 values (NaN-propagating; the producers record
// it for the amax anyway), vmax * qs <= FMAX for every active lane - the delayed-scaling steady
// state - means every product is finite and rounds to at most FMAX, so the conversion runs directly
// 4 f32 -> 4 fp8 bytes, direct conversion (caller guarantees |v * qs| <= FMAX and no NaN)
template <int FMT>
PVR_DEV uint32_t pack4_fp8_direct(float a, float b, float c, float d) {
  if constexpr (FMT == 0)
    return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c, d, __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false), true);
  else
    return (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(c, d, __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false), true);
}
// true when every active lane's vmax * qs <= FMAX (wave-uniform): pack4_fp8_direct is exact
template <int FMT>
PVR_DEV bool fp8_direct_ok(float vmax, float qs) {
  constexpr float FMAX = FMT == 0 ? 448.f : 57344.f;
  return __builtin_amdgcn_ballot_w64(!(vmax * qs <= FMAX)) == 0;  // NaN compares false
}
template <int FMT>
PVR_DEV uint2 pack8_fp8_fast(const float (&v)[8], float qs, float vmax) {
  if (!fp8_direct_ok<FMT>(vmax, qs)) return pack8_fp8<FMT>(v, qs);
  uint2 r;
  r.x = pack4_fp8_direct<FMT>(v[0] * qs, v[1] * qs, v[2] * qs, v[3] * qs);
  r.y = pack4_fp8_direct<FMT>(v[4] * qs, v[5] * qs, v[6] * qs, v[7] * qs);
  return r;
}

// Runtime-format forms for the gradient copies (fmt 1 e5m2, the default; 0 e4m3 with
// enable_fp8(grad_fmt="e4m3")): one wave-uniform branch per store, both conversions compiled in.
PVR_DEV uint32_t pack4_fp8_rt(int fmt, float a, float b, float c, float d) {
  return fmt ? (uint32_t)pack2_fp8<1, true>(c, d, pack2_fp8<1, false>(a, b, 0))
             : (uint32_t)pack2_fp8<0, true>(c, d, pack2_fp8<0, false>(a, b, 0));
}
PVR_DEV uint8_t pack1_fp8_rt(int fmt, float a) {
  return (uint8_t)((fmt ? pack2_fp8<1, false>(a, 0.f, 0) : pack2_fp8<0, false>(a, 0.f, 0)) & 0xFF);
}
PVR_DEV uint2 pack8_fp8_fast_rt(int fmt, const float (&v)[8], float qs, float vmax) {
  return fmt ? pack8_fp8_fast<1>(v, qs, vmax) : pack8_fp8_fast<0>(v, qs, vmax);
}

}  // namespace pvr
