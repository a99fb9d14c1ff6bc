// Multi-head self-attention forward/backward for ViT (no mask, head_dim 64/80/96/128), gfx950.
//
// Replaces nn.MultiheadAttention's scaled_dot_product_attention core (reference models/vit.py:86-97;
// SURVEY.md K7). Q, K and V are read in place from the fused QKV GEMM output [tokens][3*D]
// (row = token, head h at columns h*dh, D + h*dh, 2D + h*dh), so there are no head transposes.
// A head row is staged in LDS as ceil(dh/64) "half" images of 128-B rows (the swizzle below works
// on 8 chunks); for dh = 80 (ViT-H/14) the MFMA k-steps over dh run to 96 with the Q / K / V
// register fragments zeroed past dh, so the finite neighbour data staged in the LDS tail of a row
// never contributes.
//
// Forward: one workgroup = 4 waves = 64 queries of one (batch, head); each wave owns 16 queries
// and computes S^T = K . Q^T so that the query sits on the MFMA lane: the softmax row reduction
// over keys is then in-register plus two cross-lane steps, and P^T is directly the B operand of
// O^T = V^T . P^T (V^T read with ds_read_b64_tr_b16). K/V tiles of 64 keys are LDS-DMA staged
// (two stages) with an online softmax, so any sequence length works (197, 257, 577 tokens...).
// The log-sum-exp per query is saved for the backward.
//
// Backward: one workgroup covers up to 256 keys of one (batch, head); each wave keeps its 32
// keys' K and V fragments in registers and accumulates dK^T, dV^T over all query blocks of 32
// (key on the lane: S and dP accumulators are directly the B operands of the dV/dK products).
// dS crosses LDS once for dQ = dS . K, which the waves split by output fragment, so dQ needs no
// atomics when one workgroup holds every key (N <= 256). The query blocks are software-pipelined
// (dQ of block t-1 beside S/dP of block t, one barrier per block). A pre-pass per (batch, head)
// supplies delta = rowsum(dO * O), the dO column sums (v-bias gradient) and, for N = 256 + 1, the
// last key's dS / dK / dV. Heads with more keys accumulate dQ in f32 slabs (or atomics) that the
// tail launch's final pass turns into bf16 dQ, its optional fp8 (e5m2 / e4m3) copy and the q-bias partials.
#include "attn_common.h"

namespace pvr {
namespace {


// ----------------------------------------------------------------------------------- forward
// QG 16-query groups per wave (workgroup = 4 waves = 64*QG queries). With QG = 2 every K fragment
// (S^T = K.Q^T) and V^T fragment (O^T += V^T.P^T) read from LDS feeds two MFMAs instead of one, and
// the per-tile fixed costs (barrier, DMA issue, fragment address math) are shared by 32 queries.
// KT keys per tile; the dynamic LDS holds two stages of K and V images (4 x KT x 128 x NH bytes).
template <int DH, bool DROP, int QG, int KT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) attn_fwd_kernel(const uint16_t* __restrict__ qkv, int64_t ld, uint16_t* __restrict__ out,
                                                        int64_t ld_o, float* __restrict__ lse, int N, int H, int D, float scale,
                                                        AttnDrop drop, AttnQ8 q8) {
  using C = Hd<DH>;
  static_assert(KT == 32 || KT == 64, "keys per tile");
  constexpr int NFR = KT / 16;                   // 16-key S fragments per tile
  constexpr int TILE_BYTES = KT * 128 * C::NH;   // one K or V tile image
  constexpr int QW = 16 * QG;                    // queries per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [stage][K|V]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  // XCD-aware: the query blocks of one (batch, head) get consecutive logical ids on ONE XCD, so its
  // K/V tiles are fetched into that XCD's L2 once instead of once per query block
  const int nqb = (N + 4 * QW - 1) / (4 * QW);
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = L / nqb, b = bh / H, h = bh % H;
  const int q0 = (L % nqb) * 4 * QW + wave * QW;  // group gi: queries q0 + 16 gi ..

  const uint16_t* base = qkv + (int64_t)b * N * ld;
  const int64_t extent = ((int64_t)(N - 1) * ld + DH) * 2;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(base + D + h * DH, clamp_bytes(extent));
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(base + 2 * D + h * DH, clamp_bytes(extent));

  // Q fragments (B operand): lane holds Q[q0 + 16 gi + li][32ks + 8g + j]
  v8s qf[QG][C::KS];
#pragma unroll
  for (int gi = 0; gi < QG; ++gi) {
    const int q = min(q0 + 16 * gi + li, N - 1);
#pragma unroll
    for (int ks = 0; ks < C::KS; ++ks) qf[gi][ks] = load_frag<DH>(base + (int64_t)q * ld + h * DH, ks * 32 + 8 * g);
  }

  const float c = scale * LOG2E;
  float m_run[QG], l_run[QG];
  uint32_t dkey = 0, drow[QG];  // dropout: the pair's hash key, this lane's query row start idx
  if constexpr (DROP) dkey = attn_drop_key(drop, bh);
#pragma unroll
  for (int gi = 0; gi < QG; ++gi) drow[gi] = DROP ? (uint32_t)min(q0 + 16 * gi + li, N - 1) * (uint32_t)((N + 3) & ~3) : 0u;
  // The LAST key (N - 1) starts the online softmax instead of running through the tiles: ViT's
  // N = 64k + 1 (the CLS token: 257 at 224/14, 577 at 384/16) then streams exactly k full 64-key
  // tiles (no masked tail tile, no 1-key tile). Per query: s = q . k_last from the Q fragments
  // (8 dims per lane, reduced over the 4 lane groups), m = s * c, l = 1 (counted on lane group 0),
  // O^T = v_last (times the keep mask / scale with dropout).
  const int NL = N - 1;  // keys through the tiles
  const uint16_t* klast = base + (int64_t)NL * ld + D + h * DH;
  v4f o[QG][C::NE];
  {
    v8s kl[C::KS];
#pragma unroll
    for (int ks = 0; ks < C::KS; ++ks) kl[ks] = load_frag<DH>(klast, ks * 32 + 8 * g);
    uint2 vl[C::NE];
#pragma unroll
    for (int e = 0; e < C::NE; ++e) vl[e] = *(const uint2*)(klast + D + 16 * e + 4 * g);
#pragma unroll
    for (int gi = 0; gi < QG; ++gi) {
      float sl = 0.f;
#pragma unroll
      for (int ks = 0; ks < C::KS; ++ks) sl = dot8_bf16(qf[gi][ks], kl[ks], sl);
      sl += __shfl_xor(sl, 16, 64);
      sl += __shfl_xor(sl, 32, 64);
      m_run[gi] = sl * c;
      l_run[gi] = g == 0 ? 1.f : 0.f;
      float pk = 1.f;
      if constexpr (DROP) pk = attn_keep1(dkey, drow[gi] + (uint32_t)NL, drop.thr) ? drop.scale : 0.f;
#pragma unroll
      for (int e = 0; e < C::NE; ++e)
        o[gi][e] = v4f{bf2f(vl[e].x & 0xFFFF) * pk, bf2f(vl[e].x >> 16) * pk, bf2f(vl[e].y & 0xFFFF) * pk, bf2f(vl[e].y >> 16) * pk};
    }
  }

  const int ntiles = (NL + KT - 1) / KT;
  if (ntiles > 0) {
    dma_rows<C::NH>(krs, smem, KT, ld, 0, wave, 4, lane);
    dma_rows<C::NH>(vrs, smem + TILE_BYTES, KT, ld, 0, wave, 4, lane);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // Waves whose queries all lie past N only help stage K/V (no math), as do a wave's groups past N
  // (QG = 2); the running max is kept in scaled log2 units so a score costs max + fma + exp + add;
  // keys past NL exist only in the last tile, whose all-invalid 16-key fragments are skipped outright.
  const bool active = q0 < N;
  const bool g1 = QG > 1 && q0 + 16 < N;  // second group holds a valid query (uniform)
  for (int t = 0; t < ntiles; ++t) {
    const char* kimg = smem + (t & 1) * 2 * TILE_BYTES;
    const char* vimg = kimg + TILE_BYTES;
    if (t + 1 < ntiles) {
      char* nk = smem + ((t + 1) & 1) * 2 * TILE_BYTES;
      dma_rows<C::NH>(krs, nk, KT, ld, (t + 1) * KT, wave, 4, lane);
      dma_rows<C::NH>(vrs, nk + TILE_BYTES, KT, ld, (t + 1) * KT, wave, 4, lane);
    }
    if (active) {
      const int kbase = t * KT;
      const int nf = min(NFR, (NL - kbase + 15) >> 4);  // 16-key fragments holding a tile key (uniform)
      // S^T[key][q] for the key fragments: one K fragment read serves every query group
      v4f s[QG][NFR];
#pragma unroll
      for (int f = 0; f < NFR; ++f) {
#pragma unroll
        for (int gi = 0; gi < QG; ++gi) s[gi][f] = v4f{0.f, 0.f, 0.f, 0.f};
        if (f < nf) {
#pragma unroll
          for (int ks = 0; ks < C::KS; ++ks) {
            const v8s kf = frag_rows(kimg, KT, 16 * f, ks, lane);
            s[0][f] = mfma16(kf, qf[0][ks], s[0][f]);
            if (QG > 1 && g1) s[QG - 1][f] = mfma16(kf, qf[QG - 1][ks], s[QG - 1][f]);
          }
        }
      }
      if (kbase + KT > NL) {  // tail tile: mask keys >= NL
#pragma unroll
        for (int gi = 0; gi < QG; ++gi)
#pragma unroll
          for (int f = 0; f < NFR; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (kbase + 16 * f + 4 * g + r >= NL) s[gi][f][r] = -INFINITY;
      }
#pragma unroll
      for (int gi = 0; gi < QG; ++gi) {
        float tmax = s[gi][0][0];
#pragma unroll
        for (int f = 0; f < NFR; ++f)
#pragma unroll
          for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, s[gi][f][r]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        // lazy rescale: the running max (scaled log2 units, c > 0) moves only when some query of the
        // wave sees a score above it by more than 2^8; otherwise P is taken against the stale max
        // (values <= 256, exact in fp32 and bf16 range) and O / l skip the alpha multiply
        const bool grow = __builtin_amdgcn_ballot_w64(tmax * c > m_run[gi] + 8.f) != 0;
        const float m_new = grow ? fmaxf(m_run[gi], tmax * c) : m_run[gi];
        float psum = 0.f;
#pragma unroll
        for (int f = 0; f < NFR; ++f) {
          bool keep[4] = {true, true, true, true};
          if constexpr (DROP) rng_keep4_32(dkey, drow[gi] + (uint32_t)(kbase + 16 * f + 4 * g), drop.thr, keep);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(s[gi][f][r], c, -m_new));
            psum += pv;  // the normaliser sums the undropped probabilities
            if constexpr (DROP) s[gi][f][r] = keep[r] ? pv * drop.scale : 0.f;
            else s[gi][f][r] = pv;
          }
        }
        if (grow) {
          const float alpha = __builtin_amdgcn_exp2f(m_run[gi] - m_new);
          l_run[gi] *= alpha;
#pragma unroll
          for (int e = 0; e < C::NE; ++e) o[gi][e] *= alpha;
          m_run[gi] = m_new;
        }
        l_run[gi] += psum;
      }
      // O^T[d][q] += V^T[d][key] P^T[key][q]: one V^T fragment read serves every query group
#pragma unroll
      for (int kk = 0; kk < NFR / 2; ++kk) {
        if (kk * 2 < nf) {
          // asm transpose reads: the next tile's K/V DMA stays in flight under them
          v4s vlo[C::NE], vhi[C::NE];
#pragma unroll
          for (int e = 0; e < C::NE; ++e) frag_tr_async(vimg, KT, 32 * kk + 4 * g, 32 * kk + 16 + 4 * g, 16 * e, lane, vlo[e], vhi[e]);
          v8s pf[QG];
#pragma unroll
          for (int gi = 0; gi < QG; ++gi) pf[gi] = pack_p(s[gi][2 * kk], s[gi][2 * kk + 1]);
          lds_wait();
#pragma unroll
          for (int e = 0; e < C::NE; ++e) {
            const v8s vf = cat44(vlo[e], vhi[e]);
            o[0][e] = mfma16(vf, pf[0], o[0][e]);
            if (QG > 1 && g1) o[QG - 1][e] = mfma16(vf, pf[QG - 1], o[QG - 1][e]);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  float qam = 0.f;
  // Output rows through LDS (the K/V images are idle after the last barrier): each wave writes its
  // 16-query groups' bf16 O rows and e4m3 rows into its own region, then stores them as 16-B chunks
  // of whole rows (a wave instruction covers 6-16 consecutive rows' bytes instead of 16 rows x 8 B
  // (bf16) / 4 B (e4m3) per store: the direct stores were issue-bound). Needs 16-B aligned rows.
  constexpr int OB = DH * 2, QB = DH;  // bytes per bf16 / e4m3 head row
  constexpr int WB = 16 * (OB + QB);    // LDS bytes per (wave, group)
  static_assert(4 * QG * WB <= 4 * TILE_BYTES, "staged output fits the K/V images");
  const bool qon = q8.out != nullptr;
  // (dh 64 without the copy: 128-B rows, whose direct stores already fill whole lines - measured
  // 0.303 direct vs 0.308 staged at ViT-L/16@384; dh 80: 0.283 -> 0.269, with the copy 0.332 -> 0.296;
  // profiles/r4/aq8/attn_q8_ab.log)
  const bool staged = (qon || DH != 64) && (((uintptr_t)out | (uintptr_t)(ld_o * 2)) & 15) == 0 &&
                      (!qon || (((uintptr_t)q8.out | (uintptr_t)q8.ld) & 15) == 0);
  const float qs = qon ? *q8.qs : 1.f;
#pragma unroll
  for (int gi = 0; gi < QG; ++gi) {
    float l = l_run[gi];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const int q = q0 + 16 * gi + li;
    if (staged) {
      if (q0 + 16 * gi < N) {  // uniform: the group holds a valid query
        char* st = smem + (wave * QG + gi) * WB;
        const bool live = q < N;
        const float inv = live ? 1.f / l : 0.f;
        float vm = 0.f;
#pragma unroll
        for (int e = 0; e < C::NE; ++e) {
          const float v0 = o[gi][e][0] * inv, v1 = o[gi][e][1] * inv, v2 = o[gi][e][2] * inv, v3 = o[gi][e][3] * inv;
          *(uint2*)(st + li * OB + (16 * e + 4 * g) * 2) = make_uint2(pack2bf(v0, v1), pack2bf(v2, v3));
          vm = nan_max(vm, nan_max(nan_max(fabsf(v0), fabsf(v1)), nan_max(fabsf(v2), fabsf(v3))));
        }
        if (qon) {  // e4m3 copy for the fp8 out-proj GEMM
          qam = nan_max(qam, vm);
          const bool fast = fp8_direct_ok<0>(vm, qs);
#pragma unroll
          for (int e = 0; e < C::NE; ++e) {
            const float v0 = o[gi][e][0] * inv * qs, v1 = o[gi][e][1] * inv * qs, v2 = o[gi][e][2] * inv * qs,
                        v3 = o[gi][e][3] * inv * qs;
            *(uint32_t*)(st + 16 * OB + li * QB + 16 * e + 4 * g) =
                fast ? pack4_fp8_direct<0>(v0, v1, v2, v3) : (uint32_t)pack2_fp8<0, true>(v2, v3, pack2_fp8<0, false>(v0, v1, 0));
          }
        }
        if (g == 0 && live) lse[(int64_t)bh * N + q] = (m_run[gi] + __log2f(l)) * LN2;
      }
      continue;
    }
    if (q < N) {
      const float inv = 1.f / l;
      uint16_t* orow = out + ((int64_t)b * N + q) * ld_o + h * DH;
#pragma unroll
      for (int e = 0; e < C::NE; ++e) {
        uint2 w;
        w.x = pack2bf(o[gi][e][0] * inv, o[gi][e][1] * inv);
        w.y = pack2bf(o[gi][e][2] * inv, o[gi][e][3] * inv);
        if (!q8.only) *(uint2*)(orow + 16 * e + 4 * g) = w;  // only: inference reads the e4m3 copy alone
      }
      if (q8.out) {  // e4m3 copy for the fp8 out-proj GEMM
        uint8_t* qrow = q8.out + ((int64_t)b * N + q) * q8.ld + h * DH;
#pragma unroll
        for (int e = 0; e < C::NE; ++e) {
          const float v[4] = {o[gi][e][0] * inv, o[gi][e][1] * inv, o[gi][e][2] * inv, o[gi][e][3] * inv};
#pragma unroll
          for (int r = 0; r < 4; ++r) qam = nan_max(qam, fabsf(v[r]));
          *(uint32_t*)(qrow + 16 * e + 4 * g) =
              (uint32_t)pack2_fp8<0, true>(v[2] * qs, v[3] * qs, pack2_fp8<0, false>(v[0] * qs, v[1] * qs, 0));
        }
      }
      if (g == 0) lse[(int64_t)bh * N + q] = (m_run[gi] + __log2f(l)) * LN2;
    }
  }
  if (staged) {  // LDS images -> whole-row 16-B chunks (each wave reads back only its own region)
#pragma unroll
    for (int gi = 0; gi < QG; ++gi) {
      const int r0 = q0 + 16 * gi;
      const int nrow = min(16, N - r0);
      if (nrow <= 0) continue;
      const char* st = smem + (wave * QG + gi) * WB;
      constexpr int OC = OB / 16, QC = QB / 16;  // 16-B chunks per row
#pragma unroll
      for (int k = 0; k < (16 * OC + 63) / 64; ++k) {
        const int ch = lane + 64 * k, row = ch / OC, cc = ch % OC;
        if (ch < 16 * OC && row < nrow && !q8.only)
          *(uint4*)((char*)(out + ((int64_t)b * N + r0 + row) * ld_o + h * DH) + cc * 16) = *(const uint4*)(st + row * OB + cc * 16);
      }
      if (qon) {
#pragma unroll
        for (int k = 0; k < (16 * QC + 63) / 64; ++k) {
          const int ch = lane + 64 * k, row = ch / QC, cc = ch % QC;
          if (ch < 16 * QC && row < nrow)
            *(uint4*)(q8.out + ((int64_t)b * N + r0 + row) * q8.ld + h * DH + cc * 16) = *(const uint4*)(st + 16 * OB + row * QB + cc * 16);
        }
      }
    }
  }
  if (q8.out) {
    qam = wave_max_nan(qam);
    if (lane == 0) amax_record(q8.amax, qam);
  }
}

// ------------------------------------------------------------- forward: whole head in LDS
// N <= 256 and dh = 64 (ViT-B/16 and ViT-L/16 at 224 px: N = 197). One persistent workgroup per
// CU walks a contiguous range of (batch, head) pairs; wave w owns QF 16-query fragments (queries
// 16 QF w .. 16 QF w + 16 QF - 1) against every key of the head. Every key of a head fits in LDS, so
//   * each query row's softmax is exact in one pass (no running max, no rescaling of O);
//   * the head's K/V are staged once instead of once per 64-query workgroup;
//   * the next pair's K/V LDS-DMA (second buffer) and Q fragments are in flight under this pair's
//     math, and its O rows are stored one pair late, so no store sits in front of a DMA wait.
// Every wave reads the whole K and V^T images (54 KiB at N = 197) per pair. QF = 2 feeds each
// fragment read to two MFMAs, halving that LDS read traffic, but with 7 instead of 13 waves it
// measured slower (0.086 vs 0.079 ms at ViT-B/16 b256, step unchanged: profiles/r6/attn_hqf/): the
// kernel is latency-, not LDS-bound. QF = 1 is the default; PVR_ATTN_HEAD_QF / set_attn_fwd_head_qf.
// Key rows past N (padding to a multiple of 32 for the P.V k-steps) read as zero.
template <int NF, int QF>
__global__ void __launch_bounds__(((NF + QF - 1) / QF) * 64) attn_fwd_head_kernel(const uint16_t* __restrict__ qkv, int64_t ld,
                                                                                uint16_t* __restrict__ out, int64_t ld_o,
                                                                                float* __restrict__ lse, int N, int H, int D,
                                                                                int npairs, float scale) {
  constexpr int DH = 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NP = 32 * ((NF + 1) / 2);  // staged key rows
  constexpr int BUF = 2 * NP * 128;         // K | V images of one (batch, head)
  constexpr int NW = (NF + QF - 1) / QF;    // waves
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  constexpr int nf = NF;  // 16-key fragments holding a valid key
  PVR_ASSERT((N + 15) / 16 == NF && blockDim.x == NW * 64 && (int)gridDim.x <= npairs);
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int per = npairs / gridDim.x, rem = npairs % gridDim.x;
  const int p0 = L * per + min(L, rem);
  const int p1 = p0 + per + (L < rem ? 1 : 0);
  int qrow[QF];
#pragma unroll
  for (int j = 0; j < QF; ++j) qrow[j] = min((QF * wave + j) * 16 + li, N - 1);
  const uint32_t extent = clamp_bytes(((int64_t)(N - 1) * ld + DH) * 2);
  const float c = scale * LOG2E;

  auto issue = [&](int pr, char* buf) {
    const uint16_t* base = qkv + (int64_t)(pr / H) * N * ld + (pr % H) * DH;
    dma_rows<1>(make_rsrc(base + D, extent), buf, NP, ld, 0, wave, NW, lane);
    dma_rows<1>(make_rsrc(base + 2 * D, extent), buf + NP * 128, NP, ld, 0, wave, NW, lane);
  };
  auto load_q = [&](int pr, v8s (&qf)[QF][2]) {
#pragma unroll
    for (int j = 0; j < QF; ++j) {
      const uint16_t* qp = qkv + ((int64_t)(pr / H) * N + qrow[j]) * ld + (pr % H) * DH + 8 * g;
      qf[j][0] = *(const v8s*)qp;
      qf[j][1] = *(const v8s*)(qp + 32);
    }
  };
  // O^T layout: lane holds O[q = 16 (QF wave + j) + li][d = 16e + 4g + r]. Stores go through
  // range-checked buffer resources: a lane with nothing to write gets an offset past the extent and
  // its store is dropped, so every wave issues exactly STORES store instructions per pair and the
  // loop's wait below can retire the DMAs issued before them without waiting for the stores.
  constexpr int STORES = 5 * QF;
  const uint32_t o_extent = clamp_bytes(((int64_t)(N - 1) * ld_o + DH) * 2);
  auto store_o = [&](int pr, int j, const v4f (&o)[4], float m, float l) {
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    const int q = (QF * wave + j) * 16 + li;
    const bool ok = q < N;
    const float inv = 1.f / l;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(out + (int64_t)(pr / H) * N * ld_o + (pr % H) * DH, o_extent);
    const uint32_t vo = ok ? (uint32_t)((q * ld_o + 4 * g) * 2) : 0x80000000u;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const v2u w = {pack2bf(o[e][0] * inv, o[e][1] * inv), pack2bf(o[e][2] * inv, o[e][3] * inv)};
      __builtin_amdgcn_raw_buffer_store_b64(w, rs, vo + 32 * e, 0, 0);
    }
    const __amdgpu_buffer_rsrc_t ls = make_rsrc(lse + (int64_t)pr * N, (uint32_t)N * 4);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((m + __log2f(l)) * LN2), ls,
                                          ok && g == 0 ? (uint32_t)q * 4 : 0x80000000u, 0, 0);
  };

  if (p0 >= p1) return;  // uniform: the host launches at most npairs workgroups
  v8s qf[QF][2], qn[QF][2];
  issue(p0, smem);
  load_q(p0, qf);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int j = 0; j < QF; ++j) asm volatile("" : "+v"(qf[j][0]), "+v"(qf[j][1]));
  for (int pr = p0; pr < p1; ++pr) {
    const int it = pr - p0;
    const char* kimg = smem + (it & 1) * BUF;
    const char* vimg = kimg + NP * 128;
    if (pr + 1 < p1) {
      issue(pr + 1, smem + ((it + 1) & 1) * BUF);
      load_q(pr + 1, qn);
    }
    // S^T[key][q] = K . Q^T: the query on the MFMA lane, keys down the accumulator rows; each K
    // fragment read feeds the wave's QF query fragments
    v4f s[QF][16];
#pragma unroll
    for (int f = 0; f < 16; ++f) {
#pragma unroll
      for (int j = 0; j < QF; ++j) s[j][f] = v4f{0.f, 0.f, 0.f, 0.f};
      if (f < nf) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const v8s kf = frag_rows(kimg, NP, 16 * f, ks, lane);
#pragma unroll
          for (int j = 0; j < QF; ++j) s[j][f] = mfma16(kf, qf[j][ks], s[j][f]);
        }
      }
    }
    float m[QF], l[QF];
#pragma unroll
    for (int j = 0; j < QF; ++j) {
      float mx = -INFINITY;
#pragma unroll
      for (int f = 0; f < 16; ++f) {
        if (f == nf - 1) {  // keys >= N live only in the last valid fragment
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (16 * f + 4 * g + r >= N) s[j][f][r] = -INFINITY;
        }
        if (f < nf) {
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[j][f][r]);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      m[j] = mx * c;  // scaled log2 units (c > 0)
      l[j] = 0.f;
    }
    v4f o[QF][4];
#pragma unroll
    for (int j = 0; j < QF; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) o[j][e] = v4f{0.f, 0.f, 0.f, 0.f};
    // O^T[d][q] += V^T[d][key] P^T[key][q], 32 keys per k-step; each V^T fragment read feeds QF MFMAs
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      if (2 * kk < nf) {
        // V^T fragments first (asm reads: the next pair's DMA stays in flight), softmax under them
        v4s vlo[4], vhi[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) frag_tr_async(vimg, NP, 32 * kk + 4 * g, 32 * kk + 16 + 4 * g, 16 * e, lane, vlo[e], vhi[e]);
        v8s pf[QF];
#pragma unroll
        for (int j = 0; j < QF; ++j) {
          v4f pa, pb = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pa[r] = __builtin_amdgcn_exp2f(fmaf(s[j][2 * kk][r], c, -m[j]));
            l[j] += pa[r];
          }
          if (2 * kk + 1 < nf) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              pb[r] = __builtin_amdgcn_exp2f(fmaf(s[j][2 * kk + 1][r], c, -m[j]));
              l[j] += pb[r];
            }
          }
          pf[j] = pack_p(pa, pb);
        }
        lds_wait();
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const v8s vf = cat44(vlo[e], vhi[e]);
#pragma unroll
          for (int j = 0; j < QF; ++j) o[j][e] = mfma16(vf, pf[j], o[j][e]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < QF; ++j) {
      l[j] += __shfl_xor(l[j], 16, 64);
      l[j] += __shfl_xor(l[j], 32, 64);
      store_o(pr, j, o[j], m[j], l[j]);
    }
    // everything but this pair's stores has landed (the next pair's K/V images and Q fragments),
    // and every wave is done reading this buffer before the pair after next restages it
    static_assert(STORES == 5 * QF && (QF == 1 || QF == 2), "the vmcnt below counts store_o's store instructions");
    if constexpr (QF == 1)
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int j = 0; j < QF; ++j) {
      qf[j][0] = qn[j][0];
      qf[j][1] = qn[j][1];
      // re-define qf through an empty asm: the compiler's own wait for these loads then sits here
      // (already satisfied) instead of in front of the next pair's first MFMA, where it would also
      // wait for that pair's K/V prefetch
      asm volatile("" : "+v"(qf[j][0]), "+v"(qf[j][1]));
    }
  }
}

// Phase stamps of the backward (diagnostic builds only, -DPVR_ATTN_STAMPS; scripts/attn_stamps.py):
// per wave, s_memtime cycles summed over the query-block loop by phase, written once at the end
// (lane 0, vector stores) to g_attn_dbg[(workgroup * NW + wave) * 8 + phase]. Production builds
// compile every stamp out.
#ifdef PVR_ATTN_STAMPS
__device__ uint64_t* g_attn_dbg;
#define ASTAMP(k)                                          \
  do {                                                     \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();      \
    st_acc[k] += t_ - st_last;                             \
    st_last = t_;                                          \
  } while (0)
#else
#define ASTAMP(k) \
  do {            \
  } while (0)
#endif

// ------------------------------------------------------------------------- backward
// grid (nkb, B*H), block NW*64 (NW in {1,2,4,8}); workgroup keys [kb*KB, kb*KB + KB), KB = 32*NW.
// delta = rowsum(dO * O) of each query block is formed in-kernel from the staged dO and O rows
// (no separate pass over dO and O, no delta round trip through HBM).
template <int DH, bool DROP>
__global__ void __launch_bounds__(512) attn_bwd_kernel(const uint16_t* __restrict__ qkv, int64_t ld,
                                                        const uint16_t* __restrict__ dout, int64_t ld_do,
                                                        const float* __restrict__ lse, const float* __restrict__ dlt,
                                                        const float* __restrict__ dsl,
                                                        uint16_t* __restrict__ dqkv, int64_t ld_dq, float* __restrict__ dq_acc,
                                                        float* __restrict__ dbias, float* __restrict__ bpart, int N, int H,
                                                        int D, float scale, int key_off, int key_end, int dq_mode,
                                                        int64_t slab_stride, int nslab, AttnDrop drop, AttnQ8 q8) {
  using C = Hd<DH>;
  constexpr int QB = 32;
  constexpr int RB = 128 * C::NH;  // LDS bytes per staged head row
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int NW = blockDim.x >> 6;
  const int KB = NW * 32;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  // this launch owns keys [key_off, key_end) (the whole range, or the KB-aligned body / the tail)
  const int nkb = (key_end - key_off + KB - 1) / KB;
  const int L = xcd_remap(blockIdx.x, gridDim.x);  // key blocks of one (batch, head) share an XCD's L2
  const int bh = L / nkb, b = bh / H, h = bh % H;
  const int kb0 = key_off + (L % nkb) * KB;
  const int kw0 = kb0 + wave * 32;
  PVR_ASSERT(kb0 < N && L < (int)gridDim.x && (KB & (KB - 1)) == 0);

  // LDS carve: K image [KB][dh] | 2 x (Q blk [32][dh] | dO blk [32][dh]) | 2 x dS [32][KB] | 2 x (lse | delta | ds_last) [3][256]
  // Q / dO rows and the per-query constants of query block qb+1 are staged while block qb is processed.
  // delta = rowsum(dO * O) comes from attn_bwd_prep_kernel (one pass over dO and O instead of every
  // wave dotting staged O rows per block); ds_last (lastkey path): dS of key N - 1 per query.
  char* kimg = smem;
  char* qdo = kimg + KB * RB;
  char* dsimg = qdo + 4 * QB * RB;  // two dS^T buffers (software pipelining over query blocks)
  float* s_ld = (float*)(dsimg + 2 * QB * KB * 2);
  typedef uint32_t v2u __attribute__((ext_vector_type(2)));
  // dS^T image [key_local][32 queries]: 64-B rows of 8-B units (4 queries), unit XOR (key>>1)&7
  auto ds_off = [](int key, int u) { return key * 64 + ((u ^ ((key >> 1) & 7)) << 3); };
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int dsw0 = wave * 2048 + ds_off(li, g), dsw1 = wave * 2048 + ds_off(li, 4 + g);  // f adds 1024

  const uint16_t* base = qkv + (int64_t)b * N * ld;
  const int64_t extent = ((int64_t)(N - 1) * ld + DH) * 2;
  const __amdgpu_buffer_rsrc_t qrs = make_rsrc(base + h * DH, clamp_bytes(extent));
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(base + D + h * DH, clamp_bytes(extent));
  const uint16_t* dobase = dout + (int64_t)b * N * ld_do;
  const __amdgpu_buffer_rsrc_t dors = make_rsrc(dobase + h * DH, clamp_bytes(((int64_t)(N - 1) * ld_do + DH) * 2));
  // dQ destination of this batch. dq_mode 0 with dq_acc: f32 atomics into the accumulator [N][D];
  // dq_mode 3 (key-block body of a multi-block head): plain f32 stores of this key block's partial
  // dQ into slab (L % nkb) of dq_acc [slabs][B*N][D] (6 TB/s stores instead of 1.3 TB/s atomics);
  // dq_mode 4 (the tail launch after a mode-3 body): its own partial into slab nslab, then the
  // final pass at the end sums the nslab + 1 slabs of the pair in fixed order into bf16 dQ;
  // otherwise the bf16 gradient rows directly.
  const bool slab_w = dq_mode == 3 || dq_mode == 4;
  // optional fp8 copy (e5m2, or e4m3: AttnQ8::fmt) of dQKV (the fp8 recipe's grad slot: dgrad and weight-gradient operand) with
  // the slot's delayed scale, written next to every final bf16 value, amax recorded per wave
  const bool q8kv = q8.out != nullptr;  // dK / dV: every launch writes final values
  const bool q8on = q8kv && !dq_acc;     // dQ here: only a launch whose fragments are the final dQ
  float q8am = 0.f;
  const float q8s = q8kv ? *q8.qs : 1.f;
  const __amdgpu_buffer_rsrc_t q8rs = make_rsrc(q8.out + (int64_t)b * N * q8.ld, q8on ? clamp_bytes((int64_t)(N - 1) * q8.ld + D) : 0u);
  float* dq_dst = dq_acc && slab_w ? dq_acc + (dq_mode == 3 ? (L % nkb) : nslab) * slab_stride : dq_acc;
  const __amdgpu_buffer_rsrc_t dqrs = dq_acc ? make_rsrc(dq_dst + (int64_t)b * N * D, clamp_bytes((int64_t)N * D * 4))
                                             : make_rsrc(dqkv + (int64_t)b * N * ld_dq, clamp_bytes(((int64_t)(N - 1) * ld_dq + D) * 2));

  // own keys' K and V fragments (B operands): lane holds X[kw0 + 16f + li][32ks + 8g + j]
  v8s kf[2][C::KS], vf[2][C::KS];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int key = kw0 + 16 * f + li;
    const bool ok = key < N;
    const int kc = ok ? key : 0;
#pragma unroll
    for (int ks = 0; ks < C::KS; ++ks) {
      v8s kk = load_frag<DH>(base + (int64_t)kc * ld + D + h * DH, ks * 32 + 8 * g);
      v8s vv = load_frag<DH>(base + (int64_t)kc * ld + 2 * D + h * DH, ks * 32 + 8 * g);
      if (!ok) { kk = v8s{0, 0, 0, 0, 0, 0, 0, 0}; vv = kk; }
      kf[f][ks] = kk;
      vf[f][ks] = vv;
    }
  }
  // whole key block's K image for the dQ product
  dma_rows<C::NH>(krs, kimg, KB, ld, kb0, wave, NW, lane);
  // waves whose 32 keys all lie past N skip the math; dQ only reduces over key slices with a valid key
  const bool active = kw0 < N;
  const int nks_dq = min(KB, N - kb0 + 31) / 32;

  v4f dk[C::NE][2], dv[C::NE][2];
#pragma unroll
  for (int e = 0; e < C::NE; ++e)
#pragma unroll
    for (int f = 0; f < 2; ++f) dk[e][f] = dv[e][f] = v4f{0.f, 0.f, 0.f, 0.f};

  const float c = scale * LOG2E;
  const int nqb = (N + QB - 1) / QB;
  const uint32_t dkey = DROP ? attn_drop_key(drop, bh) : 0u, npad = (uint32_t)((N + 3) & ~3);
  auto stage = [&](int qb) {  // Q / dO rows and lse / delta (/ ds_last) of query block qb into slot qb & 1
    // everything by LDS-DMA: a plain load of lse here would make hipcc wait vmcnt(0) at its first
    // use, draining these DMAs right after issuing them. lse / delta of queries past N read as 0;
    // their Q and dO rows are zero, so their P = 1 meets dO = 0 and dS = 0 and contributes nothing.
    char* qi = qdo + (qb & 1) * 2 * QB * RB;
    dma_rows<C::NH>(qrs, qi, QB, ld, qb * QB, wave, NW, lane);
    dma_rows<C::NH>(dors, qi + QB * RB, QB, ld_do, qb * QB, wave, NW, lane);
    if (wave == NW - 1) {  // 1 KiB slots, first QB floats used
      const int64_t r0 = (int64_t)bh * N + qb * QB;
      const uint32_t nb = (uint32_t)(N - qb * QB) * 4;
      dma16(make_rsrc(lse + r0, nb), to_lds(s_ld + (qb & 1) * 768), (uint32_t)lane * 16);
      dma16(make_rsrc(dlt + r0, nb), to_lds(s_ld + (qb & 1) * 768 + 256), (uint32_t)lane * 16);
      if (dsl) dma16(make_rsrc(dsl + r0, nb), to_lds(s_ld + (qb & 1) * 768 + 512), (uint32_t)lane * 16);
    }
  };
  // lastkey path: K[N - 1] at this lane's dQ columns (16e + li of the wave's dQ fragments)
  float kl_dq[2] = {0.f, 0.f};
  if (dsl) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int fr = wave + j * NW;
      if (fr < 2 * C::NE) kl_dq[j] = bf2f(base[(int64_t)(N - 1) * ld + D + h * DH + 16 * (fr % C::NE) + li]);
    }
  }
#ifdef PVR_ATTN_STAMPS
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_last = __builtin_amdgcn_s_memtime();
  const uint64_t st_0 = st_last;
#endif
  stage(0);
  float dqb0 = 0.f, dqb1 = 0.f;  // q-bias gradient partials (column sums of this wave's dQ fragments)
  // dQ stores this wave issues per query block (younger than the next block's staging DMAs)
  const int nst = wave < 2 * C::NE ? 4 * ((2 * C::NE - 1 - wave) / NW + 1) : 0;
  constexpr int DS_BYTES = QB * 32 * 2;  // per 32 keys of one dS^T buffer
  const int ds_buf = KB / 32 * DS_BYTES;
  // dQ of query block qbp = sum_key dS[q][key] K[key][d] from dS^T buffer (qbp & 1); 2*NE output
  // fragments split over the waves. Both operands by transposed reads (dS^T rows 32ks + 8g + q4 (+4),
  // queries 16a + 4p4; K rows the same keys, dims 16e + 4p4), four key slices per LDS wait; the
  // stores are buffer ops, so queries past N drop in the range check and every wave issues exactly 4
  // per fragment. slq: the block's dS of key N - 1 at this lane's fragment rows (lastkey path).
  auto dq_block = [&](int qbp, const v4f (&slq)[2]) {
    const char* dsb = dsimg + (qbp & 1) * ds_buf;
    int kfr = 0;
    for (int fr = wave; fr < 2 * C::NE; fr += NW, ++kfr) {
      const int a = fr / C::NE, e = fr % C::NE;
      v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
      const char* kt0 = kimg + lds_off(KB, 8 * g + q4, 2 * e + (p4 >> 1)) + 8 * (p4 & 1);
      const char* kt1 = kimg + lds_off(KB, 8 * g + q4 + 4, 2 * e + (p4 >> 1)) + 8 * (p4 & 1);
      const char* dt0 = dsb + ds_off(8 * g + q4, 4 * a + p4);
      const char* dt1 = dsb + ds_off(8 * g + q4 + 4, 4 * a + p4);
      auto batch = [&](auto k0c) {
        constexpr int k0 = decltype(k0c)::value;
        v4s klo[4], khi[4], slo[4], shi[4];
        static_for<0, 4>([&](auto jc) {
          constexpr int ks = k0 + decltype(jc)::value;
          klo[ks - k0] = ds_read_tr_async_at<4096 * ks>(kt0);
          khi[ks - k0] = ds_read_tr_async_at<4096 * ks>(kt1);
          slo[ks - k0] = ds_read_tr_async_at<2048 * ks>(dt0);
          shi[ks - k0] = ds_read_tr_async_at<2048 * ks>(dt1);
        });
        lds_wait();
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          if (k0 + jj < nks_dq) acc = mfma16(cat44(slo[jj], shi[jj]), cat44(klo[jj], khi[jj]), acc);
      };
      batch(std::integral_constant<int, 0>{});
      if (nks_dq > 4) batch(std::integral_constant<int, 4>{});
      const uint32_t vq = (uint32_t)(qbp * QB + 16 * a + 4 * g), col = (uint32_t)(h * DH + 16 * e + li);
      float cs = 0.f;  // queries past N have dS = 0, so their dQ is exactly 0
      if (dsl) {  // + dS[q][N - 1] K[N - 1] (lastkey path: key N - 1 is not in any key block)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = fmaf(slq[kfr & 1][r], kl_dq[kfr & 1], acc[r]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float val = acc[r] * scale;
        cs += val;
        if (dq_acc && slab_w)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, val), dqrs, ((vq + r) * (uint32_t)D + col) * 4, 0, 0);
        else if (dq_acc)
          __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(val, dqrs, ((vq + r) * (uint32_t)D + col) * 4, 0, 0);
        else if (!q8.only)
          __builtin_amdgcn_raw_buffer_store_b16(f2bf(val), dqrs, ((vq + r) * (uint32_t)ld_dq + col) * 2, 0, 0);
        if (q8on) {
          q8am = nan_max(q8am, fabsf(val));
          __builtin_amdgcn_raw_buffer_store_b8(pack1_fp8_rt(q8.fmt, val * q8s), q8rs,
                                               (vq + r) * (uint32_t)q8.ld + col, 0, 0);
        }
      }
      if (kfr == 0) dqb0 += cs;  // q-bias gradient: this fragment's column sums across query blocks
      else dqb1 += cs;           // (at most two fragments per wave: host guarantees 2*NE <= 2*NW)
    }
  };
  // Software-pipelined over query blocks, one barrier per block: block qb's S / dP / dV / dK and its
  // dS^T write (buffer qb & 1) run in the same interval as the dQ of block qb - 1 (buffer (qb-1) & 1,
  // written before this block's barrier), so the dQ product's LDS reads and MFMAs interleave with
  // the next block's instead of waiting behind a second barrier.
  v4f slq_prev[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
  for (int qb = 0; qb < nqb; ++qb) {
    const int q0 = qb * QB;
    // block qb landed (issued one iteration ago, before the dQ stores of block qb - 2, which may
    // stay in flight); every wave is done with slot (qb+1)&1, with dS buffer qb&1 (block qb - 2's)
    // and has written dS buffer (qb-1)&1
    ASTAMP(7);
    if (qb < 2 || nst < 4)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (nst < 8)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    // a raw barrier: __syncthreads' release fence would drain those stores (vmcnt(0)) first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ASTAMP(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    ASTAMP(1);
    if (qb + 1 < nqb) stage(qb + 1);
    ASTAMP(2);
    const char* qimg = qdo + (qb & 1) * 2 * QB * RB;
    const char* doimg = qimg + QB * RB;
    const float* s_lse = s_ld + (qb & 1) * 768;
    const float* s_dl = s_lse + 256;
    char* dsw = dsimg + (qb & 1) * ds_buf;
    // this block's dS of key N - 1 at the rows of this wave's dQ fragments: its constants slot is
    // restaged (block qb + 2) before the dQ of this block runs (next iteration)
    v4f slq_cur[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
    if (dsl) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int fr = wave + j * NW;
        if (fr < 2 * C::NE) slq_cur[j] = *(const v4f*)(s_lse + 512 + 16 * (fr / C::NE) + 4 * g);
      }
    }

    if (active) {
    // S[q][key], dP[q][key]: lane holds [q = 16a + 4g + r][key = kw0 + 16f + li]; dP starts from
    // -delta of its row, so dS = P * dP' needs no subtraction
    v4f s[2][2], dp[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const v4f nd = DROP ? v4f{0.f, 0.f, 0.f, 0.f} : -*(const v4f*)(s_dl + 16 * a + 4 * g);
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        s[a][f] = v4f{0.f, 0.f, 0.f, 0.f};
        dp[a][f] = nd;
      }
    }
#pragma unroll
    for (int ks = 0; ks < C::KS; ++ks) {
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const v8s qa = frag_rows(qimg, QB, 16 * a, ks, lane);
        const v8s da = frag_rows(doimg, QB, 16 * a, ks, lane);
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          s[a][f] = mfma16(qa, kf[f][ks], s[a][f]);
          dp[a][f] = mfma16(da, vf[f][ks], dp[a][f]);
        }
      }
    }
    // dV / dK operands (transposed dO / Q reads) one head-dim fragment ahead of their MFMAs, the first
    // under the exp work: -2.3 % L/16-384 backward time vs read-then-wait per fragment
    // (profiles/r5/attn/readahead_ab.log; with attention dropout the extra registers spill)
    constexpr bool TR_AHEAD = !DROP;
    v4s tdlo[2], tdhi[2], tqlo[2], tqhi[2];
    auto tr_load = [&](int e, int bsel) {
      frag_tr_async(doimg, QB, 4 * g, 16 + 4 * g, 16 * e, lane, tdlo[bsel], tdhi[bsel]);
      frag_tr_async(qimg, QB, 4 * g, 16 + 4 * g, 16 * e, lane, tqlo[bsel], tqhi[bsel]);
    };
    if constexpr (TR_AHEAD) tr_load(0, 0);
    ASTAMP(3);
    // P and dS
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * a + 4 * g + r;
        const float l2 = s_lse[ql] * LOG2E;
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const float pv = __builtin_amdgcn_exp2f(fmaf(s[a][f][r], c, -l2));
          if constexpr (DROP) {
            // dropout: dV takes the dropped P, dP = mask * scale * (dO . V); rows past N have
            // dO = 0 and delta = 0, so their dS stays 0 whatever the mask
            const int key = kw0 + 16 * f + li;
            const uint32_t qi = (uint32_t)min(q0 + ql, N - 1);
            const float m = attn_keep1(dkey, qi * npad + (uint32_t)min(key, N - 1), drop.thr) ? drop.scale : 0.f;
            s[a][f][r] = pv * m;
            dp[a][f][r] = pv * (m * dp[a][f][r] - s_dl[ql]);
          } else {
            s[a][f][r] = pv;
            dp[a][f][r] = pv * dp[a][f][r];
          }
        }
      }
    // dV^T[d][key] += dO^T[d][q] P[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
    // (asm transpose reads: the next query block's DMA stays in flight under this phase)
    v8s pf[2], sf[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      pf[f] = pack_p(s[0][f], s[1][f]);
      sf[f] = pack_p(dp[0][f], dp[1][f]);
    }
    ASTAMP(4);
#pragma unroll
    for (int e = 0; e < C::NE; ++e) {
      if constexpr (!TR_AHEAD) tr_load(e, e & 1);
      lds_wait();
      if (TR_AHEAD && e + 1 < C::NE) tr_load(e + 1, (e + 1) & 1);
      const v8s dot = cat44(tdlo[e & 1], tdhi[e & 1]), qt = cat44(tqlo[e & 1], tqhi[e & 1]);
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        dv[e][f] = mfma16(dot, pf[f], dv[e][f]);
        dk[e][f] = mfma16(qt, sf[f], dk[e][f]);
      }
    }
    // dS^T -> LDS (bf16) [key_local][32 queries]: the packed dK-product operands sf, four
    // consecutive queries per 8-B write (a = 0: queries 4g.., a = 1: 16 + 4g..)
    {
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const v4u w = __builtin_bit_cast(v4u, sf[f]);
        *(__attribute__((address_space(3))) v2u*)(dsw + dsw0 + 1024 * f) = v2u{w[0], w[1]};
        *(__attribute__((address_space(3))) v2u*)(dsw + dsw1 + 1024 * f) = v2u{w[2], w[3]};
      }
    }
    }  // active
    ASTAMP(5);
    if (qb > 0) dq_block(qb - 1, slq_prev);
    ASTAMP(6);
    slq_prev[0] = slq_cur[0];
    slq_prev[1] = slq_cur[1];
  }
  // the last block's dQ, once every wave's dS^T of it is written
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  dq_block(nqb - 1, slq_prev);
#ifdef PVR_ATTN_STAMPS
  ASTAMP(7);
  st_acc[7] = __builtin_amdgcn_s_memtime() - st_0;  // whole kernel up to here (slot 7: total, not a phase)
  if (g_attn_dbg && lane == 0 && dq_mode != 4) {  // (not the tail launch of a split head)
#pragma unroll
    for (int k = 0; k < 8; ++k) g_attn_dbg[((int64_t)blockIdx.x * NW + wave) * 8 + k] = st_acc[k];
  }
#endif
  // bpart (the launch that writes the final dQ): this pair's q-bias partials, the column sums of the
  // wave's dQ fragments over all query blocks -> [bh][a][16e + li] (the pre-pass adds the v sums)
  if (bpart && dq_mode == 0) {  // (mode 4: the final pass below writes them)
    int kfr = 0;
    for (int fr = wave; fr < 2 * C::NE && kfr < 2; fr += NW, ++kfr) {
      float cs = kfr == 0 ? dqb0 : dqb1;
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      if (g == 0) bpart[((int64_t)bh * 3 + fr / C::NE) * DH + 16 * (fr % C::NE) + li] = cs;
    }
  }
  // in_proj bias gradient partials of this (batch, key block, head): column sums of dQ | dK | dV,
  // reduced across the waves in LDS and written once (no atomics) to dbias[(b * nkb + kb)][3D];
  // the host then sums over the (batch, key block) rows
  if (dbias) {
    __syncthreads();  // every wave is past its last LDS read
    float* red = (float*)smem;  // [2 (dQ row halves)][DH] q sums | [NW][DH] k | [NW][DH] v
    float* rq = red;
    float* rk = red + 2 * DH;
    float* rv = rk + NW * DH;
    int kfr = 0;
    for (int fr = wave; fr < 2 * C::NE && kfr < 2; fr += NW, ++kfr) {
      float cs = kfr == 0 ? dqb0 : dqb1;
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      if (g == 0) rq[(fr / C::NE) * DH + 16 * (fr % C::NE) + li] = cs;
    }
#pragma unroll
    for (int e = 0; e < C::NE; ++e)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sk = 0.f, sv = 0.f;
#pragma unroll
        for (int f = 0; f < 2; ++f)
          if (kw0 + 16 * f + li < N) {
            sk += dk[e][f][r];
            sv += dv[e][f][r];
          }
#pragma unroll
        for (int sh = 1; sh < 16; sh <<= 1) {
          sk += __shfl_xor(sk, sh, 64);
          sv += __shfl_xor(sv, sh, 64);
        }
        if (li == 0) {
          rk[wave * DH + 16 * e + 4 * g + r] = sk * scale;
          rv[wave * DH + 16 * e + 4 * g + r] = sv;
        }
      }
    __syncthreads();
    float* dst = dbias + ((int64_t)b * nkb + kb0 / KB) * 3 * D + h * DH;
    for (int d = threadIdx.x; d < DH; d += blockDim.x) {
      float tk = 0.f, tv = 0.f;
      for (int w = 0; w < NW; ++w) {
        tk += rk[w * DH + d];
        tv += rv[w * DH + d];
      }
      dst[d] = rq[d] + rq[DH + d];
      dst[D + d] = tk;
      dst[2 * D + d] = tv;
    }
  }
  // dK, dV stores: lane holds X^T[d = 16e + 4g + r][key = kw0 + 16f + li]
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int key = kw0 + 16 * f + li;
    if (key >= N) continue;
    uint16_t* row = dqkv + ((int64_t)b * N + key) * ld_dq;
#pragma unroll
    for (int e = 0; e < C::NE; ++e) {
      uint2 wk, wv;
      wk.x = pack2bf(dk[e][f][0] * scale, dk[e][f][1] * scale);
      wk.y = pack2bf(dk[e][f][2] * scale, dk[e][f][3] * scale);
      wv.x = pack2bf(dv[e][f][0], dv[e][f][1]);
      wv.y = pack2bf(dv[e][f][2], dv[e][f][3]);
      if (!q8.only) {
        *(uint2*)(row + D + h * DH + 16 * e + 4 * g) = wk;
        *(uint2*)(row + 2 * D + h * DH + 16 * e + 4 * g) = wv;
      }
      if (q8kv) {
        float k4[4], v4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          k4[r] = dk[e][f][r] * scale;
          v4[r] = dv[e][f][r];
          q8am = nan_max(q8am, nan_max(fabsf(k4[r]), fabsf(v4[r])));
        }
        uint8_t* qrow = q8.out + ((int64_t)b * N + key) * q8.ld + h * DH + 16 * e + 4 * g;
        *(uint32_t*)(qrow + D) = pack4_fp8_rt(q8.fmt, k4[0] * q8s, k4[1] * q8s, k4[2] * q8s, k4[3] * q8s);
        *(uint32_t*)(qrow + 2 * D) =
            pack4_fp8_rt(q8.fmt, v4[0] * q8s, v4[1] * q8s, v4[2] * q8s, v4[3] * q8s);
      }
    }
  }
  if (q8kv) {
    q8am = wave_max_nan(q8am);
    if (lane == 0) amax_record(q8.amax, q8am);
  }
  // Final dQ pass of the last launch of a multi-block head (one workgroup per (batch, head)):
  //   dq_mode 4: every key block stored its partial dQ as an f32 slab (the body launch before this
  //     one, this workgroup's own just now): sum the nslab + 1 slabs in slab order (deterministic).
  // Coalesced 16-B loads; writes the final dQ: bf16 (unless only the fp8 copy is wanted), its fp8
  // copy, and the q-bias partials (column sums in a fixed order).
  // (no agent-scope fence: it would write back the whole L2. The body launch completed before this
  // one started; this workgroup's own stores / atomics performed in its XCD's L2, which the loads
  // below go through; the CU's L1 holds no line of these rows.)
  if (dq_mode == 4 && dq_acc) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    constexpr int C4 = DH / 4, U = 4;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef uint32_t v2u_ __attribute__((ext_vector_type(2)));
    const int RG = (int)blockDim.x / C4;  // row groups; thread = (row group, fixed 4-column chunk)
    const int chunk = (int)threadIdx.x % C4, rg = (int)threadIdx.x / C4;
    const bool tact = rg < RG;
    const uint32_t sbytes = clamp_bytes((int64_t)N * D * 4);
    const __amdgpu_buffer_rsrc_t ors_q = make_rsrc(dqkv + (int64_t)b * N * ld_dq + h * DH, clamp_bytes(((int64_t)(N - 1) * ld_dq + DH) * 2));
    float csum[4] = {0.f, 0.f, 0.f, 0.f};
    float am = 0.f;
    for (int r0 = rg; r0 < N; r0 += RG * U) {
      v4f sum[U];
#pragma unroll
      for (int u = 0; u < U; ++u) sum[u] = v4f{0.f, 0.f, 0.f, 0.f};
      const int nsrc = nslab + 1;
      for (int sl = 0; sl < nsrc; ++sl) {
        const __amdgpu_buffer_rsrc_t srs = make_rsrc(dq_acc + sl * slab_stride + (int64_t)b * N * D, sbytes);
        v4u v[U];
        uint32_t off[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // rows past N (and idle threads) read as zero
          const int qrow = tact ? r0 + u * RG : N;
          off[u] = ((uint32_t)qrow * (uint32_t)D + (uint32_t)(h * DH + 4 * chunk)) * 4;
          v[u] = __builtin_amdgcn_raw_buffer_load_b128(srs, off[u], 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) sum[u] += __builtin_bit_cast(v4f, v[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int qrow = r0 + u * RG;
        if (!tact || qrow >= N) continue;
        const v4f sv = sum[u];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          csum[j] += sv[j];
          am = nan_max(am, fabsf(sv[j]));
        }
        if (!q8.only)
          __builtin_amdgcn_raw_buffer_store_b64(v2u_{pack2bf(sv[0], sv[1]), pack2bf(sv[2], sv[3])}, ors_q,
                                                ((uint32_t)qrow * (uint32_t)ld_dq + 4 * chunk) * 2, 0, 0);
        if (q8kv)
          *(uint32_t*)(q8.out + ((int64_t)b * N + qrow) * q8.ld + h * DH + 4 * chunk) =
              pack4_fp8_rt(q8.fmt, sv[0] * q8s, sv[1] * q8s, sv[2] * q8s, sv[3] * q8s);
      }
    }
    if (q8kv) {
      am = wave_max_nan(am);
      if (lane == 0) amax_record(q8.amax, am);
    }
    if (bpart) {  // q-bias partials: the row groups' column sums reduced in a fixed order
      float* red = (float*)smem;
      __syncthreads();  // every wave is past its LDS use
      if (tact) {
#pragma unroll
        for (int j = 0; j < 4; ++j) red[rg * DH + 4 * chunk + j] = csum[j];
      }
      __syncthreads();
      for (int d = (int)threadIdx.x; d < DH; d += (int)blockDim.x) {
        float t = 0.f;
        for (int g2 = 0; g2 < RG; ++g2) t += red[g2 * DH + d];
        bpart[((int64_t)bh * 3 + 0) * DH + d] = t;
        bpart[((int64_t)bh * 3 + 1) * DH + d] = 0.f;
      }
    }
  }
}

// Backward pre-pass, one workgroup per (batch, head) pair, streaming the pair's rows once:
//   delta[q] = rowsum(dO[q] * O[q]) for every query (the main kernel then stages no O rows);
//   LAST = true (the lastkey path: the main kernel covers keys [0, N - 1)): the contribution of key
//   kt = N - 1 as well: s = Q.K[kt], dp = dO.V[kt], p = exp(s*scale - lse), ds = p (dp - delta),
//   written per query (ds_last, added to dQ by the main kernel's dQ epilogue), and dV[kt] = sum p dO,
//   dK[kt] = scale * sum ds Q reduced here. For ViT's N = 256 + 1 (the CLS token of 224/14) the main
//   kernel's key blocks are then exactly full.
// Thread = (row slot, 1/8 of the head row): 8 lanes share one query row (DH / 8 consecutive elements
// each: 16 B at dh 64, 20 B at dh 80), 32 row slots per workgroup walk the queries; memory- and
// latency-bound, no MFMA. (The round-4 form gave each row 16 lanes of 16 B: at dh 80 six of every
// 16 lanes idled and a pair took 17 dependent trips instead of 9.)
template <int DH, bool LAST>
__global__ void __launch_bounds__(256) attn_bwd_prep_kernel(const uint16_t* __restrict__ qkv, int64_t ld,
                                                             const uint16_t* __restrict__ dout, int64_t ld_do,
                                                             const uint16_t* __restrict__ o, int64_t ld_o,
                                                             const float* __restrict__ lse, float* __restrict__ dlt,
                                                             float* __restrict__ dsl, float* __restrict__ bpart,
                                                             uint16_t* __restrict__ dqkv, int64_t ld_dq, int N, int H, int D,
                                                             float scale, AttnQ8 q8, int xcd) {
  constexpr int E = DH / 8;   // elements per lane (8 / 10 / 12 / 16)
  constexpr int W = E / 2;    // dwords per lane and row
  constexpr int RS = 32;      // row slots (8 per wave)
  static_assert(DH % 16 == 0 && DH <= 128, "head dim");
  __shared__ float red[3][4][DH];  // per-wave partial column sums
  // xcd: consecutive (batch, head) pairs on one XCD, so the heads of a token row share its L2 (a dh 80
  // head slice is 160 B: its 128-B lines straddle the neighbouring heads' slices)
  const int pr = xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int b = pr / H, h = pr % H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = lane & 7, rs = tid >> 3;  // this lane's eighth of the row, row slot
  const int kt = N - 1;
  const int col = h * DH + ch * E;
  auto load_row = [](const uint16_t* p, uint32_t (&w)[W]) {
#pragma unroll
    for (int j = 0; j < W; ++j) w[j] = ((const uint32_t*)p)[j];
  };
  auto unpack = [](const uint32_t (&w)[W], float (&x)[E]) {
#pragma unroll
    for (int j = 0; j < E; ++j) x[j] = bf2f(j & 1 ? w[j >> 1] >> 16 : w[j >> 1] & 0xFFFF);
  };
  auto row8_sum = [](float v) {  // the row's 8 lanes
#pragma unroll
    for (int off = 4; off > 0; off >>= 1) v += __shfl_xor(v, off, 8);
    return v;
  };
  const uint16_t* qrow0 = qkv + (int64_t)b * N * ld + col;
  float kf[E], vf[E];
#pragma unroll
  for (int j = 0; j < E; ++j) kf[j] = vf[j] = 0.f;
  if constexpr (LAST) {  // this lane's part of K and V of key kt
    uint32_t kw[W], vw[W];
    load_row(qrow0 + (int64_t)kt * ld + D, kw);
    load_row(qrow0 + (int64_t)kt * ld + 2 * D, vw);
    unpack(kw, kf);
    unpack(vw, vf);
  }
  const float c = scale * LOG2E;
  float av[E], ak[E], ov_sum[E];  // dV[kt], dK[kt] partials; column sums of dO (the v-bias gradient)
#pragma unroll
  for (int j = 0; j < E; ++j) av[j] = ak[j] = ov_sum[j] = 0.f;
  const int trips = (N + RS - 1) / RS;  // every row slot takes the same trips (rows past N: not live)
  for (int t = 0; t < trips; ++t) {
    const int q = rs + t * RS;
    const bool live = q < N;  // (uniform per row slot; the row's 8 lanes agree)
    const int qc = min(q, N - 1);
    const int64_t row = (int64_t)b * N + qc;
    uint32_t dw[W], ow[W], qw[W];
    load_row(dout + row * ld_do + col, dw);
    load_row(o + row * ld_o + col, ow);
    if constexpr (LAST) load_row(qrow0 + (int64_t)qc * ld, qw);
    const float lq = LAST ? lse[(int64_t)pr * N + qc] : 0.f;
    float dv[E], ov[E];
    unpack(dw, dv);
    unpack(ow, ov);
    float dl = 0.f;
#pragma unroll
    for (int j = 0; j < E; ++j) dl = fmaf(dv[j], ov[j], dl);
    dl = row8_sum(dl);
    if (live) {
#pragma unroll
      for (int j = 0; j < E; ++j) ov_sum[j] += dv[j];
    }
    if constexpr (LAST) {
      float qv[E];
      unpack(qw, qv);
      float sdot = 0.f, dpdot = 0.f;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        sdot = fmaf(qv[j], kf[j], sdot);
        dpdot = fmaf(dv[j], vf[j], dpdot);
      }
      sdot = row8_sum(sdot);
      dpdot = row8_sum(dpdot);
      const float p = __builtin_amdgcn_exp2f(fmaf(sdot, c, -lq * LOG2E));
      const float ds = live ? p * (dpdot - dl) : 0.f;
      const float pl = live ? p : 0.f;
      if (ch == 0 && live) dsl[(int64_t)pr * N + q] = ds;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        av[j] = fmaf(pl, dv[j], av[j]);
        ak[j] = fmaf(ds, qv[j], ak[j]);
      }
    }
    if (ch == 0 && live) dlt[(int64_t)pr * N + q] = dl;
  }
  if (!LAST && !bpart) return;
  // column sums: the wave's 8 row slots (lanes ch, ch + 8, ..) by shuffles, then the 4 waves via LDS
#pragma unroll
  for (int j = 0; j < E; ++j) {
#pragma unroll
    for (int off = 8; off < 64; off <<= 1) {
      ov_sum[j] += __shfl_xor(ov_sum[j], off);
      if constexpr (LAST) {
        av[j] += __shfl_xor(av[j], off);
        ak[j] += __shfl_xor(ak[j], off);
      }
    }
  }
  if (lane < 8) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      red[0][wave][ch * E + j] = av[j];
      red[1][wave][ch * E + j] = ak[j];
      red[2][wave][ch * E + j] = ov_sum[j];
    }
  }
  __syncthreads();
  if (tid < DH) {
    float sv = 0.f, sk = 0.f, so = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sv += red[0][r][tid];
      sk += red[1][r][tid];
      so += red[2][r][tid];
    }
    if constexpr (LAST) {
      uint16_t* krow = dqkv + ((int64_t)b * N + kt) * ld_dq + h * DH;
      if (!q8.only) {
        krow[D + tid] = f2bf(sk * scale);
        krow[2 * D + tid] = f2bf(sv);
      }
      if (q8.out) {  // fp8 copy of key kt's dK / dV (amax of the two values: the rest come from the main kernel)
        const float qs = *q8.qs;
        uint8_t* qrow = q8.out + ((int64_t)b * N + kt) * q8.ld + h * DH;
        qrow[D + tid] = pack1_fp8_rt(q8.fmt, sk * scale * qs);
        qrow[2 * D + tid] = pack1_fp8_rt(q8.fmt, sv * qs);
        amax_record(q8.amax, nan_max(fabsf(sk * scale), fabsf(sv)));
      }
    }
    // v-bias partial: sum_k dV[k] = sum_q dO[q] (softmax rows sum to 1, no attention dropout)
    if (bpart) bpart[((int64_t)pr * 3 + 2) * DH + tid] = so;
  }
}

// ------------------------------------------- backward, whole head, pipelined (dh 64, 192 < N <= 224)
// ViT-B/16 and ViT-L/16 at 224 px (N = 197). The algorithm (stated for a 4-wave form; the kernel
// below is its 8-wave version): one persistent workgroup per CU walks its (batch, head) pairs; each pair is NQ = ceil(N / 32) blocks of 32 queries, and the blocks of
// consecutive pairs form one stream. Wave w owns keys [64w, 64w + 64): their K / V fragments sit in
// registers for the pair and dK^T / dV^T accumulate in registers over the pair's blocks (key
// fragments entirely past N are skipped). Block t:
//   phase 1 (t):   S = Q K^T, dP = dO V^T (query on the accumulator rows, key on the lane),
//                  P = exp(S c - lse), dS = P (dP - delta); dV^T += dO^T P, dK^T += Q^T dS;
//                  dS^T -> LDS ([key][query] image, ds_write_b64 per 16x16 fragment, 2 buffers).
//   phase 2 (t-1): dQ^T = K^T dS^T of the PREVIOUS block: wave w owns dims 16w .. 16w + 15 of all 32
//                  queries (two 16x16 fragments); the K^T fragments of its dims stay in registers.
//   table (t+1):   lse * log2(e) and delta = rowsum(dO * O) of the NEXT block (8 queries per wave)
//                  into a small LDS table, off phase 1's critical path.
// One barrier per block. S and dP are computed once (the two-kernel backward computes them twice:
// 10 instead of 14 MFMAs per 16x16 score tile), and each Q / dO fragment read from LDS feeds four
// key fragments. LDS-DMA streams block t+3's Q / dO / O / lse rows (4-slot ring) and slices of the
// NEXT pair's K / V images under block t: exactly 7 DMAs per wave per block, issued after the
// block's stores, so one counted wait (vmcnt 7: only the newest group in flight) serves every block.
// The kernel: that algorithm (NQ = 7 blocks) with 8 waves, two per SIMD: the second wave on each
// SIMD hides the latency chains (exp -> pack -> MFMA, LDS reads, per-block waits) that leave a
// one-wave-per-SIMD form's MFMA and VALU pipes idle (measured faster in round 2). That needs <= 256 registers
// per wave, so the persistent state shrinks: wave w owns keys [32w, 32w + 32) (two key fragments:
// 64 accumulator registers), and the K image is double-buffered by pair so the K (S operand) and
// K^T (dQ operand) fragments are read from LDS each block instead of being held; only V (dP
// operand) stays in registers. Phase 2: wave w computes dQ^T dims 16(w&3) .. +15 of queries
// 16(w>>2) .. +15. LDS: K x2 | V | 3-slot Q/dO/O/lse ring | dS^T x2 (152.75 KiB). Every block issues
// one LDS-DMA group right after its barrier (4 per wave, slots 8i + wave: i = 0 Q / dO pieces, 1 O
// pieces and lse, 2-3 next-pair K / V slices) with block t+2's rows; the next barrier waits for it
// (vmcnt(0)), a whole block later. Wave 7 (no keys below N) computes the v-bias partial. Bias
// partials: [pair][NQ][192] = dQ column sums of the two query halves | dO column sums.
template <int NQ>
__global__ void __launch_bounds__(512, 1) attn_bwd_pipe8_kernel(const uint16_t* __restrict__ qkv, int64_t ld,
                                                                 const uint16_t* __restrict__ dout, int64_t ld_do,
                                                                 const uint16_t* __restrict__ o, int64_t ld_o,
                                                                 const float* __restrict__ lse, uint16_t* __restrict__ dqkv,
                                                                 int64_t ld_dq, float* __restrict__ dbp, int N, int H, int D,
                                                                 int npairs, float scale) {
  static_assert(NQ == 7, "192 < N <= 224");
  typedef unsigned int v2u __attribute__((ext_vector_type(2)));
  constexpr int DH = 64;
  constexpr int NP = 32 * NQ;               // staged rows (queries / keys) per pair
  constexpr int IMG = NP * 128;             // K or V image: [NP][128 B], swizzled (lds_off)
  constexpr int SLOT = 3 * 4096 + 1024;     // ring slot: Q | dO | O rows of one block, lse DMA slot
  constexpr int DSB = NP * 64;              // dS^T image [key][32 queries]
  constexpr int NKV = NP / 4;               // 1 KiB pieces of one pair's K + V images
  constexpr int NDMA = 4;                   // DMA instructions per wave per block
  constexpr int KV_PER_IT = 8 * (NDMA - 2); // next-pair K/V pieces per block (slots 16 .. 31)
  constexpr int DBP = 192;                  // bias-gradient partial floats per (pair, block)
  static_assert((NQ - 1) * KV_PER_IT >= NKV, "the next pair's K/V images must be issued within the pair");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* kimg0 = smem;                        // K image of even pair indices (odd: + IMG)
  char* vimg = smem + 2 * IMG;
  char* ring = vimg + IMG;
  char* dsb = ring + 3 * SLOT;
  float* s_tab = (float*)(dsb + 2 * DSB);   // [2][64]: lse * log2e [32] | delta [32] of a block
  float* vsb = s_tab + 128;                  // [64]: v-bias partial of the last block (wave 7 only)
  char* sink = (char*)(vsb + 64);           // 1 KiB target of the filler DMAs of a group

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  PVR_ASSERT(blockDim.x == 512 && (N + 31) / 32 == NQ && (int)gridDim.x <= npairs);
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int per = npairs / gridDim.x, rem = npairs % gridDim.x;
  const int p0 = L * per + min(L, rem);
  const int p1 = p0 + per + (L < rem ? 1 : 0);
  if (p0 >= p1) return;
  const int kw0 = wave * 32;
  const int nf = min(2, max(0, (N - kw0 + 15) / 16));  // this wave's key fragments holding a key < N
  const int j4 = wave & 3, qh = wave >> 2;            // staging piece / phase-2 dims 16 j4, queries 16 qh
  const float c = scale * LOG2E;
  const int64_t rows_all = (int64_t)(npairs / H) * N;
  const __amdgpu_buffer_rsrc_t rq = make_rsrc(qkv, clamp_bytes(((rows_all - 1) * ld + 3 * D) * 2));
  const __amdgpu_buffer_rsrc_t rdo = make_rsrc(dout, clamp_bytes(((rows_all - 1) * ld_do + D) * 2));
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(o, clamp_bytes(((rows_all - 1) * ld_o + D) * 2));
  const __amdgpu_buffer_rsrc_t rl = make_rsrc(lse, clamp_bytes((int64_t)npairs * N * 4));
  const __amdgpu_buffer_rsrc_t rdq = make_rsrc(dqkv, clamp_bytes(((rows_all - 1) * ld_dq + 3 * D) * 2));
  constexpr uint32_t OOR = 0x80000000u;  // dropped stores only: no DMA ever reads out of range
  const uint32_t ldq = (uint32_t)ld * 2, lddo = (uint32_t)ld_do * 2, ldoo = (uint32_t)ld_o * 2, lddq = (uint32_t)ld_dq * 2;

  // ---- lane-dependent offsets, computed once
  const int l3 = lane >> 3, l7 = lane & 7;
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int srl = 8 * j4 + l3;  // staging: row of a 32-row block (piece j4)
  const uint32_t sch = (uint32_t)((l7 ^ swz_a(srl)) << 4);
  const uint32_t stq = (uint32_t)srl * ldq + sch, std_ = (uint32_t)srl * lddo + sch, sto = (uint32_t)srl * ldoo + sch;
  const uint32_t kvo0 = (uint32_t)l3 * ldq + (uint32_t)((l7 ^ swz_a(l3)) << 4);
  const uint32_t kvo1 = (uint32_t)l3 * ldq + (uint32_t)((l7 ^ swz_a(8 + l3)) << 4);
  // A-operand rows (query 16a + li, dims 32ks + 8g ..): a adds 2048; K rows kw0 + 16f + li: f adds 2048
  const int fr0 = li * 128 + ((g ^ swz_a(li)) << 4);
  const int fr1 = li * 128 + (((4 + g) ^ swz_a(li)) << 4);
  int trq[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) trq[e] = (4 * g + q4) * 128 + (((2 * e + (p4 >> 1)) ^ swz_a(4 * g + q4)) << 4) + 8 * (p4 & 1);
  // K^T transposed reads for phase 2 (rows 32ks + 8g + q4, +4; dims 16 j4 + 4p4): ks adds 4096
  const int ktlo = lds_off(NP, 8 * g + q4, 2 * j4 + (p4 >> 1)) + 8 * (p4 & 1);
  const int kthi = lds_off(NP, 8 * g + q4 + 4, 2 * j4 + (p4 >> 1)) + 8 * (p4 & 1);
  auto ds_off = [](int key, int u) { return key * 64 + ((u ^ ((key >> 1) & 7)) << 3); };
  const int dsw0 = ds_off(li, g) + kw0 * 64, dsw1 = ds_off(li, 4 + g) + kw0 * 64;  // a = 0 / 1; f adds 1024
  // phase 2: dS^T rows 32ks + 8g + q4 (+4), queries 16 qh + 4p4; ks adds 2048
  const int p2lo = ds_off(8 * g + q4, 4 * qh + p4), p2hi = ds_off(8 * g + q4 + 4, 4 * qh + p4);
  // next-block table: queries 4 wave + g, dims 4 li .. 4 li + 3 (one 8-B piece)
  const int tq = 4 * wave + g;
  const int tbo = tq * 128 + (((li >> 1) ^ swz_a(tq)) << 4) + 8 * (li & 1);

  struct PairOff {
    uint32_t row, col;  // b * N, h * DH * 2 (bytes)
  };
  auto pair_off = [&](int pr) { return PairOff{(uint32_t)((pr / H) * N), (uint32_t)((pr % H) * DH * 2)}; };
  auto dma = [&](__amdgpu_buffer_rsrc_t rs, char* img, uint32_t voff) { dma16(rs, to_lds(img), voff); };
  // this wave's NDMA DMAs: block sqb of pair `so` into ring slot `slot` and, if kvon, K / V pieces
  // [kvc * KV_PER_IT, ...) of pair `ko` (K into `kdst`); rows past N clamped to N-1 (no DMA reads
  // out of range); filler slots reload a valid piece into `sink` at a distinct address per slot
  auto issue_group = [&](PairOff so, int sqb, char* slot, bool kvon, int kvc, PairOff ko, char* kdst) {
    const int r0 = 32 * sqb;
    const int row = min(r0 + srl, N - 1) - srl;
    const uint32_t rb = so.row + (uint32_t)row;
    if (wave < 4)
      dma(rq, slot + j4 * 1024, rb * ldq + so.col + stq);
    else
      dma(rdo, slot + 4096 + j4 * 1024, rb * lddo + so.col + std_);
    if (wave < 4) {
      dma(ro, slot + 8192 + j4 * 1024, rb * ldoo + so.col + sto);
    } else if (wave == 4) {  // lse[(b*H + h)*N + r0 ..] (lanes 8.. repeat lane 7)
      dma(rl, slot + 12288, (so.row * (uint32_t)H + (so.col >> 7) * (uint32_t)N + (uint32_t)r0) * 4 + (uint32_t)min(lane, 7) * 16);
    } else {
      dma(rq, sink, (uint32_t)lane * 16 + 1024);
    }
#pragma unroll
    for (int i = 2; i < NDMA; ++i) {
      const int k = kvc * KV_PER_IT + 8 * (i - 2) + wave;
      const bool live = kvon && k < NKV;
      const int which = k >= NP / 8, rr = (k - which * (NP / 8)) * 8;
      const int kr = min(rr + l3, N - 1) - l3;
      const uint32_t base = (ko.row + kr) * ldq + (uint32_t)(which + 1) * D * 2 + ko.col;
      dma(rq, live ? (which ? vimg : kdst) + rr * 128 : sink, live ? base + ((rr & 8) ? kvo1 : kvo0) : (uint32_t)lane * 16 + i * 1024);
    }
  };
  // lse*log2e and delta of the block in ring slot `sb` (local block qb) into table buffer `tb`
  auto block_table = [&](const char* sb, int qb, int tb) {
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
    const bf4 dw = *(const __attribute__((address_space(3))) bf4*)(sb + 4096 + tbo);
    const bf4 ow = *(const __attribute__((address_space(3))) bf4*)(sb + 8192 + tbo);
    float d = __builtin_amdgcn_fdot2_f32_bf16(bf2{dw[0], dw[1]}, bf2{ow[0], ow[1]}, 0.f, false);
    d = __builtin_amdgcn_fdot2_f32_bf16(bf2{dw[2], dw[3]}, bf2{ow[2], ow[3]}, d, false);
    d = row16_sum(d);
    if (li == 0) {
      const float l = ((const float*)(sb + 12288))[tq];
      s_tab[tb * 64 + tq] = 32 * qb + tq < N ? l * LOG2E : __builtin_huge_valf();
      s_tab[tb * 64 + 32 + tq] = d;
    }
  };
  // dQ^T fragment (dims 16 j4 + 4g + r, queries 16 qh + li) of a block (local pqb of pair index
  // ppair) from dS^T buffer `ds` and the pair's K image `kimg`; with dbp, its bias partials
  auto phase2 = [&](const char* ds, const char* kimg, int pqb, PairOff po, int ppair) {
    v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
    auto batch = [&](auto k0c, auto k1c) {
      constexpr int k0 = decltype(k0c)::value, k1 = decltype(k1c)::value;
      v4s klo[k1 - k0], khi[k1 - k0], lo[k1 - k0], hi[k1 - k0];
      static_for<k0, k1>([&](auto kc) {
        constexpr int ks = decltype(kc)::value;
        klo[ks - k0] = ds_read_tr_async_at<4096 * ks>(kimg + ktlo);
        khi[ks - k0] = ds_read_tr_async_at<4096 * ks>(kimg + kthi);
        lo[ks - k0] = ds_read_tr_async_at<2048 * ks>(ds + p2lo);
        hi[ks - k0] = ds_read_tr_async_at<2048 * ks>(ds + p2hi);
      });
      lds_wait();
#pragma unroll
      for (int j = 0; j < k1 - k0; ++j) acc = mfma16(cat44(klo[j], khi[j]), cat44(lo[j], hi[j]), acc);
    };
    batch(std::integral_constant<int, 0>{}, std::integral_constant<int, 4>{});
    batch(std::integral_constant<int, 4>{}, std::integral_constant<int, NQ>{});
    const int q = pqb * 32 + 16 * qh + li;
    const uint32_t vo = q < N ? (po.row + q) * lddq + po.col + (uint32_t)(16 * j4 + 4 * g) * 2 : OOR;
    const v2u w = {pack2bf(acc[0] * scale, acc[1] * scale), pack2bf(acc[2] * scale, acc[3] * scale)};
    __builtin_amdgcn_raw_buffer_store_b64(w, rdq, vo, 0, 0);
    if (dbp) {  // queries past N have dS = 0, so dQ = 0 exactly
      float* dst = dbp + ((int64_t)ppair * NQ + pqb) * DBP;
      float cs[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[r] = row16_sum(acc[r]) * scale;
      if (li == 0) *(float4*)(dst + 64 * qh + 16 * j4 + 4 * g) = make_float4(cs[0], cs[1], cs[2], cs[3]);
      if (wave == 7) dst[128 + lane] = vsb[lane];
    }
  };

  v8s vf[2][2];
  v4f dk[4][2], dv[4][2];  // [dims e][key fragment f]
  auto zero_acc = [&]() {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int f = 0; f < 2; ++f) dk[e][f] = dv[e][f] = v4f{0.f, 0.f, 0.f, 0.f};
  };
  auto store_dkv = [&](PairOff po) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int key = kw0 + 16 * f + li;
      const uint32_t vo = key < N ? (po.row + key) * lddq + po.col + (uint32_t)(4 * g) * 2 : OOR;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const v2u wk = {pack2bf(dk[e][f][0] * scale, dk[e][f][1] * scale), pack2bf(dk[e][f][2] * scale, dk[e][f][3] * scale)};
        const v2u wv = {pack2bf(dv[e][f][0], dv[e][f][1]), pack2bf(dv[e][f][2], dv[e][f][3])};
        __builtin_amdgcn_raw_buffer_store_b64(wk, rdq, vo + (uint32_t)(D + 16 * e) * 2, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64(wv, rdq, vo + (uint32_t)(2 * D + 16 * e) * 2, 0, 0);
      }
    }
  };

  // ---- prologue: pair p0's K (buffer 0) / V images, blocks 0 and 1; table of block 0
  const PairOff none{0u, 0u};
  PairOff cur = pair_off(p0);
  for (int k = wave; k < NKV; k += 8) {
    const int which = k >= NP / 8, rr = (k - which * (NP / 8)) * 8;
    const int kr = min(rr + l3, N - 1) - l3;
    const uint32_t base = (cur.row + kr) * ldq + (uint32_t)(which + 1) * D * 2 + cur.col;
    dma(rq, (which ? vimg : kimg0) + rr * 128, base + ((rr & 8) ? kvo1 : kvo0));
  }
  issue_group(cur, 0, ring, false, 0, none, kimg0);
  issue_group(cur, 1, ring + SLOT, false, 0, none, kimg0);
  zero_acc();
  wait_barrier_lds<0>();
  block_table(ring, 0, 0);

  const int npr = p1 - p0;
  PairOff prv = cur;
  int sl = 0;  // ring slot of block t (t mod 3)
#ifdef PVR_ATTN_STAMPS
  // slots: 0 wait + barrier, 1 DMA group issue, 2 pair switch (previous pair's dQ / dK / dV, V
  // fragments), 3 S / dP, 4 dQ, 5 next table, 6 P / dS + dV / dK, 7 loop total
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_last = __builtin_amdgcn_s_memtime();
  const uint64_t st_0 = st_last;
#endif
  // global stores of a block (dQ of the previous block, its bias partials, a pair's dK / dV) are issued
  // after the block's DMA group: the next block's wait retires the group but leaves them in flight
  // (a plain vmcnt(0) there waited for their write acknowledgements, ~1-2 us per block)
  const int pdb = dbp ? 1 + (wave == 7 ? 1 : 0) : 0;  // bias-partial stores per phase 2
  int nst = 0;                                          // stores issued in the previous block
  for (int pi = 0; pi < npr; ++pi) {
    cur = pair_off(p0 + pi);
    const bool has_next = pi + 1 < npr;
    const PairOff nxt = has_next ? pair_off(p0 + pi + 1) : none;
    const char* kimg = kimg0 + (pi & 1) * IMG;
    char* knext = kimg0 + ((pi + 1) & 1) * IMG;
#pragma unroll 1
    for (int qb = 0; qb < NQ; ++qb) {
      const int t = pi * NQ + qb;
      // block t+1's DMA group (issued a block ago) complete, the previous block's stores may still be
      // in flight; dS^T of block t-1 and the table of block t visible; every wave past its reads of
      // the reused buffers
      switch (nst) {  // wave-uniform: the count of stores younger than that group
        case 1: wait_barrier_lds<1>(); break;
        case 2: wait_barrier_lds<2>(); break;
        case 3: wait_barrier_lds<3>(); break;
        case 17: wait_barrier_lds<17>(); break;
        case 18: wait_barrier_lds<18>(); break;
        case 19: wait_barrier_lds<19>(); break;
        default: wait_barrier_lds<0>(); break;
      }
      ASTAMP(0);
      nst = (qb == 0 && pi > 0 ? 17 + pdb : 0) + (qb != 0 ? 1 + pdb : 0);
      const char* qimg = ring + sl * SLOT;
      const char* doimg = qimg + 4096;
      const int sl1 = sl == 2 ? 0 : sl + 1, sl2 = sl1 == 2 ? 0 : sl1 + 1;
      // ---- DMA: block t+2 into slot (t+2) mod 3 (block t-1's, consumed) and, in local blocks
      // 1 .. NQ-1, slices of the next pair's K (other buffer, free once block 0's phase 2 of the
      // previous pair ran) / V (this pair's V fragments are in registers by then) images
      if (qb + 2 < NQ)
        issue_group(cur, qb + 2, ring + sl2 * SLOT, qb >= 1 && has_next, qb - 1, nxt, knext);
      else
        issue_group(has_next ? nxt : cur, has_next ? qb + 2 - NQ : 0, ring + sl2 * SLOT, has_next, qb - 1, nxt, knext);
      ASTAMP(1);
      if (qb == 0) {
        if (pi > 0) {
          // the previous pair's last block (its K image is the other buffer) and its dK / dV
          phase2(dsb + ((t - 1) & 1) * DSB, knext, NQ - 1, prv, p0 + pi - 1);
          store_dkv(prv);
          zero_acc();
        }
        if (nf > 0) {
#pragma unroll
          for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) vf[f][ks] = ds_read_b128(vimg + kw0 * 128 + 2048 * f + (ks ? fr1 : fr0));
        }
      }
      ASTAMP(2);
      // ---- phase 1a: S[q][key], dP[q][key] of the wave's two key fragments
      v4f s[2][2], dp[2][2];
      if (nf > 0) {
        v8s qa[2][2], dA[2][2], kf[2][2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            const int fo = (ks ? fr1 : fr0) + 2048 * a;
            qa[ks][a] = ds_read_b128(qimg + fo);
            dA[ks][a] = ds_read_b128(doimg + fo);
            kf[a][ks] = ds_read_b128(kimg + kw0 * 128 + fo);  // key fragment f = a
          }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int f = 0; f < 2; ++f) s[a][f] = dp[a][f] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int f = 0; f < 2; ++f) {
              s[a][f] = mfma16(qa[ks][a], kf[f][ks], s[a][f]);
              dp[a][f] = mfma16(dA[ks][a], vf[f][ks], dp[a][f]);
            }
      }
      ASTAMP(3);
      // ---- phase 2 of block t-1 (same pair), while the S / dP products drain
      if (qb != 0) phase2(dsb + ((t - 1) & 1) * DSB, kimg, qb - 1, cur, p0 + pi);
      ASTAMP(4);
      // ---- table of block t+1 (landed at this block's wait)
      if (qb + 1 < NQ)
        block_table(ring + sl1 * SLOT, qb + 1, (t + 1) & 1);
      else if (has_next)
        block_table(ring + sl1 * SLOT, 0, (t + 1) & 1);
      ASTAMP(5);
      // ---- phase 1b: P, dS of both key fragments (dS^T -> LDS), then dV^T += dO^T P, dK^T += Q^T dS
      // one dims fragment at a time (transposed Q / dO reads double-buffered)
      if (nf > 0) {
        const float* tl = s_tab + (t & 1) * 64 + 4 * g;
        char* img = dsb + (t & 1) * DSB;
        v8s pf[2], sf[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const bool kin = kw0 + 16 * f + li < N;
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            const v4f l4 = *(const v4f*)(tl + 16 * a), d4 = *(const v4f*)(tl + 32 + 16 * a);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float pv = kin ? __builtin_amdgcn_exp2f(fmaf(s[a][f][r], c, -l4[r])) : 0.f;
              s[a][f][r] = pv;
              dp[a][f][r] = pv * (dp[a][f][r] - d4[r]);
            }
            const v2u w = {pack2bf(dp[a][f][0], dp[a][f][1]), pack2bf(dp[a][f][2], dp[a][f][3])};
            *(v2u*)(img + (a ? dsw1 : dsw0) + 1024 * f) = w;
          }
          pf[f] = pack_p(s[0][f], s[1][f]);
          sf[f] = pack_p(dp[0][f], dp[1][f]);
        }
        v4s dlo[2], dhi[2], qlo[2], qhi[2];
        auto tr_load = [&](int e, int bsel) {
          dlo[bsel] = ds_read_tr_async(doimg + trq[e]);
          dhi[bsel] = ds_read_tr_async(doimg + trq[e] + 2048);
          qlo[bsel] = ds_read_tr_async(qimg + trq[e]);
          qhi[bsel] = ds_read_tr_async(qimg + trq[e] + 2048);
        };
        tr_load(0, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lds_wait();
          if (e + 1 < 4) tr_load(e + 1, (e + 1) & 1);
          const v8s dot = cat44(dlo[e & 1], dhi[e & 1]), qt = cat44(qlo[e & 1], qhi[e & 1]);
#pragma unroll
          for (int f = 0; f < 2; ++f) {
            dv[e][f] = mfma16(dot, pf[f], dv[e][f]);
            dk[e][f] = mfma16(qt, sf[f], dk[e][f]);
          }
        }
      }
      if (dbp && wave == 7) {
        // v-bias partial: dO^T . 1 over the block's queries < N (the k bias gets no gradient)
        v4s vlo[4], vhi[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vlo[e] = ds_read_tr_async(doimg + trq[e]);
          vhi[e] = ds_read_tr_async(doimg + trq[e] + 2048);
        }
        v4f m0, m1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          m0[r] = 32 * qb + 4 * g + r < N ? 1.f : 0.f;
          m1[r] = 32 * qb + 16 + 4 * g + r < N ? 1.f : 0.f;
        }
        const v8s ones = pack_p(m0, m1);
        lds_wait();
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const v4f cs = mfma16(cat44(vlo[e], vhi[e]), ones, v4f{0.f, 0.f, 0.f, 0.f});
          if (li == 0) *(v4f*)(vsb + 16 * e + 4 * g) = cs;
        }
      }
      ASTAMP(6);
      sl = sl1;
    }
    prv = cur;
  }
#ifdef PVR_ATTN_STAMPS
  st_acc[7] = __builtin_amdgcn_s_memtime() - st_0;
  if (g_attn_dbg && lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g_attn_dbg[((int64_t)blockIdx.x * 8 + wave) * 8 + k] = st_acc[k];
  }
#endif
  // last block's dQ and the last pair's dK / dV
  wait_barrier_lds<0>();
  phase2(dsb + ((npr * NQ - 1) & 1) * DSB, kimg0 + ((npr - 1) & 1) * IMG, NQ - 1, prv, p1 - 1);
  store_dkv(prv);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
}

// Deterministic dQ of a multi-key-block head without the tail-split slab path: dQ = the key blocks'
// f32 partial slabs (mode-3 launch, slab s = key block s) summed in slab order, as bf16.
__global__ void __launch_bounds__(256) dq_slab_sum_kernel(const float* __restrict__ slab, int nslab, int64_t sstride,
                                                           uint16_t* __restrict__ dqkv, int64_t ld_dq, int64_t rows, int D) {
  const int64_t n = rows * D;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float v = slab[i];
    for (int k = 1; k < nslab; ++k) v += slab[k * sstride + i];
    dqkv[(i / D) * ld_dq + i % D] = f2bf(v);
  }
}

__global__ void __launch_bounds__(256) dq_convert_kernel(float* __restrict__ acc, uint16_t* __restrict__ dqkv, int64_t ld_dq,
                                                          int64_t rows, int D, int rezero) {
  const int64_t n = rows * D;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / D;
    const int d = (int)(i % D);
    dqkv[r * ld_dq + d] = f2bf(acc[i]);
    if (rezero) acc[i] = 0.f;
  }
}

// In_proj bias gradient from the pipelined backward's per-(batch, head, 32-query block) partials
// part[(b*H + h)*NQ + nq][192] (q sums of the two 16-query halves | v sums), deterministic in two
// passes: (1) grid (H, S): rows s*R .. of head h's B*NQ partial rows -> ws[s][h][128] (q | v);
// (2) grid H: dbias[q slice of h] += sum_s, dbias[v slice of h] += sum_s (the k bias gradient is 0).
// partial rows of 3 * DH floats: q sums of the two 16-query halves | v sums; block = 2 * DH threads
__global__ void __launch_bounds__(256) dbias_part_kernel(const float* __restrict__ part, float* __restrict__ ws, int B, int H,
                                                         int NQ, int R, int DH) {
  const int h = blockIdx.x, sidx = blockIdx.y, t = threadIdx.x;
  const int rows = B * NQ, r0 = sidx * R, r1 = min(rows, r0 + R);
  float a = 0.f;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) {  // unrolled: eight rows' loads in flight, not one dependent load per row
    const int b = r / NQ, nq = r - b * NQ;
    const float* row = part + ((int64_t)(b * H + h) * NQ + nq) * 3 * DH;
    a += t < DH ? row[t] + row[DH + t] : row[DH + t];
  }
  ws[((int64_t)sidx * H + h) * 2 * DH + t] = a;
}

__global__ void __launch_bounds__(256) dbias_final_kernel(const float* __restrict__ ws, float* __restrict__ dbias, int H, int D, int S,
                                                          int DH) {
  const int h = blockIdx.x, t = threadIdx.x;
  // four independent partial sums, 16 loads in flight per thread: the one-accumulator loop waited one
  // memory latency per split (32 us for 128 splits at ViT-B/16 b256); fixed order, so deterministic
  const float* col = ws + (int64_t)h * 2 * DH + t;
  const int64_t step = (int64_t)H * 2 * DH;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int sidx = 0;
#pragma unroll 4
  for (; sidx + 4 <= S; sidx += 4) {
    a0 += col[(sidx + 0) * step];
    a1 += col[(sidx + 1) * step];
    a2 += col[(sidx + 2) * step];
    a3 += col[(sidx + 3) * step];
  }
  for (; sidx < S; ++sidx) a0 += col[sidx * step];
  const float a = (a0 + a1) + (a2 + a3);
  if (t < DH)
    dbias[h * DH + t] += a;
  else
    dbias[2 * D + h * DH + (t - DH)] += a;
}

}  // namespace
}  // namespace pvr

// ws: f32 [S][H][2 * DH] scratch, S = pvr_attn_dbias_splits(B, NQ); part f32 [B*H][NQ][3 * DH]
extern "C" int pvr_attn_dbias_splits(int B, int NQ) { return B * NQ < 128 ? B * NQ : 128; }

extern "C" hipError_t pvr_attn_dbias_reduce(const float* part, float* ws, float* dbias, int B, int H, int NQ, int D, hipStream_t s) {
  using namespace pvr;
  const int S = pvr_attn_dbias_splits(B, NQ);
  if (S <= 0) return hipSuccess;
  const int DH = D / H;
  if (D % H != 0 || 2 * DH > 256) return hipErrorInvalidValue;
  const int R = (B * NQ + S - 1) / S;
  hipLaunchKernelGGL(dbias_part_kernel, dim3(H, S), dim3(2 * DH), 0, s, part, ws, B, H, NQ, R, DH);
  hipLaunchKernelGGL(dbias_final_kernel, dim3(H), dim3(2 * DH), 0, s, ws, dbias, H, D, S, DH);
  return hipGetLastError();
}

static int device_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

// whole-head kernel: one persistent workgroup per CU (its double-buffered K/V images take up to
// 128 KiB of LDS), ceil(N / (16 QF)) waves. g_attn_fwd_head_qf: query fragments per wave (A/B,
// default 1).
#ifndef PVR_ATTN_HEAD_QF
#define PVR_ATTN_HEAD_QF 1
#endif
int g_attn_fwd_head_qf = PVR_ATTN_HEAD_QF;
template <int NF, int QF>
static hipError_t attn_fwd_head_launch_qf(const uint16_t* qkv, int64_t ld, uint16_t* out, int64_t ld_o, float* lse, int B, int N,
                                          int H, int D, float scale, hipStream_t s) {
  using namespace pvr;
  constexpr int SMEM = 2 * 2 * 32 * ((NF + 1) / 2) * 128;
  constexpr int NW = (NF + QF - 1) / QF;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)attn_fwd_head_kernel<NF, QF>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int npairs = B * H;
  const int grid = npairs < device_cus() ? npairs : device_cus();
  hipLaunchKernelGGL((attn_fwd_head_kernel<NF, QF>), dim3(grid), dim3(NW * 64), SMEM, s, qkv, ld, out, ld_o, lse, N, H, D, npairs, scale);
  return hipGetLastError();
}
template <int NF>
static hipError_t attn_fwd_head_launch(const uint16_t* qkv, int64_t ld, uint16_t* out, int64_t ld_o, float* lse, int B, int N,
                                       int H, int D, float scale, hipStream_t s) {
  return g_attn_fwd_head_qf == 2 ? attn_fwd_head_launch_qf<NF, 2>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, s)
                                 : attn_fwd_head_launch_qf<NF, 1>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, s);
}

// Tiled forward launch: QG query groups per wave, KT keys per tile, dynamic LDS for two K/V stages.
// round 3 form: QG 1 (64 queries per workgroup) and 32-key tiles for two-image head rows (dh > 64);
// round 4: QG 2 (128 queries per workgroup, each K / V fragment read feeds two MFMAs) and 64-key
// tiles at every head dim (64 KiB of LDS at dh 80: two workgroups per CU). QG 2 pads the query
// count to 128 instead of 64: it is chosen only when that padding costs < 10 % more query rows
// (L/16-384, N = 577: 640 either way, QG 2 0.399 vs 0.440 ms; H/14, N = 257: 384 vs 320 rows, QG 2
// 0.376 vs 0.319 ms, scripts/attn_ab.py). g_attn_fwd_qg: 0 = that rule, 1 / 2 = forced (A/B of
// the two production forms). (Measured losers removed in round 5: QG 1 with 64-key tiles at every
// head dim; O stored straight from the registers instead of through LDS, profiles/r4/aq8.)
int g_attn_fwd_qg = 0;
static bool attn_fwd_use_qg2(int N) {
  if (g_attn_fwd_qg) return g_attn_fwd_qg == 2;
  const int r2 = (N + 127) / 128 * 128, r1 = (N + 63) / 64 * 64;
  return r2 * 10 <= r1 * 11;
}
template <int DH, bool DROP, int QG, int KT>
static hipError_t attn_fwd_tiled(const uint16_t* qkv, int64_t ld, uint16_t* out, int64_t ld_o, float* lse, int B, int N, int H, int D,
                                 float scale, const pvr::AttnDrop& drop, const pvr::AttnQ8& q8, hipStream_t s) {
  using namespace pvr;
  constexpr int SMEM = 4 * KT * 128 * Hd<DH>::NH;
  auto kern = attn_fwd_kernel<DH, DROP, QG, KT>;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int nqb = (N + 64 * QG - 1) / (64 * QG);
  hipLaunchKernelGGL(kern, dim3(nqb * B * H, 1), dim3(256), SMEM, s, qkv, ld, out, ld_o, lse, N, H, D, scale, drop, q8);
  return hipGetLastError();
}

template <int DH, bool DROP>
static hipError_t attn_fwd_tiled_pick(const uint16_t* qkv, int64_t ld, uint16_t* out, int64_t ld_o, float* lse, int B, int N, int H,
                                      int D, float scale, const pvr::AttnDrop& drop, const pvr::AttnQ8& q8, hipStream_t s) {
  if (attn_fwd_use_qg2(N)) return attn_fwd_tiled<DH, DROP, 2, 64>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, drop, q8, s);
  return attn_fwd_tiled<DH, DROP, 1, (pvr::Hd<DH>::NH == 1 ? 64 : 32)>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, drop, q8, s);
}

template <int DH>
static hipError_t attn_fwd_launch(const uint16_t* qkv, int64_t ld, uint16_t* out, int64_t ld_o, float* lse, int B, int N, int H,
                                  int D, float scale, const pvr::AttnDrop& drop, const pvr::AttnQ8& q8, hipStream_t s) {
  using namespace pvr;
  if (drop.seed)  // attention dropout: the tiled kernel with the in-register keep mask
    return attn_fwd_tiled_pick<DH, true>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, drop, q8, s);
  if (DH == 64 && N <= 256 && !q8.out) {
    // whole-head kernel: one persistent workgroup per CU (its double-buffered K/V images take
    // up to 128 KiB of LDS), ceil(N/16) waves
    switch ((N + 15) / 16) {
#define PVR_FWD_HEAD(NF) \
  case NF: return attn_fwd_head_launch<NF>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, s);
      PVR_FWD_HEAD(1) PVR_FWD_HEAD(2) PVR_FWD_HEAD(3) PVR_FWD_HEAD(4) PVR_FWD_HEAD(5) PVR_FWD_HEAD(6)
      PVR_FWD_HEAD(7) PVR_FWD_HEAD(8) PVR_FWD_HEAD(9) PVR_FWD_HEAD(10) PVR_FWD_HEAD(11) PVR_FWD_HEAD(12)
      PVR_FWD_HEAD(13) PVR_FWD_HEAD(14) PVR_FWD_HEAD(15) PVR_FWD_HEAD(16)
#undef PVR_FWD_HEAD
      default: break;
    }
  }
  return attn_fwd_tiled_pick<DH, false>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, drop, q8, s);
}

// diagnostic builds (-DPVR_ATTN_STAMPS): where the backward writes its phase stamps (null: nowhere)
extern "C" void pvr_set_attn_dbg(void* p) {
#ifdef PVR_ATTN_STAMPS
  uint64_t* q = (uint64_t*)p;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(pvr::g_attn_dbg), &q, sizeof(q));
#else
  (void)p;
#endif
}

extern "C" void pvr_set_attn_fwd_qg(int qg) { g_attn_fwd_qg = qg == 1 || qg == 2 ? qg : 0; }
extern "C" void pvr_set_attn_fwd_head_qf(int qf) { g_attn_fwd_head_qf = qf == 2 ? 2 : 1; }
// backward pre-pass: (batch, head) pairs dealt XCD-contiguously (1) or round-robin (0, default: the
// two measured equal, profiles/r6/prep/attn_ab.log); A/B
static int g_attn_prep_xcd = 0;
extern "C" void pvr_set_attn_prep_xcd(int on) { g_attn_prep_xcd = on ? 1 : 0; }

// seed (optional): attention-probability dropout with keep threshold thr16 (see AttnDrop); the
// backward must get the same seed / seed_off / thr16
extern "C" hipError_t pvr_attn_fwd(const uint16_t* qkv, int64_t ld, uint16_t* out, int64_t ld_o, float* lse, int B, int N,
                                   int H, int D, float scale, const uint64_t* seed, uint64_t seed_off, uint32_t thr16, float keep_scale,
                                   uint8_t* q8_out, int64_t q8_ld, const float* q8_qs, unsigned* q8_amax, int q8_only, hipStream_t s) {
  using namespace pvr;
  if (H <= 0 || D % H != 0 || B <= 0 || N <= 0 || N > 65536) return hipErrorInvalidValue;
  if (q8_out && (!q8_qs || !q8_amax || q8_ld % 4 != 0 || (uintptr_t)q8_out % 4 != 0)) return hipErrorInvalidValue;
  if (q8_only && !q8_out) return hipErrorInvalidValue;
  const AttnDrop drop{seed, seed_off, thr16, keep_scale};
  // only (inference): O's e4m3 copy alone is stored (bf16 O unwritten); the copy's path is the generic kernel
  const AttnQ8 q8{q8_out, q8_ld, q8_qs, q8_amax, q8_only ? 1 : 0};
  switch (D / H) {
    case 64: return attn_fwd_launch<64>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, drop, q8, s);
    case 80: return attn_fwd_launch<80>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, drop, q8, s);
    case 96: return attn_fwd_launch<96>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, drop, q8, s);
    case 128: return attn_fwd_launch<128>(qkv, ld, out, ld_o, lse, B, N, H, D, scale, drop, q8, s);
    default: return hipErrorInvalidValue;
  }
}

extern "C" int pvr_attn_head_dim_supported(int dh) { return dh == 64 || dh == 80 || dh == 96 || dh == 128; }

extern "C" int pvr_attn_bwd_waves(int N);
extern "C" int pvr_attn_bwd_key_blocks(int N) {
  const int kb = 32 * pvr_attn_bwd_waves(N);
  return (N + kb - 1) / kb;
}

extern "C" int pvr_attn_bwd_waves(int N) {
  const int need = (N + 31) / 32;
  return need >= 8 ? 8 : (need > 4 ? 8 : (need > 2 ? 4 : (need > 1 ? 2 : 1)));
}

// N = (full key blocks) + 1 key: main kernel + the pre-pass's last key, dQ written directly (no
// dq_acc); not with attention dropout (the pre-pass has no mask)
static bool attn_bwd_lastkey_path(int N, bool dbias, bool drop) {
  const int KB = 32 * pvr_attn_bwd_waves(N);
  return (N + KB - 1) / KB == 2 && N % KB == 1 && !dbias && !drop && N <= 512;
}

// key-block body + a short tail launch (ViT-L/16@384: 577 = 2 x 256 + 65; see attn_bwd_generic)
static bool attn_bwd_tail_split(int N, bool dbias, bool drop) {
  const int KB = 32 * pvr_attn_bwd_waves(N);
  const int rem = N % KB;
  return !attn_bwd_lastkey_path(N, dbias, drop) && (N + KB - 1) / KB > 1 && rem >= 16 && rem <= 128 && !dbias;
}
// dQ of the tail-split path through f32 slabs summed by the tail (the f32-atomics alternative lost:
// 1.215 vs 1.260 ms per ViT-L/16@384 b128 layer, same process, profiles/r4/ab10/attn_ab.log; removed)
static bool attn_bwd_slab_path(int N, bool dbias, bool drop) { return attn_bwd_tail_split(N, dbias, drop); }

// the generic backward's kernels write every final dQ value (no f32 atomics + conversion pass)
static bool attn_bwd_final_dq_in_kernel(int N, bool dbias, bool drop) {
  const int KB = 32 * pvr_attn_bwd_waves(N);
  return attn_bwd_lastkey_path(N, dbias, drop) || attn_bwd_tail_split(N, dbias, drop) || (N + KB - 1) / KB == 1;
}

// the generic backward can emit the in_proj bias gradient as [B*H][1][3*dh] partials (q sums of
// the two 16-query fragment rows | v sums = dO column sums): the launch that writes the final dQ
// holds every dQ fragment of a pair, at most two per wave (no attention dropout: its rows of P do
// not sum to 1, so sum_k dV != sum_q dO)
static bool attn_bwd_bpart_ok(int N, int DH) {
  const int NE = DH / 16;
  const int KB = 32 * pvr_attn_bwd_waves(N);
  if (attn_bwd_lastkey_path(N, false, false)) return NE <= pvr_attn_bwd_waves(N);
  if (attn_bwd_tail_split(N, false, false)) return true;  // the tail's final dQ pass writes them
  return (N + KB - 1) / KB == 1 && NE <= pvr_attn_bwd_waves(N);
}

// 1 if pvr_attn_bwd needs the zero-initialised f32 dQ workspace for this shape (det: deterministic
// mode, where such shapes sum per-key-block dQ slabs in a fixed order instead: no workspace)
extern "C" int pvr_attn_bwd_needs_dq_acc(int N, int dh, int dbias, int drop, int det) {
  if (pvr_attn_bwd_key_blocks(N) <= 1 || det) return 0;
  return attn_bwd_lastkey_path(N, dbias != 0, drop != 0) || attn_bwd_slab_path(N, dbias != 0, drop != 0) ? 0 : 1;
}

template <int NQ>
static hipError_t attn_bwd_pipe8_launch(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ld_o, const uint16_t* dout,
                                        int64_t ld_do, const float* lse, uint16_t* dqkv, int64_t ld_dq, float* dbp, int B, int N, int H,
                                        int D, float scale, hipStream_t s) {
  using namespace pvr;
  constexpr int SMEM = 3 * (32 * NQ) * 128 + 3 * (3 * 4096 + 1024) + 2 * (32 * NQ) * 64 + 512 + 256 + 1024;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)attn_bwd_pipe8_kernel<NQ>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int npairs = B * H;
  const int grid = npairs < device_cus() ? npairs : device_cus();
  hipLaunchKernelGGL(attn_bwd_pipe8_kernel<NQ>, dim3(grid), dim3(512), SMEM, s, qkv, ld, dout, ld_do, out, ld_o, lse, dqkv, ld_dq, dbp,
                     N, H, D, npairs, scale);
  return hipGetLastError();
}

// the pipelined backward serves this shape / these layouts (dh 64, 192 < N <= 224: the K double
// buffer fits LDS; 31-bit offsets)
static bool attn_bwd_pipe_ok(int B, int N, int H, int D, int64_t ld, int64_t ld_do, int64_t ld_o, int64_t ld_dq) {
  const int64_t rows_all = (int64_t)B * N;
  const bool off31 = ((rows_all - 1) * std::max(std::max(ld, ld_do), std::max(ld_o, ld_dq)) + 3 * D) * 2 < (1ll << 31) &&
                     (int64_t)B * H * N * 4 < (1ll << 31);
  return H > 0 && D == 64 * H && N > 192 && N <= 224 && off31;
}

template <int DH, bool DROP>
static hipError_t attn_bwd_generic(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ld_o, const uint16_t* dout,
                                   int64_t ld_do, const float* lse, uint16_t* dqkv, int64_t ld_dq, float* dq_acc,
                                   int dq_rezero, float* dbias, float* bpart, float* ws, int B, int N, int H, int D, float scale,
                                   const pvr::AttnDrop& drop, const pvr::AttnQ8& q8, hipStream_t s) {
  using namespace pvr;
  if (bpart && (DROP || dbias || !attn_bwd_bpart_ok(N, DH))) return hipErrorInvalidValue;
  if (q8.out && !attn_bwd_final_dq_in_kernel(N, dbias != nullptr, DROP)) return hipErrorInvalidValue;
  const int NW = pvr_attn_bwd_waves(N);
  const int KB = NW * 32;
  const int nkb = (N + KB - 1) / KB;
  const bool lastkey = attn_bwd_lastkey_path(N, dbias != nullptr, DROP);
  const int rem_ = N % KB;
  const bool tail_split = !lastkey && nkb > 1 && rem_ >= 16 && rem_ <= 128 && !dbias;
  const bool slab_path = tail_split;
  // no dQ accumulator for a shape that would need one: deterministic mode (pvr_attn_bwd_needs_dq_acc),
  // per-key-block slabs in the scratch past the pre-pass outputs, summed in a fixed order
  const bool det_slab = nkb > 1 && !dq_acc && !lastkey && !slab_path;
  if (dbias && 2 * Hd<DH>::NE > 2 * NW) return hipErrorInvalidValue;  // q-bias sums: <= 2 fragments per wave
  if (!ws) return hipErrorInvalidValue;
  const int RB = 128 * Hd<DH>::NH;
  // K image | 2 x (Q | dO) blocks | dS | 2 x (lse | delta | ds_last) 1 KiB DMA slots
  auto smem_of = [&](int kb) { return (size_t)kb * RB + 4 * 32 * RB + 2 * 32 * kb * 2 + 6 * 1024; };
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)attn_bwd_kernel<DH, DROP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)smem_of(8 * 32));
    if (e != hipSuccess) return e;
    attr = true;
  }
  // pre-pass: delta (and, on the lastkey path, key N - 1's dS / dK / dV)
  float* dlt = ws;
  float* dsl = lastkey ? ws + (int64_t)B * H * N : nullptr;
  float* slab = slab_path || det_slab ? ws + 2 * (int64_t)B * H * N : nullptr;  // [N / KB + 1][B*N][D] f32 partial dQ
  if (lastkey)
    hipLaunchKernelGGL((attn_bwd_prep_kernel<DH, true>), dim3(B * H), dim3(256), 0, s, qkv, ld, dout, ld_do, out, ld_o, lse, dlt, dsl,
                       bpart, dqkv, ld_dq, N, H, D, scale, q8, g_attn_prep_xcd);
  else
    hipLaunchKernelGGL((attn_bwd_prep_kernel<DH, false>), dim3(B * H), dim3(256), 0, s, qkv, ld, dout, ld_do, out, ld_o, lse, dlt,
                       nullptr, bpart, dqkv, ld_dq, N, H, D, scale, q8, g_attn_prep_xcd);
  // bp: q-bias partials, passed only to the launch that writes the final dQ
  auto launch = [&](int nw, int k0, int k1, int dq_mode, float* dqa, int64_t sstride, int nslab, float* bp) {
    const int kb = nw * 32;
    hipLaunchKernelGGL((attn_bwd_kernel<DH, DROP>), dim3((k1 - k0 + kb - 1) / kb * B * H), dim3(nw * 64), smem_of(kb), s, qkv, ld,
                       dout, ld_do, lse, dlt, dsl, dqkv, ld_dq, dqa, dbias, bp, N, H, D, scale, k0, k1, dq_mode, sstride, nslab, drop,
                       q8);
  };
  if (lastkey) {
    // one key past a full key block: the main kernel over keys [0, N - 1) writes dQ directly (adding
    // the pre-pass's dS of key N - 1 times K[N - 1]); that key's dK / dV come from the pre-pass
    launch(NW, 0, N - 1, 0, nullptr, 0, 0, bpart);
    return hipGetLastError();
  }
  const int rem = N % KB;
  if (tail_split) {
    // N = a multiple of KB plus a short tail (ViT-L/16@384: 577 = 2 x 256 + 65): the KB-aligned body
    // in full-size workgroups, the tail in workgroups sized for it, instead of 8-wave workgroups with
    // 3 live waves holding a CU each (818 vs 862 us at B64 H16). A 1-key tail (257 = 256 + 1, the
    // CLS token of 224/14) takes the lastkey path above instead.
    // The tail launch, one workgroup per (batch, head) running after the body, ends with a final
    // dQ pass over the pair's rows: every key block's f32 slab summed there in slab order; the
    // final pass also writes the fp8 copy and the q-bias partials.
    const int nslab = (N - rem) / KB;
    const int64_t sstride = (int64_t)B * N * D;
    launch(NW, 0, N - rem, 3, slab, sstride, nslab, nullptr);
    launch(pvr_attn_bwd_waves(rem), N - rem, N, 4, slab, sstride, nslab, bpart);
    return hipGetLastError();
  }
  if (det_slab) {
    const int64_t rows = (int64_t)B * N, sstride = rows * D;
    launch(NW, 0, N, 3, slab, sstride, 0, nullptr);
    int64_t blocks = (rows * D + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(dq_slab_sum_kernel, dim3((unsigned)blocks), dim3(256), 0, s, slab, nkb, sstride, dqkv, ld_dq, rows, D);
    return hipGetLastError();
  }
  launch(NW, 0, N, 0, nkb > 1 ? dq_acc : nullptr, 0, 0, nkb > 1 ? nullptr : bpart);
  if (nkb > 1) {
    const int64_t rows = (int64_t)B * N;
    int64_t blocks = (rows * D + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(dq_convert_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dq_acc, dqkv, ld_dq, rows, D, dq_rezero);
  }
  return hipGetLastError();
}

template <int DH>
static hipError_t attn_bwd_launch(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ld_o, const uint16_t* dout,
                                  int64_t ld_do, const float* lse, uint16_t* dqkv, int64_t ld_dq, float* dq_acc,
                                  int dq_rezero, float* dbias, float* bpart, float* ws, int B, int N, int H, int D, float scale,
                                  const pvr::AttnDrop& drop, const pvr::AttnQ8& q8, hipStream_t s) {
  if (drop.seed)  // attention dropout: the generic kernel regenerates the forward's keep mask
    return attn_bwd_generic<DH, true>(qkv, ld, out, ld_o, dout, ld_do, lse, dqkv, ld_dq, dq_acc, dq_rezero, dbias, bpart, ws, B, N, H, D, scale,
                                      drop, q8, s);
  if (DH == 64 && !q8.out && attn_bwd_pipe_ok(B, N, H, D, ld, ld_do, ld_o, ld_dq))  // dbias: [B*H][NQ][192] partials
    return attn_bwd_pipe8_launch<7>(qkv, ld, out, ld_o, dout, ld_do, lse, dqkv, ld_dq, dbias, B, N, H, D, scale, s);
  return attn_bwd_generic<DH, false>(qkv, ld, out, ld_o, dout, ld_do, lse, dqkv, ld_dq, dq_acc, dq_rezero, dbias, bpart, ws, B, N, H, D, scale,
                                     drop, q8, s);
}

// floats of the f32 scratch pvr_attn_bwd needs (per-query delta and, on the lastkey path, ds_last;
// dQ slabs on the tail-split path, and in deterministic mode (det) on multi-key-block shapes without it)
extern "C" int64_t pvr_attn_bwd_ws_floats(int B, int N, int H, int D, int dbias, int drop, int det) {
  int64_t n = 2 * (int64_t)B * H * N;
  const int KB = 32 * pvr_attn_bwd_waves(N);
  if (attn_bwd_slab_path(N, dbias != 0, drop != 0))
    n += (int64_t)(N / KB + 1) * B * N * D;
  else if (det && pvr_attn_bwd_key_blocks(N) > 1 && !attn_bwd_lastkey_path(N, dbias != 0, drop != 0))
    n += (int64_t)((N + KB - 1) / KB) * B * N * D;
  return n;
}

// 1 if pvr_attn_bwd can write dQKV's e5m2 copy (q8_out) for this shape: the generic kernels must
// write every final dQ value
extern "C" int pvr_attn_bwd_q8_ok(int N, int drop) { return attn_bwd_final_dq_in_kernel(N, false, drop != 0) ? 1 : 0; }

// 1 if pvr_attn_bwd takes the pipelined whole-head backward for this shape and these layouts; its
// dbias is then f32 [B*H][ceil(N/32)][192] partials instead: per (batch, head, 32-query block) the
// column sums of dQ over its two 16-query halves (2 x 64, the head's q-bias slice; summed) and of dO
// (64: the v-bias slice, sum_k dV = sum_q dO since softmax rows sum to 1); the k-bias gradient is
// exactly 0 (sum_k dS = 0 per query)
extern "C" int pvr_attn_bwd_uses_pipe(int B, int N, int H, int D, int64_t ld, int64_t ld_do, int64_t ld_o, int64_t ld_dq, int drop) {
  return !drop && attn_bwd_pipe_ok(B, N, H, D, ld, ld_do, ld_o, ld_dq) ? 1 : 0;
}

// Rows R of the f32 [B*H][R][3*dh] bias-gradient partials (q half 0 | q half 1 | v) that pvr_attn_bwd
// writes for this shape: pipelined kernel (into `dbias`): R = 32-query blocks; generic kernel (into
// `bpart`): R = 1 where attn_bwd_bpart_ok; 0: none (`dbias` then means the generic kernel's
// [B * key blocks][3D] layout).
extern "C" int pvr_attn_bwd_part_rows(int B, int N, int H, int D, int64_t ld, int64_t ld_do, int64_t ld_o, int64_t ld_dq, int drop) {
  if (pvr_attn_bwd_uses_pipe(B, N, H, D, ld, ld_do, ld_o, ld_dq, drop)) return (N + 31) / 32;
  return !drop && H > 0 && D % H == 0 && pvr_attn_head_dim_supported(D / H) && attn_bwd_bpart_ok(N, D / H) ? 1 : 0;
}

// dq_acc: f32 [B*N][D] zero-initialised workspace, required iff N > 256 (several key blocks per head);
// dq_rezero = 1 leaves it zeroed again afterwards (a persistent workspace reused across calls).
// dbias: optional f32 [B * nkb][3D] partial column sums of dQ | dK | dV (nkb = pvr_attn_bwd_key_blocks;
// every element is written), whose row sum is the in_proj bias gradient; on the pipelined path
// (pvr_attn_bwd_uses_pipe) the per-block partials described there.
// ws: f32 scratch of pvr_attn_bwd_ws_floats(B, N, H) floats (the generic path's pre-pass outputs).
extern "C" hipError_t pvr_attn_bwd(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ld_o, const uint16_t* dout,
                                   int64_t ld_do, const float* lse, uint16_t* dqkv, int64_t ld_dq, float* dq_acc,
                                   int dq_rezero, float* dbias, float* bpart, float* ws, int B, int N, int H, int D, float scale,
                                   const uint64_t* seed, uint64_t seed_off, uint32_t thr16, float keep_scale, uint8_t* q8_out,
                                   int64_t q8_ld, const float* q8_qs, unsigned* q8_amax, int q8_only, int q8_fmt, hipStream_t s) {
  if (H <= 0 || D % H != 0 || B <= 0 || N <= 0 || N > 65536) return hipErrorInvalidValue;
  if (q8_fmt != 0 && q8_fmt != 1) return hipErrorInvalidValue;
  if (q8_out && (!q8_qs || !q8_amax || q8_ld % 4 != 0 || (uintptr_t)q8_out % 4 != 0)) return hipErrorInvalidValue;
  const pvr::AttnDrop drop{seed, seed_off, thr16, keep_scale};
  if (q8_only && !q8_out) return hipErrorInvalidValue;
  const pvr::AttnQ8 q8{q8_out, q8_ld, q8_qs, q8_amax, q8_only, q8_fmt};
  switch (D / H) {
#define PVR_BWD_DH(DH) \
  case DH:             \
    return attn_bwd_launch<DH>(qkv, ld, out, ld_o, dout, ld_do, lse, dqkv, ld_dq, dq_acc, dq_rezero, dbias, bpart, ws, B, N, H, D, scale, \
                               drop, q8, s);
    PVR_BWD_DH(64) PVR_BWD_DH(80) PVR_BWD_DH(96) PVR_BWD_DH(128)
#undef PVR_BWD_DH
    default: return hipErrorInvalidValue;
  }
}
