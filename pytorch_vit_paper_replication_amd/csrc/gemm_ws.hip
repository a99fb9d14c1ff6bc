// Wave-specialized persistent GEMM for gfx950: the fused epilogue runs on its own waves, beside the
// matrix cores, instead of after each tile's MFMAs.
//
//   C[m][n] = epilogue( sum_k A[m][k] * B[n][k] )      A, B k-contiguous bf16; fp32 accumulation
//
// Why: the 256x256 ping-pong kernels (gemm.hip) finish every tile with an epilogue that the same
// waves run while the matrix cores idle - the fc1 GELU + dropout + derivative epilogue is ~22k of a
// ~70k-cycle tile, the dGELU one ~21k, and their stores then drain under the next tile's K loop
// (profiles/r5/README.md). Here one 1024-thread workgroup per CU has two roles:
//
//   * 8 MFMA waves (two per SIMD, ping-ponging a barrier apart as in gemm.hip) compute 256 x 128
//     output tiles (each wave 64 x 64: 4 x 4 v_mfma_f32_16x16x32_bf16 fragments) from a 6-slot ring
//     of 32-deep K-steps that LDS-DMA (buffer_load ... lds) fills 4 steps ahead, continuously across
//     the workgroup's tiles. Their accumulators start at the bias; at a tile end they store the tile
//     as bf16 u = A.B^T + bias (64 KiB, register order) to a per-workgroup scratch slot in L2 and go
//     straight on with the next tile.
//   * 8 epilogue waves (two per SIMD) turn tile t - 2's u into the outputs while the MFMA waves run
//     tile t: GELU + dropout + GELU-derivative (fc1 forward), x dGELU-factor + column sums (fc2
//     dgrad), or dropout + residual. Their VALU work and HBM stores overlap the matrix-core work on
//     the same SIMDs (an MFMA blocks its SIMD's vector issue for 8 of its 16 cycles).
//
// Both roles execute the same s_barrier sequence (every barrier counts all 16 waves): the epilogue
// waves spread a tile's work over the barrier intervals of the MFMA waves' next-next tile, so the
// protocol needs no flags. Register budget: 4 waves per SIMD, <= 128 VGPRs each (__launch_bounds__).
// LDS: 6 K-step slots x 24 KiB + bias staging + column-sum exchange.
//
// Numerics: u is rounded to bf16 before the elementwise epilogue, as PyTorch's autocast Linear
// output is (reference models/vit.py:118-126 under autocast); the epilogue math is gemm.hip's.
// Reference: /root/reference/models/vit.py:118-126 (MLP block), :166-169; SURVEY.md K9, K10, K11.
#include "common.h"
#include "gemm_params.h"

namespace pvr {
namespace {

constexpr int EPI_BF16_ = 0, EPI_GELU_ = 1, EPI_DGELU_ = 2;  // = GemmEpi of gemm.hip

constexpr int WS_BM = 256, WS_BN = 128;       // output tile (rows of A x rows of B)
constexpr int WS_A = WS_BM * 64;              // A image of one K-step: [256 rows][32 k] bf16 = 16 KiB
constexpr int WS_B = WS_BN * 64;              // B image: 8 KiB
constexpr int WS_SLOT = WS_A + WS_B;          // 24 KiB
constexpr int WS_NSLOT = 6;                   // K-step ring
constexpr int WS_AHEAD = 4;                   // K-steps of LDS-DMA in flight ahead of the reads
constexpr int WS_DMA = 3;                     // DMA instructions per MFMA wave per K-step
constexpr int WS_VM = (WS_AHEAD - 1) * WS_DMA;  // vmcnt that retires the next K-step
constexpr int WS_USTORES = 8;                 // u stores per MFMA wave at a tile end
constexpr int WS_BIAS_OFF = WS_NSLOT * WS_SLOT;           // 2 x 128 fp32 bias staging slots
constexpr int WS_CS_OFF = WS_BIAS_OFF + 2 * WS_BN * 4;    // column-sum exchange [8 waves][64] fp32
constexpr int WS_LDS = WS_CS_OFF + 8 * 64 * 4;
constexpr int WS_U_BYTES = WS_BM * WS_BN * 2;  // one scratch slot (bf16 u of a tile)
constexpr int WS_SC1 = 16;                    // buffer cache policy sc1: L2-served (no stale L1 line)

PVR_DEV int ws_swz(int row) { return (row >> 1) & 3; }  // 64-B rows: conflict-free ds_read_b128

PVR_DEV void ws_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS-DMA of one 32-deep K-step of a tile into `slot`: image rows of 64 B (4 chunks of 16 B, the
// chunk index XOR-swizzled by the row on the SOURCE side). A: 16 wave-instructions of 16 rows,
// B: 8; MFMA wave w issues A rows 16w.., 16(w+8).. and B rows 16w.. The per-lane offsets (row and
// chunk, range-checked) are fixed per wave (WsDma); the K-step's byte offset kb rides in the SGPR
// offset, which stays inside the row.
struct WsDma {
  uint32_t a0, a1, b;
};
PVR_DEV WsDma ws_dma_offsets(int64_t lda, int64_t ldb, int w, int lane) {
  WsDma d;
  int row = w * 16 + (lane >> 2);
  d.a0 = (uint32_t)(row * lda * 2 + (((lane & 3) ^ ((row >> 1) & 3)) * 16));
  d.b = (uint32_t)(row * ldb * 2 + (((lane & 3) ^ ((row >> 1) & 3)) * 16));
  row += 128;
  d.a1 = (uint32_t)(row * lda * 2 + (((lane & 3) ^ ((row >> 1) & 3)) * 16));
  return d;
}
PVR_DEV void ws_issue(__amdgpu_buffer_rsrc_t ars, __amdgpu_buffer_rsrc_t brs, char* slot, const WsDma& d, int kb, int w) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, to_lds(slot + w * 1024), 16, d.a0, kb, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, to_lds(slot + (w + 8) * 1024), 16, d.a1, kb, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, to_lds(slot + WS_A + w * 1024), 16, d.b, kb, 0, 0);
}

// 16 rows x 32 k MFMA operand fragment: lane l holds X[r0 + (l & 15)][8 (l >> 4) .. + 7]
PVR_DEV v8s ws_frag(const char* img, int r0, int lane) {
  const int row = r0 + (lane & 15);
  return ds_read_b128(img + row * 64 + (((lane >> 4) ^ ws_swz(row)) << 4));
}

struct WsTile {
  int m0, n0;
  __amdgpu_buffer_rsrc_t ars, brs;
};

PVR_DEV int ws_ntn(const GemmParams& p) { return (p.N + WS_BN - 1) / WS_BN; }
PVR_DEV int ws_ntiles(const GemmParams& p) { return ((p.M + WS_BM - 1) / WS_BM) * ws_ntn(p); }

PVR_DEV uint32_t ws_bytes(int64_t extent, int64_t base) {
  int64_t b = (extent - base) * 2;
  if (b < 0) b = 0;
  if (b > 0xFFFFFFFFll) b = 0xFFFFFFFFll;
  return (uint32_t)b;
}

PVR_DEV void ws_coords(const GemmParams& p, int v, int& m0, int& n0) {
  const int t = xcd_remap(v, ws_ntiles(p));
  m0 = (t / ws_ntn(p)) * WS_BM;
  n0 = (t % ws_ntn(p)) * WS_BN;
}

PVR_DEV WsTile ws_tile(const GemmParams& p, int v) {
  WsTile t;
  if (v >= ws_ntiles(p)) {  // past the workgroup's last tile: every DMA reads as out of range
    t.m0 = t.n0 = 0;
    t.ars = make_rsrc(p.A, 0);
    t.brs = make_rsrc(p.B, 0);
    return t;
  }
  ws_coords(p, v, t.m0, t.n0);
  t.ars = make_rsrc(p.A + (int64_t)t.m0 * p.lda, ws_bytes((int64_t)(p.M - 1) * p.lda + p.K, (int64_t)t.m0 * p.lda));
  t.brs = make_rsrc(p.B + (int64_t)t.n0 * p.ldb, ws_bytes((int64_t)(p.N - 1) * p.ldb + p.K, (int64_t)t.n0 * p.ldb));
  return t;
}

// One K-step of an MFMA wave (a barrier apart from its SIMD partner): read this step's fragments,
// issue the DMA of step G + WS_AHEAD (this tile's or the next one's), retire step G + 1, MFMAs.
// infl: the first K-steps after a tile end, whose counted wait leaves the WS_USTORES u stores (younger
// than the DMAs it retires) in flight.
PVR_DEV void ws_step(v4f (&acc)[4][4], char* smem, int G, int G0, int nk, const WsTile& cur, const WsTile& nxt,
                     const WsDma& d, bool infl, int w, int lane, int wm, int wn) {
  const char* slot = smem + (G % WS_NSLOT) * WS_SLOT;
  v8s a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = ws_frag(slot, wm * 64 + 16 * i, lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = ws_frag(slot + WS_A, wn * 64 + 16 * j, lane);
  {
    const int Gi = G + WS_AHEAD, rel = Gi - G0;
    const bool same = rel < nk;
    ws_issue(same ? cur.ars : nxt.ars, same ? cur.brs : nxt.brs, smem + (Gi % WS_NSLOT) * WS_SLOT, d,
             (same ? rel : rel - nk) * 64, w);
  }
  if (infl)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WS_VM + WS_USTORES) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WS_VM) : "memory");
  ws_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(b[j], a[i], acc[i][j]);  // lane: C[16i + li][16j + 4g + r]
  __builtin_amdgcn_s_setprio(0);
  ws_barrier();
}

// ---------------------------------------------------------------- epilogue waves
// Epilogue wave e processes MFMA wave e's 64 x 64 block of a tile: fragment rows i = 0..3, column
// pairs jp = 0..1. Its u words come from the scratch in the MFMA lane order; one v_permlane16_swap
// per word pair gives every lane 8 contiguous columns c0 = nb + 32 jp + {0, 16, 8, 24}[g] of row
// mb + 16 i + li (the register-direct layout of gemm.hip's epilogue_direct), so every load / store
// below is 16 B per lane.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct WsEpi {
  int mb, nb, e;                       // block origin, epilogue wave
  uint32_t vc[2], vx[2];               // per-jp lane offsets in C and in the resid / aux tensor
  __amdgpu_buffer_rsrc_t crs, xrs, srs;  // C, resid (BF16) or aux (GELU store / DGELU load), scratch
  int ldx;
  bool has_in;
  v4u pu[2], px[2];                    // u / per-row input of units s and s + 1 (ring of 2, by unit & 1)
  float cs[2][8];                      // column sums (DGELU)
};

// unit s = (fragment row s >> 1, column pair s & 1): its u words (scratch, MFMA lane order) and input
template <int S>
PVR_DEV void ws_epi_load(WsEpi& E, int lane) {
  constexpr int I = S >> 1, JP = S & 1;
  E.pu[S & 1] = __builtin_amdgcn_raw_buffer_load_b128(E.srs, (uint32_t)(E.e * 8192 + (I * 2 + JP) * 1024 + lane * 16), 0, WS_SC1);
  if (E.has_in) E.px[S & 1] = __builtin_amdgcn_raw_buffer_load_b128(E.xrs, E.vx[JP] + (uint32_t)(I * 16 * E.ldx * 2), 0, 0);
}

template <int EPI>
PVR_DEV void ws_epi_begin(const GemmParams& p, WsEpi& E, int m0, int n0, const char* scratch, int e, int lane) {
  const int wm = e >> 1, wn = e & 1, li = lane & 15, g = lane >> 4;
  E.e = e;
  E.mb = m0 + wm * 64;
  E.nb = n0 + wn * 64;
  const int rows = max(0, min(64, p.M - E.mb));
  const uint32_t OOB = 0x80000000u;
  E.crs = make_rsrc((const uint16_t*)p.C + (int64_t)E.mb * p.ldc, rows ? (uint32_t)(((int64_t)(rows - 1) * p.ldc + p.N) * 2) : 0);
  E.xrs = E.crs;
  E.ldx = (int)p.ldc;
  E.has_in = EPI == EPI_DGELU_;
  if constexpr (EPI == EPI_BF16_) {
    if (p.resid) {
      E.xrs = make_rsrc(p.resid + (int64_t)E.mb * p.ld_resid, rows ? (uint32_t)(((int64_t)(rows - 1) * p.ld_resid + p.N) * 2) : 0);
      E.ldx = (int)p.ld_resid;
      E.has_in = true;
    }
  } else {
    const bool has = p.aux != nullptr;
    E.xrs = make_rsrc(has ? p.aux + (int64_t)E.mb * p.ld_aux : p.aux, has && rows ? (uint32_t)(((int64_t)(rows - 1) * p.ld_aux + p.N) * 2) : 0);
    E.ldx = (int)p.ld_aux;
  }
  E.srs = make_rsrc(scratch, WS_U_BYTES);
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    const int c0 = E.nb + 32 * jp + ((g & 1) << 4) + ((g & 2) << 2);
    const bool okc = c0 < p.N;
    E.vc[jp] = okc ? (uint32_t)((li * (int)p.ldc + c0) * 2) : OOB;
    E.vx[jp] = okc ? (uint32_t)((li * E.ldx + c0) * 2) : OOB;
#pragma unroll
    for (int k = 0; k < 8; ++k) E.cs[jp][k] = 0.f;
  }
  ws_epi_load<0>(E, lane);
  ws_epi_load<1>(E, lane);
}

PVR_DEV float bfw_lo(uint32_t w) { return __uint_as_float(w << 16); }
PVR_DEV float bfw_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }

// Unit S: 8 elements per lane. Consumes ring slot S & 1, then refills it with unit S + 2.
template <int EPI, int S>
PVR_DEV void ws_epi_unit(const GemmParams& p, WsEpi& E, uint32_t key, uint64_t seed, bool idx32, int lane) {
  constexpr int I = S >> 1, JP = S & 1;
  const int li = lane & 15, g = lane >> 4;
  const int m = E.mb + 16 * I + li;
  const int c0 = E.nb + 32 * JP + ((g & 1) << 4) + ((g & 2) << 2);
  const uint32_t so_c = (uint32_t)(I * 16 * (int)p.ldc * 2), so_x = (uint32_t)(I * 16 * E.ldx * 2);
  // words 0, 1: columns 16 (2 JP) + 4g .. +3 of the pair's first fragment, 2, 3: of the second
  const v4u uu = E.pu[S & 1], xin = E.px[S & 1];
  if constexpr (S + 2 < 8) ws_epi_load<S + 2>(E, lane);
  uint32_t q[4] = {uu[0], uu[1], uu[2], uu[3]};
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(q[0]), "+v"(q[2]));
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(q[1]), "+v"(q[3]));
  float v[8] = {bfw_lo(q[0]), bfw_hi(q[0]), bfw_lo(q[1]), bfw_hi(q[1]), bfw_lo(q[2]), bfw_hi(q[2]), bfw_lo(q[3]), bfw_hi(q[3])};
  bool keep[8] = {true, true, true, true, true, true, true, true};
  if constexpr (EPI == EPI_BF16_ || EPI == EPI_GELU_) {
    if (p.drop_thr) {
      const uint64_t idx = (uint64_t)m * p.N + c0;
      if (idx32) {
        bool k0[4], k1[4];
        rng_keep4_32(key, (uint32_t)idx, p.drop_thr, k0);
        rng_keep4_32(key, (uint32_t)idx + 4, p.drop_thr, k1);
#pragma unroll
        for (int k = 0; k < 4; ++k) { keep[k] = k0[k]; keep[4 + k] = k1[k]; }
      } else {
#pragma unroll
        for (int k = 0; k < 8; k += 2) rng_keep2(seed, idx + k, p.drop_thr, keep[k], keep[k + 1]);
      }
    }
  }
  v4u out;
  if constexpr (EPI == EPI_BF16_) {
    if (p.drop_thr) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = keep[k] ? v[k] * p.drop_scale : 0.f;
    }
    if (E.has_in) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] += bfw_lo(xin[k]);
        v[2 * k + 1] += bfw_hi(xin[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = pack2bf(v[2 * k], v[2 * k + 1]);
  } else if constexpr (EPI == EPI_GELU_) {
    v4u ax;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const v2f s2 = {keep[2 * k] ? p.drop_scale : 0.f, keep[2 * k + 1] ? p.drop_scale : 0.f};
      v2f g2, d2;
      gelu_and_grad2((v2f){v[2 * k], v[2 * k + 1]}, g2, d2);
      g2 *= s2;
      d2 *= s2;
      ax[k] = pack2bf(d2.x, d2.y);
      out[k] = pack2bf(g2.x, g2.y);
    }
    __builtin_amdgcn_raw_buffer_store_b128(ax, E.xrs, E.vx[JP] + so_x, 0, 0);  // no aux (inference): 0-byte resource
  } else {  // EPI_DGELU
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] *= bfw_lo(xin[k]);
      v[2 * k + 1] *= bfw_hi(xin[k]);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) E.cs[JP][k] += v[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = pack2bf(v[2 * k], v[2 * k + 1]);
  }
  __builtin_amdgcn_raw_buffer_store_b128(out, E.crs, E.vc[JP] + so_c, 0, 0);
}

template <int EPI>
PVR_DEV void ws_epi_stage(const GemmParams& p, WsEpi& E, int s, uint32_t key, uint64_t seed, bool idx32, int lane) {
  switch (s) {
    case 0: ws_epi_unit<EPI, 0>(p, E, key, seed, idx32, lane); break;
    case 1: ws_epi_unit<EPI, 1>(p, E, key, seed, idx32, lane); break;
    case 2: ws_epi_unit<EPI, 2>(p, E, key, seed, idx32, lane); break;
    case 3: ws_epi_unit<EPI, 3>(p, E, key, seed, idx32, lane); break;
    case 4: ws_epi_unit<EPI, 4>(p, E, key, seed, idx32, lane); break;
    case 5: ws_epi_unit<EPI, 5>(p, E, key, seed, idx32, lane); break;
    case 6: ws_epi_unit<EPI, 6>(p, E, key, seed, idx32, lane); break;
    default: ws_epi_unit<EPI, 7>(p, E, key, seed, idx32, lane); break;
  }
}

// DGELU column sums, part 1: each wave's 64 column sums (over its 64 rows) into the LDS exchange
PVR_DEV void ws_cs_put(WsEpi& E, char* smem, int e, int lane) {
  const int li = lane & 15, g = lane >> 4;
  float* red = (float*)(smem + WS_CS_OFF) + e * 64;
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float c = row16_sum(E.cs[jp][k]);
      if (li == 0) red[32 * jp + ((g & 1) << 4) + ((g & 2) << 2) + k] = c;
    }
}
// part 2 (after a barrier): the wm = 0 waves add the four partials of their 64 columns, one atomic
// per column
PVR_DEV void ws_cs_add(const GemmParams& p, const WsEpi& E, const char* smem, int e, int lane) {
  if ((e >> 1) != 0 || !p.colsum) return;
  const float* red = (const float*)(smem + WS_CS_OFF);
  const int wn = e & 1, c = E.nb + lane;
  const float s = red[(0 + wn) * 64 + lane] + red[(2 + wn) * 64 + lane] + red[(4 + wn) * 64 + lane] + red[(6 + wn) * 64 + lane];
  if (c < p.N) atomicAdd(p.colsum + c, s);
}

template <int EPI>
__global__ void __launch_bounds__(1024, 1) gemm_ws_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = ws_ntiles(p);
  const int nk = p.K / 32;                   // K-steps per tile (K % 64 == 0, K >= 256: host check)
  const int nbar = 2 * nk + 1;               // barriers per tile, both roles
  char* scratch = (char*)p.tail_ws + (int64_t)blockIdx.x * 2 * WS_U_BYTES;
  if ((int)blockIdx.x >= ntiles) return;
  constexpr bool HAS_BIAS = EPI != EPI_DGELU_;

  if (w < 8) {
    // ============================================================ MFMA waves
    const int grp = w >> 2, wm = w >> 1, wn = w & 1;
    const int g = lane >> 4;
    int v = blockIdx.x;
    WsTile cur = ws_tile(p, v);
    WsTile nxt = ws_tile(p, v + gridDim.x);
    const WsDma dma = ws_dma_offsets(p.lda, p.ldb, w, lane);
#pragma unroll
    for (int s = 0; s < WS_AHEAD; ++s) ws_issue(cur.ars, cur.brs, smem + s * WS_SLOT, dma, s * 64, w);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WS_VM) : "memory");  // K-step 0 landed
    ws_barrier();                                                  // P0 (the epilogue waves staged tile 0's bias)
    int G0 = 0, k = 0;
    for (;;) {
      v4f acc[4][4];
      if (HAS_BIAS && p.bias) {  // accumulators start at the bias (staged in LDS by the epilogue waves)
        const float* bs = (const float*)(smem + WS_BIAS_OFF + (k & 1) * WS_BN * 4) + wn * 64 + 4 * g;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const v4f b4 = *(const __attribute__((address_space(3))) v4f*)(bs + 16 * j);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = b4;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
      }
      if (grp == 1) ws_barrier();  // group 1 runs one barrier behind
      // first K-steps after a tile end: the u stores are younger than the DMAs these steps wait for;
      // step 3's plain wait retires them
      for (int ks = 0; ks < nk; ++ks) ws_step(acc, smem, G0 + ks, G0, nk, cur, nxt, dma, G0 > 0 && ks < 3, w, lane, wm, wn);
      if (grp == 0) ws_barrier();  // re-align the groups
      // u = bf16(acc) to scratch slot k & 1 in register order: 8 x 16 B per lane (fragments j, j + 1)
      {
        typedef uint32_t v4u_ __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t srs = make_rsrc(scratch + (k & 1) * WS_U_BYTES, WS_U_BYTES);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jp = 0; jp < 2; ++jp) {
            const v4f a0 = acc[i][2 * jp], a1 = acc[i][2 * jp + 1];
            const v4u_ o = {pack2bf(a0[0], a0[1]), pack2bf(a0[2], a0[3]), pack2bf(a1[0], a1[1]), pack2bf(a1[2], a1[3])};
            __builtin_amdgcn_raw_buffer_store_b128(o, srs, (uint32_t)(w * 8192 + (i * 2 + jp) * 1024 + lane * 16), 0, 0);
          }
      }
      v += gridDim.x;
      ++k;
      if (v >= ntiles) break;
      G0 += nk;
      cur = nxt;
      nxt = ws_tile(p, v + gridDim.x);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // u stores retired; no LDS-DMA outlives the workgroup
    ws_barrier();                                      // F: the epilogue waves may read the last tiles
    return;
  }

  // ============================================================== epilogue waves
  const int e = w - 8;
  const uint64_t seed = (p.drop_thr ? *p.seed_ptr : 0ull) + p.seed_offset;
  const uint32_t key = p.drop_thr ? rng_key(seed) : 0u;
  const bool idx32 = (uint64_t)p.M * (uint64_t)p.N + 8 <= 0xFFFFFFFFull;
  const int tid = threadIdx.x - 512;
  auto stage_bias = [&](int vt, int kslot) {  // bias of tile vt -> LDS slot kslot & 1 (before the MFMA waves read it)
    if (!HAS_BIAS || !p.bias || vt >= ntiles) return;
    int m0, n0;
    ws_coords(p, vt, m0, n0);
    if (tid < WS_BN) {
      const int n = n0 + tid;
      ((float*)(smem + WS_BIAS_OFF + (kslot & 1) * WS_BN * 4))[tid] = n < p.N ? p.bias[n] : 0.f;
    }
  };
  stage_bias(blockIdx.x, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ws_barrier();  // P0
  WsEpi E;
  // stage s of the block runs after barrier interval at(s) of the MFMA waves' tile: spread over the
  // tile's 2 nk + 1 intervals, loads at interval 0
  auto at = [&](int s) { return 1 + (s * (nbar - 4)) / 8; };
  int k = 0;
  for (int v = blockIdx.x; v < ntiles; v += gridDim.x, ++k) {
    // MFMA tile k is running; process tile k - 2 (its u stores retired during tile k - 1)
    const bool work = k >= 2;
    int s = 0;
    for (int b = 0; b < nbar; ++b) {
      if (b == 0) {
        stage_bias(v + gridDim.x, k + 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (work) {
          int m0, n0;
          ws_coords(p, v - 2 * gridDim.x, m0, n0);
          ws_epi_begin<EPI>(p, E, m0, n0, scratch + (k & 1) * WS_U_BYTES, e, lane);
        }
      }
      if (work) {
        while (s < 8 && b >= at(s)) ws_epi_stage<EPI>(p, E, s++, key, seed, idx32, lane);
        if constexpr (EPI == EPI_DGELU_) {
          if (b == nbar - 2) {
            ws_cs_put(E, smem, e, lane);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          if (b == nbar - 1) ws_cs_add(p, E, smem, e, lane);
        }
      }
      ws_barrier();
    }
  }
  ws_barrier();  // F: every u store of the MFMA waves retired; they have exited
  // the last one or two tiles: no barriers needed beside the (exited) MFMA waves, except the
  // column-sum exchange between the epilogue waves themselves
  const int ktot = k;
  for (int kk = max(0, ktot - 2); kk < ktot; ++kk) {
    int m0, n0;
    ws_coords(p, blockIdx.x + kk * gridDim.x, m0, n0);
    ws_epi_begin<EPI>(p, E, m0, n0, scratch + (kk & 1) * WS_U_BYTES, e, lane);
    for (int s = 0; s < 8; ++s) ws_epi_stage<EPI>(p, E, s, key, seed, idx32, lane);
    if constexpr (EPI == EPI_DGELU_) {
      ws_cs_put(E, smem, e, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ws_barrier();
      ws_cs_add(p, E, smem, e, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ws_barrier();
    }
  }
}

template <int EPI>
hipError_t launch_ws(const GemmParams& p, hipStream_t s, int cus) {
  auto kern = gemm_ws_kernel<EPI>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, WS_LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int ntiles = ((p.M + WS_BM - 1) / WS_BM) * ((p.N + WS_BN - 1) / WS_BN);
  const int grid = ntiles < cus ? ntiles : cus;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), WS_LDS, s, p);
  return hipGetLastError();
}

}  // namespace
}  // namespace pvr

// 1 if the wave-specialized kernel takes this GEMM (k-contiguous bf16 operands, bf16-output
// epilogue without row remap / addend / fp8 copy, K a multiple of 64 and >= 256, the per-stream
// scratch present and large enough)
extern "C" int pvr_gemm_ws_ok(const pvr::GemmParams* pp, int cus) {
  const pvr::GemmParams& p = *pp;
  if (p.elem8 || !p.a_kcontig || !p.b_kcontig || p.epi > 2 || p.addend || p.row_group || p.c_skip || p.q_out) return 0;
  if (p.K % 64 || p.K < 256 || p.k_split_len < p.K || (p.N & 7) || p.M <= 0) return 0;
  if (!p.tail_ws || p.tail_ws_elems * 4 < (int64_t)cus * 2 * pvr::WS_U_BYTES) return 0;
  const int64_t l1 = p.ldc > p.ld_resid ? p.ldc : p.ld_resid;
  const int64_t ld = l1 > p.ld_aux ? l1 : p.ld_aux;
  if ((int64_t)p.M * ld * 2 >= (1ll << 31) || 256ll * p.lda * 2 >= (1ll << 31) || 128ll * p.ldb * 2 >= (1ll << 31)) return 0;
  return 1;
}

extern "C" hipError_t pvr_gemm_ws(const pvr::GemmParams* pp, int cus, hipStream_t s) {
  using namespace pvr;
  const GemmParams& p = *pp;
  if (!pvr_gemm_ws_ok(pp, cus)) return hipErrorInvalidValue;
  switch (p.epi) {
    case EPI_BF16_: return launch_ws<EPI_BF16_>(p, s, cus);
    case EPI_GELU_: return launch_ws<EPI_GELU_>(p, s, cus);
    case EPI_DGELU_: return launch_ws<EPI_DGELU_>(p, s, cus);
  }
  return hipErrorInvalidValue;
}
