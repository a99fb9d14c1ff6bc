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
//     the workgroup's tiles. At a tile end they hand the accumulators to the epilogue waves through
//     LDS (the two ring slots just consumed + a 16 KiB spare region = 64 KiB) and go on with the next
//     tile. They issue no global store: their vmcnt waits count LDS-DMA only.
//   * 8 epilogue waves (two per SIMD) hold the handed-off tile in registers and turn it into the
//     outputs while the MFMA waves run the next tile: bias + GELU + dropout + GELU-derivative (fc1
//     forward), x dGELU-factor + bias-gradient column sums (fc2 dgrad), bias + dropout + residual.
//     Their VALU work and HBM traffic overlap the matrix-core work on the same SIMDs (an MFMA blocks
//     its SIMD's vector issue for 8 of its 16 cycles).
//
// Both roles execute the same s_barrier sequence (every barrier counts all 16 waves): the epilogue
// waves spread a tile's 8 work units over the barrier intervals of the next tile, so the protocol
// needs no flags. Register budget: 4 waves per SIMD, <= 128 VGPRs each (__launch_bounds__).
// An earlier form of this kernel handed u over through an L2 scratch buffer: its stores sat in the
// MFMA waves' in-order vmcnt queue and every CU's burst at the tile end stalled their next K-steps
// (+35 % on the qkv forward; profiles/r6/README.md).
//
// Numerics: the bf16 hand-off rounds A.B^T to bf16 before the bias and the elementwise epilogue, as
// PyTorch's autocast Linear output is (reference models/vit.py:118-126 under autocast); the dGELU
// hand-off stays fp32 (two rounds), so the bias-gradient column sums keep the fp32 accumulator.
// Reference: /root/reference/models/vit.py:118-126 (MLP block), :166-169; SURVEY.md K9, K10, K11.
#include "common.h"
#include "gemm_params.h"
#include <type_traits>

namespace pvr {
namespace {

constexpr int EPI_BF16_ = 0, EPI_GELU_ = 1, EPI_DGELU_ = 2;  // = GemmEpi of gemm.hip

// 1: the MFMA waves raise their priority over their MFMA bursts (A/B knob)
#ifndef PVR_WS_PRIO
#define PVR_WS_PRIO 1
#endif
// diagnostic ablations (timing only, wrong results): 1 = the epilogue waves only keep the barrier
// count, 3 = and no hand-off (the compiler then deletes the MFMAs too: DMA + barriers only), 4 = the
// full epilogue math without its stores, 5 = the stores without the math
#ifndef PVR_WS_ABL
#define PVR_WS_ABL 0
#endif
constexpr bool WS_EPI_ON = PVR_WS_ABL == 0 || PVR_WS_ABL >= 4;

constexpr int WS_BM = 256, WS_BN = 128;       // output tile (rows of A x rows of B)
constexpr int WS_A = WS_BM * 64;              // A image of one K-step: [256 rows][32 k] bf16 = 16 KiB
constexpr int WS_B = WS_BN * 64;              // B image: 8 KiB
constexpr int WS_SLOT = WS_A + WS_B;          // 24 KiB
constexpr int WS_NSLOT = 6;                   // K-step ring
constexpr int WS_AHEAD = 4;                   // K-steps of LDS-DMA in flight ahead of the reads
constexpr int WS_DMA = 3;                     // DMA instructions per MFMA wave per K-step
constexpr int WS_VM = (WS_AHEAD - 1) * WS_DMA;  // vmcnt that retires the next K-step
constexpr int WS_SPARE = WS_NSLOT * WS_SLOT;  // 16 KiB: hand-off chunks 6, 7; column-sum exchange between hand-offs
constexpr int WS_LDS = WS_SPARE + 16384;      // 160 KiB
// hand-off: bf16 (one round, 8 KiB per MFMA wave) or fp32 for the dGELU epilogue (two rounds, one
// wave group at a time, 16 KiB per wave)
template <int EPI> constexpr bool ws_f32u() { return EPI == 2; }

PVR_DEV int ws_swz(int row) { return (row >> 1) & 3; }  // 64-B rows: conflict-free ds_read_b128

template <int I, int N, class F>
PVR_DEV void ws_static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    ws_static_for<I + 1, N>(f);
  }
}

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
// issue the DMA of step G + WS_AHEAD (this tile's or the next one's), retire step G + 1 (the MFMA
// waves issue no other vector-memory operation, so the count is exact), MFMAs.
PVR_DEV void ws_step(v4f (&acc)[4][4], char* smem, int G, int G0, int nk, const WsTile& cur, const WsTile& nxt,
                     const WsDma& d, int w, int lane, int wm, int wn) {
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
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WS_VM) : "memory");
  ws_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (PVR_WS_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(b[j], a[i], acc[i][j]);  // lane: C[16i + li][16j + 4g + r]
  if (PVR_WS_PRIO) __builtin_amdgcn_s_setprio(0);
  ws_barrier();
}

// ---------------------------------------------------------------- hand-off and epilogue waves
// The 64 KiB hand-off area of the tile ending at K-step G0 - 1: 8 chunks of 8 KiB, chunks 0-2 in the
// ring slot of K-step G0 - 2, 3-5 in that of G0 - 1 (both consumed: their next DMAs, of steps G0 + 4
// and G0 + 5, are issued after the hand-off), 6-7 in the spare region.
PVR_DEV char* ws_chunk(char* smem, int G0, int c) {
  const int sa = (G0 + WS_NSLOT - 2) % WS_NSLOT, sb = (G0 + WS_NSLOT - 1) % WS_NSLOT;
  return c < 3 ? smem + sa * WS_SLOT + c * 8192 : c < 6 ? smem + sb * WS_SLOT + (c - 3) * 8192 : smem + WS_SPARE + (c - 6) * 8192;
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// A handed-off 64 x 64 block in register order: bf16: word group (2i + jp) = fragments (i, 2 jp),
// (i, 2 jp + 1) packed (NU = 8); fp32: group (4i + j) = fragment (i, j) (NU = 16).
template <int NU>
struct WsBlock {
  v4u q[NU];
};

// MFMA wave side: write the accumulators (register order, 16 B per lane and instruction)
template <bool F32>
PVR_DEV void ws_put(const v4f (&acc)[4][4], char* smem, int G0, int q, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const v4f a0 = acc[i][2 * jp], a1 = acc[i][2 * jp + 1];
      if constexpr (F32) {  // 16 KiB per wave: chunks 2q, 2q + 1
        const int o0 = (i * 4 + 2 * jp) * 1024, o1 = o0 + 1024;
        *(__attribute__((address_space(3))) v4f*)(ws_chunk(smem, G0, 2 * q + (o0 >> 13)) + (o0 & 8191) + lane * 16) = a0;
        *(__attribute__((address_space(3))) v4f*)(ws_chunk(smem, G0, 2 * q + (o1 >> 13)) + (o1 & 8191) + lane * 16) = a1;
      } else {  // 8 KiB per wave: chunk q
        const v4u o = {pack2bf(a0[0], a0[1]), pack2bf(a0[2], a0[3]), pack2bf(a1[0], a1[1]), pack2bf(a1[2], a1[3])};
        *(__attribute__((address_space(3))) v4u*)(ws_chunk(smem, G0, q) + (i * 2 + jp) * 1024 + lane * 16) = o;
      }
    }
}

// epilogue wave side: the same words back, into registers
template <bool F32, int NU>
PVR_DEV void ws_get(WsBlock<NU>& B, char* smem, int G0, int q, int lane) {
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int o = u * 1024;
    const char* base = F32 ? ws_chunk(smem, G0, 2 * q + (o >> 13)) + (o & 8191) : ws_chunk(smem, G0, q) + o;
    B.q[u] = *(const __attribute__((address_space(3))) v4u*)(base + lane * 16);
  }
}

struct WsEpi {
  int mb, nb;                             // block origin (rows, columns)
  uint32_t vc0, vc1, vx0, vx1;            // per-jp lane offsets in C and in the resid / aux tensor
  __amdgpu_buffer_rsrc_t crs, xrs;        // C, resid (BF16) or aux (GELU store / DGELU load)
  int ldc2, ldx2;                         // row strides in bytes
  bool has_in;
  v4u x[2];                               // per-row inputs of the next even / odd unit (two units ahead)
  float bias[2][8];                       // this lane's 8 + 8 bias columns (BF16 / GELU)
  float* red;                             // DGELU: this wave's 64 column sums in the exchange area (LDS)
  uint32_t ow[4], aw[4];                  // the unit's packed outputs (and GELU aux) until its last pair
};

template <int S>
PVR_DEV void ws_epi_load_x(WsEpi& E) {
  constexpr int I = S >> 1, JP = S & 1;
  if (E.has_in) E.x[S & 1] = __builtin_amdgcn_raw_buffer_load_b128(E.xrs, (JP ? E.vx1 : E.vx0) + (uint32_t)(I * 16 * E.ldx2), 0, 0);
}

template <int EPI>
PVR_DEV void ws_epi_begin(const GemmParams& p, WsEpi& E, int m0, int n0, int e, int lane) {
  const int wm = e >> 1, wn = e & 1, li = lane & 15, g = lane >> 4;
  E.mb = m0 + wm * 64;
  E.nb = n0 + wn * 64;
  const int rows = max(0, min(64, p.M - E.mb));
  const uint32_t OOB = 0x80000000u;
  E.crs = make_rsrc((const uint16_t*)p.C + (int64_t)E.mb * p.ldc, rows ? (uint32_t)(((int64_t)(rows - 1) * p.ldc + p.N) * 2) : 0);
  E.xrs = E.crs;
  int ldx = (int)p.ldc;
  E.has_in = EPI == EPI_DGELU_;
  if constexpr (EPI == EPI_BF16_) {
    if (p.resid) {
      E.xrs = make_rsrc(p.resid + (int64_t)E.mb * p.ld_resid, rows ? (uint32_t)(((int64_t)(rows - 1) * p.ld_resid + p.N) * 2) : 0);
      ldx = (int)p.ld_resid;
      E.has_in = true;
    }
  } else {
    const bool has = p.aux != nullptr;
    E.xrs = make_rsrc(has ? p.aux + (int64_t)E.mb * p.ld_aux : p.aux, has && rows ? (uint32_t)(((int64_t)(rows - 1) * p.ld_aux + p.N) * 2) : 0);
    ldx = (int)p.ld_aux;
  }
  E.ldc2 = (int)p.ldc * 2;
  E.ldx2 = ldx * 2;
  const int cb = E.nb + ((g & 1) << 4) + ((g & 2) << 2);  // this lane's first column (jp = 0)
  E.vc0 = cb < p.N ? (uint32_t)((li * (int)p.ldc + cb) * 2) : OOB;
  E.vx0 = cb < p.N ? (uint32_t)((li * ldx + cb) * 2) : OOB;
  E.vc1 = cb + 32 < p.N ? (uint32_t)((li * (int)p.ldc + cb + 32) * 2) : OOB;
  E.vx1 = cb + 32 < p.N ? (uint32_t)((li * ldx + cb + 32) * 2) : OOB;
#pragma unroll
  for (int k = 0; k < 8; ++k) E.bias[0][k] = E.bias[1][k] = 0.f;
  if constexpr (EPI != EPI_DGELU_) {
    if (p.bias) {
      const __amdgpu_buffer_rsrc_t brs = make_rsrc(p.bias, (uint32_t)p.N * 4);
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const uint32_t vb = cb + 32 * jp < p.N ? (uint32_t)((cb + 32 * jp) * 4) : OOB;
        const v4f b0 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(brs, vb, 0, 0));
        const v4f b1 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(brs, vb + 16, 0, 0));
#pragma unroll
        for (int k = 0; k < 4; ++k) { E.bias[jp][k] = b0[k]; E.bias[jp][4 + k] = b1[k]; }
      }
    }
  }
  ws_epi_load_x<0>(E);
  ws_epi_load_x<1>(E);
}

PVR_DEV float bfw_lo(uint32_t w) { return __uint_as_float(w << 16); }
PVR_DEV float bfw_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }

// Unit S = (fragment row I = S >> 1, column half JP = S & 1): 8 elements per lane, columns c0 .. c0 + 7,
// in 4 pairs P (columns c0 + 2P, +1) run in the order 0, 2, 1, 3 (one permlane swap serves two pairs).
// A unit is split into pieces of 1, 2 or 4 pairs, one piece per K-loop barrier interval: a whole
// unit (~160 VALU incl. 16 transcendentals per wave) is several MFMA intervals of issue time and
// would hold the MFMA waves at the next barrier. The results collect in E.ow / E.aw and the last pair
// stores them (16 B per lane). Dropout: one 32-bit hash per pair (the rng_keep4_32 bits; host check
// M * N < 2^32).
template <int EPI, int S, int P, int NU>
PVR_DEV void ws_epi_pair(const GemmParams& p, WsEpi& E, WsBlock<NU>& B, uint32_t key, int lane) {
  constexpr int I = S >> 1, JP = S & 1;
  const int li = lane & 15, g = lane >> 4;
  float v0, v1;
  if constexpr (NU == 16) {  // fp32 words: a = group 4I + 2JP, b = a + 1; swap r pairs (0, 1) / (2, 3)
    constexpr int ga = I * 4 + 2 * JP, r0 = (P & 1) * 2;
    if constexpr (P < 2) {
#pragma unroll
      for (int r = r0; r < r0 + 2; ++r) {
        uint32_t x = B.q[ga][r], y = B.q[ga + 1][r];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
        B.q[ga][r] = x;
        B.q[ga + 1][r] = y;
      }
    }
    constexpr int src = P < 2 ? ga : ga + 1;
    v0 = __uint_as_float(B.q[src][r0]);
    v1 = __uint_as_float(B.q[src][r0 + 1]);
  } else {  // bf16 words 0, 1: the pair's first fragment, 2, 3: its second; swaps (0, 2), (1, 3)
    constexpr int gw = I * 2 + JP;
    if constexpr (P < 2) {
      uint32_t x = B.q[gw][P], y = B.q[gw][P + 2];
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
      B.q[gw][P] = x;
      B.q[gw][P + 2] = y;
    }
    v0 = bfw_lo(B.q[gw][P]);
    v1 = bfw_hi(B.q[gw][P]);
  }
  const uint32_t xw = E.x[S & 1][P];
  if constexpr (EPI != EPI_DGELU_) {
    v0 += E.bias[JP][2 * P];
    v1 += E.bias[JP][2 * P + 1];
  }
  bool k0 = true, k1 = true;
  if constexpr (EPI == EPI_BF16_ || EPI == EPI_GELU_) {
    if (p.drop_thr) {
      const int m = E.mb + 16 * I + li;
      const int c = E.nb + 32 * JP + ((g & 1) << 4) + ((g & 2) << 2) + 2 * P;
      const uint32_t h = rng_mix32((((uint32_t)m * (uint32_t)p.N + (uint32_t)c) >> 1) ^ key);
      k0 = (h & 0xFFFFu) >= p.drop_thr;
      k1 = (h >> 16) >= p.drop_thr;
    }
  }
  if constexpr (PVR_WS_ABL == 5) {  // ablation: no epilogue math, the raw words stored
    E.ow[P] = __float_as_uint(v0) ^ __float_as_uint(v1);
    E.aw[P] = E.ow[P];
  } else if constexpr (EPI == EPI_BF16_) {
    if (p.drop_thr) {
      v0 = k0 ? v0 * p.drop_scale : 0.f;
      v1 = k1 ? v1 * p.drop_scale : 0.f;
    }
    if (E.has_in) {
      v0 += bfw_lo(xw);
      v1 += bfw_hi(xw);
    }
    E.ow[P] = pack2bf(v0, v1);
  } else if constexpr (EPI == EPI_GELU_) {
    const v2f s2 = {k0 ? p.drop_scale : 0.f, k1 ? p.drop_scale : 0.f};
    v2f g2, d2;
    gelu_and_grad2((v2f){v0, v1}, g2, d2);
    g2 *= s2;
    d2 *= s2;
    E.aw[P] = pack2bf(d2.x, d2.y);
    E.ow[P] = pack2bf(g2.x, g2.y);
  } else {  // EPI_DGELU: bias-gradient column sums over the unit's 16 rows by DPP, one LDS add per column
    v0 *= bfw_lo(xw);
    v1 *= bfw_hi(xw);
    const float c0s = row16_sum(v0), c1s = row16_sum(v1);
    float* r = E.red + 32 * JP + ((g & 1) << 4) + ((g & 2) << 2) + 2 * P;
    if (li == 0) {
      atomicAdd(r, c0s);
      atomicAdd(r + 1, c1s);
    }
    E.ow[P] = pack2bf(v0, v1);
  }
  // pin the pair's results here: without it the compiler sinks the arithmetic across the barriers
  // to the unit's store, re-forming one interval-sized lump
  asm volatile("" : "+v"(E.ow[P]));
  if constexpr (EPI == EPI_GELU_) asm volatile("" : "+v"(E.aw[P]));
  if (PVR_WS_ABL == 4 && p.M > 0) return;  // ablation: all the math, no stores (runtime-opaque skip)
  if constexpr (P == 3) {
    const uint32_t vc = (JP ? E.vc1 : E.vc0) + (uint32_t)(I * 16 * E.ldc2);
    if constexpr (EPI == EPI_GELU_) {  // no aux (inference): 0-byte resource
      const uint32_t vx = (JP ? E.vx1 : E.vx0) + (uint32_t)(I * 16 * E.ldx2);
      __builtin_amdgcn_raw_buffer_store_b128((v4u){E.aw[0], E.aw[1], E.aw[2], E.aw[3]}, E.xrs, vx, 0, 0);
    }
    __builtin_amdgcn_raw_buffer_store_b128((v4u){E.ow[0], E.ow[1], E.ow[2], E.ow[3]}, E.crs, vc, 0, 0);
    if constexpr (S + 2 < 8) ws_epi_load_x<S + 2>(E);  // the ring slot of unit S is free now
  }
}

// piece H of NQ of unit S: pairs 4H / NQ .. 4(H + 1) / NQ - 1 of the order 0, 2, 1, 3
template <int EPI, int S, int H, int NQ, int NU>
PVR_DEV void ws_epi_piece(const GemmParams& p, WsEpi& E, WsBlock<NU>& B, uint32_t key, int lane) {
  constexpr int PER = 4 / NQ;
  ws_static_for<0, PER>([&](auto pc) {
    constexpr int k = H * PER + decltype(pc)::value;
    ws_epi_pair<EPI, S, (k == 0 ? 0 : k == 1 ? 2 : k == 2 ? 1 : 3), NU>(p, E, B, key, lane);
  });
}

// DGELU column sums, part 1: zero this wave's exchange row (the spare region, free between
// hand-offs); the units add into it
PVR_DEV void ws_cs_zero(WsEpi& E, char* smem, int e, int lane) {
  E.red = (float*)(smem + WS_SPARE) + e * 64;
  E.red[lane] = 0.f;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
// part 2 (after a barrier): the wm = 0 waves add the four partials of their 64 columns, one atomic
// per column
PVR_DEV void ws_cs_add(const GemmParams& p, const WsEpi& E, const char* smem, int e, int lane) {
  if ((e >> 1) != 0 || !p.colsum) return;
  const float* red = (const float*)(smem + WS_SPARE);
  const int wn = e & 1, c = E.nb + lane;
  const float s = red[(0 + wn) * 64 + lane] + red[(2 + wn) * 64 + lane] + red[(4 + wn) * 64 + lane] + red[(6 + wn) * 64 + lane];
  if (c < p.N) atomicAdd(p.colsum + c, s);
}


template <int EPI, int NQ, int SPC>
__global__ void __launch_bounds__(1024, 1) gemm_ws_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntiles = ws_ntiles(p);
  const int nk = p.K / 32;                   // K-steps per tile (K % 64 == 0, K >= 256: host check)
  const int nbar = 2 * nk + 1;               // barriers of a tile's K loop, both roles
  constexpr bool F32 = ws_f32u<EPI>();
  constexpr int R = F32 ? 2 : 1;             // hand-off rounds
  constexpr int NU = F32 ? 16 : 8;
  if ((int)blockIdx.x >= ntiles) return;

  if (w < 8) {
    // ============================================================ MFMA waves
    const int grp = w >> 2, wm = w >> 1, wn = w & 1;
    int v = blockIdx.x;
    WsTile cur = ws_tile(p, v);
    WsTile nxt = ws_tile(p, v + gridDim.x);
    const WsDma dma = ws_dma_offsets(p.lda, p.ldb, w, lane);
#pragma unroll
    for (int s = 0; s < WS_AHEAD; ++s) ws_issue(cur.ars, cur.brs, smem + s * WS_SLOT, dma, s * 64, w);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WS_VM) : "memory");  // K-step 0 landed
    ws_barrier();                                                  // P0
    int G0 = 0;
    for (;;) {
      v4f acc[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
      if (grp == 1) ws_barrier();  // group 1 runs one barrier behind
      for (int ks = 0; ks < nk; ++ks) ws_step(acc, smem, G0 + ks, G0, nk, cur, nxt, dma, w, lane, wm, wn);
      if (grp == 0) ws_barrier();  // re-align the groups
      G0 += nk;
      // hand-off: round r writes, the epilogue waves read, both barrier-fenced
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (PVR_WS_ABL != 3 && (R == 1 || grp == r)) ws_put<F32>(acc, smem, G0, R == 1 ? w : w & 3, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        ws_barrier();  // H1
        ws_barrier();  // H2: the epilogue waves hold it
      }
      v += gridDim.x;
      if (v >= ntiles) break;
      cur = nxt;
      nxt = ws_tile(p, v + gridDim.x);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup (null steps)
    return;
  }

  // ============================================================== epilogue waves
  const int e = w - 8;
  const uint32_t key = p.drop_thr ? rng_key(*p.seed_ptr + p.seed_offset) : 0u;
  ws_barrier();  // P0
  WsBlock<NU> B;
  bool have = false;  // B holds a tile (handed off at the end of the previous MFMA tile)
  int vprev = 0;
  int G0 = 0;
  for (int v = blockIdx.x; v < ntiles; v += gridDim.x) {
    // the MFMA waves run tile v; process tile vprev (if any) over the K loop's barrier intervals:
    // interval 0 loads its bias and first per-row inputs, piece x runs after barrier SPC (x + 1)
    if (have && WS_EPI_ON) {
      WsEpi E;
      int m0, n0;
      ws_coords(p, vprev, m0, n0);
      ws_epi_begin<EPI>(p, E, m0, n0, e, lane);
      if constexpr (EPI == EPI_DGELU_) ws_cs_zero(E, smem, e, lane);
      ws_barrier();
      ws_static_for<0, 8 * NQ>([&](auto sc) {
        constexpr int X = decltype(sc)::value;
#pragma unroll
        for (int t = 1; t < SPC; ++t) ws_barrier();
        ws_epi_piece<EPI, X / NQ, X % NQ, NQ, NU>(p, E, B, key, lane);
        ws_barrier();
      });
      int rest = nbar - 1 - 8 * NQ * SPC;
      if constexpr (EPI == EPI_DGELU_) {  // the exchange area (spare region) is free until the hand-off
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        ws_barrier();
        ws_cs_add(p, E, smem, e, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        rest -= 1;
      }
      for (; rest > 0; --rest) ws_barrier();
    } else {
      for (int b = 0; b < nbar; ++b) ws_barrier();
    }
    G0 += nk;
    // hand-off of tile v
#pragma unroll
    for (int r = 0; r < R; ++r) {
      ws_barrier();  // H1
      if (WS_EPI_ON && (R == 1 || (e >> 2) == r)) ws_get<F32, NU>(B, smem, G0, R == 1 ? e : e & 3, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ws_barrier();  // H2
    }
    have = true;
    vprev = v;
  }
  // the last tile, after the MFMA waves have exited: no barriers needed beside them, except the
  // column-sum exchange between the epilogue waves themselves
  if (have && WS_EPI_ON) {
    WsEpi E;
    int m0, n0;
    ws_coords(p, vprev, m0, n0);
    ws_epi_begin<EPI>(p, E, m0, n0, e, lane);
    if constexpr (EPI == EPI_DGELU_) ws_cs_zero(E, smem, e, lane);
    ws_static_for<0, 8>([&](auto sc) {
      constexpr int S = decltype(sc)::value;
      ws_epi_piece<EPI, S, 0, 1, NU>(p, E, B, key, lane);
    });
    if constexpr (EPI == EPI_DGELU_) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ws_barrier();
      ws_cs_add(p, E, smem, e, lane);
    }
  }
}

template <int EPI, int NQ, int SPC>
hipError_t launch_ws_spc(const GemmParams& p, hipStream_t s, int grid) {
  auto kern = gemm_ws_kernel<EPI, NQ, SPC>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, WS_LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), WS_LDS, s, p);
  return hipGetLastError();
}

// the epilogue waves' pieces: one pair per piece (NQ = 4) spaced SPC barriers apart, the widest
// spacing that fits the K loop's 2 nk + 1 barriers (32 pieces + interval 0 + 2 for the column-sum
// exchange); short K loops take 2- or 4-pair pieces
template <int EPI>
hipError_t launch_ws(const GemmParams& p, hipStream_t s, int cus) {
  const int ntiles = ((p.M + WS_BM - 1) / WS_BM) * ((p.N + WS_BN - 1) / WS_BN);
  const int grid = ntiles < cus ? ntiles : cus;
  const int nbar = 2 * (p.K / 32) + 1;
  if (3 + 32 * 4 <= nbar) return launch_ws_spc<EPI, 4, 4>(p, s, grid);
  if (3 + 32 * 2 <= nbar) return launch_ws_spc<EPI, 4, 2>(p, s, grid);
  if (3 + 32 <= nbar) return launch_ws_spc<EPI, 4, 1>(p, s, grid);
  if (3 + 16 <= nbar) return launch_ws_spc<EPI, 2, 1>(p, s, grid);
  return launch_ws_spc<EPI, 1, 1>(p, s, grid);
}

}  // namespace
}  // namespace pvr

// 1 if the wave-specialized kernel takes this GEMM (k-contiguous bf16 operands, bf16-output
// epilogue without row remap / addend / fp8 copy, K a multiple of 64 and >= 256, 32-bit element
// indices, 31-bit buffer offsets)
extern "C" int pvr_gemm_ws_ok(const pvr::GemmParams* pp, int cus) {
  (void)cus;
  const pvr::GemmParams& p = *pp;
  if (p.elem8 || !p.a_kcontig || !p.b_kcontig || p.epi > 2 || p.addend || p.row_group || p.c_skip || p.q_out) return 0;
  if (p.K % 64 || p.K < 256 || p.k_split_len < p.K || (p.N & 7) || p.M <= 0) return 0;
  const int64_t l1 = p.ldc > p.ld_resid ? p.ldc : p.ld_resid;
  const int64_t ld = l1 > p.ld_aux ? l1 : p.ld_aux;
  if ((int64_t)p.M * ld * 2 >= (1ll << 31) || 256ll * p.lda * 2 >= (1ll << 31) || 128ll * p.ldb * 2 >= (1ll << 31)) return 0;
  if ((uint64_t)p.M * (uint64_t)p.N + 8 > 0xFFFFFFFFull) return 0;  // 32-bit dropout element index
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
