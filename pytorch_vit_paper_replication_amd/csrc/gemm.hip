// MFMA bf16 GEMM for gfx950 with fused ViT epilogues.
//
//   C[m][n] = sum_k A[m][k] * B[n][k]        (fp32 accumulation, v_mfma_f32_16x16x32_bf16)
//
// Each operand is either "k-contiguous" (row-major [rows][k], e.g. activations and nn.Linear
// weights) or "mn-contiguous" (stored [k][rows], e.g. the token-major tensors reduced over in the
// weight-gradient GEMM). This single template therefore covers the three GEMMs of a Linear layer:
//   forward  Y  = X  . W^T   (A=X k-contig,   B=W k-contig)
//   dgrad    dX = dY . W     (A=dY k-contig,  B=W mn-contig)
//   wgrad    dW = dY^T . X   (A=dY mn-contig, B=X mn-contig, split over tokens, f32 atomics)
// which replaces the reference's nn.Linear / F.multi_head_attention_forward in_proj/out_proj GEMMs
// (reference models/vit.py:86-90, :118-126).
//
// Staging: tiles go HBM/L2 -> LDS by LDS-DMA (buffer_load ... lds, 16 B per lane), with the
// buffer's range check zero-filling every row past the operand's end (M/N tails, token tails).
// LDS images are lane-linear per wave-instruction; bank conflicts are removed by XOR-swizzling the
// per-lane SOURCE address and applying the same XOR on the read (ds_read_b128 for k-contig,
// ds_read_b64_tr_b16 hardware transpose for mn-contig). Two LDS stages: the DMA for tile t+1 is in
// flight while the MFMAs of tile t run.
#include "common.h"
#include "gemm_params.h"
#include <type_traits>

namespace pvr {

enum GemmEpi : int {
  EPI_BF16 = 0,        // out = resid + dropout(acc + bias + addend[row])      (bf16)
  EPI_GELU = 1,        // u = acc + bias; out = dropout(gelu(u)); aux = mask * scale * gelu'(u)
  EPI_DGELU = 2,       // out = acc * aux   (aux as saved by EPI_GELU)            (bf16)
  EPI_F32_ATOMIC = 3,  // out += acc                                             (f32 atomics)
  EPI_F32_STORE = 4,   // out = acc                                              (f32)
};



namespace {

PVR_DEV void stamp(const GemmParams& p, int slot) {
#ifdef PVR_GEMM_PHASE_STAMPS
  return;  // p.dbg holds the per-wave phase sums instead (PpStamps)
#endif
  if (p.dbg && threadIdx.x == 0) {
    const int b = blockIdx.x + gridDim.x * blockIdx.z;
    p.dbg[(int64_t)b * 8 + slot] = __builtin_amdgcn_s_memtime();
  }
}

constexpr int TK = 64;  // K depth of one LDS stage

// Ping-pong K loops: read the next K-tile's A0 first-k-step fragments in the read-free (1,0) phase
// (A/B switch while it is measured; 0 = the round-5 phase reads 12 / 4 / 8 / 0)
#ifndef PVR_PP_PRE
#define PVR_PP_PRE 1
#endif

PVR_DEV int swz_k(int row) { return (row >> 1) & 7; }                                // 128-B rows
PVR_DEV int swz_mn(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }  // 16-B chunk XOR
// 16-B chunk XOR of the fp8 mn images' 128-B k-rows: the 16 rows a 32-lane half reads with
// ds_read_b64_tr_b8 (rows 8q' + q of its two 16-lane groups, 32 apart) land on 64 distinct banks
PVR_DEV int swz8(int row) { return ((row >> 1) & 3) | (((row >> 5) & 1) << 2); }

// Issue the LDS-DMA of one operand tile (R rows of the operand x 64 k) into `lds`.
template <int R, bool KC, int NW>
PVR_DEV void stage_tile(__amdgpu_buffer_rsrc_t rs, char* lds, int64_t ld, int k0, int wave, int lane) {
  if constexpr (KC) {
    // image [R][8 chunks of 16 B]; one wave-instruction = 8 rows
    constexpr int NI = R / 8;
#pragma unroll
    for (int i = 0; i < NI / NW; ++i) {
      const int s = wave + NW * i;
      const int row = s * 8 + (lane >> 3);
      const int c = (lane & 7) ^ swz_k(row);
      const uint32_t voff = (uint32_t)(row * ld * 2 + (int64_t)(k0 + c * 8) * 2);
      dma16(rs, to_lds(lds + s * 1024), voff);
    }
  } else {
    // image [64 k-rows][R/8 chunks]; one wave-instruction = 64/(R/8) rows
    constexpr int CPR = R / 8, RPI = 64 / CPR, NI = TK / RPI;
#pragma unroll
    for (int i = 0; i < NI / NW; ++i) {
      const int s = wave + NW * i;
      const int row = s * RPI + lane / CPR;
      const int pc = lane % CPR;
      const int c = (pc & ~15) | ((pc & 15) ^ swz_mn(row));
      const uint32_t voff = (uint32_t)((int64_t)(k0 + row) * ld * 2 + c * 16);
      dma16(rs, to_lds(lds + s * 1024), voff);
    }
  }
}

// Read one 16(rows) x 32(k) MFMA operand fragment: lane holds X[r0 + (l&15)][ks*32 + 8(l>>4) + j].
template <int R, bool KC>
PVR_DEV v8s read_frag(const char* lds, int r0, int ks, int lane) {
  if constexpr (KC) {
    const int row = r0 + (lane & 15);
    const int c = ks * 4 + (lane >> 4);
    return ds_read_b128(lds + row * 128 + ((c ^ swz_k(row)) << 4));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int c = (r0 >> 3) + (p >> 1);
    const int kr0 = ks * 32 + 8 * g + q;
    const int kr1 = kr0 + 4;
    const int pc0 = (c & ~15) | ((c & 15) ^ swz_mn(kr0));
    const int pc1 = (c & ~15) | ((c & 15) ^ swz_mn(kr1));
    v4s lo = ds_read_tr(lds + kr0 * (R * 2) + pc0 * 16 + 8 * (p & 1));
    v4s hi = ds_read_tr(lds + kr1 * (R * 2) + pc1 * 16 + 8 * (p & 1));
    return cat44(lo, hi);
  }
}

// read_frag<R, false> as two ds_read_tr_async halves (no compiler-inserted drain of in-flight
// LDS-DMA); the caller combines them with cat44 after lds_wait()
template <int R>
PVR_DEV void read_frag_mn_async(const char* lds, int r0, int ks, int lane, v4s& lo, v4s& hi) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int c = (r0 >> 3) + (p >> 1);
  const int kr0 = ks * 32 + 8 * g + q;
  const int kr1 = kr0 + 4;
  const int pc0 = (c & ~15) | ((c & 15) ^ swz_mn(kr0));
  const int pc1 = (c & ~15) | ((c & 15) ^ swz_mn(kr1));
  lo = ds_read_tr_async(lds + kr0 * (R * 2) + pc0 * 16 + 8 * (p & 1));
  hi = ds_read_tr_async(lds + kr1 * (R * 2) + pc1 * 16 + 8 * (p & 1));
}

PVR_DEV uint32_t rsrc_bytes(int64_t extent_elems, int64_t base_elems) {
  int64_t b = (extent_elems - base_elems) * 2;
  if (b < 0) b = 0;
  if (b > 0xFFFFFFFFll) b = 0xFFFFFFFFll;
  return (uint32_t)b;
}

// Shared epilogue: acc[i][j] is the 16x16 fragment at rows mb + 16i, cols nb + 16j.
// SWAP layout (bf16 / fp32-store outputs): bias is loaded once, and the per-row inputs (residual,
// GELU pre-activation, position addend) of fragment row i+1 are issued BEFORE the stores of row i:
// vmcnt counts stores too, so a load issued after a store would wait for that store's completion.
template <int FN, int EPI>
struct RowIn {
  uint2 r[FN];   // residual (EPI_BF16) or aux pre-activation (EPI_DGELU), 4 bf16
  float4 a[FN];  // addend (EPI_BF16)
};

template <int FN, int EPI>
PVR_DEV void load_row(const GemmParams& p, int m, int64_t orow, int nb, int g, RowIn<FN, EPI>& in) {
  if (m >= p.M) return;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = nb + 16 * j + 4 * g;
    if (n >= p.N) continue;
    if constexpr (EPI == EPI_BF16) {
      if (p.resid) in.r[j] = *(const uint2*)(p.resid + (int64_t)m * p.ld_resid + n);
      if (p.addend) in.a[j] = *(const float4*)(p.addend + (orow % p.addend_period) * p.N + n);
    } else if constexpr (EPI == EPI_DGELU) {
      in.r[j] = *(const uint2*)(p.aux + (int64_t)m * p.ld_aux + n);
    }
  }
}

PVR_DEV int64_t out_row(const GemmParams& p, int m) {
  return p.row_group ? (int64_t)(m / p.row_group) * p.row_stride_group + p.row_offset + m % p.row_group : (int64_t)m;
}

template <int FM, int FN, bool SWAP, int EPI>
PVR_DEV void epilogue(const GemmParams& p, v4f (&acc)[FM][FN], int mb, int nb, int lane) {
  const int g = lane >> 4, li = lane & 15;
  if constexpr (SWAP) {
    // lane holds C[m = mb + 16i + li][n = nb + 16j + 4g + r], r = 0..3 (4 consecutive columns)
    const uint64_t seed = (p.drop_thr ? *p.seed_ptr : 0ull) + p.seed_offset;
    const float deq = p.scale_a ? (*p.scale_a) * (*p.scale_b) : 1.f;
    float4 bias[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bias[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
        const int n = nb + 16 * j + 4 * g;
        if (p.bias && n < p.N) bias[j] = *(const float4*)(p.bias + n);
      }
    }
    float csum[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j) csum[j][0] = csum[j][1] = csum[j][2] = csum[j][3] = 0.f;
    RowIn<FN, EPI> cur, nxt;
    load_row<FN, EPI>(p, mb + li, out_row(p, mb + li), nb, g, cur);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = mb + 16 * i + li;
      const int64_t orow = out_row(p, m);
      if (i + 1 < FM) load_row<FN, EPI>(p, m + 16, out_row(p, m + 16), nb, g, nxt);
      if (m < p.M) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = nb + 16 * j + 4 * g;
          if (n >= p.N) continue;
          float v[4] = {acc[i][j][0] * deq, acc[i][j][1] * deq, acc[i][j][2] * deq, acc[i][j][3] * deq};
          bool keep[4] = {true, true, true, true};
          if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
            if (p.drop_thr) {
              const uint64_t idx = (uint64_t)orow * p.N + n;
              rng_keep2(seed, idx, p.drop_thr, keep[0], keep[1]);
              rng_keep2(seed, idx + 2, p.drop_thr, keep[2], keep[3]);
            }
          }
          if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
            v[0] += bias[j].x; v[1] += bias[j].y; v[2] += bias[j].z; v[3] += bias[j].w;
          }
          if constexpr (EPI == EPI_BF16) {
            if (p.addend) {
              v[0] += cur.a[j].x; v[1] += cur.a[j].y; v[2] += cur.a[j].z; v[3] += cur.a[j].w;
            }
            if (p.drop_thr) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = keep[r] ? v[r] * p.drop_scale : 0.f;
            }
            if (p.resid) {
              const uint2 rr = cur.r[j];
              v[0] += bf2f(rr.x & 0xFFFF); v[1] += bf2f(rr.x >> 16);
              v[2] += bf2f(rr.y & 0xFFFF); v[3] += bf2f(rr.y >> 16);
            }
            uint2 o; o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
            *(uint2*)((uint16_t*)p.C + orow * p.ldc + n) = o;
          } else if constexpr (EPI == EPI_GELU) {
            // h = dropout(gelu(u)); aux = dropout-mask * scale * gelu'(u): the backward's whole
            // elementwise chain, computed while erf(u) is at hand (one exp more, no recompute later).
            float gp[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float gv, gd;
              gelu_and_grad(v[r], gv, gd);
              const float sc = keep[r] ? p.drop_scale : 0.f;
              v[r] = gv * sc;
              gp[r] = gd * sc;
            }
            if (p.aux) {  // no aux: inference (nothing to save for a backward)
              uint2 a; a.x = pack2bf(gp[0], gp[1]); a.y = pack2bf(gp[2], gp[3]);
              *(uint2*)(p.aux + (int64_t)m * p.ld_aux + n) = a;
            }
            uint2 o; o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
            *(uint2*)((uint16_t*)p.C + orow * p.ldc + n) = o;
          } else if constexpr (EPI == EPI_DGELU) {
            const uint2 gg = cur.r[j];  // mask * scale * gelu'(u) saved by the forward epilogue
            v[0] *= bf2f(gg.x & 0xFFFF); v[1] *= bf2f(gg.x >> 16);
            v[2] *= bf2f(gg.y & 0xFFFF); v[3] *= bf2f(gg.y >> 16);
            csum[j][0] += v[0]; csum[j][1] += v[1]; csum[j][2] += v[2]; csum[j][3] += v[3];
            uint2 o; o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
            *(uint2*)((uint16_t*)p.C + orow * p.ldc + n) = o;
          } else if constexpr (EPI == EPI_F32_STORE) {
            *(float4*)((float*)p.C + orow * p.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) atomicAdd((float*)p.C + orow * p.ldc + n + r, v[r]);
          }
        }
      }
      cur = nxt;
    }
    if constexpr (EPI == EPI_DGELU) {
      if (p.colsum) {
        // reduce over the 16 rows held by lanes li = 0..15 of each 16-lane group, one atomic per column
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float c = csum[j][r];
            c += __shfl_xor(c, 1, 64);
            c += __shfl_xor(c, 2, 64);
            c += __shfl_xor(c, 4, 64);
            c += __shfl_xor(c, 8, 64);
            csum[j][r] = c;
          }
        if (li == 0) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int n = nb + 16 * j + 4 * g;
            if (n < p.N)
#pragma unroll
              for (int r = 0; r < 4; ++r) atomicAdd(p.colsum + n + r, csum[j][r]);
          }
        }
      }
    }
  } else {
    // lane holds C[m = mb + 16i + 4g + r][n = nb + 16j + li]; f32 outputs (64-B row segments per instruction)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = nb + 16 * j + li;
        if (n >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mb + 16 * i + 4 * g + r;
          if (m >= p.M) continue;
          float* dst = (float*)p.C + (int64_t)m * p.ldc + n;
          if constexpr (EPI == EPI_F32_ATOMIC)
            atomicAdd(dst, acc[i][j][r]);
          else
            *dst = acc[i][j][r];
        }
      }
  }
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, bool SWAP, int EPI>
__global__ void __launch_bounds__(WM* WN * 64) gemm_kernel(GemmParams p) {
  constexpr int NW = WM * WN;
  constexpr int A_BYTES = BM * TK * 2, B_BYTES = BN * TK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;

  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int nb = ntm * ntn;
  const int t = xcd_remap(blockIdx.x, nb);
  const int tm = t / ntn, tn = t % ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kbeg = blockIdx.z * p.k_split_len;
  const int kend = min(p.K, kbeg + p.k_split_len);
  const int nk = (kend - kbeg + TK - 1) / TK;

  // Buffer resources start at this block's tile; every byte past the operand's logical extent reads 0.
  const uint16_t* abase;
  uint32_t abytes;
  if constexpr (AK) {
    abase = p.A + (int64_t)m0 * p.lda + kbeg;
    abytes = rsrc_bytes((int64_t)(p.M - 1) * p.lda + p.K, (int64_t)m0 * p.lda + kbeg);
  } else {
    abase = p.A + (int64_t)kbeg * p.lda + m0;
    abytes = rsrc_bytes((int64_t)(p.K - 1) * p.lda + p.M, (int64_t)kbeg * p.lda + m0);
  }
  const uint16_t* bbase;
  uint32_t bbytes;
  if constexpr (BKC) {
    bbase = p.B + (int64_t)n0 * p.ldb + kbeg;
    bbytes = rsrc_bytes((int64_t)(p.N - 1) * p.ldb + p.K, (int64_t)n0 * p.ldb + kbeg);
  } else {
    bbase = p.B + (int64_t)kbeg * p.ldb + n0;
    bbytes = rsrc_bytes((int64_t)(p.K - 1) * p.ldb + p.N, (int64_t)kbeg * p.ldb + n0);
  }
  const __amdgpu_buffer_rsrc_t ars = make_rsrc(abase, abytes);
  const __amdgpu_buffer_rsrc_t brs = make_rsrc(bbase, bbytes);

  v4f acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  stamp(p, 0);
  if (nk > 0) {
    stage_tile<BM, AK, NW>(ars, smem, p.lda, 0, wave, lane);
    stage_tile<BN, BKC, NW>(brs, smem + A_BYTES, p.ldb, 0, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  stamp(p, 1);
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * STAGE;
      stage_tile<BM, AK, NW>(ars, nxt, p.lda, (kt + 1) * TK, wave, lane);
      stage_tile<BN, BKC, NW>(brs, nxt + A_BYTES, p.ldb, (kt + 1) * TK, wave, lane);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8s af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = read_frag<BM, AK>(cur, wm * WTM + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = read_frag<BN, BKC>(cur + A_BYTES, wn * WTN + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (SWAP)
            acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
          else
            acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  stamp(p, 2);
  epilogue<FM, FN, SWAP, EPI>(p, acc, m0 + wm * WTM, n0 + wn * WTN, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp(p, 3);
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, bool SWAP, int EPI>
hipError_t launch_cfg(const GemmParams& p, hipStream_t s) {
  constexpr int SMEM = 2 * (BM + BN) * TK * 2;
  auto kern = gemm_kernel<BM, BN, WM, WN, AK, BKC, SWAP, EPI>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int nsplit = (p.K + p.k_split_len - 1) / p.k_split_len;
  dim3 grid(ntm * ntn, 1, nsplit);
  hipLaunchKernelGGL(kern, grid, dim3(WM * WN * 64), SMEM, s, p);
  return hipGetLastError();
}

// ===================================================================================== BK = 32 staging
// (the 4-stage ring of the v3 kernel below)
constexpr int BK32 = 32;
// LDS-DMA wave-instructions per wave per BK=32 stage of a BM x BN tile (1 KiB each)
#define LPS_OF(BM, BN, NW) (((BM) * BK32 * 2 / 1024 + (BN) * BK32 * 2 / 1024) / (NW))

PVR_DEV int swz_k32(int row) { return (row >> 1) & 3; }  // 64-B rows: conflict-free ds_read_b128

template <int R, bool KC, int NW>
PVR_DEV void stage32(__amdgpu_buffer_rsrc_t rs, char* lds, int64_t ld, int k0, int wave, int lane) {
  if constexpr (KC) {
    constexpr int NI = R / 16;  // image [R][4 chunks], one wave-instruction = 16 rows
#pragma unroll
    for (int i = 0; i < NI / NW; ++i) {
      const int s = wave + NW * i;
      const int row = s * 16 + (lane >> 2);
      const int c = (lane & 3) ^ swz_k32(row);
      const uint32_t voff = (uint32_t)(row * ld * 2 + (int64_t)(k0 + c * 8) * 2);
      dma16(rs, to_lds(lds + s * 1024), voff);
    }
  } else {
    constexpr int CPR = R / 8, RPI = 64 / CPR, NI = BK32 / RPI;  // image [32 k-rows][R/8 chunks]
#pragma unroll
    for (int i = 0; i < NI / NW; ++i) {
      const int s = wave + NW * i;
      const int row = s * RPI + lane / CPR;
      const int pc = lane % CPR;
      const int c = (pc & ~15) | ((pc & 15) ^ swz_mn(row));
      const uint32_t voff = (uint32_t)((int64_t)(k0 + row) * ld * 2 + c * 16);
      dma16(rs, to_lds(lds + s * 1024), voff);
    }
  }
}

template <int R, bool KC>
PVR_DEV v8s frag32(const char* lds, int r0, int lane) {
  if constexpr (KC) {
    const int row = r0 + (lane & 15);
    return ds_read_b128(lds + row * 64 + (((lane >> 4) ^ swz_k32(row)) << 4));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int c = (r0 >> 3) + (p >> 1);
    const int kr0 = 8 * g + q, kr1 = kr0 + 4;
    const int pc0 = (c & ~15) | ((c & 15) ^ swz_mn(kr0));
    const int pc1 = (c & ~15) | ((c & 15) ^ swz_mn(kr1));
    return cat44(ds_read_tr(lds + kr0 * (R * 2) + pc0 * 16 + 8 * (p & 1)),
                 ds_read_tr(lds + kr1 * (R * 2) + pc1 * 16 + 8 * (p & 1)));
  }
}


// ===================================================================================== v3
// 4 waves (2x2) per workgroup, wave tile (BM/2)x(BN/2) (128x128 at 256x256: 256 fp32 accumulators
// per lane in the AGPR half of the unified register file, one wave per SIMD), BK = 32, 4-stage
// LDS-DMA ring. Fragments are register double-buffered: the ds_reads of stage k+1 are issued while
// the MFMAs of stage k run, so LDS latency is hidden behind the matrix pipe instead of exposed after
// every barrier. The barrier ending stage k waits (counted vmcnt) for stage k+2 to land, so stage
// k+1 is already visible when its fragments are read; one DMA stage stays in flight across it.
template <int FM, int FN, int BM, int BN, bool AK, bool BKC>
PVR_DEV void load_frags(const char* stage, int wm, int wn, int lane, v8s (&af)[FM], v8s (&bf)[FN]) {
  constexpr int A_BYTES = BM * BK32 * 2;
#pragma unroll
  for (int i = 0; i < FM; ++i) af[i] = frag32<BM, AK>(stage, wm * (16 * FM) + 16 * i, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) bf[j] = frag32<BN, BKC>(stage + A_BYTES, wn * (16 * FN) + 16 * j, lane);
}

template <int FM, int FN, bool SWAP>
PVR_DEV void mfma_block(v4f (&acc)[FM][FN], const v8s (&af)[FM], const v8s (&bf)[FN]) {
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (SWAP)
        acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
      else
        acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    }
}

// One LDS-DMA wave-instruction (the idx-th of this wave) of a BK=32 operand tile.
template <int R, bool KC, int NW>
PVR_DEV void dma_one(__amdgpu_buffer_rsrc_t rs, char* lds, int64_t ld, int k0, int wave, int lane, int idx) {
  const int s = wave + NW * idx;
  if constexpr (KC) {
    const int row = s * 16 + (lane >> 2);
    const int c = (lane & 3) ^ swz_k32(row);
    dma16(rs, to_lds(lds + s * 1024), (uint32_t)(row * ld * 2 + (int64_t)(k0 + c * 8) * 2));
  } else {
    constexpr int CPR = R / 8, RPI = 64 / CPR;
    const int row = s * RPI + lane / CPR;
    const int pc = lane % CPR;
    const int c = (pc & ~15) | ((pc & 15) ^ swz_mn(row));
    dma16(rs, to_lds(lds + s * 1024), (uint32_t)((int64_t)(k0 + row) * ld * 2 + c * 16));
  }
}

PVR_DEV __amdgpu_buffer_rsrc_t pick_rsrc(bool live, __amdgpu_buffer_rsrc_t r, __amdgpu_buffer_rsrc_t dead) {
  return live ? r : dead;
}

template <int I, int N, class F>
PVR_DEV void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// One pipeline stage: 16x16x32 MFMAs of fragment set (ac, bc) into acc, interleaved with (a) this
// wave's LDS-DMA instructions for the stage `ds` (into LDS `dst`) and (b) the ds_reads of the next
// stage's fragments (from `nxt`) into (an, bn). Branch-free, so the whole stage is one scheduling
// region and sched_group_barrier pins the interleave: per fragment row, {DMA, ds_reads, MFMAs}.
template <int BM, int BN, int WM, int WN, bool AK, bool BKC, bool SWAP>
PVR_DEV void v3_stage(v4f (&acc)[BM / WM / 16][BN / WN / 16], const v8s (&ac)[BM / WM / 16], const v8s (&bc)[BN / WN / 16],
                      v8s (&an)[BM / WM / 16], v8s (&bn)[BN / WN / 16], const char* nxt, char* dst,
                      __amdgpu_buffer_rsrc_t ars, __amdgpu_buffer_rsrc_t brs, int64_t lda, int64_t ldb, int dk0,
                      int wave, int lane, int wm, int wn) {
  constexpr int NW = WM * WN, FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr int A_BYTES = BM * BK32 * 2;
  constexpr int NIA = (BM * BK32 * 2 / 1024) / NW, NIB = (BN * BK32 * 2 / 1024) / NW, ND = NIA + NIB;
  static_for<0, FM>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    constexpr int d0 = i * ND / FM, d1 = (i + 1) * ND / FM;
    constexpr int j0 = i * FN / FM, j1 = (i + 1) * FN / FM;
#pragma unroll
    for (int d = d0; d < d1; ++d) {
      if (d < NIA)
        dma_one<BM, AK, NW>(ars, dst, lda, dk0, wave, lane, d);
      else
        dma_one<BN, BKC, NW>(brs, dst + A_BYTES, ldb, dk0, wave, lane, d - NIA);
    }
    an[i] = frag32<BM, AK>(nxt, wm * (16 * FM) + 16 * i, lane);
#pragma unroll
    for (int j = j0; j < j1; ++j) bn[j] = frag32<BN, BKC>(nxt + A_BYTES, wn * (16 * FN) + 16 * j, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (SWAP)
        acc[i][j] = mfma16(bc[j], ac[i], acc[i][j]);
      else
        acc[i][j] = mfma16(ac[i], bc[j], acc[i][j]);
    }
    constexpr int nds = (AK ? 1 : 2) + (j1 - j0) * (BKC ? 1 : 2);  // b128 per k-contig frag, 2 tr reads otherwise
    if constexpr (d1 > d0) __builtin_amdgcn_sched_group_barrier(0x020, d1 - d0, 0);  // VMEM read (LDS-DMA)
    __builtin_amdgcn_sched_group_barrier(0x100, nds, 0);                              // DS read
    __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);                               // MFMA
  });
}

template <int BM, int BN, int WM, int WN, int STAGES, int WPE, bool AK, bool BKC, bool SWAP, int EPI>
__global__ void __launch_bounds__(WM* WN * 64, WPE) gemm_v3_kernel(GemmParams p) {
  static_assert(STAGES == 3 || STAGES == 4, "ring depth");
  constexpr int NW = WM * WN;
  constexpr int INFL = (STAGES - 2) * LPS_OF(BM, BN, NW);  // DMA instructions allowed in flight at a stage barrier
  constexpr int A_BYTES = BM * BK32 * 2, B_BYTES = BN * BK32 * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;  // wave tile in 16x16 fragments
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;

  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, ntm * ntn);
  const int tm = t / ntn, tn = t % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * p.k_split_len;
  const int kend = min(p.K, kbeg + p.k_split_len);
  const int nk = (kend - kbeg + BK32 - 1) / BK32;

  const uint16_t* abase;
  uint32_t abytes;
  if constexpr (AK) {
    abase = p.A + (int64_t)m0 * p.lda + kbeg;
    abytes = rsrc_bytes((int64_t)(p.M - 1) * p.lda + p.K, (int64_t)m0 * p.lda + kbeg);
  } else {
    abase = p.A + (int64_t)kbeg * p.lda + m0;
    abytes = rsrc_bytes((int64_t)(p.K - 1) * p.lda + p.M, (int64_t)kbeg * p.lda + m0);
  }
  const uint16_t* bbase;
  uint32_t bbytes;
  if constexpr (BKC) {
    bbase = p.B + (int64_t)n0 * p.ldb + kbeg;
    bbytes = rsrc_bytes((int64_t)(p.N - 1) * p.ldb + p.K, (int64_t)n0 * p.ldb + kbeg);
  } else {
    bbase = p.B + (int64_t)kbeg * p.ldb + n0;
    bbytes = rsrc_bytes((int64_t)(p.K - 1) * p.ldb + p.N, (int64_t)kbeg * p.ldb + n0);
  }
  const __amdgpu_buffer_rsrc_t ars = make_rsrc(abase, abytes);
  const __amdgpu_buffer_rsrc_t brs = make_rsrc(bbase, bbytes);
  const __amdgpu_buffer_rsrc_t nul = make_rsrc(abase, 0);  // every access out of range: no traffic

  v4f acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  stamp(p, 0);
  // Prologue: stages 0..STAGES-1 (stages >= nk use the null resource, keeping every vmcnt count uniform).
#pragma unroll
  for (int s = 0; s < STAGES; ++s) {
    char* dst = smem + s * STAGE_BYTES;
    stage32<BM, AK, NW>(pick_rsrc(s < nk, ars, nul), dst, p.lda, s * BK32, wave, lane);
    stage32<BN, BKC, NW>(pick_rsrc(s < nk, brs, nul), dst + A_BYTES, p.ldb, s * BK32, wave, lane);
  }
  wait_barrier<INFL>();  // stages 0 and 1 landed
  v8s a0[FM], b0[FN], a1[FM], b1[FN];
  load_frags<FM, FN, BM, BN, AK, BKC>(smem, wm, wn, lane, a0, b0);
  wait_barrier_lds<INFL>();  // every wave holds stage 0 in registers: slot 0 may be refilled
  stamp(p, 1);

  // Invariant at stage kt: its fragments are in registers, its LDS slot receives stage kt+STAGES,
  // stage kt+1 is visible. The barrier after stage kt waits for stage kt+2 and retires the LDS reads.
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    v3_stage<BM, BN, WM, WN, AK, BKC, SWAP>(acc, a0, b0, a1, b1, smem + ((kt + 1) % STAGES) * STAGE_BYTES,
                                    smem + (kt % STAGES) * STAGE_BYTES, pick_rsrc(kt + STAGES < nk, ars, nul),
                                    pick_rsrc(kt + STAGES < nk, brs, nul), p.lda, p.ldb, (kt + STAGES) * BK32, wave, lane,
                                    wm, wn);
    wait_barrier_lds<INFL>();
    v3_stage<BM, BN, WM, WN, AK, BKC, SWAP>(acc, a1, b1, a0, b0, smem + ((kt + 2) % STAGES) * STAGE_BYTES,
                                    smem + ((kt + 1) % STAGES) * STAGE_BYTES, pick_rsrc(kt + 1 + STAGES < nk, ars, nul),
                                    pick_rsrc(kt + 1 + STAGES < nk, brs, nul), p.lda, p.ldb, (kt + 1 + STAGES) * BK32, wave,
                                    lane, wm, wn);
    wait_barrier_lds<INFL>();
  }
  if (kt < nk) mfma_block<FM, FN, SWAP>(acc, a0, b0);  // odd tail: set 0 holds the last stage
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // no LDS-DMA may outlive the workgroup
  stamp(p, 2);
  epilogue<FM, FN, SWAP, EPI>(p, acc, m0 + wm * (16 * FM), n0 + wn * (16 * FN), lane);
  if (p.dbg) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp(p, 3);
}

template <int BM, int BN, int WM, int WN, int STAGES, int WPE, bool AK, bool BKC, bool SWAP, int EPI>
hipError_t launch_v3(const GemmParams& p, hipStream_t s) {
  constexpr int SMEM = STAGES * (BM + BN) * BK32 * 2;
  auto kern = gemm_v3_kernel<BM, BN, WM, WN, STAGES, WPE, AK, BKC, SWAP, EPI>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int nsplit = (p.K + p.k_split_len - 1) / p.k_split_len;
  hipLaunchKernelGGL(kern, dim3(ntm * ntn, 1, nsplit), dim3(WM * WN * 64), SMEM, s, p);
  return hipGetLastError();
}

// ===================================================================================== ping-pong
// 256x256 tile, BK = 64, 8 waves as 2 groups of 4 (group = wm: one wave of each group per SIMD),
// k-contiguous operands only. Each wave owns a 128x64 output (8x4 fragments) processed as four
// 64x32 quadrants per K-tile ("phases"). A phase is
//     R: ds_read this quadrant's register subtile | issue one half-tile of LDS-DMA | counted vmcnt
//     barrier | lgkmcnt(0) | prio 1: 16 MFMAs (quadrant x K 64) | prio 0 | barrier
// and group 1 runs one barrier behind group 0, so on every SIMD one wave's MFMA block overlaps the
// other wave's fragment reads and DMA issue (the two never compete for the same phase).
//
// LDS: two 64 KiB buffers (K-tile t in buffer t&1), each an A image [256][64] and a B image
// [256][64] of 128-B swizzled rows. "Half-tiles" are the rows one quadrant reads:
//   A0 = A rows {0-63, 128-191} (qm = 0 of both wave rows), A1 = {64-127, 192-255},
//   B0 = B rows {32-row blocks 0,2,4,6} (qn = 0 of every wave column), B1 = blocks {1,3,5,7}.
// Phase order per K-tile: (qm,qn) = (0,0) reads A0,B0 | (0,1) reads B1 | (1,1) reads A1 | (1,0) -.
// A half-tile is dead two phases after its last read, so K-tile t+2 is staged into buffer t&1 in
// the order A0,B0 (phases 3,4 of t), B1,A1 (phases 1,2 of t+1): half-tile h = 4t + {0:A0,1:B0,2:B1,
// 3:A1} is issued at global phase h - 6, and the vmcnt(8) before each phase's first barrier (four
// half-tiles = 8 DMA instructions per wave stay in flight) retires exactly what the next phase
// reads — every read is one phase after the wait that retires it, across one barrier more than
// the group stagger needs.
constexpr int PP_BK = 64;
constexpr int PP_BUF = 2 * 256 * 128;  // A + B image of one K-tile

// k-contiguous operand half-tile: rows of a [256][64] image (128-B rows), see the layout above.
// mn-contiguous operand half-tile (wgrad: dY / X are [tokens][features]): its own [64 k][128 col]
// image (256-B rows, 16-B chunks XOR-swizzled by swz_mn for the transposed reads); image column c
// is tile row (c >> 6) * 128 + hh * 64 + (c & 63) for A, (c >> 5) * 64 + hh * 32 + (c & 31) for B.
template <int W, bool AK, bool BKC, int ES>
PVR_DEV void pp_issue(__amdgpu_buffer_rsrc_t ars, __amdgpu_buffer_rsrc_t brs, __amdgpu_buffer_rsrc_t nul, char* smem,
                      int64_t lda, int64_t ldb, int t, int nk, int wave, int lane) {
  static_assert(ES == 2 || ES == 1, "bf16 or fp8 operands");
  char* buf = smem + (t & 1) * PP_BUF;
  const int k0 = t * PP_BK;   // bf16 element offset (mn path)
  const int kb = t * 128;     // byte offset of this K-tile within a k-contiguous row (64 bf16 / 128 fp8)
  const bool live = t < nk;
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int d = wave + 8 * x;  // 16 wave-instructions of 1 KiB per half-tile
    if constexpr (W == 0 || W == 3) {
      constexpr int hh = W == 3;
      if constexpr (AK) {
        const int rowb = (2 * (d >> 3) + hh) * 64 + (d & 7) * 8;  // first image row of this instruction
        const int row = rowb + (lane >> 3);
        const int c = (lane & 7) ^ swz_k(row);
        dma16(live ? ars : nul, to_lds(buf + rowb * 128), (uint32_t)(row * lda * ES + kb + c * 16));
      } else if constexpr (ES == 1) {
        // fp8 mn-contiguous half-tile: [128 k][128 B] image, 16-B chunk cl of k-row kr at byte 16 cl
        // holds tile rows (cl >> 2) * 128 + hh * 64 + (cl & 3) * 16 .. +15 (lda in bytes)
        const int kr = 8 * d + (lane >> 3), cl = (lane & 7) ^ swz8(kr);
        const int m = (cl >> 2) * 128 + hh * 64 + (cl & 3) * 16;
        dma16(live ? ars : nul, to_lds(buf + hh * 16384 + d * 1024), (uint32_t)((int64_t)(t * 128 + kr) * lda + m));
      } else {
        const int kr = 4 * d + (lane >> 4);
        const int cl = (lane & 15) ^ swz_mn(kr);  // logical chunk stored at this lane's LDS slot
        const int m = (cl >> 3) * 128 + hh * 64 + (cl & 7) * 8;
        dma16(live ? ars : nul, to_lds(buf + hh * 16384 + d * 1024), (uint32_t)(((int64_t)(k0 + kr) * lda + m) * 2));
      }
    } else {
      constexpr int hh = W == 2;
      if constexpr (BKC) {
        const int rowb = (2 * (d >> 2) + hh) * 32 + (d & 3) * 8;
        const int row = rowb + (lane >> 3);
        const int c = (lane & 7) ^ swz_k(row);
        dma16(live ? brs : nul, to_lds(buf + 256 * 128 + rowb * 128), (uint32_t)(row * ldb * ES + kb + c * 16));
      } else if constexpr (ES == 1) {
        // chunk cl holds tile rows (cl >> 1) * 64 + hh * 32 + (cl & 1) * 16 .. +15
        const int kr = 8 * d + (lane >> 3), cl = (lane & 7) ^ swz8(kr);
        const int n = (cl >> 1) * 64 + hh * 32 + (cl & 1) * 16;
        dma16(live ? brs : nul, to_lds(buf + 256 * 128 + hh * 16384 + d * 1024), (uint32_t)((int64_t)(t * 128 + kr) * ldb + n));
      } else {
        const int kr = 4 * d + (lane >> 4);
        const int cl = (lane & 15) ^ swz_mn(kr);
        const int n = (cl >> 2) * 64 + hh * 32 + (cl & 3) * 8;
        dma16(live ? brs : nul, to_lds(buf + 256 * 128 + hh * 16384 + d * 1024), (uint32_t)(((int64_t)(k0 + kr) * ldb + n) * 2));
      }
    }
  }
}

PVR_DEV void pp_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// fp8 fragment half h of a 16 x 128 (k) operand tile: lane (row r0 + (l&15)) gets 16-B chunk
// (l>>4) + 4h of its 128-B row. A and B use the same read, so the k order the MFMA assigns to the
// 32 bytes of a lane is the same for both operands and the product is unchanged by which chunks a
// lane holds. Chunk (l>>4) + 4h (the bf16 read_frag order) keeps each ds_read_b128 lane group on 16
// distinct bank quads of the swz_k image; the former 2 (l>>4) + h hit 8 (2-way conflicts on every
// fragment read: SQ_LDS_BANK_CONFLICT ~4 cycles per LDS instruction, profiles/r4/pmc_gemm).
// The fp8 kernels never mix a k-contiguous operand with an mn-contiguous one (read_frag_mn8_async).
PVR_DEV v8s frag_fp8(const char* img, int r0, int h, int lane) {
  const int row = r0 + (lane & 15);
  const int c = (lane >> 4) + 4 * h;
  return ds_read_b128(img + row * 128 + ((c ^ swz_k(row)) << 4));
}

typedef uint32_t v2u8 __attribute__((ext_vector_type(2)));
// fp8 operand fragment of an mn-contiguous [128 k][128 B] image (4 x ds_read_b64_tr_b8, async: the
// caller waits with lds_wait): lane (g = l >> 4, i = l & 15) gets image column c0 + i at k-rows
// 32g + 8j .. +7 in r[j], i.e. k = 32g .. 32g + 31 of its row (both operands of the wgrad kernel
// use this read). Per 16-lane group, lane 2q + p supplies row q, bytes 8p .. 8p + 7.
PVR_DEV void read_frag_mn8_async(const char* img, int c0, int lane, v2u8 (&r)[4]) {
  const int g = lane >> 4, i = lane & 15;
  const int row = 32 * g + (i >> 1);  // + 8j for read j: swz8 is the same on all four
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(
      img + row * 128 + ((((c0 >> 4) ^ swz8(row)) << 4) | 8 * (i & 1)));
  asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(r[0]) : "v"(a));
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:1024" : "=v"(r[1]) : "v"(a));
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:2048" : "=v"(r[2]) : "v"(a));
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:3072" : "=v"(r[3]) : "v"(a));
}
PVR_DEV v8s cat8_fp8(v2u8 lo, v2u8 hi) {
  typedef uint32_t v4u_ __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(v8s, (v4u_){lo.x, lo.y, hi.x, hi.y});
}

template <int FA, int FB>
PVR_DEV v4f mfma_fp8(const v8s& a0, const v8s& a1, const v8s& b0, const v8s& b1, v4f c) {
  typedef int v8i __attribute__((ext_vector_type(8)));
  typedef int v4i __attribute__((ext_vector_type(4)));
  const v4i x0 = __builtin_bit_cast(v4i, a0), x1 = __builtin_bit_cast(v4i, a1);
  const v4i y0 = __builtin_bit_cast(v4i, b0), y1 = __builtin_bit_cast(v4i, b1);
  const v8i a = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  const v8i b = {y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
  // scale operands 127 = 2^0 in E8M0: per-tensor dequant happens in the epilogue
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, FA, FB, 0, 127, 0, 127);
}

// Per-wave phase-segment cycle sums of the ping-pong K loop (diagnostic builds, -DPVR_GEMM_PHASE_STAMPS;
// scripts/gemm_phase_stamps.py): reads issue | DMA issue | vmcnt wait | barrier 1 | lgkmcnt wait |
// MFMA issue | barrier 2 | (slot 7: whole K loop), summed over every phase, written once per wave to
// p.dbg[(workgroup * 8 + wave) * 8 + segment]. Production builds compile the stamps out.
// -DPVR_GEMM_PHASE_ONLY_TYPE=t (with -DPVR_GEMM_PHASE_STAMPS): the same segments, phases of type t only.
// -DPVR_GEMM_PHASE_BY_TYPE (with -DPVR_GEMM_PHASE_STAMPS): slots 0-3 = whole phase by phase type
// (quadrant order (0,0) (0,1) (1,1) (1,0)), 4-7 = its reads + DMA issue + vmcnt wait part.
struct PpStamps {
#ifdef PVR_GEMM_PHASE_STAMPS
  uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t last = 0;
  uint64_t t0 = 0;
#endif
  // pt: the calling phase's type; -DPVR_GEMM_PHASE_ONLY_TYPE=t sums the segments of type-t phases only
  PVR_DEV void at(int k, int pt) {
#if defined(PVR_GEMM_PHASE_STAMPS) && !defined(PVR_GEMM_PHASE_BY_TYPE)
    const uint64_t t = __builtin_amdgcn_s_memtime();
#ifdef PVR_GEMM_PHASE_ONLY_TYPE
    if (pt == PVR_GEMM_PHASE_ONLY_TYPE) acc[k] += t - last;
#else
    (void)pt;
    acc[k] += t - last;
#endif
    last = t;
#else
    (void)k;
    (void)pt;
#endif
  }
  PVR_DEV void type_mark(int pt, int what) {  // what 0: phase start, 1: R-part end, 2: phase end
#if defined(PVR_GEMM_PHASE_STAMPS) && defined(PVR_GEMM_PHASE_BY_TYPE)
    const uint64_t t = __builtin_amdgcn_s_memtime();
    if (what == 0) t0 = t;
    else if (what == 1) acc[4 + pt] += t - t0;
    else acc[pt] += t - t0;
#else
    (void)pt;
    (void)what;
#endif
  }
  PVR_DEV void begin() {
#ifdef PVR_GEMM_PHASE_STAMPS
    last = __builtin_amdgcn_s_memtime();
#endif
  }
};

// PR (bf16 k-contiguous A only, see PVR_PP_PRE): 1 = this (0,0) phase takes A0's first k-step
// fragments from `pre` (read one phase earlier) and reads only the second; 2 = this (1,0) phase
// reads the NEXT K-tile's A0 first-k-step fragments from `nbuf` into `pre`.
template <int QM, int QN, int RD_A, int RD_B, int KIND, bool AK, bool BKC, bool SWAP, int ES = 2, int FA = 0, int FB = 0, int PR = 0>
PVR_DEV void pp_phase(v4f (&acc)[8][4], v8s (&af)[4][2], v8s (&bf)[2][2][2], v8s (&pre)[4], const char* buf, const char* nbuf,
                      __amdgpu_buffer_rsrc_t ars, __amdgpu_buffer_rsrc_t brs, __amdgpu_buffer_rsrc_t nul, char* smem, int64_t lda,
                      int64_t ldb, int t_issue, int nk, int wave, int lane, int wm, int wn, PpStamps& pst) {
  static_assert(PR == 0 || (AK && ES == 2), "A0 read-ahead: bf16 k-contiguous A only");
  constexpr int PT_ = QM == 0 ? QN : 3 - QN;  // phase type: (0,0) (0,1) (1,1) (1,0)
  pst.type_mark(PT_, 0);

  // R: register subtile for this quadrant. mn-contiguous operands are read with the asm transpose
  // read (halves combined after the wait below): the builtin would make hipcc drain the in-flight
  // half-tile DMAs (vmcnt(0)) in front of the read.
  v4s alo[4][2], ahi[4][2], blo[2][2], bhi[2][2];
  constexpr bool MN8A = ES == 1 && !AK, MN8B = ES == 1 && !BKC;
  v2u8 a8r[MN8A ? 4 : 1][4], b8r[MN8B ? 2 : 1][4];
  if constexpr (RD_A && MN8A) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) read_frag_mn8_async(buf + QM * 16384, wm * 64 + 16 * ii, lane, a8r[ii]);
  } else if constexpr (RD_A) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (ES == 1)
          af[ii][ks] = frag_fp8(buf, wm * 128 + QM * 64 + 16 * ii, ks, lane);
        else if constexpr (AK && PR == 1)
          af[ii][ks] = ks == 0 ? pre[ii] : read_frag<256, true>(buf, wm * 128 + QM * 64 + 16 * ii, ks, lane);
        else if constexpr (AK)
          af[ii][ks] = read_frag<256, true>(buf, wm * 128 + QM * 64 + 16 * ii, ks, lane);
        else
          read_frag_mn_async<128>(buf + QM * 16384, wm * 64 + 16 * ii, ks, lane, alo[ii][ks], ahi[ii][ks]);
      }
  }
  if constexpr (PR == 2) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) pre[ii] = read_frag<256, true>(nbuf, wm * 128 + 16 * ii, 0, lane);
  }
  if constexpr (RD_B && MN8B) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) read_frag_mn8_async(buf + 256 * 128 + QN * 16384, wn * 32 + 16 * jj, lane, b8r[jj]);
  } else if constexpr (RD_B) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (ES == 1)
          bf[QN][jj][ks] = frag_fp8(buf + 256 * 128, wn * 64 + QN * 32 + 16 * jj, ks, lane);
        else if constexpr (BKC)
          bf[QN][jj][ks] = read_frag<256, true>(buf + 256 * 128, wn * 64 + QN * 32 + 16 * jj, ks, lane);
        else
          read_frag_mn_async<128>(buf + 256 * 128 + QN * 16384, wn * 32 + 16 * jj, ks, lane, blo[jj][ks], bhi[jj][ks]);
      }
  }
  pst.at(0, PT_);
  pp_issue<KIND, AK, BKC, ES>(ars, brs, nul, smem, lda, ldb, t_issue, nk, wave, lane);
  pst.at(1, PT_);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  pst.type_mark(PT_, 1);
  pst.at(2, PT_);
  pp_barrier();
  pst.at(3, PT_);
  if constexpr (AK && BKC)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else
    lds_wait();  // asm reads in flight: the wait must also fence their consumers
  if constexpr (RD_A && MN8A) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      af[ii][0] = cat8_fp8(a8r[ii][0], a8r[ii][1]);
      af[ii][1] = cat8_fp8(a8r[ii][2], a8r[ii][3]);
    }
  }
  if constexpr (RD_B && MN8B) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      bf[QN][jj][0] = cat8_fp8(b8r[jj][0], b8r[jj][1]);
      bf[QN][jj][1] = cat8_fp8(b8r[jj][2], b8r[jj][3]);
    }
  }
  if constexpr (RD_A && !AK && ES == 2) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[ii][ks] = cat44(alo[ii][ks], ahi[ii][ks]);
  }
  if constexpr (RD_B && !BKC && ES == 2) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bf[QN][jj][ks] = cat44(blo[jj][ks], bhi[jj][ks]);
  }
  pst.at(4, PT_);
  __builtin_amdgcn_s_setprio(1);
  if constexpr (ES == 1) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        v4f& c = acc[QM * 4 + ii][QN * 2 + jj];
        if constexpr (SWAP)
          c = mfma_fp8<FB, FA>(bf[QN][jj][0], bf[QN][jj][1], af[ii][0], af[ii][1], c);
        else
          c = mfma_fp8<FA, FB>(af[ii][0], af[ii][1], bf[QN][jj][0], bf[QN][jj][1], c);
      }
    __builtin_amdgcn_s_setprio(0);
    pst.at(5, PT_);
    pp_barrier();
    pst.at(6, PT_);
    pst.type_mark(PT_, 2);
    return;
  }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        v4f& c = acc[QM * 4 + ii][QN * 2 + jj];
        if constexpr (SWAP)
          c = mfma16(bf[QN][jj][ks], af[ii][ks], c);
        else
          c = mfma16(af[ii][ks], bf[QN][jj][ks], c);
      }
  __builtin_amdgcn_s_setprio(0);
  pst.at(5, PT_);
  pp_barrier();
  pst.at(6, PT_);
  pst.type_mark(PT_, 2);
}

// Register-direct epilogue of the ping-pong kernels (SWAP layout, bf16-output epilogues, no row
// remap / position addend, N % 8 == 0). Each wave finishes its own 128x64 output block straight
// from the accumulators: no LDS staging, no barriers (DGELU colsum excepted), so a wave whose main
// loop ended early starts storing while its SIMD partner still runs MFMAs.
//   lane (li = l & 15, g = l >> 4) holds C[mb + 16i + li][nb + 16j + 4g + r] in acc[i][j][r];
//   one v_permlane16_swap per dword of fragments (j0, j1) = (2jp, 2jp+1) (rows 1, 3 of j0 <-> rows
//   0, 2 of j1) leaves every lane 8 contiguous columns c0 = nb + 32jp + {0, 16, 8, 24}[g] .. +7,
// so bias / residual / dGELU-factor loads and output / GELU-derivative stores are 16 B per lane,
// 16 rows x 64 B per wave instruction (16 stores per wave and output instead of 32 x 8 B through
// LDS). Buffer resources start at the wave's first row: rows past M read 0 and are not written;
// lanes whose columns are past N use an out-of-range offset. Same fp32 math as `epilogue` above.
// epilogue_direct's preconditions: plain row mapping, 16-B column groups, 31-bit buffer offsets
__host__ __device__ inline bool direct_ok(const GemmParams& p) {
  const int64_t l1 = p.ldc > p.ld_resid ? p.ldc : p.ld_resid;
  const int64_t ld = l1 > p.ld_aux ? l1 : p.ld_aux;
  return !p.addend && !p.row_group && (p.N & 7) == 0 && (int64_t)p.M * ld * 2 < (1ll << 31);
}

template <int EPI, bool RES, bool SCALED = false>
PVR_DEV void epilogue_direct(const GemmParams& p, v4f (&acc)[8][4], char* smem, int mb, int nb, int wm, int wn, int lane) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  typedef uint32_t v2u_q __attribute__((ext_vector_type(2)));
  const int li = lane & 15, g = lane >> 4;
  const float deq = SCALED ? (*p.scale_a) * (*p.scale_b) : 1.f;  // fp8 operands: per-tensor dequant
  // rows [mb, min(M, mb + 128)) of C (and of the residual / aux tensors) from the wave's first row
  const int rows = max(0, min(128, p.M - mb));
  const uint32_t OOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t crs =
      make_rsrc((const uint16_t*)p.C + (int64_t)mb * p.ldc, rows && !p.c_skip ? (uint32_t)(((int64_t)(rows - 1) * p.ldc + p.N) * 2) : 0);
  __amdgpu_buffer_rsrc_t xrs = crs;  // residual (BF16) / aux (GELU store, DGELU load)
  int64_t ldx = p.ldc;
  if constexpr (EPI == EPI_BF16 && RES) {
    xrs = make_rsrc(p.resid + (int64_t)mb * p.ld_resid, rows ? (uint32_t)(((int64_t)(rows - 1) * p.ld_resid + p.N) * 2) : 0);
    ldx = p.ld_resid;
  } else if constexpr (EPI == EPI_GELU || EPI == EPI_DGELU) {
    const bool has = p.aux != nullptr;
    xrs = make_rsrc(has ? p.aux + (int64_t)mb * p.ld_aux : p.aux, has && rows ? (uint32_t)(((int64_t)(rows - 1) * p.ld_aux + p.N) * 2) : 0);
    ldx = p.ld_aux;
  }
  const __amdgpu_buffer_rsrc_t brs = make_rsrc(p.bias, p.bias ? (uint32_t)p.N * 4 : 0);
  int c0[2];
  uint32_t vc[2], vx[2];
  float bias[2][8];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    c0[jp] = nb + 32 * jp + ((g & 1) << 4) + ((g & 2) << 2);
    const bool okc = c0[jp] < p.N;
    vc[jp] = okc ? (uint32_t)((li * p.ldc + c0[jp]) * 2) : OOB;
    vx[jp] = okc ? (uint32_t)((li * ldx + c0[jp]) * 2) : OOB;
#pragma unroll
    for (int e = 0; e < 8; ++e) bias[jp][e] = 0.f;
    if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
      const uint32_t vb = okc ? (uint32_t)(c0[jp] * 4) : OOB;
      const v4f b0 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(brs, vb, 0, 0));
      const v4f b1 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(brs, vb + 16, 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) { bias[jp][e] = b0[e]; bias[jp][4 + e] = b1[e]; }
    }
  }
  const uint64_t seed = (p.drop_thr ? *p.seed_ptr : 0ull) + p.seed_offset;
  const uint32_t key = p.drop_thr ? rng_key(seed) : 0u;
  const bool idx32 = (uint64_t)p.M * (uint64_t)p.N + 8 <= 0xFFFFFFFFull;
  float csum[2][8];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[jp][e] = 0.f;
  // the row inputs (residual / dGELU factor) of the wave's 128 rows go through a ring of RING fragment
  // rows (8 VGPRs each), each requested RING rows ahead of its use: the loads' latency overlaps the
  // rows before it without holding all 64 VGPRs at once (which spilled to scratch next to the 128
  // accumulators). Row offsets go into the VGPR offset: the SGPR offset of a buffer access is outside
  // its range check, so rows past M would be accessed.
  constexpr bool HAS_IN = (EPI == EPI_BF16 && RES) || EPI == EPI_DGELU;
  constexpr int RING = 4;
  // fp8 copy of the GELU / dGELU output (fp8 GEMMs only): 8 bytes per lane and fragment row
  constexpr bool QOK = SCALED && (EPI == EPI_GELU || EPI == EPI_DGELU);
  const bool qon = QOK && p.q_out != nullptr;
  const __amdgpu_buffer_rsrc_t qrs = make_rsrc(qon ? p.q_out + (int64_t)mb * p.ld_q : p.q_out,
                                               qon && rows ? (uint32_t)((int64_t)(rows - 1) * p.ld_q + p.N) : 0u);
  const float qsc = qon ? *p.q_scale : 1.f;
  float qam = 0.f;
  v4u xring[HAS_IN ? RING : 1][2];
  if constexpr (HAS_IN) {
#pragma unroll
    for (int i = 0; i < RING; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp)
        xring[i][jp] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vx[jp] + (uint32_t)(i * 16 * (int)ldx * 2), 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i == 1) stamp(p, 4);  // diagnostic builds only (p.dbg): row 0 done (bias / first inputs landed)
    const uint32_t so_c = (uint32_t)(i * 16 * (int)p.ldc * 2), so_x = (uint32_t)(i * 16 * (int)ldx * 2);
    const int m = mb + 16 * i + li;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      v4u xin = {0u, 0u, 0u, 0u};
      if constexpr (HAS_IN) {
        xin = xring[i % RING][jp];
        if (i + RING < 8)  // refill the slot with the row RING ahead
          xring[i % RING][jp] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vx[jp] + (uint32_t)((i + RING) * 16 * (int)ldx * 2), 0, 0);
      }
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // inline asm: hipcc merged the four builtin swaps of a fragment pair into one (wrong values)
        float a = acc[i][2 * jp][r], b = acc[i][2 * jp + 1][r];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
        v[r] = SCALED ? a * deq : a;
        v[4 + r] = SCALED ? b * deq : b;
      }
      bool keep[8] = {true, true, true, true, true, true, true, true};
      if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bias[jp][e];
        if (p.drop_thr) {
          const uint64_t idx = (uint64_t)m * p.N + c0[jp];
          if (idx32) {
            bool k0[4], k1[4];
            rng_keep4_32(key, (uint32_t)idx, p.drop_thr, k0);
            rng_keep4_32(key, (uint32_t)idx + 4, p.drop_thr, k1);
#pragma unroll
            for (int e = 0; e < 4; ++e) { keep[e] = k0[e]; keep[4 + e] = k1[e]; }
          } else {
#pragma unroll
            for (int e = 0; e < 8; e += 2) rng_keep2(seed, idx + e, p.drop_thr, keep[e], keep[e + 1]);
          }
        }
      }
      v4u out;
      if constexpr (EPI == EPI_BF16) {
        if (p.drop_thr) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = keep[e] ? v[e] * p.drop_scale : 0.f;
        }
        if constexpr (RES) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[2 * q] += bf2f(xin[q] & 0xFFFF);
            v[2 * q + 1] += bf2f(xin[q] >> 16);
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) out[q] = pack2bf(v[2 * q], v[2 * q + 1]);
      } else if constexpr (EPI == EPI_GELU) {
        v4u ax;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const v2f s2 = {keep[2 * q] ? p.drop_scale : 0.f, keep[2 * q + 1] ? p.drop_scale : 0.f};
          v2f g2, d2;
          gelu_and_grad2((v2f){v[2 * q], v[2 * q + 1]}, g2, d2);
          g2 *= s2;
          d2 *= s2;
          ax[q] = pack2bf(d2.x, d2.y);
          v[2 * q] = g2.x;  // the output (bf16 below, the fp8 copy)
          v[2 * q + 1] = g2.y;
        }
        if (!p.c_skip) {  // uniform; c_skip: stored to a 0-byte range (the store count stays fixed)
#pragma unroll
          for (int q = 0; q < 4; ++q) out[q] = pack2bf(v[2 * q], v[2 * q + 1]);
        } else {
          out = v4u{0u, 0u, 0u, 0u};
        }
        __builtin_amdgcn_raw_buffer_store_b128(ax, xrs, vx[jp] + so_x, 0, 0);  // no aux (inference): 0-byte resource
      } else {  // EPI_DGELU
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[2 * q] *= bf2f(xin[q] & 0xFFFF);
          v[2 * q + 1] *= bf2f(xin[q] >> 16);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[jp][e] += v[e];
        if (!p.c_skip) {  // uniform; c_skip: stored to a 0-byte range (the store count stays fixed)
#pragma unroll
          for (int q = 0; q < 4; ++q) out[q] = pack2bf(v[2 * q], v[2 * q + 1]);
        } else {
          out = v4u{0u, 0u, 0u, 0u};
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(out, crs, vc[jp] + so_c, 0, 0);
      if constexpr (QOK) {
        if (qon) {
          // rows past M / columns past N: out-of-range offset (dropped); their values are 0 anyway
          const uint32_t vq = c0[jp] < p.N ? (uint32_t)((int64_t)(16 * i + li) * p.ld_q + c0[jp]) : OOB;
          float vm = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) vm = nan_max(vm, fabsf(v[e]));
          qam = nan_max(qam, vm);
          const uint2 q8 = p.q_fmt ? pack8_fp8_fast<1>(v, qsc, vm) : pack8_fp8_fast<0>(v, qsc, vm);
          __builtin_amdgcn_raw_buffer_store_b64((v2u_q){q8.x, q8.y}, qrs, vq, 0, 0);
        }
      }
    }
  }
  stamp(p, 5);  // every row's stores issued
  if constexpr (EPI == EPI_DGELU) {
    {  // without colsum the atomics go to a 0-byte resource: the store count stays fixed
      // column sums over the wave's 128 rows (16 lanes of a row x 8 fragment rows: rows past M
      // and columns past N hold zeros). The two wave groups hold the same 64 columns: group g
      // hands its other column half (jp = 1 - g) to its partner through LDS and adds the
      // partner's half jp = g, then 8 buffer atomics per wave (lanes li = 0; columns past N are
      // out of range). Every wave issues exactly 8: the persistent kernel counts them.
#pragma unroll
      for (int jp = 0; jp < 2; ++jp)
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[jp][e] = row16_sum(csum[jp][e]);
      float* red = (float*)smem;  // [2 column halves][4 wave columns][32 columns]
      if (li == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float give = wm == 0 ? csum[1][e] : csum[0][e];
          red[(1 - wm) * 128 + wn * 32 + (c0[1 - wm] - nb - 32 * (1 - wm)) + e] = give;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // raw barrier: no vmcnt drain of the in-flight stores
      asm volatile("" ::: "memory");
      const __amdgpu_buffer_rsrc_t srs = make_rsrc(p.colsum, p.colsum ? (uint32_t)p.N * 4 : 0);
      if (li == 0) {
        const int jp = wm;
        const uint32_t vo = c0[jp] < p.N ? (uint32_t)c0[jp] * 4 : OOB;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float mine = wm == 0 ? csum[0][e] : csum[1][e];
          __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(mine + red[jp * 128 + wn * 32 + (c0[jp] - nb - 32 * jp) + e], srs, vo + 4 * e, 0, 0);
        }
      }
    }
  }
  if constexpr (QOK) {
    if (qon) {
      // max |out| of the workgroup's tile: waves -> LDS (past the colsum exchange area), one atomic
      // per workgroup (same-address atomics serialise at L2)
      qam = wave_max_nan(qam);
      float* qred = (float*)(smem + 2048);
      const int w = (int)(threadIdx.x >> 6);
      if (lane == 0) qred[w] = qam;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // raw barrier: the output stores stay in flight
      asm volatile("" ::: "memory");
      if (threadIdx.x == 0) {
        float b = qred[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) b = nan_max(b, qred[k]);
        if (!(b <= 0.f)) atomicMax(p.q_amax, __float_as_uint(b));
      }
    }
  }
}

constexpr int CPOL_SC1 = 16;  // buffer-instruction cache policy: sc1 (write-through / L2-bypassing read)

// LDS-staged epilogue of the ping-pong kernel (SWAP layout, bf16-output epilogues): the fp32
// accumulators cross LDS in two 128-row halves (the 128 KiB of K-tile buffers are free by then),
// and every thread then owns 4 consecutive columns of rows t/64 + 8k, so each wave instruction
// reads/writes one whole 512-B row segment — residual / aux loads and bf16 stores are fully
// coalesced instead of 16 rows x 32 B per instruction. The math is the per-element epilogue above,
// in fp32, unchanged. Row images are 1 KiB (256 fp32) with the 16-B chunk index XOR-swizzled by
// the row (ds_write_b128 2-way, ds_read_b128 conflict-free).
// RP = tile rows per staging pass (128: the two K-tile buffers, 128 KiB; 32: the persistent
// kernel's separate 32 KiB region, while the next tile's K-tiles stream into the buffers).
template <int EPI, int RP = 128, bool RES = false>
PVR_DEV void epilogue_staged(const GemmParams& p, v4f (&acc)[8][4], char* smem, int m0, int n0, int wm, int wn, int lane) {
  static_assert(RP == 128 || RP == 64 || RP == 32, "rows per pass");
  const int tid = threadIdx.x;
  const int g = lane >> 4, li = lane & 15;
  const int cq = tid & 63;           // this thread's 4-column group within the tile row
  const int n = n0 + 4 * cq;
  const bool ncol = n < p.N;
  float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
    if (p.bias && ncol) bias = *(const float4*)(p.bias + n);
  }
  const uint64_t seed = (p.drop_thr ? *p.seed_ptr : 0ull) + p.seed_offset;
  const uint32_t key = p.drop_thr ? rng_key(seed) : 0u;
  // every dropout element index of the tensor fits in 32 bits (the usual case): 32-bit hash path
  const bool idx32 = (uint64_t)p.M * (uint64_t)p.N + 4 <= 0xFFFFFFFFull;
  const float deq = p.scale_a ? (*p.scale_a) * (*p.scale_b) : 1.f;
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int NPASS = 256 / RP, FPP = RP / 16;  // passes; fragment rows (of 8 per wave) per pass
#pragma unroll
  for (int half = 0; half < NPASS; ++half) {
    if constexpr (EPI == EPI_F32_ATOMIC) {
      // split-K partial sums: each wave instruction adds one dense 256-B run of a row (thread =
      // column), two cache lines per request instead of 4 rows x 64 B
      __syncthreads();
      if (wm == (half * RP) / 128) {
        const int i0 = ((half * RP) % 128) / 16;
#pragma unroll
        for (int ii = 0; ii < FPP; ++ii)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 16 * ii + li;
            const int ch = wn * 16 + 4 * j + g;
            *(v4f*)(smem + r * 1024 + ((ch ^ (r & 63)) << 4)) = acc[i0 + ii][j];
          }
      }
      __syncthreads();
      const int c = tid & 255;
      const bool okc = n0 + c < p.N;
#pragma unroll 8
      for (int k = 0; k < RP / 2; ++k) {
        const int r = (tid >> 8) + 2 * k;
        const int m = m0 + half * RP + r;
        const float a = *(const float*)(smem + r * 1024 + (((c >> 2) ^ (r & 63)) << 4) + 4 * (c & 3));
        if (okc && m < p.M) atomicAdd((float*)p.C + (int64_t)m * p.ldc + n0 + c, a * deq);
      }
      continue;
    }
    __syncthreads();  // previous pass's LDS reads (or the main loop's) are done
    if (wm == (half * RP) / 128) {
      const int i0 = ((half * RP) % 128) / 16;
#pragma unroll
      for (int ii = 0; ii < FPP; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 16 * ii + li;                // row within the pass
          const int ch = wn * 16 + 4 * j + g;        // 16-B chunk (4 fp32 columns) within the row
          *(v4f*)(smem + r * 1024 + ((ch ^ (r & 63)) << 4)) = acc[i0 + ii][j];
        }
    }
    __syncthreads();
    // Per-row inputs of this pass (residual / dGELU factor) are loaded up front and unconditionally
    // (rows / columns clamped into range): a load under a per-row branch makes the compiler wait
    // vmcnt(0) after each one, serialising them and draining every in-flight LDS-DMA.
    constexpr int RPT = RP / 8;  // rows per thread per pass
    constexpr bool HAS_IN = EPI == EPI_DGELU || (EPI == EPI_BF16 && RES);
    // Row k of this thread is mrow0 + 8k: every per-row address and the dropout element index are
    // a base plus k times a wave-uniform step, so no 64-bit multiply (quarter rate) runs per row.
    const int mrow0 = m0 + half * RP + (tid >> 6);
    const int nn = ncol ? n : 0;
    const bool rows_in = m0 + half * RP + RP <= p.M;  // uniform: no row of this pass past M
    uint2 pin[HAS_IN ? RPT : 1];
    if constexpr (HAS_IN) {
      const uint16_t* src = EPI == EPI_DGELU ? p.aux : p.resid;
      const int64_t lsrc = EPI == EPI_DGELU ? p.ld_aux : p.ld_resid;
      const uint16_t* s0 = src + (int64_t)mrow0 * lsrc + nn;
      if (rows_in) {
#pragma unroll
        for (int k = 0; k < RPT; ++k) pin[k] = *(const uint2*)(s0 + (int64_t)k * (8 * lsrc));
      } else {
#pragma unroll
        for (int k = 0; k < RPT; ++k) pin[k] = *(const uint2*)(src + (int64_t)min(mrow0 + 8 * k, p.M - 1) * lsrc + nn);
      }
    }
    const uint64_t idx0 = (uint64_t)mrow0 * p.N + n, idx_step = 8ull * p.N;
    uint16_t* c0 = (uint16_t*)p.C + (int64_t)mrow0 * p.ldc + n;
    uint16_t* x0 = EPI == EPI_GELU && p.aux ? p.aux + (int64_t)mrow0 * p.ld_aux + n : nullptr;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = (tid >> 6) + 8 * k;
      const int m = mrow0 + 8 * k;
      const v4f a = *(const v4f*)(smem + r * 1024 + ((cq ^ (r & 63)) << 4));
      const bool ok = m < p.M && ncol;
      float v[4] = {a[0] * deq, a[1] * deq, a[2] * deq, a[3] * deq};
      if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
        v[0] += bias.x; v[1] += bias.y; v[2] += bias.z; v[3] += bias.w;
        bool keep[4] = {true, true, true, true};
        if (p.drop_thr) {
          const uint64_t idx = idx0 + (uint64_t)k * idx_step;
          if (EPI == EPI_GELU && idx32) {
            rng_keep4_32(key, (uint32_t)idx, p.drop_thr, keep);
          } else {
            rng_keep2(seed, idx, p.drop_thr, keep[0], keep[1]);
            rng_keep2(seed, idx + 2, p.drop_thr, keep[2], keep[3]);
          }
        }
        if constexpr (EPI == EPI_BF16) {
          if (p.drop_thr) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = keep[q] ? v[q] * p.drop_scale : 0.f;
          }
          if constexpr (RES) {
            const uint2 rr = pin[k];
            v[0] += bf2f(rr.x & 0xFFFF); v[1] += bf2f(rr.x >> 16);
            v[2] += bf2f(rr.y & 0xFFFF); v[3] += bf2f(rr.y >> 16);
          }
        } else {
          // two lanes per packed-fp32 instruction (v_pk_fma_f32 / v_pk_mul_f32)
          const v2f s01 = {keep[0] ? p.drop_scale : 0.f, keep[1] ? p.drop_scale : 0.f};
          const v2f s23 = {keep[2] ? p.drop_scale : 0.f, keep[3] ? p.drop_scale : 0.f};
          v2f g01, d01, g23, d23;
          gelu_and_grad2((v2f){v[0], v[1]}, g01, d01);
          gelu_and_grad2((v2f){v[2], v[3]}, g23, d23);
          g01 *= s01; g23 *= s23; d01 *= s01; d23 *= s23;
          v[0] = g01.x; v[1] = g01.y; v[2] = g23.x; v[3] = g23.y;
          uint2 ax; ax.x = pack2bf(d01.x, d01.y); ax.y = pack2bf(d23.x, d23.y);
          if (ok && p.aux) *(uint2*)(x0 + (int64_t)k * (8 * p.ld_aux)) = ax;  // no aux: inference
        }
      } else if constexpr (EPI == EPI_DGELU) {
        const uint2 gg = pin[k];
        v[0] *= bf2f(gg.x & 0xFFFF); v[1] *= bf2f(gg.x >> 16);
        v[2] *= bf2f(gg.y & 0xFFFF); v[3] *= bf2f(gg.y >> 16);
        if (ok) {
          csum[0] += v[0]; csum[1] += v[1]; csum[2] += v[2]; csum[3] += v[3];
        }
      }
      if constexpr (EPI == EPI_F32_STORE) {
        if (p.sk_out) {  // in-launch reduction: write-through (sc1) slab stores, read by other CUs
          typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));
          const __amdgpu_buffer_rsrc_t srs = make_rsrc((float*)p.C + (int64_t)blockIdx.z * p.split_stride, (uint32_t)(p.split_stride * 4));
          if (ok)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, make_float4(v[0], v[1], v[2], v[3])), srs,
                                                   (uint32_t)(((int64_t)m * p.ldc + n) * 4), 0, CPOL_SC1);
        } else if (ok) {
          *(float4*)((float*)p.C + (int64_t)blockIdx.z * p.split_stride + (int64_t)m * p.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {
        uint2 o; o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
        if (ok) *(uint2*)(c0 + (int64_t)k * (8 * p.ldc)) = o;
      }
    }
  }
  if constexpr (EPI == EPI_DGELU) {
    if (p.colsum) {
      // the 8 waves hold partial sums of the same 256 columns (different rows): reduce them in LDS,
      // then one atomic per column per workgroup (atomics on 3072 bias addresses from ~2400
      // workgroups contend at L2, so their number matters more than their size)
      __syncthreads();
      float* red = (float*)smem;  // [8 waves][256 columns]
      *(float4*)(red + (tid >> 6) * 256 + 4 * cq) = make_float4(csum[0], csum[1], csum[2], csum[3]);
      __syncthreads();
      if (tid < 256 && n0 + tid < p.N) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) t += red[w * 256 + tid];
        atomicAdd(p.colsum + n0 + tid, t);
      }
    }
  }
}

// Split-tail hand-off (see GemmParams::tail_*): this K-part of tail tile `tloc` publishes its fp32
// partial tile, and the part that arrives last adds every part's partial in the fixed order 0..S-1
// into `acc` and returns true (it then runs the epilogue); the others return false. Partials are
// stored in register order (accumulator (i, j) of thread t at float4 (i*4 + j)*512 + t of the
// part's 256 KiB slab): every wave instruction moves one contiguous KiB and each thread re-reads
// only its own values. Publication is the write-through form of the agent-scope hand-off (one
// workgroup per CU, hipMalloc'ed buffers, 16-B accesses): every slab byte is stored sc1, every
// storing wave drains (vmcnt(0)) before the workgroup barrier, one lane then adds to the tile's
// arrival counter (agent scope), and the last arriver's waves read every slab with sc1 loads. No
// release / acquire fences: a release writes back the XCD's whole L2, which with the GEMM's own
// output dirty in it measured ~30 us per tail tile (profiles/r4/tail_ab.md).

template <int S>
PVR_DEV void tail_sum(v4f (&acc)[8][4], __amdgpu_buffer_rsrc_t rs, int tid) {
  constexpr int SLAB_BYTES = 256 * 256 * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t off = (uint32_t)(((i * 4 + j) * 512 + tid) * 16);
      v4f s = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, CPOL_SC1));
#pragma unroll
      for (int q = 1; q < S; ++q)
        s += __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rs, off, q * SLAB_BYTES, CPOL_SC1));
      acc[i][j] = s;
    }
}

PVR_DEV bool tail_gather(const GemmParams& p, v4f (&acc)[8][4], char* smem, int tloc, int tpart) {
  typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));
  constexpr int SLAB = 256 * 256;  // floats per part
  const int tid = threadIdx.x;
  const int S = p.tail_split;
  float* base = p.tail_ws + (int64_t)tloc * S * SLAB;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(base, (uint32_t)S * SLAB * 4);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, acc[i][j]), rs, (uint32_t)(((i * 4 + j) * 512 + tid) * 16),
                                             tpart * SLAB * 4, CPOL_SC1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave, before the barrier
  __syncthreads();
  unsigned* flag = (unsigned*)smem;  // K-tile buffers are idle: every DMA and read has retired
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(p.tail_cnt + tloc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned last = old == (unsigned)(S - 1) ? 1u : 0u;
    // every part of this tile has arrived: re-arm the counter for the next launch
    if (last) __hip_atomic_store(p.tail_cnt + tloc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *(volatile unsigned*)flag = last;
  }
  __syncthreads();  // the other waves load only after the adding lane's result is in
  const unsigned last = *(volatile unsigned*)flag;
  if (!last) return false;
  switch (S) {
    case 2: tail_sum<2>(acc, rs, tid); break;
    case 3: tail_sum<3>(acc, rs, tid); break;
    default: tail_sum<4>(acc, rs, tid); break;
  }
  __syncthreads();  // the flag word is LDS the epilogue may reuse
  return true;
}

// The rows [rb, rb + nrow) of one tile of the in-launch split-K reduction: thread t owns columns
// n0 + 4 (t % 64) .. + 3 of rows rb + t / 64 + 8 i (i < RPT), and sums the S slabs in the order
// 0..S-1. U slabs x RPT rows of sc1 loads are issued before their adds (16 in flight per thread: one
// dependent load at a time left the reduction latency-bound, ~25 us per tile at S = 28). Slabs past
// S and rows past the slice read zero through the resource's range check.
template <int RPT, int U>
PVR_DEV void splitk_rows(const GemmParams& p, __amdgpu_buffer_rsrc_t wrs, int S, int rb, int nrow, int n0, int tid) {
  const int n = n0 + 4 * (tid & 63);
  const uint32_t far = (uint32_t)(p.split_stride * 4 * S);  // past the resource (host: 2 S + 16 slabs < 4 GiB)
  uint32_t off[RPT];
  v4f a[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = (tid >> 6) + 8 * i, m = rb + r;
    off[i] = r < nrow && m < p.M && n < p.N ? (uint32_t)(((int64_t)m * p.ldc + n) * 4) : far;
    a[i] = v4f{0.f, 0.f, 0.f, 0.f};
  }
  for (int q0 = 0; q0 < S; q0 += U) {
    v4f l[U][RPT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < RPT; ++i)
        l[u][i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(wrs, off[i], (uint32_t)((q0 + u) * p.split_stride * 4), CPOL_SC1));
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < RPT; ++i) a[i] += l[u][i];
  }
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    if (off[i] == far) continue;
    const int m = rb + (tid >> 6) + 8 * i;
    float4* dst = (float4*)(p.sk_out + (int64_t)m * p.sk_ldo + n);
    const v4f prev = p.sk_acc ? __builtin_bit_cast(v4f, *dst) : v4f{0.f, 0.f, 0.f, 0.f};
    *dst = __builtin_bit_cast(float4, prev + a[i]);
  }
}

// In-launch split-K reduction (GemmParams::sk_*), after this split's slab is stored write-through.
// The hand-off is the sc1 form of the agent-scope publish: every storing wave drains, one lane adds
// to the tile's arrival counter, one lane polls it relaxed (s_sleep between polls, bounded), and
// every slab byte is then read with sc1 loads, so no release / acquire fence (a release writes back
// the XCD's whole L2). Unlike the split tail's last-arriver gather, every split reduces 1/S of the
// tile: each workgroup reads 256 KiB in total whatever S is, instead of one workgroup reading S x
// 256 KiB. The second counter re-arms both once every split has finished reading.
PVR_DEV void splitk_fixup(const GemmParams& p, char* smem, int tile, int m0, int n0) {
  typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));
  const int S = gridDim.z, z = blockIdx.z, tid = threadIdx.x;
  unsigned* arrive = p.sk_cnt + 2 * tile;
  unsigned* done = arrive + 1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave, before the barrier
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)S) {
      __builtin_amdgcn_s_sleep(4);
      if (++spins == (1u << 24)) {  // ~1 s: a split never arrived (not co-resident); give up
        __hip_atomic_fetch_add(p.sk_cnt + 2 * p.sk_cnt_tiles, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the poll
  const __amdgpu_buffer_rsrc_t wrs = make_rsrc(p.C, (uint32_t)(p.split_stride * 4 * S));
  const int r0 = 256 * z / S, nrow = 256 * (z + 1) / S - r0;
  const int rpt = (nrow + 7) / 8;  // rows per thread
  if (rpt <= 1) splitk_rows<1, 16>(p, wrs, S, m0 + r0, nrow, n0, tid);
  else if (rpt <= 2) splitk_rows<2, 8>(p, wrs, S, m0 + r0, nrow, n0, tid);
  else if (rpt <= 4) splitk_rows<4, 4>(p, wrs, S, m0 + r0, nrow, n0, tid);
  else if (rpt <= 8) splitk_rows<8, 2>(p, wrs, S, m0 + r0, nrow, n0, tid);
  else splitk_rows<16, 1>(p, wrs, S, m0 + r0, nrow, n0, tid);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)(S - 1)) {  // every split has read: re-arm for the next launch
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  (void)smem;
}

template <bool AK, bool BKC, bool SWAP, int EPI, int ES = 2, int FA = 0, int FB = 0>
__global__ void __launch_bounds__(512, 2) gemm_pp_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // group = wm

  const int ntm = (p.M + 255) / 256, ntn = (p.N + 255) / 256;
  constexpr int BKE = 128 / ES;  // K-tile depth in elements (64 bf16 / 128 fp8)
  PVR_ASSERT(blockDim.x == 512);
  PVR_ASSERT(ES == 2 || (p.K % 128 == 0 && p.scale_a && p.scale_b));
  // Tile and K range of this workgroup. Plain grid: one whole tile per workgroup (split-K over
  // blockIdx.z for the weight gradients). Split tail (tail_split > 1): workgroups < tail_from own
  // one whole tile each; the rest are K-parts of the tail tiles, the parts of one tile on
  // consecutive remapped ids (usually one XCD; a locality hint only, some tiles straddle two XCDs:
  // the sc1 partial stores / loads and the agent-scope arrival counter make the hand-off correct).
  int tt, kbeg, kend, tloc = 0, tpart = -1;
  const TailPlan tp{p.tail_from, p.tail_split};
  PVR_ASSERT((int)blockIdx.x < tail_grid(tp, ntm * ntn));
  const TailUnit tu = tail_unit_c(tp, ntm * ntn, (int)blockIdx.x);
  tt = tu.tile;
  if (tu.part >= 0) {
    tpart = tu.part;
    tloc = tt - p.tail_from;
    const int nkt = p.K / BKE;  // k-contiguous operands: K % BKE == 0 (host check)
    kbeg = tail_kbeg(tpart, p.tail_split, nkt) * BKE;
    kend = tail_kbeg(tpart + 1, p.tail_split, nkt) * BKE;
  } else {
    kbeg = blockIdx.z * p.k_split_len;
    kend = min(p.K, kbeg + p.k_split_len);
  }
  const int m0 = (tt / ntn) * 256, n0 = (tt % ntn) * 256;
  const int nk = (kend - kbeg + BKE - 1) / BKE;  // k-contiguous operands: K % BKE == 0 (host check)
  PVR_ASSERT(!(AK || BKC) || (p.K % BKE == 0 && kbeg % BKE == 0));

  const void* abase;
  uint32_t abytes;
  if constexpr (ES == 1 && !AK) {  // fp8 mn-contiguous [K][M] bytes: rows past kend, columns past M read 0
    const uint8_t* a8 = (const uint8_t*)p.A;
    abase = a8 + (int64_t)kbeg * p.lda + m0;
    abytes = rsrc_bytes((int64_t)(kend - 1) * p.lda + p.M, (int64_t)kbeg * p.lda + m0) / 2;
  } else if constexpr (ES == 1) {
    const uint8_t* a8 = (const uint8_t*)p.A;
    abase = a8 + (int64_t)m0 * p.lda + kbeg;
    abytes = rsrc_bytes((int64_t)(p.M - 1) * p.lda + p.K, (int64_t)m0 * p.lda + kbeg) / 2;
  } else if constexpr (AK) {
    abase = p.A + (int64_t)m0 * p.lda + kbeg;
    abytes = rsrc_bytes((int64_t)(p.M - 1) * p.lda + p.K, (int64_t)m0 * p.lda + kbeg);
  } else {  // rows past K and columns past M read as zero (range check of the last row)
    abase = p.A + (int64_t)kbeg * p.lda + m0;
    abytes = rsrc_bytes((int64_t)(kend - 1) * p.lda + p.M, (int64_t)kbeg * p.lda + m0);
  }
  const void* bbase;
  uint32_t bbytes;
  if constexpr (ES == 1 && !BKC) {
    const uint8_t* b8 = (const uint8_t*)p.B;
    bbase = b8 + (int64_t)kbeg * p.ldb + n0;
    bbytes = rsrc_bytes((int64_t)(kend - 1) * p.ldb + p.N, (int64_t)kbeg * p.ldb + n0) / 2;
  } else if constexpr (ES == 1) {
    const uint8_t* b8 = (const uint8_t*)p.B;
    bbase = b8 + (int64_t)n0 * p.ldb + kbeg;
    bbytes = rsrc_bytes((int64_t)(p.N - 1) * p.ldb + p.K, (int64_t)n0 * p.ldb + kbeg) / 2;
  } else if constexpr (BKC) {
    bbase = p.B + (int64_t)n0 * p.ldb + kbeg;
    bbytes = rsrc_bytes((int64_t)(p.N - 1) * p.ldb + p.K, (int64_t)n0 * p.ldb + kbeg);
  } else {
    bbase = p.B + (int64_t)kbeg * p.ldb + n0;
    bbytes = rsrc_bytes((int64_t)(kend - 1) * p.ldb + p.N, (int64_t)kbeg * p.ldb + n0);
  }
  const __amdgpu_buffer_rsrc_t ars = make_rsrc(abase, abytes);
  const __amdgpu_buffer_rsrc_t brs = make_rsrc(bbase, bbytes);
  const __amdgpu_buffer_rsrc_t nul = make_rsrc(abase, 0);

  v4f acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s af[4][2], bf[2][2][2];
  PpStamps pst;

  stamp(p, 0);
  // prologue: half-tiles 0..5 = all of K-tile 0, A0/B0 of K-tile 1
  pp_issue<0, AK, BKC, ES>(ars, brs, nul, smem, p.lda, p.ldb, 0, nk, wave, lane);
  pp_issue<1, AK, BKC, ES>(ars, brs, nul, smem, p.lda, p.ldb, 0, nk, wave, lane);
  pp_issue<2, AK, BKC, ES>(ars, brs, nul, smem, p.lda, p.ldb, 0, nk, wave, lane);
  pp_issue<3, AK, BKC, ES>(ars, brs, nul, smem, p.lda, p.ldb, 0, nk, wave, lane);
  pp_issue<0, AK, BKC, ES>(ars, brs, nul, smem, p.lda, p.ldb, 1, nk, wave, lane);
  pp_issue<1, AK, BKC, ES>(ars, brs, nul, smem, p.lda, p.ldb, 1, nk, wave, lane);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A0, B0 of K-tile 0 landed
  pp_barrier();
  if (wm == 1) pp_barrier();  // group 1 runs one barrier behind
  stamp(p, 1);
  pst.begin();
#ifdef PVR_GEMM_PHASE_STAMPS
  const uint64_t pst0 = pst.last;
#endif

  // A0 read-ahead (PVR_PP_PRE): K-tile 0's first k-step A0 fragments now (landed: vmcnt(8) above)
  constexpr int PRE = (PVR_PP_PRE && AK && ES == 2) ? 1 : 0;
  v8s pre[4];
  if constexpr (PRE) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) pre[ii] = read_frag<256, true>(smem, wm * 128 + 16 * ii, 0, lane);
  }
  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * PP_BUF;
    const char* nbuf = smem + ((t + 1) & 1) * PP_BUF;  // (the last K-tile's read-ahead reads dead data)
    // phase P = 4t + ph issues half-tile P + 6 = 4(t+1) + ph + 2
    pp_phase<0, 0, 1, 1, 2, AK, BKC, SWAP, ES, FA, FB, PRE>(acc, af, bf, pre, buf, nbuf, ars, brs, nul, smem, p.lda, p.ldb, t + 1, nk, wave, lane, wm, wn, pst);
    pp_phase<0, 1, 0, 1, 3, AK, BKC, SWAP, ES, FA, FB>(acc, af, bf, pre, buf, nbuf, ars, brs, nul, smem, p.lda, p.ldb, t + 1, nk, wave, lane, wm, wn, pst);
    pp_phase<1, 1, 1, 0, 0, AK, BKC, SWAP, ES, FA, FB>(acc, af, bf, pre, buf, nbuf, ars, brs, nul, smem, p.lda, p.ldb, t + 2, nk, wave, lane, wm, wn, pst);
    pp_phase<1, 0, 0, 0, 1, AK, BKC, SWAP, ES, FA, FB, 2 * PRE>(acc, af, bf, pre, buf, nbuf, ars, brs, nul, smem, p.lda, p.ldb, t + 2, nk, wave, lane, wm, wn, pst);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // null stages too: no LDS-DMA may outlive the workgroup
  if (wm == 0) pp_barrier();  // equal barrier counts for both groups
  stamp(p, 2);
#ifdef PVR_GEMM_PHASE_STAMPS
  pst.acc[7] = __builtin_amdgcn_s_memtime() - pst0;
  if (p.dbg && lane == 0) {
    const int64_t b = blockIdx.x + (int64_t)gridDim.x * blockIdx.z;
#pragma unroll
    for (int k = 0; k < 8; ++k) p.dbg[(b * 8 + wave) * 8 + k] = pst.acc[k];
  }
#endif
  if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_DGELU) {
    if (tpart >= 0 && !tail_gather(p, acc, smem, tloc, tpart)) return;  // another part finishes the tile
  }
  if constexpr (SWAP && (EPI == EPI_F32_ATOMIC || EPI == EPI_F32_STORE)) {
    if ((p.N & 3) == 0 && !p.row_group)
      epilogue_staged<EPI, 128, false>(p, acc, smem, m0, n0, wm, wn, lane);
    else
      epilogue<8, 4, SWAP, EPI>(p, acc, m0 + wm * 128, n0 + wn * 64, lane);
    if constexpr (EPI == EPI_F32_STORE) {
      if (p.sk_out) splitk_fixup(p, smem, tt, m0, n0);  // host: staged path (N % 4 == 0, no row groups)
    }
  } else if constexpr (SWAP && (EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_DGELU)) {
    if (!p.epi_staged && direct_ok(p)) {
      // (one instance per epilogue actually reachable: a residual exists for BF16 only; a second,
      // identical GELU / dGELU copy doubled the kernel's code, and its hot path's I-cache footprint)
      if (EPI == EPI_BF16 && p.resid)
        epilogue_direct<EPI, EPI == EPI_BF16, ES == 1>(p, acc, smem, m0 + wm * 128, n0 + wn * 64, wm, wn, lane);
      else
        epilogue_direct<EPI, false, ES == 1>(p, acc, smem, m0 + wm * 128, n0 + wn * 64, wm, wn, lane);
    } else if (!p.addend && !p.row_group && (p.N & 3) == 0) {
      if (EPI == EPI_BF16 && p.resid)
        epilogue_staged<EPI, 128, EPI == EPI_BF16>(p, acc, smem, m0, n0, wm, wn, lane);
      else
        epilogue_staged<EPI, 128, false>(p, acc, smem, m0, n0, wm, wn, lane);
    }
    else
      epilogue<8, 4, SWAP, EPI>(p, acc, m0 + wm * 128, n0 + wn * 64, lane);
  } else {
    epilogue<8, 4, SWAP, EPI>(p, acc, m0 + wm * 128, n0 + wn * 64, lane);
  }
  if (p.dbg) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp(p, 3);
}

// compute units of the current device (cached per device)
int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    hipDeviceProp_t prop;
    const int n = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 0;
    cache[dev] = n > 0 ? n : 256;
  }
  return cache[dev];
}

// Split of the last, partial dispatch round into K-parts (GemmParams::tail_*). A 256x256 tile owns a
// CU for its whole K loop, so with R full rounds and r < CUs tiles left over the last round runs r
// tiles on CUs / r times fewer CUs than it could: e.g. the N = 768 GEMMs of ViT-B/16 at batch 256
// (591 tiles) spend 3 tile-times on 2.31 rounds of work. Splitting each leftover tile's K loop into
// S parts puts S*r <= CUs workgroups on the last round, at the price of an fp32 partial-tile
// exchange (256 KiB written per part, S x 256 KiB read by the last). That exchange runs at a
// workgroup's own bandwidth (~60-120 GB/s), i.e. ~10 us per tail tile, so the split only pays where a
// tile's K loop is long: each part keeps >= 12 K-tiles (K >= 2304 at S = 3) and S <= 4. Measured on
// ViT-B/16 b256 (profiles/r4/tail_ab.md): the K = 768 GEMMs lost 20-35 us with 3 x 4-K-tile parts.
void plan_tail(GemmParams& q, int ntiles, int bke) {
  q.tail_from = 0;
  q.tail_split = 0;
  if (!q.tail_ws || !q.tail_cnt) return;
  const TailPlan t = plan_tail_c(ntiles, q.K / bke, device_cus(), q.tail_ws_elems, q.tail_cnt_elems, q.tail_max_units,
                                    q.tail_min_kt > 0 ? q.tail_min_kt : 12);
  q.tail_from = t.from;
  q.tail_split = t.split;
}

template <bool AK, bool BKC, bool SWAP, int EPI, int ES = 2, int FA = 0, int FB = 0>
hipError_t launch_pp(const GemmParams& p, hipStream_t s) {
  constexpr int SMEM = 2 * PP_BUF;
  auto kern = gemm_pp_kernel<AK, BKC, SWAP, EPI, ES, FA, FB>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int ntm = (p.M + 255) / 256, ntn = (p.N + 255) / 256;
  const int nsplit = (p.K + p.k_split_len - 1) / p.k_split_len;
  GemmParams q = p;
  q.tail_from = q.tail_split = 0;
  int grid = ntm * ntn;
  if constexpr (AK && BKC && (EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_DGELU)) {
    if (nsplit == 1) {
      plan_tail(q, ntm * ntn, 128 / ES);
      grid = tail_grid(TailPlan{q.tail_from, q.tail_split}, ntm * ntn);
    }
  }
  hipLaunchKernelGGL(kern, dim3(grid, 1, nsplit), dim3(512), SMEM, s, q);
  return hipGetLastError();
}

// ===================================================================================== persistent ping-pong
// One resident 8-wave workgroup per CU walks tiles v = blockIdx.x, +gridDim.x, ... (XCD-remapped as
// above). The half-tile LDS-DMA stream is continuous across a workgroup's tiles: the last phases
// of tile i already stage K-tiles 0 and 1 of tile i+1 into the two buffers, so the next tile starts
// with its operands landed and its prologue latency is hidden under tile i's tail and epilogue.
// The epilogue stages through a separate 32 KiB LDS region (8 passes of 32 rows) so it never
// touches the K-tile buffers the in-flight DMAs are writing. k-contiguous bf16 operands, K >= 128.
template <int ES = 2>
PVR_DEV void ppp_issue_kind(int kind, __amdgpu_buffer_rsrc_t ars, __amdgpu_buffer_rsrc_t brs, char* buf, int64_t lda, int64_t ldb,
                            int kb, int wave, int lane) {
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int d = wave + 8 * x;
    if (kind == 0 || kind == 3) {
      const int hh = kind == 3;
      const int rowb = (2 * (d >> 3) + hh) * 64 + (d & 7) * 8;
      const int row = rowb + (lane >> 3);
      const int c = (lane & 7) ^ swz_k(row);
      dma16(ars, to_lds(buf + rowb * 128), (uint32_t)(row * lda * ES + kb + c * 16));
    } else {
      const int hh = kind == 2;
      const int rowb = (2 * (d >> 2) + hh) * 32 + (d & 3) * 8;
      const int row = rowb + (lane >> 3);
      const int c = (lane & 7) ^ swz_k(row);
      dma16(brs, to_lds(buf + 256 * 128 + rowb * 128), (uint32_t)(row * ldb * ES + kb + c * 16));
    }
  }
}

struct PppTile {
  int m0, n0;
  __amdgpu_buffer_rsrc_t ars, brs;
};

template <int ES = 2>
PVR_DEV PppTile ppp_tile(const GemmParams& p, int v, int ntiles, int ntn) {
  PppTile t;
  if (v >= ntiles) {  // past this workgroup's last tile: every DMA reads as out of range
    t.m0 = t.n0 = 0;
    t.ars = make_rsrc(p.A, 0);
    t.brs = make_rsrc(p.B, 0);
    return t;
  }
  const int tt = xcd_remap(v, ntiles);
  t.m0 = (tt / ntn) * 256;
  t.n0 = (tt % ntn) * 256;
  if constexpr (ES == 1) {  // fp8: lda / ldb / K in bytes (rsrc_bytes counts 2-B elements)
    t.ars = make_rsrc((const uint8_t*)p.A + (int64_t)t.m0 * p.lda, rsrc_bytes((int64_t)(p.M - 1) * p.lda + p.K, (int64_t)t.m0 * p.lda) / 2);
    t.brs = make_rsrc((const uint8_t*)p.B + (int64_t)t.n0 * p.ldb, rsrc_bytes((int64_t)(p.N - 1) * p.ldb + p.K, (int64_t)t.n0 * p.ldb) / 2);
  } else {
    t.ars = make_rsrc(p.A + (int64_t)t.m0 * p.lda, rsrc_bytes((int64_t)(p.M - 1) * p.lda + p.K, (int64_t)t.m0 * p.lda));
    t.brs = make_rsrc(p.B + (int64_t)t.n0 * p.ldb, rsrc_bytes((int64_t)(p.N - 1) * p.ldb + p.K, (int64_t)t.n0 * p.ldb));
  }
  return t;
}

// Phase of the continuous stream: reads / MFMAs of K-tile (current buffer) and the DMA of global
// half-tile `h_issue`, which belongs to this tile (K-tile kt_i) or to the next one.
// PR: the A0 read-ahead of pp_phase (bf16 only); the next K-tile's buffer is the other one, also
// across a tile boundary (the K-tile stream is continuous).
template <int QM, int QN, int RD_A, int RD_B, bool SWAP, int VM = 8, int ES = 2, int FA = 0, int FB = 0, int PR = 0>
PVR_DEV void ppp_phase(v4f (&acc)[8][4], v8s (&af)[4][2], v8s (&bf)[2][2][2], v8s (&pre)[4], const char* buf, char* smem,
                       const PppTile& cur, const PppTile& nxt, int G_issue, int kind, int tile_first_G, int nk, const GemmParams& p,
                       int wave, int lane, int wm, int wn) {
  static_assert(PR == 0 || ES == 2, "A0 read-ahead: bf16 only");
  if constexpr (RD_A) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        af[ii][ks] = ES == 1 ? frag_fp8(buf, wm * 128 + QM * 64 + 16 * ii, ks, lane)
                     : (PR == 1 && ks == 0) ? pre[ii]
                                            : read_frag<256, true>(buf, wm * 128 + QM * 64 + 16 * ii, ks, lane);
  }
  if constexpr (PR == 2) {
    const char* nbuf = smem + (((buf - smem) / PP_BUF) ^ 1) * PP_BUF;
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) pre[ii] = read_frag<256, true>(nbuf, wm * 128 + 16 * ii, 0, lane);
  }
  if constexpr (RD_B) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        bf[QN][jj][ks] = ES == 1 ? frag_fp8(buf + 256 * 128, wn * 64 + QN * 32 + 16 * jj, ks, lane)
                                 : read_frag<256, true>(buf + 256 * 128, wn * 64 + QN * 32 + 16 * jj, ks, lane);
  }
  {
    const int rel = G_issue - tile_first_G;  // K-tile index relative to the current tile
    const bool same = rel < nk;
    const PppTile& t = same ? cur : nxt;
    const int kt = same ? rel : rel - nk;
    ppp_issue_kind<ES>(kind, t.ars, t.brs, smem + (G_issue & 1) * PP_BUF, p.lda, p.ldb, kt * 128, wave, lane);
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
  pp_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_setprio(1);
  if constexpr (ES == 1) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        v4f& c = acc[QM * 4 + ii][QN * 2 + jj];
        if constexpr (SWAP)
          c = mfma_fp8<FB, FA>(bf[QN][jj][0], bf[QN][jj][1], af[ii][0], af[ii][1], c);
        else
          c = mfma_fp8<FA, FB>(af[ii][0], af[ii][1], bf[QN][jj][0], bf[QN][jj][1], c);
      }
    __builtin_amdgcn_s_setprio(0);
    pp_barrier();
    return;
  }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        v4f& c = acc[QM * 4 + ii][QN * 2 + jj];
        if constexpr (SWAP)
          c = mfma16(bf[QN][jj][ks], af[ii][ks], c);
        else
          c = mfma16(af[ii][ks], bf[QN][jj][ks], c);
      }
  __builtin_amdgcn_s_setprio(0);
  pp_barrier();
}

// ES = 1: fp8 operands (register-direct epilogue only; the GELU epilogue's e4m3 copy adds 16 stores
// per wave beyond INFL, which only makes the counted waits retire more of them: still correct)
template <bool SWAP, int EPI, bool DIRECT, int ES = 2, int FA = 0, int FB = 0>
__global__ void __launch_bounds__(512, 2) gemm_ppp_kernel(GemmParams p) {
  static_assert(ES == 2 || DIRECT, "fp8 persistent GEMM: register-direct epilogue");
  // epilogue stores per wave left in flight across the tile boundary (0: drain): the register-direct
  // BF16 epilogue issues 16 x 16 B, GELU 32 (output + derivative), dGELU 16 + 8 column-sum atomics
  // (to a 0-byte resource without colsum)
  constexpr int INFL = !DIRECT ? 0 : EPI == EPI_BF16 ? 16 : EPI == EPI_GELU ? 32 : 24;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int ntm = (p.M + 255) / 256, ntn = (p.N + 255) / 256, ntiles = ntm * ntn;
  const int nk = p.K / (128 / ES);  // K-tiles of 128 B (64 bf16 / 128 fp8); >= 2 (host check)
  int v = blockIdx.x;
  if (v >= ntiles) return;

  PppTile cur = ppp_tile<ES>(p, v, ntiles, ntn);
  PppTile nxt = ppp_tile<ES>(p, v + gridDim.x, ntiles, ntn);
  // prologue of the first tile: half-tiles 0..5 (global K-tiles 0 and 1 of the stream)
  ppp_issue_kind<ES>(0, cur.ars, cur.brs, smem, p.lda, p.ldb, 0, wave, lane);
  ppp_issue_kind<ES>(1, cur.ars, cur.brs, smem, p.lda, p.ldb, 0, wave, lane);
  ppp_issue_kind<ES>(2, cur.ars, cur.brs, smem, p.lda, p.ldb, 0, wave, lane);
  ppp_issue_kind<ES>(3, cur.ars, cur.brs, smem, p.lda, p.ldb, 0, wave, lane);
  ppp_issue_kind<ES>(0, cur.ars, cur.brs, smem + PP_BUF, p.lda, p.ldb, 128, wave, lane);
  ppp_issue_kind<ES>(1, cur.ars, cur.brs, smem + PP_BUF, p.lda, p.ldb, 128, wave, lane);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  pp_barrier();
  constexpr int PRE = (PVR_PP_PRE && ES == 2) ? 1 : 0;
  v8s pre[4];  // A0 read-ahead: live across each epilogue into the next tile's first phase
  if constexpr (PRE) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) pre[ii] = read_frag<256, true>(smem, wm * 128 + 16 * ii, 0, lane);
  }

  // diagnostic stamps (p.dbg set, scripts/gemm_stamps.py --persistent): per workgroup, cycles in the
  // K loops and in the epilogues summed over its tiles, the whole kernel, and its tile count
  const bool dstamp = p.dbg != nullptr;
  const uint64_t ts0 = dstamp ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t ts_loop = 0, ts_epi = 0, ts_a = 0;
  int ntile_done = 0;
  int G0 = 0;  // global index (in this workgroup's K-tile stream) of the current tile's K-tile 0
  for (;;) {
    if (dstamp) ts_a = __builtin_amdgcn_s_memtime();
    v4f acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    v8s af[4][2], bf[2][2][2];
    if (wm == 1) pp_barrier();  // group 1 runs one barrier behind
    int kt = 0;
    if constexpr (INFL > 0) {
      if (G0 > 0) {
        // first K-tile after a register-direct epilogue: its INFL stores per wave are younger than
        // the four half-tiles this K-tile waits for, so every wait leaves them in flight (counted);
        // the first wait for a half-tile issued after them (next K-tile) retires them
        const char* buf = smem + (G0 & 1) * PP_BUF;
        ppp_phase<0, 0, 1, 1, SWAP, 8 + INFL, ES, FA, FB, PRE>(acc, af, bf, pre, buf, smem, cur, nxt, G0 + 1, 2, G0, nk, p, wave, lane, wm, wn);
        ppp_phase<0, 1, 0, 1, SWAP, 8 + INFL, ES, FA, FB>(acc, af, bf, pre, buf, smem, cur, nxt, G0 + 1, 3, G0, nk, p, wave, lane, wm, wn);
        ppp_phase<1, 1, 1, 0, SWAP, 8 + INFL, ES, FA, FB>(acc, af, bf, pre, buf, smem, cur, nxt, G0 + 2, 0, G0, nk, p, wave, lane, wm, wn);
        ppp_phase<1, 0, 0, 0, SWAP, 8 + INFL, ES, FA, FB, 2 * PRE>(acc, af, bf, pre, buf, smem, cur, nxt, G0 + 2, 1, G0, nk, p, wave, lane, wm, wn);
        kt = 1;
      }
    }
    for (; kt < nk; ++kt) {
      const int G = G0 + kt;
      const char* buf = smem + (G & 1) * PP_BUF;
      ppp_phase<0, 0, 1, 1, SWAP, 8, ES, FA, FB, PRE>(acc, af, bf, pre, buf, smem, cur, nxt, G + 1, 2, G0, nk, p, wave, lane, wm, wn);
      ppp_phase<0, 1, 0, 1, SWAP, 8, ES, FA, FB>(acc, af, bf, pre, buf, smem, cur, nxt, G + 1, 3, G0, nk, p, wave, lane, wm, wn);
      ppp_phase<1, 1, 1, 0, SWAP, 8, ES, FA, FB>(acc, af, bf, pre, buf, smem, cur, nxt, G + 2, 0, G0, nk, p, wave, lane, wm, wn);
      ppp_phase<1, 0, 0, 0, SWAP, 8, ES, FA, FB, 2 * PRE>(acc, af, bf, pre, buf, smem, cur, nxt, G + 2, 1, G0, nk, p, wave, lane, wm, wn);
    }
    if (wm == 0) pp_barrier();  // re-align the groups for the epilogue
    uint64_t ts_b = 0;
    if (dstamp) {
      ts_b = __builtin_amdgcn_s_memtime();
      ts_loop += ts_b - ts_a;
    }
    // The next tile's first DMAs are in flight into the K-tile buffers; the epilogue works from
    // registers (DIRECT; the DGELU column-sum exchange uses the separate region) or stages in the
    // separate region behind them.
    if constexpr (DIRECT) {
      if (EPI == EPI_BF16 && p.resid)  // (see gemm_pp_kernel: one instance per reachable epilogue)
        epilogue_direct<EPI, EPI == EPI_BF16, ES == 1>(p, acc, smem + 2 * PP_BUF, cur.m0 + wm * 128, cur.n0 + wn * 64, wm, wn, lane);
      else
        epilogue_direct<EPI, false, ES == 1>(p, acc, smem + 2 * PP_BUF, cur.m0 + wm * 128, cur.n0 + wn * 64, wm, wn, lane);
    } else if constexpr (ES == 2) {
      if (EPI == EPI_BF16 && p.resid)
        epilogue_staged<EPI, 32, EPI == EPI_BF16>(p, acc, smem + 2 * PP_BUF, cur.m0, cur.n0, wm, wn, lane);
      else
        epilogue_staged<EPI, 32, false>(p, acc, smem + 2 * PP_BUF, cur.m0, cur.n0, wm, wn, lane);
    }
    if (dstamp) {
      ts_epi += __builtin_amdgcn_s_memtime() - ts_b;
      ++ntile_done;
    }
    v += gridDim.x;
    if (v >= ntiles) break;
    G0 += nk;
    cur = nxt;
    nxt = ppp_tile<ES>(p, v + gridDim.x, ntiles, ntn);
    if constexpr (INFL == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain (stores + the K-tiles already issued)
      __syncthreads();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
  if (dstamp && threadIdx.x == 0) {
    uint64_t* d = p.dbg + (int64_t)blockIdx.x * 8;
    d[0] = __builtin_amdgcn_s_memtime() - ts0;
    d[1] = ts_loop;
    d[2] = ts_epi;
    d[3] = (uint64_t)ntile_done;
  }
}

template <bool SWAP, int EPI, int ES = 2, int FA = 0, int FB = 0>
hipError_t launch_ppp(const GemmParams& p, hipStream_t s) {
  constexpr int SMEM = 2 * PP_BUF + 32 * 1024;
  auto kd = gemm_ppp_kernel<SWAP, EPI, true, ES, FA, FB>;
  auto ks = gemm_ppp_kernel<SWAP, EPI, ES == 1, ES, FA, FB>;  // fp8: the direct form only
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kd, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    if (e == hipSuccess) e = hipFuncSetAttribute((const void*)ks, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const bool direct = !p.epi_staged && direct_ok(p);
  if (ES == 1 && !direct) return hipErrorInvalidValue;  // caller checks (fp8_persistent_ok)
  auto kern = direct ? kd : ks;
  const int ntiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  const int cus = device_cus();
  const int grid = ntiles < cus ? ntiles : cus;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), SMEM, s, p);
  return hipGetLastError();
}

// Tile configs (ops/gemm.py `_tile`): 0 = 128x128 (small GEMMs), 6 = 256x256 BK-32 ring (K % 64 != 0),
// 12 = 256x256 8-wave ping-pong (one tile per workgroup, split-K tail), 13 = its persistent form.
template <bool AK, bool BKC, bool SWAP, int EPI>
hipError_t launch_tile(const GemmParams& p, hipStream_t s) {
  switch (p.tile_cfg) {
    case 6: return launch_v3<256, 256, 2, 4, 4, 2, AK, BKC, SWAP, EPI>(p, s);
    case 13:  // persistent ping-pong (k-contiguous bf16, bf16-output epilogues, no split-K)
      if constexpr (AK && BKC && SWAP && (EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_DGELU)) {
        if (p.K % PP_BK == 0 && p.K >= 2 * PP_BK && p.k_split_len >= p.K && !p.addend && !p.row_group && (p.N & 3) == 0)
          return launch_ppp<SWAP, EPI>(p, s);
      }
      [[fallthrough]];
    case 12:
      // k-contiguous pair (fwd / dgrad with W^T), mn pair (wgrad) or k-contiguous A with an
      // mn-contiguous B (dgrad straight from W, transposed B reads)
      if constexpr (AK || !BKC) {
        if ((!AK || (p.K % PP_BK == 0 && p.k_split_len % PP_BK == 0)) && (AK || p.k_split_len % PP_BK == 0))
          return launch_pp<AK, BKC, SWAP, EPI>(p, s);
      }
      return launch_v3<256, 256, 2, 4, 4, 2, AK, BKC, SWAP, EPI>(p, s);
    default: return launch_cfg<128, 128, 2, 2, AK, BKC, SWAP, EPI>(p, s);
  }
}

}  // namespace

}  // namespace pvr

// The split-K tail plan a one-tile-per-workgroup GEMM of this shape gets (0: none): tests / tools.
extern "C" int pvr_gemm_tail_split(int M, int N, int K, int elem_bytes, int max_units) {
  pvr::GemmParams q{};
  q.K = K;
  q.tail_max_units = max_units;
  q.tail_ws = reinterpret_cast<float*>(16);  // any non-null: plan only
  q.tail_cnt = reinterpret_cast<unsigned*>(16);
  q.tail_ws_elems = (int64_t)pvr::device_cus() * 65536;
  q.tail_cnt_elems = pvr::device_cus();
  pvr::plan_tail(q, ((M + 255) / 256) * ((N + 255) / 256), elem_bytes == 1 ? 128 : 64);
  return q.tail_split;
}

// fp8 forward / dgrad GEMMs on the persistent ping-pong (see pvr_gemm): 1 = when the epilogue has
// no per-row input (default), 0 = never (A/B of the two production forms; the residual and dGELU
// epilogues lost on the persistent form and stay one tile per workgroup: profiles/r4/g8b, g8c)
static int g_fp8_persistent = 1;
extern "C" void pvr_set_fp8_persistent(int mode) { g_fp8_persistent = mode ? 1 : 0; }

extern "C" int pvr_gemm_ws_ok(const pvr::GemmParams* pp, int cus);
extern "C" hipError_t pvr_gemm_ws(const pvr::GemmParams* pp, int cus, hipStream_t s);

// 1 if tile config 15 (the wave-specialized kernel, gemm_ws.hip) runs this GEMM as given
extern "C" int pvr_gemm_ws_takes(const pvr::GemmParams* pp) { return pvr_gemm_ws_ok(pp, pvr::device_cus()); }

// Host entry. Returns hipSuccess, or hipErrorInvalidValue for an unsupported layout/epilogue pair.
extern "C" hipError_t pvr_gemm(const pvr::GemmParams* pp, hipStream_t s) {
  using namespace pvr;
  const GemmParams& p = *pp;
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return hipSuccess;
  // tile 15: wave-specialized persistent kernel (epilogue waves beside the MFMA waves); shapes it
  // does not take fall through to the 256x256 ping-pong
  if (p.tile_cfg == 15) {
    if (pvr_gemm_ws_ok(pp, device_cus())) return pvr_gemm_ws(pp, device_cus(), s);
    GemmParams q = p;
    q.tile_cfg = 13;
    return pvr_gemm(&q, s);
  }
  const bool ak = p.a_kcontig, bk = p.b_kcontig;
  if (p.elem8) {  // fp8 operands: k-contiguous ping-pong only (forward e4m3 x e4m3, dgrad / wgrad e5m2 or e4m3 x e4m3)
    const int f = p.fmt_a * 2 + p.fmt_b;
    if ((p.N & 3) || !p.scale_a || !p.scale_b) return hipErrorInvalidValue;
    if (!ak && !bk) {
      // weight gradient straight from the row-major fp8 copies ([tokens][features], mn-contiguous,
      // transposed LDS reads): split-K over the tokens, per-split partials (tile 14); 16-B rows
      if (p.epi != EPI_F32_STORE || p.tile_cfg != 14 || p.k_split_len % 128 != 0 || (f != 2 && f != 0) || (p.M & 15) ||
          (p.N & 15) || (p.lda & 15) || (p.ldb & 15))
        return hipErrorInvalidValue;
      if (f == 0) return launch_pp<false, false, true, EPI_F32_STORE, 1, 0, 0>(p, s);  // e4m3 gradients
      return launch_pp<false, false, true, EPI_F32_STORE, 1, 1, 0>(p, s);
    }
    if (!ak || !bk || p.K % 128 != 0) return hipErrorInvalidValue;
    if (p.epi == EPI_F32_STORE) {
      // weight gradient: split-K over the (128-padded) token dim, per-split partials (tile 14)
      if (p.tile_cfg != 14 || p.k_split_len % 128 != 0 || (f != 2 && f != 0)) return hipErrorInvalidValue;
      if (f == 0) return launch_pp<true, true, true, EPI_F32_STORE, 1, 0, 0>(p, s);
      return launch_pp<true, true, true, EPI_F32_STORE, 1, 1, 0>(p, s);
    }
    if (p.k_split_len < p.K) return hipErrorInvalidValue;
    // persistent form (tile 13) when there are >= 4 output tiles per CU, the K loop is short
    // (<= 16 K-tiles: the next tile's prologue / this tile's epilogue are a large share of a tile)
    // and the register-direct epilogue applies (epilogues without per-row inputs; g_fp8_persistent
    // 0 = never, A/B). ViT-H/14 b256 (profiles/r4/g8b):
    // fc1 GELU fwd 0.800 -> 0.688 ms, qkv fwd 0.363 -> 0.357, out dgrad 0.126 -> 0.121; the K = 3840 /
    // 5120 GEMMs lose 3-8 % persistent and stay one tile per workgroup
    const int ntiles8 = ((p.M + 255) / 256) * ((p.N + 255) / 256);
    const bool pers = g_fp8_persistent > 0 && ntiles8 >= 4 * device_cus() && p.K >= 256 && p.K <= 2048 && !p.epi_staged &&
                      direct_ok(p) && !p.resid;
    switch (p.epi) {
      case EPI_BF16:
        if (pers && f == 0) return launch_ppp<true, EPI_BF16, 1, 0, 0>(p, s);
        if (pers && f == 2) return launch_ppp<true, EPI_BF16, 1, 1, 0>(p, s);
        if (f == 0) return launch_pp<true, true, true, EPI_BF16, 1, 0, 0>(p, s);
        if (f == 2) return launch_pp<true, true, true, EPI_BF16, 1, 1, 0>(p, s);
        break;
      case EPI_GELU:
        if (pers && f == 0) return launch_ppp<true, EPI_GELU, 1, 0, 0>(p, s);
        if (f == 0) return launch_pp<true, true, true, EPI_GELU, 1, 0, 0>(p, s);
        break;
      case EPI_DGELU:
        if (f == 0) return launch_pp<true, true, true, EPI_DGELU, 1, 0, 0>(p, s);  // e4m3 gradients
        if (f == 2) return launch_pp<true, true, true, EPI_DGELU, 1, 1, 0>(p, s);
        break;
    }
    return hipErrorInvalidValue;
  }
  switch (p.epi) {
    case EPI_BF16:
      if (ak && bk) return launch_tile<true, true, true, EPI_BF16>(p, s);
      if (ak && !bk) return launch_tile<true, false, true, EPI_BF16>(p, s);
      break;
    case EPI_GELU:
      if (ak && bk) return launch_tile<true, true, true, EPI_GELU>(p, s);
      break;
    case EPI_DGELU:
      if (ak && bk) return launch_tile<true, true, true, EPI_DGELU>(p, s);
      if (ak && !bk) return launch_tile<true, false, true, EPI_DGELU>(p, s);
      break;
    case EPI_F32_ATOMIC:
      // tile 14: ping-pong with the LDS-staged f32 epilogue (split-K wgrad)
      if (p.tile_cfg == 14 && ak == bk && p.k_split_len % PP_BK == 0 && (!ak || p.K % PP_BK == 0))
        return ak ? launch_pp<true, true, true, EPI_F32_ATOMIC>(p, s) : launch_pp<false, false, true, EPI_F32_ATOMIC>(p, s);
      if (!ak && !bk) return launch_tile<false, false, false, EPI_F32_ATOMIC>(p, s);
      if (ak && bk) return launch_tile<true, true, false, EPI_F32_ATOMIC>(p, s);
      break;
    case EPI_F32_STORE:
      // tile 14: per-split partials C + z * split_stride (split_stride 0: one K range only)
      if (p.tile_cfg == 14 && ak == bk && p.k_split_len % PP_BK == 0 && (!ak || p.K % PP_BK == 0))
        return ak ? launch_pp<true, true, true, EPI_F32_STORE>(p, s) : launch_pp<false, false, true, EPI_F32_STORE>(p, s);
      if (p.split_stride) return hipErrorInvalidValue;
      if (!ak && !bk) return launch_tile<false, false, false, EPI_F32_STORE>(p, s);
      if (ak && bk) return launch_tile<true, true, false, EPI_F32_STORE>(p, s);
      break;
  }
  return hipErrorInvalidValue;
}
