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

namespace pvr {

enum GemmEpi : int {
  EPI_BF16 = 0,        // out = resid + dropout(acc + bias + addend[row])      (bf16)
  EPI_GELU = 1,        // aux = acc + bias (pre-act, bf16); out = dropout(gelu(aux))
  EPI_DGELU = 2,       // out = acc * dropmask * gelu'(aux)                       (bf16)
  EPI_F32_ATOMIC = 3,  // out += acc                                             (f32 atomics)
  EPI_F32_STORE = 4,   // out = acc                                              (f32)
};

struct GemmParams {
  int M, N, K;
  const uint16_t* A; int64_t lda; int a_kcontig;
  const uint16_t* B; int64_t ldb; int b_kcontig;
  void* C; int64_t ldc;
  const float* bias;
  const uint16_t* resid; int64_t ld_resid;
  const float* addend; int addend_period;
  uint16_t* aux; int64_t ld_aux;
  int row_group, row_stride_group, row_offset;
  const uint64_t* seed_ptr; uint64_t seed_offset; uint32_t drop_thr; float drop_scale;
  int k_split_len;
  int epi;
  int tile_cfg;
};

namespace {

constexpr int TK = 64;  // K depth of one LDS stage

PVR_DEV int swz_k(int row) { return (row >> 1) & 7; }                                // 128-B rows
PVR_DEV int swz_mn(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }  // 16-B chunk XOR

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

PVR_DEV uint32_t rsrc_bytes(int64_t extent_elems, int64_t base_elems) {
  int64_t b = (extent_elems - base_elems) * 2;
  if (b < 0) b = 0;
  if (b > 0xFFFFFFFFll) b = 0xFFFFFFFFll;
  return (uint32_t)b;
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

  if (nk > 0) {
    stage_tile<BM, AK, NW>(ars, smem, p.lda, 0, wave, lane);
    stage_tile<BN, BKC, NW>(brs, smem + A_BYTES, p.ldb, 0, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
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

  // ------------------------------------------------------------------ epilogue
  const int g = lane >> 4, li = lane & 15;
  if constexpr (SWAP) {
    // lane holds C[m = .. + li][n = .. + 4g + r], r = 0..3 (4 consecutive columns)
    const uint64_t seed = (p.drop_thr ? *p.seed_ptr : 0ull) + p.seed_offset;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * WTM + 16 * i + li;
      if (m >= p.M) continue;
      int64_t orow = m;
      if (p.row_group) orow = (int64_t)(m / p.row_group) * p.row_stride_group + p.row_offset + m % p.row_group;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + 16 * j + 4 * g;
        if (n >= p.N) continue;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
          if (p.bias) {
            const float4 bb = *(const float4*)(p.bias + n);
            v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
          }
        }
        if constexpr (EPI == EPI_BF16) {
          if (p.addend) {
            const float4 ad = *(const float4*)(p.addend + (orow % p.addend_period) * p.N + n);
            v[0] += ad.x; v[1] += ad.y; v[2] += ad.z; v[3] += ad.w;
          }
          if (p.drop_thr) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              v[r] = rng_keep(seed, (uint64_t)orow * p.N + n + r, p.drop_thr) ? v[r] * p.drop_scale : 0.f;
          }
          if (p.resid) {
            const uint2 rr = *(const uint2*)(p.resid + (int64_t)m * p.ld_resid + n);
            v[0] += bf2f(rr.x & 0xFFFF); v[1] += bf2f(rr.x >> 16);
            v[2] += bf2f(rr.y & 0xFFFF); v[3] += bf2f(rr.y >> 16);
          }
          uint2 o; o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
          *(uint2*)((uint16_t*)p.C + orow * p.ldc + n) = o;
        } else if constexpr (EPI == EPI_GELU) {
          uint2 u; u.x = pack2bf(v[0], v[1]); u.y = pack2bf(v[2], v[3]);
          *(uint2*)(p.aux + (int64_t)m * p.ld_aux + n) = u;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float h = gelu_erf(v[r]);
            if (p.drop_thr) h = rng_keep(seed, (uint64_t)orow * p.N + n + r, p.drop_thr) ? h * p.drop_scale : 0.f;
            v[r] = h;
          }
          uint2 o; o.x = pack2bf(v[0], v[1]); o.y = pack2bf(v[2], v[3]);
          *(uint2*)((uint16_t*)p.C + orow * p.ldc + n) = o;
        } else if constexpr (EPI == EPI_DGELU) {
          const uint2 uu = *(const uint2*)(p.aux + (int64_t)m * p.ld_aux + n);
          const float u[4] = {bf2f(uu.x & 0xFFFF), bf2f(uu.x >> 16), bf2f(uu.y & 0xFFFF), bf2f(uu.y >> 16)};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float d = v[r];
            if (p.drop_thr) d = rng_keep(seed, (uint64_t)orow * p.N + n + r, p.drop_thr) ? d * p.drop_scale : 0.f;
            v[r] = d * gelu_erf_grad(u[r]);
          }
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
  } else {
    // lane holds C[m = .. + 4g + r][n = .. + li]; used for f32 outputs (64-B row segments per instruction)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + 16 * j + li;
        if (n >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + 16 * i + 4 * g + r;
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

template <bool AK, bool BKC, bool SWAP, int EPI>
hipError_t launch_tile(const GemmParams& p, hipStream_t s) {
  switch (p.tile_cfg) {
    case 1: return launch_cfg<256, 128, 4, 2, AK, BKC, SWAP, EPI>(p, s);
    case 2: return launch_cfg<128, 256, 2, 4, AK, BKC, SWAP, EPI>(p, s);
    default: return launch_cfg<128, 128, 2, 2, AK, BKC, SWAP, EPI>(p, s);
  }
}

}  // namespace

}  // namespace pvr

// Host entry. Returns hipSuccess, or hipErrorInvalidValue for an unsupported layout/epilogue pair.
extern "C" hipError_t pvr_gemm(const pvr::GemmParams* pp, hipStream_t s) {
  using namespace pvr;
  const GemmParams& p = *pp;
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return hipSuccess;
  const bool ak = p.a_kcontig, bk = p.b_kcontig;
  switch (p.epi) {
    case EPI_BF16:
      if (ak && bk) return launch_tile<true, true, true, EPI_BF16>(p, s);
      if (ak && !bk) return launch_tile<true, false, true, EPI_BF16>(p, s);
      break;
    case EPI_GELU:
      if (ak && bk) return launch_tile<true, true, true, EPI_GELU>(p, s);
      break;
    case EPI_DGELU:
      if (ak && !bk) return launch_tile<true, false, true, EPI_DGELU>(p, s);
      break;
    case EPI_F32_ATOMIC:
      if (!ak && !bk) return launch_tile<false, false, false, EPI_F32_ATOMIC>(p, s);
      if (ak && bk) return launch_tile<true, true, false, EPI_F32_ATOMIC>(p, s);
      break;
    case EPI_F32_STORE:
      if (!ak && !bk) return launch_tile<false, false, false, EPI_F32_STORE>(p, s);
      if (ak && bk) return launch_tile<true, true, false, EPI_F32_STORE>(p, s);
      break;
  }
  return hipErrorInvalidValue;
}
