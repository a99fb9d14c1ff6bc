// Launch parameters of the GEMM kernels (csrc/gemm.hip), shared with the host bindings
// (bindings.cpp, compiled by g++): plain C++, no HIP headers.
#pragma once
#include <stdint.h>

namespace pvr {

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
  uint64_t* dbg;  // diagnostic s_memtime stamps [block][4] (null in normal runs)
  float* colsum;  // optional: += column sums of the bf16-type output (a fused bias gradient)
  // fp8 operands (elem8 = 1): A / B hold 1-byte OCP fp8 (fmt 0 = e4m3, 1 = e5m2), lda / ldb in
  // bytes; the accumulator is multiplied by (*scale_a) * (*scale_b) (per-tensor dequant factors)
  const float* scale_a; const float* scale_b;
  int elem8, fmt_a, fmt_b;
  // EPI_F32_STORE with split-K (tile 14): split z writes its partial to C + z * split_stride
  int64_t split_stride;
  int epi_staged;  // A/B: ping-pong bf16 epilogues through LDS (1) instead of register-direct (0)
  // optional fp8 copy of a GELU / dGELU output written by the fp8 GEMM's epilogue (the producer-side
  // quantization of the delayed-scaling recipe): q_out[m][n] = fp8(out * (*q_scale)) (fmt 0 e4m3,
  // 1 e5m2, row stride ld_q bytes), *q_amax = max(*q_amax, max |out|) (float bits, NaN-propagating)
  uint8_t* q_out; int64_t ld_q; const float* q_scale; unsigned* q_amax; int q_fmt;
  // c_skip = 1: the bf16 output is not stored (register-direct epilogue: 0-byte C resource, every
  // store dropped by the range check) - only its fp8 copy / aux / column sums are consumed
  int c_skip;
  // split-K tail of the one-tile-per-workgroup ping-pong (bf16-output epilogues): the output tiles of
  // the last, partial dispatch round (tiles >= tail_from) are computed as tail_split K-parts each;
  // every part stores its fp32 partial tile into tail_ws and the last part to arrive (per-tile
  // arrival counter in tail_cnt, zero between launches) sums them and runs the epilogue. tail_ws /
  // tail_cnt are per-stream buffers from the host (null: no tail split); tail_from / tail_split are
  // chosen by the launcher from the tile and CU counts.
  float* tail_ws; unsigned* tail_cnt; int64_t tail_ws_elems; int tail_cnt_elems;
  int tail_from, tail_split;
  // at most this many workgroups in the split round (0: no limit). The backward passes a small
  // limit: there the weight-gradient side stream's long workgroups occupy the CUs a wide split
  // round would need, and the dgrad chain then waits for them (measured -0.6 % per step).
  int tail_max_units;
  // fewest K-tiles a split part may keep (default 12: measured on the K = 768 bf16 GEMMs)
  int tail_min_kt;
  // in-launch split-K reduction of EPI_F32_STORE (weight gradients): with sk_out set, every split
  // stores its partial slab write-through, arrives on its tile's counter (sk_cnt[2 tile], zero
  // between launches), waits for the tile's other splits and then adds rows [256 z / S, 256 (z+1) / S)
  // of the tile, summed over the S slabs in order 0..S-1, into sk_out (row stride sk_ldo; sk_acc = 0:
  // overwrite). Needs every workgroup of the launch co-resident (host: tiles x splits <= CUs).
  // sk_cnt[2 * sk_cnt_tiles] counts spin timeouts (0 in a healthy run).
  float* sk_out; int64_t sk_ldo; unsigned* sk_cnt; int sk_acc; int sk_cnt_tiles;
};

}  // namespace pvr
