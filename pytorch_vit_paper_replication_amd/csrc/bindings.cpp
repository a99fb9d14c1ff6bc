#include <cstdlib>
// pybind11 / ATen bindings for the gfx950 kernels. Every entry point launches on PyTorch's current
// HIP stream (so it composes with torch streams, events and hipGraph capture) and validates dtypes,
// shapes and strides before touching device memory.
#include <algorithm>
#include <map>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "gemm_params.h"


namespace pvr {

struct AdamGroup {
  float lr, beta1, beta2, eps, weight_decay;
  float bc1, bc2_sqrt;
  int decoupled;
};
}  // namespace pvr

extern "C" {
hipError_t pvr_gemm(const pvr::GemmParams* p, hipStream_t s);
int pvr_gemm_tail_split(int M, int N, int K, int elem_bytes, int max_units);
void pvr_set_attn_fwd_qg(int qg);
void pvr_set_attn_fwd_head_qf(int qf);
void pvr_set_ln_fwd_q8_grid(int per_cu);
void pvr_set_attn_prep_xcd(int on);
void pvr_set_attn_dbg(void* p);
void pvr_set_fp8_persistent(int mode);
hipError_t pvr_layernorm_fwd(const uint16_t*, int64_t, const float*, const float*, uint16_t*, int64_t, float*, float*, int, int, float, hipStream_t);
hipError_t pvr_layernorm_fwd_q8(const uint16_t*, int64_t, const float*, const float*, uint16_t*, int64_t, uint8_t*, int64_t, const float*,
                                unsigned*, float*, float*, int, int, float, hipStream_t);
hipError_t pvr_layernorm_bwd(const uint16_t*, int64_t, const uint16_t*, int64_t, const float*, const float*, const float*, const uint16_t*, int64_t, uint16_t*, int64_t, float*, float*, float*, uint16_t*, int64_t, const uint64_t*, uint64_t, uint32_t, float, int, uint8_t*, int64_t, const float*, unsigned*, int, int, int, float*, hipStream_t);
int pvr_layernorm_bwd_blocks(int, int);
int pvr_colsum_part_rows(int);
hipError_t pvr_cast_f32_bf16(const float*, uint16_t*, int64_t, hipStream_t);
hipError_t pvr_splitk_reduce(const float*, int, int64_t, float*, int64_t, int, int, int, hipStream_t);
hipError_t pvr_pad_cols_bf16(const uint16_t*, int, int, uint16_t*, int, hipStream_t);
hipError_t pvr_transpose_batched(const uint16_t*, uint16_t*, const int64_t*, int, int, hipStream_t);
hipError_t pvr_colsum(const uint16_t*, int64_t, int, int, float*, uint16_t*, int64_t, const uint64_t*, uint64_t, uint32_t, float, uint8_t*, int64_t,
                      const float*, unsigned*, int, float*, hipStream_t);
hipError_t pvr_im2col(const float*, uint16_t*, int, int, int, int, int, int, hipStream_t);
hipError_t pvr_cls_rows(const float*, const float*, uint16_t*, int, int, int64_t, const uint64_t*, uint64_t, uint32_t, float, hipStream_t);
hipError_t pvr_patch_bwd(const uint16_t*, int, int, int, float*, float*, float*, uint16_t*, float*, const uint64_t*, uint64_t, uint32_t, float, hipStream_t);
int pvr_patch_bwd_groups(int);
int64_t pvr_patch_bwd_ws_floats(int, int, int);
hipError_t pvr_head_fwd(const uint16_t*, int64_t, int, int, const float*, const float*, float, const float*, const float*, int, float*, float*,
                        float*, hipStream_t);
hipError_t pvr_head_bwd(const float*, const float*, const float*, const float*, const float*, const float*, int, int, int, int, float*,
                        float*, float*, float*, float*, uint16_t*, float*, hipStream_t);
hipError_t pvr_scale_by(const float*, const float*, float*, int64_t, hipStream_t);
hipError_t pvr_mean(const float*, int, float*, hipStream_t);
hipError_t pvr_metrics_accum(float*, const float*, const int*, int, hipStream_t);
hipError_t pvr_rng_next(int64_t*, int64_t*, hipStream_t);
hipError_t pvr_zero_f32(float*, int64_t, hipStream_t);
hipError_t pvr_xent(const float*, int64_t, const int64_t*, int, int, float*, float*, int*, float, hipStream_t);
int pvr_norm_partial_blocks();
hipError_t pvr_grad_norm(const float*, int64_t, float, float*, float*, hipStream_t);
hipError_t pvr_adam(float*, const float*, float*, float*, uint16_t*, int64_t, const int64_t*, const int*, int, const pvr::AdamGroup*,
                    const pvr::AdamGroup*, int, const float*, int, hipStream_t);
hipError_t pvr_scale_by_clip(float*, int64_t, const float*, hipStream_t);
hipError_t pvr_adam_t(float*, const float*, float*, float*, uint16_t*, uint16_t*, const int64_t*, int, int, const int64_t*, int, int64_t,
                      const pvr::AdamGroup*, const pvr::AdamGroup*, int, const float*, int, hipStream_t);
hipError_t pvr_fp8_quant(const uint16_t*, int64_t, uint8_t*, int64_t, int64_t, int, const float*, unsigned*, int, hipStream_t);
hipError_t pvr_fp8_dequant(const uint8_t*, float*, int64_t, const float*, int, hipStream_t);
hipError_t pvr_fp8_scale_update(float*, int, unsigned*, float*, float*, const float*, int, int, float, hipStream_t);
hipError_t pvr_fp8_quant_t(const uint16_t*, int64_t, uint8_t*, int64_t, int, int, const float*, int, hipStream_t);
hipError_t pvr_fp8_transpose(const uint8_t*, int64_t, uint8_t*, int64_t, int, int, hipStream_t);
hipError_t pvr_fp8_quant_multi(const int64_t*, int, int64_t, const float*, unsigned*, int, int, hipStream_t);
int pvr_attn_bwd_key_blocks(int);
int pvr_attn_bwd_needs_dq_acc(int, int, int, int, int);
int pvr_attn_bwd_waves(int);
int pvr_attn_bwd_uses_pipe(int, int, int, int, int64_t, int64_t, int64_t, int64_t, int);
int pvr_attn_bwd_part_rows(int, int, int, int, int64_t, int64_t, int64_t, int64_t, int);
hipError_t pvr_attn_fwd(const uint16_t*, int64_t, uint16_t*, int64_t, float*, int, int, int, int, float, const uint64_t*, uint64_t,
                        uint32_t, float, uint8_t*, int64_t, const float*, unsigned*, int, hipStream_t);
int pvr_attn_dbias_splits(int, int);
hipError_t pvr_splitk_epilogue(const float*, int, int64_t, int, int, const float*, const uint16_t*, int64_t, int, uint16_t*, int64_t,
                               hipStream_t);
hipError_t pvr_attn_dbias_reduce(const float*, float*, float*, int, int, int, int, hipStream_t);
hipError_t pvr_attn_bwd(const uint16_t*, int64_t, const uint16_t*, int64_t, const uint16_t*, int64_t, const float*, uint16_t*, int64_t, float*, int, float*, float*, float*, int, int, int, int, float,
                        const uint64_t*, uint64_t, uint32_t, float, uint8_t*, int64_t, const float*, unsigned*,
                        int, int, hipStream_t);
int64_t pvr_attn_bwd_ws_floats(int, int, int, int, int, int, int);
int pvr_attn_bwd_q8_ok(int, int);
}

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }
// Per-(device, stream) scratch caches are keyed by the stream's id (a pooled raw handle can be
// reused by a different stream) and live in heap maps that free_scratch() empties (never in
// static-storage destructors, which would run after the HIP runtime's teardown).
using ScratchKey = std::pair<int, int64_t>;
ScratchKey scratch_key(int dev) { return std::make_pair(dev, (int64_t)c10::hip::getCurrentHIPStream().id()); }
template <class T>
std::map<ScratchKey, T>& scratch_map() {
  static auto* m = new std::map<ScratchKey, T>();
  return *m;
}
struct SkCounters { torch::Tensor t; };
struct DetWs { torch::Tensor t; };
struct DqWs { torch::Tensor t; };
struct AttnWs { torch::Tensor t; };

// compute units of the current device (the persistent kernels' grid)
int num_cus() {
  static std::map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  hipDeviceProp_t prop;
  int n = hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  cache[dev] = n;
  return n;
}

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "pvr kernel '", what, "' failed: ", hipGetErrorString(e));
}

const uint16_t* bf(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, " must be bfloat16, got ", t.scalar_type());
  return reinterpret_cast<const uint16_t*>(t.data_ptr());
}
uint16_t* bf_mut(torch::Tensor& t, const char* name) { return const_cast<uint16_t*>(bf(t, name)); }
const float* f32(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32, got ", t.scalar_type());
  return t.data_ptr<float>();
}
float* f32_mut(torch::Tensor& t, const char* name) { return const_cast<float*>(f32(t, name)); }

template <class T>
T* opt_ptr(const c10::optional<torch::Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// 2-D row-major view check: last-dim contiguous, returns leading dimension (elements)
int64_t ld_of(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D");
  TORCH_CHECK(t.stride(1) == 1, name, " must have unit stride in its last dim");
  TORCH_CHECK(t.stride(0) % 8 == 0 || t.size(0) == 1, name, " leading dimension must be a multiple of 8 elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
  return t.size(0) == 1 ? t.size(1) : t.stride(0);
}

// Split-K tail of the one-tile-per-workgroup GEMMs (GemmParams::tail_*): per (device, stream) a
// slab workspace of CUs x 256x256 fp32 partial tiles and CUs arrival counters (zeroed once; each
// launch leaves them zero). GEMMs on one stream are serialised, so they share the buffers.
bool g_gemm_tail = true;
struct TailBufs {
  torch::Tensor ws, cnt;
};
void attach_tail(pvr::GemmParams& p, const torch::Tensor& like) {
  if (!g_gemm_tail) return;
  auto& bufs = scratch_map<TailBufs>();
  const auto key = scratch_key((int)like.get_device());
  auto it = bufs.find(key);
  if (it == bufs.end()) {
    const int64_t cus = num_cus();
    TailBufs b;
    b.ws = torch::empty({cus * 65536}, like.options().dtype(torch::kFloat32));
    b.cnt = torch::zeros({cus}, like.options().dtype(torch::kInt32));
    it = bufs.emplace(key, b).first;
  }
  p.tail_ws = it->second.ws.data_ptr<float>();
  p.tail_cnt = reinterpret_cast<unsigned*>(it->second.cnt.data_ptr<int32_t>());
  p.tail_ws_elems = it->second.ws.numel();
  p.tail_cnt_elems = (int)it->second.cnt.numel();
}
void set_gemm_tail(bool on) { g_gemm_tail = on; }

// Counters of the in-launch split-K reduction (GemmParams::sk_*): per (device, stream) two words
// per output tile plus a timeout count, zeroed once; every launch leaves the tile words zero.
constexpr int g_sk_tiles = 4096;
torch::Tensor& splitk_counters(const torch::Tensor& like) {
  auto& bufs = scratch_map<SkCounters>();
  const auto key = scratch_key((int)like.get_device());
  auto it = bufs.find(key);
  if (it == bufs.end()) it = bufs.emplace(key, SkCounters{torch::zeros({2 * g_sk_tiles + 4}, like.options().dtype(torch::kInt32))}).first;
  return it->second.t;
}
// spin timeouts of the in-launch split-K reduction on the current stream (0 unless a split's
// workgroups were not co-resident); reset = true zeroes the count
int64_t splitk_timeouts(torch::Tensor like, bool reset) {
  torch::Tensor& c = splitk_counters(like);
  const int64_t v = c[2 * g_sk_tiles].item<int32_t>();
  if (reset) c[2 * g_sk_tiles].zero_();
  return v;
}
// fewest K-tiles per split-tail part: 12 (6 / 4 / 3 measured no better or worse on the short-K
// GEMMs, profiles/r4/ab14/tail_kt.log)
constexpr int g_tail_min_kt = 12;

// Deterministic mode (set_deterministic): the reductions that otherwise add float atomics in
// arrival order (LayerNorm backward dgamma / dbeta / fused bias sums, the column-sum kernel, the
// classifier LayerNorm's dgamma / dbeta) write one partial row per workgroup instead and an ordered
// pass sums the rows: every run of a step produces the same bits (bit-exact resume).
bool g_deterministic = [] {
  const char* e = std::getenv("PVR_DETERMINISTIC");
  return e && std::atoi(e) != 0;
}();
void set_deterministic(bool on) { g_deterministic = on; }
bool deterministic() { return g_deterministic; }
// partial-row scratch of the deterministic reductions, one per (device, stream), grown on demand
float* det_scratch(int64_t numel, const torch::TensorOptions& opts) {
  DetWs& d = scratch_map<DetWs>()[scratch_key((int)opts.device().index())];
  if (!d.t.defined() || d.t.numel() < numel) d.t = torch::empty({numel}, opts.dtype(torch::kFloat32));
  return d.t.data_ptr<float>();
}

// C = A . B^T with the given operand layouts; see csrc/gemm.hip for the epilogue contract.
void gemm(torch::Tensor A, bool a_kcontig, torch::Tensor B, bool b_kcontig, torch::Tensor C, int64_t M, int64_t N, int64_t K,
          int64_t epi, c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> resid, c10::optional<torch::Tensor> addend,
          int64_t addend_period, c10::optional<torch::Tensor> aux, int64_t row_group, int64_t row_stride_group,
          int64_t row_offset, c10::optional<torch::Tensor> seed, int64_t seed_offset, double drop_p, int64_t k_split,
          int64_t tile_cfg, c10::optional<torch::Tensor> dbg, c10::optional<torch::Tensor> colsum,
          int64_t epi_staged, int64_t tail_limit, c10::optional<torch::Tensor> reduce_out, bool reduce_acc) {
  pvr::GemmParams p{};
  p.epi_staged = (int)epi_staged;
  if (colsum.has_value() && colsum->defined()) p.colsum = f32_mut(*colsum, "colsum");
  if (dbg.has_value() && dbg->defined()) p.dbg = reinterpret_cast<uint64_t*>(dbg->data_ptr());
  p.drop_scale = 1.f;
  p.M = (int)M; p.N = (int)N; p.K = (int)K;
  p.A = bf(A, "A"); p.lda = ld_of(A, "A"); p.a_kcontig = a_kcontig;
  p.B = bf(B, "B"); p.ldb = ld_of(B, "B"); p.b_kcontig = b_kcontig;
  TORCH_CHECK(N % 8 == 0, "gemm: N must be a multiple of 8");
  if (a_kcontig) TORCH_CHECK(K % 64 == 0, "gemm: K must be a multiple of 64 for a k-contiguous A");
  if (b_kcontig) TORCH_CHECK(K % 64 == 0, "gemm: K must be a multiple of 64 for a k-contiguous B");
  if (a_kcontig) {
    TORCH_CHECK(A.size(0) >= M && A.size(1) >= K, "gemm: A too small");
  } else {
    TORCH_CHECK(A.size(0) >= K && A.size(1) >= M, "gemm: A too small");
  }
  if (b_kcontig) {
    TORCH_CHECK(B.size(0) >= N && B.size(1) >= K, "gemm: B too small");
  } else {
    TORCH_CHECK(B.size(0) >= K && B.size(1) >= N, "gemm: B too small");
  }
  const bool f32out = epi >= 3;
  TORCH_CHECK(C.is_cuda() && C.scalar_type() == (f32out ? torch::kFloat32 : torch::kBFloat16), "gemm: C dtype mismatch for epilogue");
  if (C.dim() == 3) {  // split-K partials [splits, M, N] (EPI_F32_STORE, tile 14)
    TORCH_CHECK(epi == 4 && tile_cfg == 14, "gemm: a 3-D C is the split-K workspace of EPI_F32_STORE / tile 14");
    TORCH_CHECK(C.stride(2) == 1 && C.size(1) >= M && C.size(2) >= N, "gemm: workspace shape");
    const int64_t ks = k_split > 0 ? ((k_split + 63) / 64) * 64 : ((K + 63) / 64) * 64;
    TORCH_CHECK(C.size(0) >= (K + ks - 1) / ks, "gemm: workspace has fewer slices than K splits");
    p.C = C.data_ptr(); p.ldc = C.stride(1); p.split_stride = C.stride(0);
  } else {
    p.C = C.data_ptr(); p.ldc = ld_of(C, "C");
  }
  if (bias.has_value() && bias->defined()) { TORCH_CHECK(bias->numel() >= N && bias->is_contiguous(), "bias"); p.bias = f32(*bias, "bias"); }
  if (resid.has_value() && resid->defined()) { p.resid = bf(*resid, "resid"); p.ld_resid = ld_of(*resid, "resid"); }
  if (addend.has_value() && addend->defined()) { p.addend = f32(*addend, "addend"); p.addend_period = (int)addend_period; TORCH_CHECK(addend_period > 0, "addend_period"); }
  if (aux.has_value() && aux->defined()) { p.aux = const_cast<uint16_t*>(bf(*aux, "aux")); p.ld_aux = ld_of(*aux, "aux"); }
  if (epi == 2) TORCH_CHECK(p.aux != nullptr, "gemm: the dGELU epilogue needs aux");  // GELU: aux optional (inference)
  p.row_group = (int)row_group; p.row_stride_group = (int)row_stride_group; p.row_offset = (int)row_offset;
  if (drop_p > 0.0) {
    TORCH_CHECK(seed.has_value() && seed->defined() && seed->scalar_type() == torch::kInt64, "dropout needs an int64 seed tensor");
    p.seed_ptr = reinterpret_cast<const uint64_t*>(seed->data_ptr());
    p.seed_offset = (uint64_t)seed_offset;
    uint32_t thr = (uint32_t)llround(drop_p * 65536.0);
    if (thr > 65535) thr = 65535;
    p.drop_thr = thr;
    p.drop_scale = (float)(65536.0 / (65536.0 - thr));
  }
  p.k_split_len = k_split > 0 ? (int)(((k_split + 63) / 64) * 64) : (int)(((K + 63) / 64) * 64);
  p.epi = (int)epi;
  p.tile_cfg = (int)tile_cfg;
  // tail_limit: -1 = no split tail, 0 = unlimited, n > 0 = at most n workgroups in the split round
  if (epi <= 2 && p.k_split_len >= K && tail_limit >= 0) {
    attach_tail(p, C);
    p.tail_max_units = (int)tail_limit;
    p.tail_min_kt = g_tail_min_kt;
  }
  if (reduce_out.has_value() && reduce_out->defined()) {
    // in-launch reduction of the K splits into reduce_out [M, N] fp32 (GemmParams::sk_*): the
    // ping-pong weight-gradient kernel, every workgroup co-resident
    const torch::Tensor& o = *reduce_out;
    TORCH_CHECK(C.dim() == 3 && epi == 4 && tile_cfg == 14, "gemm: reduce_out needs the split-K workspace form");
    TORCH_CHECK(o.is_cuda() && o.scalar_type() == torch::kFloat32 && o.dim() == 2 && o.stride(1) == 1 && o.size(0) >= M && o.size(1) >= N &&
                    o.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(o.data_ptr()) % 16 == 0,
                "gemm: reduce_out must be a 16-B aligned fp32 [M, N] tensor with unit column stride");
    const int64_t splits = (K + p.k_split_len - 1) / p.k_split_len;
    const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
    TORCH_CHECK(N % 4 == 0 && tiles <= g_sk_tiles && tiles * splits <= num_cus(), "gemm: reduce_out: too many workgroups to be co-resident");
    TORCH_CHECK(p.split_stride * 4 * (2 * splits + 16) < (int64_t(1) << 32) && M * p.ldc * 4 < (int64_t(1) << 31),
                "gemm: reduce_out: workspace too large for 32-bit buffer offsets");
    torch::Tensor& cnt = splitk_counters(o);
    p.sk_out = o.data_ptr<float>();
    p.sk_ldo = o.stride(0);
    p.sk_acc = reduce_acc ? 1 : 0;
    p.sk_cnt = reinterpret_cast<unsigned*>(cnt.data_ptr<int32_t>());
    p.sk_cnt_tiles = g_sk_tiles;
  }
  check(pvr_gemm(&p, stream()), "gemm");
}

std::vector<torch::Tensor> layernorm_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor b, double eps, int64_t rows,
                                         int64_t x_row_stride) {
  const int64_t D = w.numel();
  auto y = torch::empty({rows, D}, x.options());
  auto mean = torch::empty({rows}, x.options().dtype(torch::kFloat32));
  auto rstd = torch::empty({rows}, x.options().dtype(torch::kFloat32));
  TORCH_CHECK(x.stride(-1) == 1, "layernorm: x last dim must be contiguous");
  check(pvr_layernorm_fwd(bf(x, "x"), x_row_stride, f32(w, "w"), f32(b, "b"), bf_mut(y, "y"), D, f32_mut(mean, "mean"),
                          f32_mut(rstd, "rstd"), (int)rows, (int)D, (float)eps, stream()),
        "layernorm_fwd");
  return {y, mean, rstd};
}

// layernorm_fwd + the output's e4m3 copy q_out [rows][D] (uint8) quantized with *q_scale, amax
// recorded into *q_amax (int32 float bits): the fp8 forward's quantize pass folded into the LayerNorm
std::vector<torch::Tensor> layernorm_fwd_q8(torch::Tensor x, torch::Tensor w, torch::Tensor b, double eps, int64_t rows,
                                            int64_t x_row_stride, torch::Tensor q_out, torch::Tensor q_scale, torch::Tensor q_amax,
                                            bool skip_y) {
  const int64_t D = w.numel();
  auto y = torch::empty({rows, D}, x.options());
  auto mean = torch::empty({rows}, x.options().dtype(torch::kFloat32));
  auto rstd = torch::empty({rows}, x.options().dtype(torch::kFloat32));
  TORCH_CHECK(x.stride(-1) == 1, "layernorm: x last dim must be contiguous");
  TORCH_CHECK(q_out.is_cuda() && q_out.scalar_type() == torch::kUInt8 && q_out.dim() == 2 && q_out.size(0) >= rows &&
                  q_out.size(1) >= D && q_out.stride(1) == 1 && q_out.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(q_out.data_ptr()) % 8 == 0,
              "layernorm_fwd_q8: q_out uint8 [rows][D], 8-byte aligned rows");
  TORCH_CHECK(q_amax.is_cuda() && q_amax.scalar_type() == torch::kInt32, "layernorm_fwd_q8: q_amax int32");
  // skip_y: only the e4m3 copy is consumed (the bf16 y stays allocated, unwritten)
  check(pvr_layernorm_fwd_q8(bf(x, "x"), x_row_stride, f32(w, "w"), f32(b, "b"), skip_y ? nullptr : bf_mut(y, "y"), D,
                             reinterpret_cast<uint8_t*>(q_out.data_ptr()), q_out.stride(0), f32(q_scale, "q_scale"),
                             reinterpret_cast<unsigned*>(q_amax.data_ptr<int32_t>()), f32_mut(mean, "mean"), f32_mut(rstd, "rstd"),
                             (int)rows, (int)D, (float)eps, stream()),
        "layernorm_fwd_q8");
  return {y, mean, rstd};
}

// Dropout parameters shared by every kernel that recomputes a mask: keep iff the element's 16-bit
// hash >= thr16 = round(p * 65536); kept values scale by 65536 / (65536 - thr16).
struct DropArgs {
  const uint64_t* seed = nullptr;
  uint32_t thr = 0;
  float scale = 1.f;
};
DropArgs drop_args(const c10::optional<torch::Tensor>& seed, double drop_p, const char* what) {
  DropArgs d;
  if (drop_p > 0.0) {
    TORCH_CHECK(seed.has_value() && seed->defined(), what, ": dropout needs a seed");
    d.seed = reinterpret_cast<const uint64_t*>(seed->data_ptr());
    d.thr = (uint32_t)llround(drop_p * 65536.0);
    if (d.thr > 65535) d.thr = 65535;
    d.scale = (float)(65536.0 / (65536.0 - d.thr));
  }
  return d;
}

// dz (optional, needs drop_p > 0): dropout backward of the layer that produced x's residual stream,
// dz = mask(seed + seed_offset) * scale * dx; dsum then receives the column sums of dz instead of dx.
void layernorm_bwd(torch::Tensor dy, int64_t dy_stride, torch::Tensor x, int64_t x_stride, torch::Tensor mean, torch::Tensor rstd,
                   torch::Tensor w, c10::optional<torch::Tensor> dres, int64_t dres_stride, torch::Tensor dx, int64_t dx_stride,
                   c10::optional<torch::Tensor> dw, c10::optional<torch::Tensor> db, int64_t rows,
                   c10::optional<torch::Tensor> dsum, c10::optional<torch::Tensor> dz, c10::optional<torch::Tensor> seed,
                   int64_t seed_offset, double drop_p, c10::optional<torch::Tensor> q_out,
                   c10::optional<torch::Tensor> q_scale, c10::optional<torch::Tensor> q_amax, bool dz_nostore,
                   int64_t q_fmt) {
  const int64_t D = w.numel();
  // optional e5m2 copy of the last-written gradient (dz if given, else dx) with a delayed scale
  // and an amax record: the producer-side quantization for the next fp8 dgrad GEMM
  uint8_t* qp = nullptr;
  int64_t ldq = 0;
  const float* qs = nullptr;
  unsigned* qa = nullptr;
  if (q_out.has_value() && q_out->defined()) {
    TORCH_CHECK(q_out->is_cuda() && q_out->scalar_type() == torch::kUInt8 && q_out->dim() == 2 && q_out->stride(1) == 1 &&
                    q_out->size(0) >= rows && q_out->size(1) >= D && q_out->stride(0) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(q_out->data_ptr()) % 8 == 0,
                "layernorm_bwd: q_out uint8 [>= rows][>= D], row stride a multiple of 8, 8-byte aligned");
    TORCH_CHECK(q_scale.has_value() && q_scale->defined() && q_amax.has_value() && q_amax->defined() &&
                    q_amax->is_cuda() && q_amax->scalar_type() == torch::kInt32,
                "layernorm_bwd: q_out needs q_scale (f32) and q_amax (int32)");
    qp = q_out->data_ptr<uint8_t>();
    ldq = q_out->stride(0);
    qs = f32(*q_scale, "q_scale");
    qa = reinterpret_cast<unsigned*>(q_amax->data_ptr());
  }
  uint16_t* dzp = nullptr;
  int64_t ldz = 0;
  DropArgs d;
  if (dz.has_value() && dz->defined()) {
    TORCH_CHECK(drop_p > 0.0, "layernorm_bwd: dz is the dropout backward, it needs drop_p > 0");
    dzp = const_cast<uint16_t*>(bf(*dz, "dz"));
    ldz = ld_of(*dz, "dz");
    d = drop_args(seed, drop_p, "layernorm_bwd");
  }
  check(pvr_layernorm_bwd(bf(dy, "dy"), dy_stride, bf(x, "x"), x_stride, f32(mean, "mean"), f32(rstd, "rstd"), f32(w, "w"),
                          opt_ptr<const uint16_t>(dres), dres_stride, bf_mut(dx, "dx"), dx_stride, opt_ptr<float>(dw),
                          opt_ptr<float>(db), opt_ptr<float>(dsum), dzp, ldz, d.seed, (uint64_t)seed_offset, d.thr, d.scale,
                          dz_nostore ? 1 : 0, qp, ldq, qs, qa, (int)q_fmt, (int)rows, (int)D,
                          g_deterministic && (opt_ptr<float>(dw) || opt_ptr<float>(db) || opt_ptr<float>(dsum)) ? det_scratch((int64_t)pvr_layernorm_bwd_blocks((int)rows, (int)D) * 3 * D, x.options()) : nullptr,
                          stream()),
        "layernorm_bwd");
}

// out (+)= ws.sum(0) for a split-K workspace ws [S, rows, cols] (out: contiguous [rows, cols])
// out (+)= ws[:S].sum(0) for ws [S, rows, wcols]; out [rows, ocols] contiguous with ocols <= wcols
// (the leading columns of each workspace row: a K-padded weight gradient reduced into the unpadded one)
void splitk_reduce(torch::Tensor ws, int64_t S, torch::Tensor out, bool accumulate) {
  TORCH_CHECK(ws.dim() == 3 && ws.size(0) >= S && S >= 1, "splitk_reduce: ws must be [S, rows, cols]");
  TORCH_CHECK(out.is_contiguous() && ws.stride(2) == 1 && ws.stride(1) == ws.size(2), "splitk_reduce: layouts");
  const int64_t rows = ws.size(1), wcols = ws.size(2);
  TORCH_CHECK(out.numel() % rows == 0, "splitk_reduce: out must hold [rows, ocols]");
  const int64_t ocols = out.numel() / rows;
  TORCH_CHECK(ocols <= wcols && ocols % 4 == 0 && wcols % 4 == 0, "splitk_reduce: out columns must be a 4-aligned prefix of ws columns");
  check(pvr_splitk_reduce(f32(ws, "ws"), (int)S, ws.stride(0), f32_mut(out, "out"), out.numel(), (int)ocols, (int)wcols,
                          accumulate ? 1 : 0, stream()),
        "splitk_reduce");
}

// dst [rows, ld] bf16 = src [rows, cols] zero-padded on the right (cols, ld % 4 == 0)
void pad_cols_bf16(torch::Tensor src, torch::Tensor dst) {
  TORCH_CHECK(src.is_contiguous() && dst.is_contiguous() && src.dim() == 2 && dst.dim() == 2 && src.size(0) == dst.size(0) &&
                  src.size(1) <= dst.size(1) && src.size(1) % 4 == 0 && dst.size(1) % 4 == 0,
              "pad_cols_bf16: src [rows, cols], dst [rows, ld >= cols], contiguous, 4-aligned");
  check(pvr_pad_cols_bf16(bf(src, "src"), (int)src.size(0), (int)src.size(1), bf_mut(dst, "dst"), (int)dst.size(1), stream()),
        "pad_cols_bf16");
}

// out = bf16(epilogue(ws.sum(0))) for a split-K workspace ws [S, M, N]: + bias, GELU (inference: no
// derivative), + resid (the small-M forward GEMM's reduction pass)
void splitk_epilogue(torch::Tensor ws, int64_t S, torch::Tensor out, c10::optional<torch::Tensor> bias,
                     c10::optional<torch::Tensor> resid, bool gelu) {
  TORCH_CHECK(ws.dim() == 3 && ws.size(0) >= S && S >= 1 && ws.stride(2) == 1 && ws.stride(1) == ws.size(2),
              "splitk_epilogue: ws must be [S, M, N] with contiguous rows");
  const int64_t M = ws.size(1), N = ws.size(2);
  TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N && N % 4 == 0, "splitk_epilogue: out shape");
  const int64_t ldc = ld_of(out, "out");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() >= N && bias->is_contiguous(), "splitk_epilogue: bias");
    bp = f32(*bias, "bias");
  }
  const uint16_t* rp = nullptr;
  int64_t ldr = 0;
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->dim() == 2 && resid->size(0) >= M && resid->size(1) >= N, "splitk_epilogue: resid must cover [M, N]");
    rp = bf(*resid, "resid");
    ldr = ld_of(*resid, "resid");
  }
  check(pvr_splitk_epilogue(f32(ws, "ws"), (int)S, ws.stride(0), (int)M, (int)N, bp, rp, ldr, gelu ? 1 : 0, bf_mut(out, "out"), ldc,
                            stream()),
        "splitk_epilogue");
}

void cast_f32_bf16(torch::Tensor in, torch::Tensor out) {
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && in.numel() == out.numel(), "cast: shape/contiguity");
  check(pvr_cast_f32_bf16(f32(in, "in"), bf_mut(out, "out"), in.numel(), stream()), "cast_f32_bf16");
}

void transpose_batched(torch::Tensor src, torch::Tensor dst, torch::Tensor meta, int64_t total_tiles) {
  TORCH_CHECK(meta.scalar_type() == torch::kInt64 && meta.is_cuda() && meta.dim() == 2 && meta.size(1) == 5, "meta");
  check(pvr_transpose_batched(bf(src, "src"), bf_mut(dst, "dst"), meta.data_ptr<int64_t>(), (int)meta.size(0), (int)total_tiles,
                              stream()),
        "transpose_batched");
}

void colsum(torch::Tensor dy, int64_t rows, int64_t N, c10::optional<torch::Tensor> db, c10::optional<torch::Tensor> dz,
            c10::optional<torch::Tensor> seed, int64_t seed_offset, double drop_p, c10::optional<torch::Tensor> q_out,
            c10::optional<torch::Tensor> q_scale, c10::optional<torch::Tensor> q_amax, int64_t q_fmt) {
  const DropArgs d = drop_args(seed, drop_p, "colsum");
  int64_t ldz = 0;
  uint16_t* dzp = nullptr;
  if (dz.has_value() && dz->defined()) { dzp = const_cast<uint16_t*>(bf(*dz, "dz")); ldz = ld_of(*dz, "dz"); }
  // optional fp8 copy (q_fmt 1 e5m2, 0 e4m3) of the (masked) gradient + amax record (the fp8 dgrad operand)
  uint8_t* qp = nullptr;
  int64_t ldq = 0;
  const float* qs = nullptr;
  unsigned* qa = nullptr;
  if (q_out.has_value() && q_out->defined()) {
    TORCH_CHECK(q_out->is_cuda() && q_out->scalar_type() == torch::kUInt8 && q_out->dim() == 2 && q_out->stride(1) == 1 &&
                    q_out->size(0) >= rows && q_out->size(1) >= N && q_out->stride(0) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(q_out->data_ptr()) % 8 == 0,
                "colsum: q_out uint8 [>= rows][>= N], row stride a multiple of 8, 8-byte aligned");
    TORCH_CHECK(q_scale.has_value() && q_scale->defined() && q_amax.has_value() && q_amax->defined() && q_amax->is_cuda() &&
                    q_amax->scalar_type() == torch::kInt32,
                "colsum: q_out needs q_scale (f32) and q_amax (int32)");
    qp = q_out->data_ptr<uint8_t>();
    ldq = q_out->stride(0);
    qs = f32(*q_scale, "q_scale");
    qa = reinterpret_cast<unsigned*>(q_amax->data_ptr());
  }
  check(pvr_colsum(bf(dy, "dy"), ld_of(dy, "dy"), (int)rows, (int)N, opt_ptr<float>(db), dzp, ldz, d.seed, (uint64_t)seed_offset,
                   d.thr, d.scale, qp, ldq, qs, qa, (int)q_fmt,
                   g_deterministic && opt_ptr<float>(db) ? det_scratch((int64_t)pvr_colsum_part_rows((int)rows) * N, dy.options()) : nullptr, stream()),
        "colsum");
}

void im2col(torch::Tensor img, torch::Tensor out, int64_t P, int64_t Kp) {
  TORCH_CHECK(img.is_contiguous() && img.dim() == 4, "im2col: img must be contiguous NCHW");
  check(pvr_im2col(f32(img, "img"), bf_mut(out, "out"), (int)img.size(0), (int)img.size(1), (int)img.size(2), (int)img.size(3),
                   (int)P, (int)Kp, stream()),
        "im2col");
}

void cls_rows(torch::Tensor cls, torch::Tensor pos, torch::Tensor out, int64_t B, int64_t D, int64_t row_stride,
              c10::optional<torch::Tensor> seed, int64_t seed_offset, double drop_p) {
  uint32_t thr = 0;
  float scale = 1.f;
  const uint64_t* sp = nullptr;
  if (drop_p > 0.0) {
    sp = reinterpret_cast<const uint64_t*>(seed->data_ptr());
    thr = (uint32_t)llround(drop_p * 65536.0);
    if (thr > 65535) thr = 65535;
    scale = (float)(65536.0 / (65536.0 - thr));
  }
  check(pvr_cls_rows(f32(cls, "cls"), f32(pos, "pos"), bf_mut(out, "out"), (int)B, (int)D, row_stride, sp, (uint64_t)seed_offset,
                     thr, scale, stream()),
        "cls_rows");
}

void patch_bwd(torch::Tensor dE, int64_t B, int64_t ntok, int64_t D, c10::optional<torch::Tensor> dpos, c10::optional<torch::Tensor> dcls,
               c10::optional<torch::Tensor> dconv, c10::optional<torch::Tensor> dbias, c10::optional<torch::Tensor> seed,
               int64_t seed_offset, double drop_p) {
  uint32_t thr = 0;
  float scale = 1.f;
  const uint64_t* sp = nullptr;
  if (drop_p > 0.0) {
    sp = reinterpret_cast<const uint64_t*>(seed->data_ptr());
    thr = (uint32_t)llround(drop_p * 65536.0);
    if (thr > 65535) thr = 65535;
    scale = (float)(65536.0 / (65536.0 - thr));
  }
  TORCH_CHECK(dE.numel() == B * ntok * D, "patch_bwd: dE must hold B * ntok * D elements");
  auto ws = torch::empty({pvr_patch_bwd_ws_floats((int)B, (int)ntok, (int)D)}, dE.options().dtype(torch::kFloat32));
  check(pvr_patch_bwd(bf(dE, "dE"), (int)B, (int)ntok, (int)D, ws.data_ptr<float>(), opt_ptr<float>(dpos), opt_ptr<float>(dcls), opt_ptr<uint16_t>(dconv),
                      opt_ptr<float>(dbias), sp, (uint64_t)seed_offset, thr, scale, stream()),
        "patch_bwd");
}

// returns per-row losses; writes dlogits (if given)
// correct (optional): int32 [B], receives 1 where argmax(logits) == label. mean (optional): f32 [1],
// receives the batch mean of the row losses (a second, one-workgroup launch).
torch::Tensor xent(torch::Tensor logits, torch::Tensor labels, c10::optional<torch::Tensor> dlogits, c10::optional<torch::Tensor> correct,
                   double grad_scale, c10::optional<torch::Tensor> mean) {
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "xent: logits must be [B, C] row-major");
  TORCH_CHECK(labels.scalar_type() == torch::kInt64 && labels.is_contiguous(), "xent: labels must be contiguous int64");
  const int64_t B = logits.size(0), C = logits.size(1);
  if (correct.has_value() && correct->defined())
    TORCH_CHECK(correct->is_cuda() && correct->numel() >= B && correct->scalar_type() == torch::kInt32, "xent: correct int32 [B]");
  if (dlogits.has_value() && dlogits->defined())
    TORCH_CHECK(dlogits->is_contiguous() && dlogits->numel() == B * C && dlogits->scalar_type() == torch::kFloat32, "xent: dlogits f32 [B][C]");
  if (mean.has_value() && mean->defined()) TORCH_CHECK(mean->numel() >= 1, "xent: mean [1]");
  auto loss = torch::empty({B}, logits.options().dtype(torch::kFloat32));
  check(pvr_xent(f32(logits, "logits"), logits.stride(0), labels.data_ptr<int64_t>(), (int)B, (int)C, loss.data_ptr<float>(),
                 opt_ptr<float>(dlogits), opt_ptr<int>(correct), (float)grad_scale, stream()),
        "xent");
  if (mean.has_value() && mean->defined()) check(pvr_mean(loss.data_ptr<float>(), (int)B, f32_mut(*mean, "mean"), stream()), "xent mean");
  return loss;
}

void grad_norm(torch::Tensor g, double max_norm, torch::Tensor workspace, torch::Tensor out) {
  TORCH_CHECK(g.is_contiguous(), "grad_norm: flat grad must be contiguous");
  TORCH_CHECK(workspace.numel() >= pvr_norm_partial_blocks(), "grad_norm: workspace too small");
  check(pvr_grad_norm(f32(g, "g"), g.numel(), (float)max_norm, f32_mut(workspace, "ws"), f32_mut(out, "out"), stream()), "grad_norm");
}

// Param-group table float32 [G][8] (csrc/optim.hip AdamGroup): a CUDA tensor is read by the kernel
// (graph-captured steps); a CPU tensor is copied into the launch's kernel arguments (G <= 8), so an
// eager step needs no host-to-device copy of its per-step lr / bias corrections.
struct GroupTable {
  const pvr::AdamGroup* dev = nullptr;
  const pvr::AdamGroup* host = nullptr;
  int n = 0;
};
GroupTable group_table(const torch::Tensor& groups, const char* who) {
  TORCH_CHECK(groups.scalar_type() == torch::kFloat32 && groups.dim() == 2 && groups.size(1) == 8 && groups.is_contiguous(), who,
              ": groups must be contiguous float32 [G, 8]");
  GroupTable t;
  t.n = (int)groups.size(0);
  auto* ptr = reinterpret_cast<const pvr::AdamGroup*>(groups.data_ptr<float>());
  if (groups.is_cuda()) {
    t.dev = ptr;
  } else {
    TORCH_CHECK(t.n >= 1 && t.n <= 8, who, ": a host group table holds 1..8 groups (pass a device table for more)");
    t.host = ptr;
  }
  return t;
}

void adam(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow, torch::Tensor seg_start,
          torch::Tensor seg_group, torch::Tensor groups, c10::optional<torch::Tensor> clip, bool skip_nonfinite) {
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adam: size mismatch");
  const GroupTable gt = group_table(groups, "adam");
  TORCH_CHECK(seg_start.scalar_type() == torch::kInt64 && seg_group.scalar_type() == torch::kInt32, "adam: segment table dtypes");
  uint16_t* sh = nullptr;
  if (shadow.has_value() && shadow->defined()) sh = const_cast<uint16_t*>(bf(*shadow, "shadow"));
  check(pvr_adam(f32_mut(p, "p"), f32(g, "g"), f32_mut(m, "m"), f32_mut(v, "v"), sh, p.numel(), seg_start.data_ptr<int64_t>(),
                 seg_group.data_ptr<int>(), (int)seg_start.numel(), gt.dev, gt.host, gt.n, opt_ptr<const float>(clip), skip_nonfinite ? 1 : 0, stream()),
        "adam");
}

// Adam + bf16 shadow + transposed bf16 shadow (W^T of the registered 2-D weights) in one launch.
// tmeta int64 [nmat][6] {flat offset, shadow_t offset, R, C, first tile, group} (R, C % 64 == 0),
// fmeta int64 [nflat][4] {flat start, elements % 4 == 0, group, first float4} for everything else.
void adam_t(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, torch::Tensor shadow, torch::Tensor shadow_t,
            torch::Tensor tmeta, int64_t ntiles, torch::Tensor fmeta, int64_t flat4, torch::Tensor groups,
            c10::optional<torch::Tensor> clip, bool skip_nonfinite) {
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel() && shadow.numel() == p.numel(),
              "adam_t: size mismatch");
  const GroupTable gt = group_table(groups, "adam_t");
  TORCH_CHECK(tmeta.is_cuda() && tmeta.scalar_type() == torch::kInt64 && tmeta.dim() == 2 && tmeta.size(1) == 6 && tmeta.is_contiguous(),
              "adam_t: tmeta int64 [n][6]");
  TORCH_CHECK(fmeta.is_cuda() && fmeta.scalar_type() == torch::kInt64 && fmeta.dim() == 2 && fmeta.size(1) == 4 && fmeta.is_contiguous(),
              "adam_t: fmeta int64 [n][4]");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous() && shadow.is_contiguous() &&
                  shadow_t.is_contiguous(),
              "adam_t: contiguous buffers");
  check(pvr_adam_t(f32_mut(p, "p"), f32(g, "g"), f32_mut(m, "m"), f32_mut(v, "v"), bf_mut(shadow, "shadow"), bf_mut(shadow_t, "shadow_t"),
                   tmeta.data_ptr<int64_t>(), (int)tmeta.size(0), (int)ntiles, fmeta.data_ptr<int64_t>(), (int)fmeta.size(0), flat4,
                   gt.dev, gt.host, gt.n, opt_ptr<const float>(clip), skip_nonfinite ? 1 : 0,
                   stream()),
        "adam_t");
}

// Classifier head forward: LayerNorm of each image's CLS row (token 0 of tokens [B*N][D] bf16) and
// logits = LN(x) . W^T + bias in fp32. Returns {logits [B][C], xhat [B][D], rstd [B]} (the latter two
// saved for head_bwd).
std::vector<torch::Tensor> head_fwd(torch::Tensor tokens, int64_t B, int64_t N, torch::Tensor gamma, torch::Tensor beta, double eps,
                                    torch::Tensor W, c10::optional<torch::Tensor> bias) {
  const int64_t D = tokens.size(1);
  TORCH_CHECK(tokens.dim() == 2 && tokens.size(0) == B * N && tokens.is_contiguous(), "head_fwd: tokens [B*N][D] contiguous");
  TORCH_CHECK(D % 16 == 0 && D <= 1536, "head_fwd: D % 16 == 0, D <= 1536");
  TORCH_CHECK(W.dim() == 2 && W.size(1) == D && W.is_contiguous() && gamma.numel() == D && beta.numel() == D, "head_fwd: shapes");
  const int64_t C = W.size(0);
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) { TORCH_CHECK(bias->numel() == C && bias->is_contiguous(), "head_fwd: bias [C]"); bp = f32(*bias, "bias"); }
  auto f = tokens.options().dtype(torch::kFloat32);
  auto logits = torch::empty({B, C}, f);
  auto xhat = torch::empty({B, D}, f);
  auto rstd = torch::empty({B}, f);
  check(pvr_head_fwd(bf(tokens, "tokens"), N * D, (int)B, (int)D, f32(gamma, "gamma"), f32(beta, "beta"), (float)eps, f32(W, "W"), bp,
                     (int)C, xhat.data_ptr<float>(), rstd.data_ptr<float>(), logits.data_ptr<float>(), stream()),
        "head_fwd");
  return {logits, xhat, rstd};
}

// Classifier head backward: dW / db / dgamma / dbeta accumulate (+=) into the given fp32 gradients
// (each optional), returns d(tokens) [B*N][D] bf16: the LayerNorm backward in every CLS row, zeros
// elsewhere (written by the same launch).
torch::Tensor head_bwd(torch::Tensor dlogits, torch::Tensor xhat, torch::Tensor rstd, torch::Tensor gamma, torch::Tensor beta,
                       torch::Tensor W, int64_t B, int64_t N, c10::optional<torch::Tensor> dW, c10::optional<torch::Tensor> db,
                       c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta) {
  const int64_t C = W.size(0), D = W.size(1);
  TORCH_CHECK(dlogits.dim() == 2 && dlogits.size(0) == B && dlogits.size(1) == C && dlogits.is_contiguous(), "head_bwd: dlogits [B][C]");
  TORCH_CHECK(xhat.numel() == B * D && rstd.numel() == B && W.is_contiguous(), "head_bwd: saved tensors");
  float* pdw = opt_ptr<float>(dW);
  if (pdw) TORCH_CHECK(dW->numel() == C * D && dW->is_contiguous() && dW->scalar_type() == torch::kFloat32, "head_bwd: dW");
  auto dy = torch::empty({B, D}, xhat.options());
  auto dtok = torch::empty({B * N, D}, xhat.options().dtype(torch::kBFloat16));
  check(pvr_head_bwd(f32(dlogits, "dlogits"), f32(xhat, "xhat"), f32(rstd, "rstd"), f32(gamma, "gamma"), f32(beta, "beta"), f32(W, "W"),
                     (int)B, (int)C, (int)D, (int)N, pdw, opt_ptr<float>(db), opt_ptr<float>(dgamma), opt_ptr<float>(dbeta),
                     dy.data_ptr<float>(), reinterpret_cast<uint16_t*>(dtok.data_ptr()),
                     g_deterministic && (opt_ptr<float>(dgamma) || opt_ptr<float>(dbeta)) ? det_scratch(((B + 15) / 16) * 2 * D, xhat.options()) : nullptr, stream()),
        "head_bwd");
  return dtok;
}

// y = x * s[0] (s a 1-element device tensor): the cross-entropy backward's upstream-gradient scale
torch::Tensor scale_by(torch::Tensor x, torch::Tensor s) {
  TORCH_CHECK(x.is_contiguous() && s.numel() >= 1, "scale_by: contiguous x, scalar s");
  auto y = torch::empty_like(x);
  check(pvr_scale_by(f32(x, "x"), f32(s, "s"), y.data_ptr<float>(), x.numel(), stream()), "scale_by");
  return y;
}

// sums[0] += loss[0]; sums[1] += sum(correct) / B with correct = xent's per-row flags [B] (per-batch
// metrics accumulated on the device)
void metrics_accum(torch::Tensor sums, torch::Tensor loss, torch::Tensor correct) {
  TORCH_CHECK(sums.numel() >= 2 && correct.scalar_type() == torch::kInt32 && correct.is_contiguous(),
              "metrics_accum: sums [2] f32, correct int32 [B]");
  check(pvr_metrics_accum(f32_mut(sums, "sums"), f32(loss, "loss"), correct.data_ptr<int>(), (int)correct.numel(), stream()),
        "metrics_accum");
}

void rng_next(torch::Tensor rng, torch::Tensor seed) {
  TORCH_CHECK(rng.is_cuda() && seed.is_cuda() && rng.scalar_type() == torch::kInt64 && seed.scalar_type() == torch::kInt64 &&
                  rng.numel() >= 1 && seed.numel() >= 1,
              "rng_next: int64 device tensors");
  check(pvr_rng_next(rng.data_ptr<int64_t>(), seed.data_ptr<int64_t>(), stream()), "rng_next");
}

void zero_f32(torch::Tensor x) {
  TORCH_CHECK(x.is_contiguous() && x.numel() % 4 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "zero_f32: contiguous, 16-B aligned, numel % 4 == 0");
  check(pvr_zero_f32(f32_mut(x, "x"), x.numel(), stream()), "zero_f32");
}

void scale_by_clip(torch::Tensor g, torch::Tensor clip) {
  check(pvr_scale_by_clip(f32_mut(g, "g"), g.numel(), f32(clip, "clip"), stream()), "scale_by_clip");
}

const uint8_t* u8(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kUInt8, name, " must hold fp8 bytes (uint8), got ", t.scalar_type());
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.stride(0) % 16 == 0, name, " must be 2-D with a 16-byte multiple row stride");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
  return reinterpret_cast<const uint8_t*>(t.data_ptr());
}

// C[M][N] = epilogue(dscale_a * dscale_b * A[M][K] . B[N][K]^T), A/B OCP fp8 (fmt 0 e4m3, 1 e5m2)
void gemm_fp8(torch::Tensor A, int64_t fmt_a, torch::Tensor B, int64_t fmt_b, torch::Tensor C, int64_t M, int64_t N, int64_t K,
              int64_t epi, torch::Tensor scale_a, torch::Tensor scale_b, c10::optional<torch::Tensor> bias,
              c10::optional<torch::Tensor> resid, c10::optional<torch::Tensor> aux, c10::optional<torch::Tensor> seed, int64_t seed_offset,
              double drop_p, c10::optional<torch::Tensor> colsum, c10::optional<torch::Tensor> q_out,
              c10::optional<torch::Tensor> q_scale, c10::optional<torch::Tensor> q_amax, int64_t q_fmt, bool c_skip,
              int64_t tail_limit) {
  pvr::GemmParams p{};
  // c_skip: only the fp8 copy (or aux / column sums) of the output is consumed; the bf16 stores are
  // dropped (register-direct epilogue; other epilogues still write C, which is allocated)
  TORCH_CHECK(!c_skip || epi == 1 || epi == 2, "gemm_fp8: c_skip with the GELU / dGELU epilogues only");
  p.c_skip = c_skip ? 1 : 0;
  p.drop_scale = 1.f;
  p.M = (int)M; p.N = (int)N; p.K = (int)K;
  p.A = reinterpret_cast<const uint16_t*>(u8(A, "A")); p.lda = A.stride(0); p.a_kcontig = 1;
  p.B = reinterpret_cast<const uint16_t*>(u8(B, "B")); p.ldb = B.stride(0); p.b_kcontig = 1;
  TORCH_CHECK(A.size(0) >= M && A.size(1) >= K && B.size(0) >= N && B.size(1) >= K, "gemm_fp8: operand too small");
  TORCH_CHECK(K % 128 == 0 && N % 8 == 0, "gemm_fp8: K must be a multiple of 128, N of 8");
  TORCH_CHECK(C.is_cuda() && C.scalar_type() == torch::kBFloat16, "gemm_fp8: bf16 output");
  p.C = C.data_ptr(); p.ldc = ld_of(C, "C");
  p.scale_a = f32(scale_a, "scale_a"); p.scale_b = f32(scale_b, "scale_b");
  p.elem8 = 1; p.fmt_a = (int)fmt_a; p.fmt_b = (int)fmt_b;
  if (bias.has_value() && bias->defined()) { TORCH_CHECK(bias->numel() >= N && bias->is_contiguous(), "bias"); p.bias = f32(*bias, "bias"); }
  if (resid.has_value() && resid->defined()) { p.resid = bf(*resid, "resid"); p.ld_resid = ld_of(*resid, "resid"); }
  if (aux.has_value() && aux->defined()) { p.aux = const_cast<uint16_t*>(bf(*aux, "aux")); p.ld_aux = ld_of(*aux, "aux"); }
  // GELU without aux: the inference epilogue (no derivative stored; its stores go to a 0-byte range)
  if (epi == 2) TORCH_CHECK(p.aux != nullptr, "gemm_fp8: the dGELU epilogue needs aux");
  if (colsum.has_value() && colsum->defined()) p.colsum = f32_mut(*colsum, "colsum");
  if (q_out.has_value() && q_out->defined()) {
    // fp8 copy of the GELU / dGELU output from the register-direct epilogue (its preconditions:
    // 16-B column groups, 31-bit offsets of every row-major operand it touches)
    TORCH_CHECK(epi == 1 || epi == 2, "gemm_fp8: q_out with the GELU / dGELU epilogues only");
    TORCH_CHECK(q_out->is_cuda() && q_out->scalar_type() == torch::kUInt8 && q_out->dim() == 2 && q_out->stride(1) == 1 &&
                    q_out->size(0) >= M && q_out->size(1) >= N && q_out->stride(0) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(q_out->data_ptr()) % 8 == 0,
                "gemm_fp8: q_out uint8 [M][N], row stride and base 8-byte aligned");
    TORCH_CHECK(q_scale.has_value() && q_scale->defined() && q_amax.has_value() && q_amax->defined() &&
                    q_amax->scalar_type() == torch::kInt32 && q_amax->is_cuda() && (q_fmt == 0 || q_fmt == 1),
                "gemm_fp8: q_out needs q_scale (f32), q_amax (int32) and q_fmt 0 / 1");
    const int64_t ld_max = std::max(std::max(p.ldc, p.ld_aux), std::max(p.ld_resid, (int64_t)N));
    TORCH_CHECK(M * ld_max * 2 < (1ll << 31), "gemm_fp8: q_out path needs 31-bit output offsets");
    p.q_out = reinterpret_cast<uint8_t*>(q_out->data_ptr());
    p.ld_q = q_out->stride(0);
    p.q_scale = f32(*q_scale, "q_scale");
    p.q_amax = reinterpret_cast<unsigned*>(q_amax->data_ptr<int32_t>());
    p.q_fmt = (int)q_fmt;
  }
  if (drop_p > 0.0) {
    TORCH_CHECK(seed.has_value() && seed->defined() && seed->scalar_type() == torch::kInt64, "dropout needs an int64 seed tensor");
    p.seed_ptr = reinterpret_cast<const uint64_t*>(seed->data_ptr());
    p.seed_offset = (uint64_t)seed_offset;
    uint32_t thr = (uint32_t)llround(drop_p * 65536.0);
    if (thr > 65535) thr = 65535;
    p.drop_thr = thr;
    p.drop_scale = (float)(65536.0 / (65536.0 - thr));
  }
  p.k_split_len = (int)K;
  p.epi = (int)epi;
  p.tile_cfg = 12;
  if (epi <= 2 && tail_limit >= 0) {  // tail_limit: as for gemm()
    attach_tail(p, C);
    p.tail_max_units = (int)tail_limit;
    p.tail_min_kt = g_tail_min_kt;
  }
  check(pvr_gemm(&p, stream()), "gemm_fp8");
}

// yT[cols][ldy] (uint8 fp8) = sat(x^T * qscale), zero past x's rows (ldy: token dim padded to 128)
void fp8_quant_t(torch::Tensor x, torch::Tensor yt, torch::Tensor qscale, int64_t fmt) {
  TORCH_CHECK(x.dim() == 2 && yt.dim() == 2 && yt.size(0) == x.size(1) && yt.size(1) >= x.size(0) && yt.stride(1) == 1,
              "fp8_quant_t: yT [cols][>= rows]");
  TORCH_CHECK(yt.is_cuda() && yt.scalar_type() == torch::kUInt8 && yt.stride(0) % 64 == 0 && yt.size(1) == yt.stride(0),
              "fp8_quant_t: yT uint8, row stride a multiple of 64");
  check(pvr_fp8_quant_t(bf(x, "x"), ld_of(x, "x"), yt.data_ptr<uint8_t>(), yt.stride(0), (int)x.size(0), (int)x.size(1),
                        f32(qscale, "qscale"), (int)fmt, stream()),
        "fp8_quant_t");
}

// yT[cols][ldy] = x8^T (fp8 bytes), zero past x8's rows: the transposed wgrad operand from a row-major fp8 copy
void fp8_transpose(torch::Tensor x8, torch::Tensor yt) {
  TORCH_CHECK(x8.is_cuda() && x8.scalar_type() == torch::kUInt8 && x8.dim() == 2 && x8.stride(1) == 1 && x8.stride(0) % 16 == 0 &&
                  x8.size(1) % 16 == 0 && reinterpret_cast<uintptr_t>(x8.data_ptr()) % 16 == 0,
              "fp8_transpose: x8 uint8 [rows][cols], cols and row stride multiples of 16, 16-byte aligned");
  TORCH_CHECK(yt.is_cuda() && yt.scalar_type() == torch::kUInt8 && yt.dim() == 2 && yt.size(0) == x8.size(1) &&
                  yt.size(1) >= x8.size(0) && yt.stride(1) == 1 && yt.stride(0) % 64 == 0 && yt.size(1) == yt.stride(0) &&
                  reinterpret_cast<uintptr_t>(yt.data_ptr()) % 16 == 0,
              "fp8_transpose: yT uint8 [cols][>= rows], row stride a multiple of 64");
  check(pvr_fp8_transpose(x8.data_ptr<uint8_t>(), x8.stride(0), yt.data_ptr<uint8_t>(), yt.stride(0), (int)x8.size(0), (int)x8.size(1),
                          stream()),
        "fp8_transpose");
}

// fp8 weight gradient partials straight from the row-major fp8 copies: ws[s][N][K] = dscale_a *
// dscale_b * dy8[Ts][N]^T . x8[Ts][K] over token split s (ksplit tokens, a multiple of 128), dy8 e5m2
// (fmt_a 1) or e4m3 (fmt_a 0)
// and x8 e4m3 [T][features] (mn-contiguous operands: transposed LDS reads, no transposed copies)
void gemm_fp8_wgrad_mn(torch::Tensor dy8, torch::Tensor x8, torch::Tensor ws, int64_t N, int64_t K, int64_t T, torch::Tensor scale_a,
                       torch::Tensor scale_b, int64_t ksplit, int64_t fmt_a) {
  TORCH_CHECK((fmt_a == 0 || fmt_a == 1), "gemm_fp8_wgrad_mn: fmt_a 0 (e4m3) / 1 (e5m2)");
  TORCH_CHECK(dy8.dim() == 2 && x8.dim() == 2 && dy8.size(0) >= T && x8.size(0) >= T && dy8.size(1) >= N && x8.size(1) >= K &&
                  dy8.stride(1) == 1 && x8.stride(1) == 1,
              "gemm_fp8_wgrad_mn: dy8 [T][N], x8 [T][K] row-major");
  TORCH_CHECK(N % 16 == 0 && K % 16 == 0 && dy8.stride(0) % 16 == 0 && x8.stride(0) % 16 == 0 && ksplit % 128 == 0 &&
                  reinterpret_cast<uintptr_t>(dy8.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(x8.data_ptr()) % 16 == 0,
              "gemm_fp8_wgrad_mn: 16-byte rows and bases, ksplit a multiple of 128");
  TORCH_CHECK(T * std::max(dy8.stride(0), x8.stride(0)) < (1ll << 31), "gemm_fp8_wgrad_mn: 31-bit operand offsets");
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == torch::kFloat32 && ws.dim() == 3 && ws.stride(2) == 1 && ws.size(1) >= N &&
                  ws.size(2) >= K && ws.size(0) >= (T + ksplit - 1) / ksplit,
              "gemm_fp8_wgrad_mn: workspace [splits][N][K] f32");
  pvr::GemmParams p{};
  p.drop_scale = 1.f;
  p.M = (int)N; p.N = (int)K; p.K = (int)T;
  p.A = reinterpret_cast<const uint16_t*>(u8(dy8, "dy8")); p.lda = dy8.stride(0); p.a_kcontig = 0;
  p.B = reinterpret_cast<const uint16_t*>(u8(x8, "x8")); p.ldb = x8.stride(0); p.b_kcontig = 0;
  p.C = ws.data_ptr(); p.ldc = ws.stride(1); p.split_stride = ws.stride(0);
  p.scale_a = f32(scale_a, "scale_a"); p.scale_b = f32(scale_b, "scale_b");
  p.elem8 = 1; p.fmt_a = (int)fmt_a; p.fmt_b = 0;
  p.k_split_len = (int)ksplit;
  p.epi = 4;  // EPI_F32_STORE
  p.tile_cfg = 14;
  check(pvr_gemm(&p, stream()), "gemm_fp8_wgrad_mn");
}

// fp8 weight gradient partials: ws[s][N][K] = dscale_a * dscale_b * A8[N][Ks] . B8[K][Ks]^T over split s
// of the (padded) token dim, A e5m2 / e4m3 (fmt_a 1 / 0; gradient^T), B e4m3 (activation^T)
void gemm_fp8_wgrad(torch::Tensor A8, torch::Tensor B8, torch::Tensor ws, int64_t N, int64_t K, int64_t Tp, torch::Tensor scale_a,
                    torch::Tensor scale_b, int64_t ksplit, int64_t fmt_a) {
  TORCH_CHECK((fmt_a == 0 || fmt_a == 1), "gemm_fp8_wgrad: fmt_a 0 (e4m3) / 1 (e5m2)");
  pvr::GemmParams p{};
  p.drop_scale = 1.f;
  p.M = (int)N; p.N = (int)K; p.K = (int)Tp;
  p.A = reinterpret_cast<const uint16_t*>(u8(A8, "A8")); p.lda = A8.stride(0); p.a_kcontig = 1;
  p.B = reinterpret_cast<const uint16_t*>(u8(B8, "B8")); p.ldb = B8.stride(0); p.b_kcontig = 1;
  TORCH_CHECK(A8.size(0) >= N && A8.size(1) >= Tp && B8.size(0) >= K && B8.size(1) >= Tp, "gemm_fp8_wgrad: operand too small");
  TORCH_CHECK(Tp % 128 == 0 && ksplit % 128 == 0 && K % 8 == 0, "gemm_fp8_wgrad: Tp, ksplit multiples of 128");
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == torch::kFloat32 && ws.dim() == 3 && ws.stride(2) == 1 && ws.size(1) >= N &&
                  ws.size(2) >= K && ws.size(0) >= (Tp + ksplit - 1) / ksplit,
              "gemm_fp8_wgrad: workspace [splits][N][K] f32");
  p.C = ws.data_ptr(); p.ldc = ws.stride(1); p.split_stride = ws.stride(0);
  p.scale_a = f32(scale_a, "scale_a"); p.scale_b = f32(scale_b, "scale_b");
  p.elem8 = 1; p.fmt_a = (int)fmt_a; p.fmt_b = 0;
  p.k_split_len = (int)ksplit;
  p.epi = 4;  // EPI_F32_STORE
  p.tile_cfg = 14;
  check(pvr_gemm(&p, stream()), "gemm_fp8_wgrad");
}

// y[rows][cols] (uint8 fp8) = sat(x * qscale); amax (int32 holding float bits) = max(amax, max|x|).
// y / qscale None: amax only.
void fp8_quant(torch::Tensor x, c10::optional<torch::Tensor> y, c10::optional<torch::Tensor> qscale, torch::Tensor amax, int64_t fmt) {
  const uint16_t* xp = bf(x, "x");
  const int64_t ldx = ld_of(x, "x");
  uint8_t* yp = nullptr;
  int64_t ldy = 0;
  if (y.has_value() && y->defined()) {
    yp = const_cast<uint8_t*>(u8(*y, "y"));
    ldy = y->stride(0);
    TORCH_CHECK(y->size(0) == x.size(0) && y->size(1) == x.size(1), "fp8_quant: shape mismatch");
  }
  TORCH_CHECK(amax.is_cuda() && amax.scalar_type() == torch::kInt32 && amax.numel() >= 1, "fp8_quant: amax int32");
  const float* qs = nullptr;
  if (qscale.has_value() && qscale->defined()) qs = f32(*qscale, "qscale");
  TORCH_CHECK(yp == nullptr || qs != nullptr, "fp8_quant: y needs qscale");
  check(pvr_fp8_quant(xp, ldx, yp, ldy, x.size(0), (int)x.size(1), qs, reinterpret_cast<unsigned*>(amax.data_ptr()), (int)fmt, stream()),
        "fp8_quant");
}

torch::Tensor fp8_dequant(torch::Tensor x, c10::optional<torch::Tensor> dscale, int64_t fmt) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kUInt8 && x.is_contiguous(), "fp8_dequant: contiguous uint8");
  auto y = torch::empty(x.sizes(), x.options().dtype(torch::kFloat32));
  const float* ds = nullptr;
  if (dscale.has_value() && dscale->defined()) ds = f32(*dscale, "dscale");
  check(pvr_fp8_dequant(x.data_ptr<uint8_t>(), y.data_ptr<float>(), x.numel(), ds, (int)fmt, stream()), "fp8_dequant");
  return y;
}

// multi-tensor weight quantization: segs = int64 [nseg][5] {src bf16 ptr, dst fp8 ptr, n, slot, first
// chunk} on the device (built once by the caller), nchunks = total chunks; amax_only: record max|x|
// per slot instead of quantizing
void fp8_quant_multi(torch::Tensor segs, int64_t nchunks, c10::optional<torch::Tensor> qscale, torch::Tensor amax, int64_t fmt,
                     bool amax_only) {
  TORCH_CHECK(segs.is_cuda() && segs.scalar_type() == torch::kInt64 && segs.dim() == 2 && segs.size(1) == 5 && segs.is_contiguous(),
              "fp8_quant_multi: segs int64 [n][5]");
  TORCH_CHECK(amax.is_cuda() && amax.scalar_type() == torch::kInt32, "fp8_quant_multi: amax int32");
  const float* qs = qscale.has_value() && qscale->defined() ? f32(*qscale, "qscale") : nullptr;
  TORCH_CHECK(amax_only || qs != nullptr, "fp8_quant_multi: quantizing needs qscale");
  check(pvr_fp8_quant_multi(segs.data_ptr<int64_t>(), (int)segs.size(0), nchunks, qs, reinterpret_cast<unsigned*>(amax.data_ptr()),
                            (int)fmt, amax_only ? 1 : 0, stream()),
        "fp8_quant_multi");
}

void fp8_scale_update(torch::Tensor hist, torch::Tensor amax, torch::Tensor qscale, torch::Tensor dscale, torch::Tensor fmax, int64_t s0,
                      int64_t s1, double margin_mul) {
  TORCH_CHECK(hist.dim() == 2 && hist.is_contiguous(), "hist [n][H]");
  TORCH_CHECK(amax.scalar_type() == torch::kInt32, "amax int32");
  TORCH_CHECK(s0 >= 0 && s1 <= hist.size(0), "slot range");
  check(pvr_fp8_scale_update(f32_mut(hist, "hist"), (int)hist.size(1), reinterpret_cast<unsigned*>(amax.data_ptr()), f32_mut(qscale, "qscale"),
                             f32_mut(dscale, "dscale"), f32(fmax, "fmax"), (int)s0, (int)s1, (float)margin_mul, stream()),
        "fp8_scale_update");
}

// seed / seed_offset / drop_p: attention-probability dropout (the backward gets the same three)
std::vector<torch::Tensor> attn_fwd(torch::Tensor qkv, int64_t B, int64_t N, int64_t H, double scale, c10::optional<torch::Tensor> seed,
                                    int64_t seed_offset, double drop_p, c10::optional<torch::Tensor> q_out,
                                    c10::optional<torch::Tensor> q_scale, c10::optional<torch::Tensor> q_amax, bool q_only) {
  const int64_t D = qkv.size(1) / 3;
  auto out = torch::empty({B * N, D}, qkv.options());
  auto lse = torch::empty({B * H, N}, qkv.options().dtype(torch::kFloat32));
  TORCH_CHECK(!q_only || (q_out.has_value() && q_out->defined()), "attn_fwd: q_only needs q_out");
  TORCH_CHECK(qkv.size(0) == B * N, "attn_fwd: qkv rows != B*N");
  const DropArgs d = drop_args(seed, drop_p, "attn_fwd");
  uint8_t* q8 = nullptr;
  int64_t q8_ld = 0;
  const float* q8_qs = nullptr;
  unsigned* q8_amax = nullptr;
  if (q_out.has_value() && q_out->defined()) {
    // e4m3 copy of the output (producer-side quantization for an fp8 out-proj GEMM)
    TORCH_CHECK(q_out->is_cuda() && q_out->scalar_type() == torch::kUInt8 && q_out->dim() == 2 && q_out->size(0) >= B * N &&
                    q_out->size(1) >= D && q_out->stride(1) == 1 && q_out->stride(0) % 4 == 0,
                "attn_fwd: q_out uint8 [B*N][D]");
    TORCH_CHECK(q_scale.has_value() && q_scale->defined() && q_amax.has_value() && q_amax->defined() &&
                    q_amax->scalar_type() == torch::kInt32,
                "attn_fwd: q_out needs q_scale (f32) and q_amax (int32)");
    q8 = reinterpret_cast<uint8_t*>(q_out->data_ptr());
    q8_ld = q_out->stride(0);
    q8_qs = f32(*q_scale, "q_scale");
    q8_amax = reinterpret_cast<unsigned*>(q_amax->data_ptr<int32_t>());
  }
  check(pvr_attn_fwd(bf(qkv, "qkv"), ld_of(qkv, "qkv"), bf_mut(out, "out"), D, f32_mut(lse, "lse"), (int)B, (int)N, (int)H, (int)D,
                     (float)scale, d.seed, (uint64_t)seed_offset, d.thr, d.scale, q8, q8_ld, q8_qs, q8_amax, q_only ? 1 : 0,
                     stream()),
        "attn_fwd");
  return {out, lse};
}

// dbias[3D] += the in_proj bias gradient from the pipelined backward's [B*H][NQ][192] partials
// (per query block: dQ column sums of two query halves | dO column sums; the k slice gets none)
void attn_dbias_reduce(torch::Tensor part, int64_t B, int64_t H, torch::Tensor dbias) {
  TORCH_CHECK(dbias.is_cuda() && dbias.scalar_type() == torch::kFloat32 && dbias.is_contiguous() && dbias.numel() % (3 * H) == 0,
              "attn_dbias_reduce: f32 [3D] bias gradient");
  const int64_t DH = dbias.numel() / (3 * H);
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == torch::kFloat32 && part.is_contiguous() && part.numel() % (B * H * 3 * DH) == 0,
              "attn_dbias_reduce: f32 [B*H][R][3 * head dim] partials");
  const int64_t NQ = part.numel() / (B * H * 3 * DH);
  auto ws = torch::empty({(int64_t)pvr_attn_dbias_splits((int)B, (int)NQ) * H * 2 * DH}, part.options());
  check(pvr_attn_dbias_reduce(part.data_ptr<float>(), ws.data_ptr<float>(), dbias.data_ptr<float>(), (int)B, (int)H, (int)NQ,
                              (int)(DH * H), stream()),
        "attn_dbias_reduce");
}

// Persistent f32 dQ accumulator of the multi-key-block attention backward, one per (device, stream),
// zero-initialised once: the backward converts the accumulated dQ and zeroes it again, so no
// per-call zero fill (a 151 MB memset per layer at ViT-L/16 384 px). Deliberately never freed (a
// static tensor's destructor would run after the HIP runtime's teardown).
// drop = true: forget the cached accumulator of this (device, stream) (after a failed backward, whose
// partial sums it may still hold); the next call re-creates it with torch::zeros.
torch::Tensor dq_workspace(int64_t numel, const torch::TensorOptions& opts, bool drop = false) {
  DqWs& d = scratch_map<DqWs>()[scratch_key((int)opts.device().index())];
  if (drop) {
    d.t = torch::Tensor();
    return torch::Tensor();
  }
  // (a replaced tensor's memory returns to the caching allocator, stream-ordered)
  if (!d.t.defined() || d.t.numel() < numel) d.t = torch::zeros({numel}, opts.dtype(torch::kFloat32));
  return d.t;
}

// Scratch of the generic attention backward, one per (device, stream), grown to the largest request
// (never freed: see dq_workspace). Calls on one stream are serialised, so they share it.
torch::Tensor attn_scratch(int64_t numel, const torch::TensorOptions& opts) {
  AttnWs& d = scratch_map<AttnWs>()[scratch_key((int)opts.device().index())];
  if (!d.t.defined() || d.t.numel() < numel) d.t = torch::empty({numel}, opts.dtype(torch::kFloat32));
  return d.t;
}

// Release every per-(device, stream) scratch buffer above (split tails, split-K counters,
// deterministic partial rows, the attention backward's dQ accumulator and scratch) to the caching
// allocator. The caller makes sure no kernel still uses them (ops: _ext.free_scratch synchronizes
// first); the next call on a stream re-creates what it needs (counters zeroed again).
void free_scratch() {
  scratch_map<TailBufs>().clear();
  scratch_map<SkCounters>().clear();
  scratch_map<DetWs>().clear();
  scratch_map<DqWs>().clear();
  scratch_map<AttnWs>().clear();
}

// R > 0: for the standard layouts of this shape (qkv [T][3D], dO / O [T][D]) the backward emits the
// in_proj bias gradient as f32 [B*H][R][192] partials (pipelined or chunked kernel); 0: it does not
int64_t attn_bwd_bias_rows(int64_t B, int64_t N, int64_t H, int64_t D, bool drop) {
  return pvr_attn_bwd_part_rows((int)B, (int)N, (int)H, (int)D, 3 * D, D, D, 3 * D, drop ? 1 : 0);
}

// 1 if attn_bwd can write dQKV's e5m2 copy (q_out) for this shape with the standard layouts (the
// generic kernels write every final dQ value; not the pipelined ViT-B/16 kernel)
bool attn_bwd_q8_ok(int64_t B, int64_t N, int64_t H, int64_t D, bool drop) {
  return pvr_attn_bwd_q8_ok((int)N, drop ? 1 : 0) && !pvr_attn_bwd_uses_pipe((int)B, (int)N, (int)H, (int)D, 3 * D, D, D, 3 * D, drop ? 1 : 0);
}

// dbias: [3D] f32 accumulated with the in_proj bias gradient. dbias_part (pipelined path only,
// [B*H][ceil(N/32)][192] f32): receives the kernel's per-block partials instead, left unreduced (the
// caller reduces them, e.g. on the weight-gradient side stream: attn_dbias_reduce).
torch::Tensor attn_bwd(torch::Tensor dout, torch::Tensor qkv, torch::Tensor out, torch::Tensor lse, int64_t B, int64_t N, int64_t H,
                       double scale, c10::optional<torch::Tensor> dbias, c10::optional<torch::Tensor> dbias_part_out,
                       c10::optional<torch::Tensor> seed, int64_t seed_offset, double drop_p, c10::optional<torch::Tensor> q_out,
                       c10::optional<torch::Tensor> q_scale, c10::optional<torch::Tensor> q_amax, bool q_only,
                       int64_t q_fmt) {
  const int64_t D = qkv.size(1) / 3;
  auto dqkv = torch::empty_like(qkv);
  torch::Tensor dq_acc;
  int dq_rezero = 0;
  const DropArgs drop = drop_args(seed, drop_p, "attn_bwd");
  const int has_drop = drop.seed ? 1 : 0;
  const int64_t dh = D / H;
  // fused in_proj bias gradient: per-(batch, head, row) partials written by the kernels (no atomics;
  // pipelined kernel: per 32-query block, generic kernel: one row per pair), reduced below
  torch::Tensor dbias_part, old_part;
  const bool want_db = dbias.has_value() && dbias->defined();
  const int64_t lds[4] = {ld_of(qkv, "qkv"), ld_of(dout, "dout"), ld_of(out, "out"), ld_of(dqkv, "dqkv")};
  const int prow = pvr_attn_bwd_part_rows((int)B, (int)N, (int)H, (int)D, lds[0], lds[1], lds[2], lds[3], has_drop);
  const bool parts = prow > 0;  // the kernels write [B*H][prow][3*dh] partials
  const bool pipe = pvr_attn_bwd_uses_pipe((int)B, (int)N, (int)H, (int)D, lds[0], lds[1], lds[2], lds[3], has_drop) != 0;
  const bool part_out = dbias_part_out.has_value() && dbias_part_out->defined();
  if (part_out) {
    TORCH_CHECK(parts && !want_db, "dbias_part: shapes with attn_bwd_bias_rows > 0 only, and not together with dbias");
    TORCH_CHECK(dbias_part_out->is_cuda() && dbias_part_out->scalar_type() == torch::kFloat32 && dbias_part_out->is_contiguous() &&
                    dbias_part_out->numel() == B * H * prow * 3 * dh,
                "dbias_part [B*H][attn_bwd_bias_rows][3 * head dim] f32");
    dbias_part = *dbias_part_out;
  }
  if (want_db) {
    TORCH_CHECK(dbias->numel() == 3 * D && dbias->scalar_type() == torch::kFloat32 && dbias->is_contiguous(), "dbias [3D] f32");
    if (parts)  // q sums of the two 16-query fragment rows | v sums, per (batch, head, row)
      dbias_part = torch::empty({B * H, (int64_t)prow, 3 * dh}, qkv.options().dtype(torch::kFloat32));
    else if (2 * (dh / 16) <= 2 * pvr_attn_bwd_waves((int)N))
      old_part = torch::empty({B * pvr_attn_bwd_key_blocks((int)N), 3 * D}, qkv.options().dtype(torch::kFloat32));
  }
  const int old_db = old_part.defined() ? 1 : 0;
  if (pvr_attn_bwd_needs_dq_acc((int)N, (int)dh, old_db, has_drop, g_deterministic ? 1 : 0)) {
    // several key blocks per head and neither the lastkey nor the tail-split slab path (e.g. N = 677):
    // dQ is summed with f32 atomics (deterministic mode: per-key-block slabs summed in order instead)
    dq_acc = dq_workspace(B * N * D, qkv.options());
    dq_rezero = dq_acc.defined() ? 1 : 0;
    if (!dq_acc.defined()) dq_acc = torch::zeros({B * N, D}, qkv.options().dtype(torch::kFloat32));
  }
  // optional e5m2 copy of dQKV + amax record (the fp8 recipe's dgrad / weight-gradient operand)
  uint8_t* qp = nullptr;
  int64_t ldq = 0;
  const float* qs = nullptr;
  unsigned* qa = nullptr;
  if (q_out.has_value() && q_out->defined()) {
    TORCH_CHECK(pvr_attn_bwd_q8_ok((int)N, has_drop) && !old_db && !pipe, "attn_bwd: no e5m2 dQKV copy for this shape (see attn_bwd_q8_ok)");
    TORCH_CHECK(q_out->is_cuda() && q_out->scalar_type() == torch::kUInt8 && q_out->dim() == 2 && q_out->stride(1) == 1 &&
                    q_out->size(0) >= B * N && q_out->size(1) >= 3 * D && q_out->stride(0) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(q_out->data_ptr()) % 4 == 0,
                "attn_bwd: q_out uint8 [B*N][>= 3D], row stride a multiple of 4");
    TORCH_CHECK(q_scale.has_value() && q_scale->defined() && q_amax.has_value() && q_amax->defined() && q_amax->is_cuda() &&
                    q_amax->scalar_type() == torch::kInt32,
                "attn_bwd: q_out needs q_scale (f32) and q_amax (int32)");
    qp = q_out->data_ptr<uint8_t>();
    ldq = q_out->stride(0);
    qs = f32(*q_scale, "q_scale");
    qa = reinterpret_cast<unsigned*>(q_amax->data_ptr());
  }
  float* dbias_arg = pipe && dbias_part.defined() ? dbias_part.data_ptr<float>() : old_db ? old_part.data_ptr<float>() : nullptr;
  float* bpart_arg = !pipe && dbias_part.defined() ? dbias_part.data_ptr<float>() : nullptr;
  // pre-pass outputs of the generic backward (per-query delta, lastkey path: ds_last; slab path: dQ
  // slabs): a persistent per-(device, stream) scratch, so the slab path (~0.9 GB per ViT-L/16@384
  // b128 layer) is not allocated on every backward
  auto ws = attn_scratch(pvr_attn_bwd_ws_floats((int)B, (int)N, (int)H, (int)D, old_db, has_drop, g_deterministic ? 1 : 0), qkv.options());
  const hipError_t err = pvr_attn_bwd(bf(qkv, "qkv"), lds[0], bf(out, "out"), lds[2], bf(dout, "dout"), lds[1], f32(lse, "lse"),
                                      bf_mut(dqkv, "dqkv"), lds[3], dq_acc.defined() ? dq_acc.data_ptr<float>() : nullptr, dq_rezero,
                                      dbias_arg, bpart_arg, ws.data_ptr<float>(), (int)B, (int)N, (int)H, (int)D, (float)scale,
                                      drop.seed, (uint64_t)seed_offset, drop.thr, drop.scale, qp, ldq, qs, qa, q_only && qp ? 1 : 0,
                                      (int)q_fmt, stream());
  // a persistent accumulator is re-zeroed only by a completed backward: after a failed launch it
  // may hold stale partial sums, so it is dropped (re-created zeroed by the next call)
  if (err != hipSuccess && dq_rezero) dq_workspace(0, qkv.options(), true);
  check(err, "attn_bwd");
  if (want_db) {
    if (parts)
      attn_dbias_reduce(dbias_part, B, H, *dbias);
    else if (old_db)
      dbias->add_(old_part.sum(0));
    else
      dbias->add_(dqkv.sum(0, false, torch::kFloat32));
  }
  return dqkv;
}

}  // namespace

extern "C" const char* pvr_src_hash(void);  // _build/src_hash.c (build.py): hash of csrc/*

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X (gfx950) HIP kernels for pytorch_vit_paper_replication_amd";
  m.def("source_hash", []() { return std::string(pvr_src_hash()); },
        "content hash of the csrc/ sources this binary was built from (build.source_hash())");
  m.def("gemm_tail_split", [](int64_t M, int64_t N, int64_t K, int64_t elem_bytes, int64_t max_units) {
    return pvr_gemm_tail_split((int)M, (int)N, (int)K, (int)elem_bytes, (int)max_units); },
    py::arg("M"), py::arg("N"), py::arg("K"), py::arg("elem_bytes"), py::arg("max_units") = 0,
    "K-parts of the split tail round this GEMM shape gets (0: none)");
  m.def("set_attn_dbg", [](torch::Tensor t) { pvr_set_attn_dbg(t.defined() && t.numel() ? t.data_ptr() : nullptr); },
        "diagnostic builds (-DPVR_ATTN_STAMPS): int64 buffer for the attention backward's phase stamps "
        "[workgroup * waves + wave][8] (scripts/attn_stamps.py); a no-op otherwise");
  m.def("set_attn_prep_xcd", &pvr_set_attn_prep_xcd, "attention backward pre-pass: XCD-contiguous (batch, head) pairs (1) or round-robin (0, default); A/B");
  m.def("set_ln_fwd_q8_grid", &pvr_set_ln_fwd_q8_grid, "LayerNorm forward with the e4m3 copy: grid cap in workgroups per CU (A/B)");
  m.def("set_attn_fwd_head_qf", &pvr_set_attn_fwd_head_qf, "whole-head attention forward (dh 64, N <= 256): 16-query fragments per wave (1 = default, 2 = half the LDS reads with 7 waves; A/B)");
  m.def("set_attn_fwd_qg", &pvr_set_attn_fwd_qg, "tiled attention forward: 16-query groups per wave (0 = auto by query padding, 1 = round-3 form, 2 = forced; A/B)");
  m.def("set_fp8_persistent", &pvr_set_fp8_persistent, "fp8 fwd/dgrad GEMMs on the persistent ping-pong: 1 when the epilogue has no per-row input (default), 0 never (A/B)");
  m.def("set_deterministic", &set_deterministic, "deterministic reductions (partial rows + ordered sum) instead of float atomics");
  m.def("deterministic", &deterministic);
  m.def("set_gemm_tail", &set_gemm_tail, "split-K tail of the last dispatch round on (True, default) / off (A/B)");
  m.def("gemm", &gemm,py::arg("A"), py::arg("a_kcontig"), py::arg("B"), py::arg("b_kcontig"), py::arg("C"),
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("epi"), py::arg("bias"), py::arg("resid"), py::arg("addend"),
        py::arg("addend_period"), py::arg("aux"), py::arg("row_group"), py::arg("row_stride_group"),
        py::arg("row_offset"), py::arg("seed"), py::arg("seed_offset"), py::arg("drop_p"), py::arg("k_split"),
        py::arg("tile_cfg"), py::arg("dbg") = py::none(), py::arg("colsum") = py::none(),
        py::arg("epi_staged") = 0, py::arg("tail_limit") = 0, py::arg("reduce_out") = py::none(), py::arg("reduce_acc") = true);
  m.def("splitk_timeouts", &splitk_timeouts, py::arg("like"), py::arg("reset") = false);
  m.def("num_cus", &num_cus);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("free_scratch", &free_scratch);
  m.def("layernorm_fwd_q8", &layernorm_fwd_q8);
  m.def("layernorm_bwd", &layernorm_bwd, py::arg("dy"), py::arg("dy_stride"), py::arg("x"), py::arg("x_stride"),
        py::arg("mean"), py::arg("rstd"), py::arg("w"), py::arg("dres"), py::arg("dres_stride"), py::arg("dx"),
        py::arg("dx_stride"), py::arg("dw"), py::arg("db"), py::arg("rows"), py::arg("dsum") = py::none(),
        py::arg("dz") = py::none(), py::arg("seed") = py::none(), py::arg("seed_offset") = 0, py::arg("drop_p") = 0.0,
        py::arg("q_out") = py::none(), py::arg("q_scale") = py::none(), py::arg("q_amax") = py::none(),
        py::arg("dz_nostore") = false, py::arg("q_fmt") = 1);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("splitk_epilogue", &splitk_epilogue);
  m.def("attn_bwd_bias_rows", &attn_bwd_bias_rows, py::arg("B"), py::arg("N"), py::arg("H"), py::arg("D"), py::arg("drop") = false);
  m.def("attn_dbias_reduce", &attn_dbias_reduce);
  m.def("splitk_reduce", &splitk_reduce);
  m.def("pad_cols_bf16", &pad_cols_bf16);
  m.def("transpose_batched", &transpose_batched);
  m.def("colsum", &colsum, py::arg("dy"), py::arg("rows"), py::arg("N"), py::arg("db"), py::arg("dz"), py::arg("seed"),
        py::arg("seed_offset"), py::arg("drop_p"), py::arg("q_out") = py::none(), py::arg("q_scale") = py::none(),
        py::arg("q_amax") = py::none(), py::arg("q_fmt") = 1);
  m.def("im2col", &im2col);
  m.def("cls_rows", &cls_rows);
  m.def("patch_bwd", &patch_bwd);
  m.def("xent", &xent, py::arg("logits"), py::arg("labels"), py::arg("dlogits"), py::arg("correct"), py::arg("grad_scale"),
        py::arg("mean") = py::none());
  m.def("grad_norm", &grad_norm);
  m.def("norm_partial_blocks", []() { return pvr_norm_partial_blocks(); });
  m.def("adam", &adam);
  m.def("adam_t", &adam_t);
  m.def("scale_by_clip", &scale_by_clip);
  m.def("head_fwd", &head_fwd);
  m.def("head_bwd", &head_bwd, py::arg("dlogits"), py::arg("xhat"), py::arg("rstd"), py::arg("gamma"), py::arg("beta"), py::arg("W"),
        py::arg("B"), py::arg("N"), py::arg("dW") = py::none(), py::arg("db") = py::none(), py::arg("dgamma") = py::none(),
        py::arg("dbeta") = py::none());
  m.def("scale_by", &scale_by);
  m.def("metrics_accum", &metrics_accum);
  m.def("rng_next", &rng_next);
  m.def("zero_f32", &zero_f32);
  m.def("gemm_fp8", &gemm_fp8, py::arg("A"), py::arg("fmt_a"), py::arg("B"), py::arg("fmt_b"), py::arg("C"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("epi"), py::arg("scale_a"), py::arg("scale_b"), py::arg("bias") = py::none(),
        py::arg("resid") = py::none(), py::arg("aux") = py::none(), py::arg("seed") = py::none(), py::arg("seed_offset") = 0,
        py::arg("drop_p") = 0.0, py::arg("colsum") = py::none(), py::arg("q_out") = py::none(), py::arg("q_scale") = py::none(),
        py::arg("q_amax") = py::none(), py::arg("q_fmt") = 0, py::arg("c_skip") = false, py::arg("tail_limit") = 0);
  m.def("fp8_transpose", &fp8_transpose);
  m.def("gemm_fp8_wgrad_mn", &gemm_fp8_wgrad_mn, py::arg("dy8"), py::arg("x8"), py::arg("ws"), py::arg("N"), py::arg("K"),
        py::arg("T"), py::arg("scale_a"), py::arg("scale_b"), py::arg("ksplit"), py::arg("fmt_a") = 1);
  m.def("fp8_quant", &fp8_quant, py::arg("x"), py::arg("y"), py::arg("qscale"), py::arg("amax"), py::arg("fmt"));
  m.def("fp8_dequant", &fp8_dequant, py::arg("x"), py::arg("dscale") = py::none(), py::arg("fmt") = 0);
  m.def("fp8_scale_update", &fp8_scale_update);
  m.def("fp8_quant_t", &fp8_quant_t);
  m.def("gemm_fp8_wgrad", &gemm_fp8_wgrad, py::arg("A8"), py::arg("B8"), py::arg("ws"), py::arg("N"), py::arg("K"), py::arg("Tp"),
        py::arg("scale_a"), py::arg("scale_b"), py::arg("ksplit"), py::arg("fmt_a") = 1);
  m.def("fp8_quant_multi", &fp8_quant_multi, py::arg("segs"), py::arg("nchunks"), py::arg("qscale"), py::arg("amax"), py::arg("fmt"),
        py::arg("amax_only"));
  m.def("attn_fwd", &attn_fwd, py::arg("qkv"), py::arg("B"), py::arg("N"), py::arg("H"), py::arg("scale"),
        py::arg("seed") = py::none(), py::arg("seed_offset") = 0, py::arg("drop_p") = 0.0, py::arg("q_out") = py::none(),
        py::arg("q_scale") = py::none(), py::arg("q_amax") = py::none(), py::arg("q_only") = false);
  m.def("attn_bwd", &attn_bwd, py::arg("dout"), py::arg("qkv"), py::arg("out"), py::arg("lse"), py::arg("B"), py::arg("N"),
        py::arg("H"), py::arg("scale"), py::arg("dbias") = py::none(), py::arg("dbias_part") = py::none(),
        py::arg("seed") = py::none(), py::arg("seed_offset") = 0, py::arg("drop_p") = 0.0, py::arg("q_out") = py::none(),
        py::arg("q_scale") = py::none(), py::arg("q_amax") = py::none(), py::arg("q_only") = false,
        py::arg("q_fmt") = 1);
  m.def("attn_bwd_q8_ok", &attn_bwd_q8_ok, "attn_bwd can write dQKV's e5m2 copy for this shape");
  m.def("arch", []() { return std::string("gfx950"); });
}
