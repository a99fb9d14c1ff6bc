// Native RCCL communicator for data-parallel gradient exchange over xGMI.
//
// The reference trains on one device (no collectives at all); this is the
// MI355X-native DP transport the framework adds:
//   * one communicator per process (one process per GPU), bootstrapped from an ncclUniqueId that
//     rank 0 creates and the Python side broadcasts over the torch.distributed store;
//   * every collective runs on the communicator's own (normal-priority) HIP stream, ordered after the
//     work already queued on the caller's stream by an event (no host synchronisation), so bucket
//     all-reduces overlap the rest of the backward pass;
//   * completion is joined back into the caller's stream with hipStreamWaitEvent — the optimizer
//     kernels queue behind the last bucket without a host round trip;
//   * RCCL entry points are resolved with dlsym from the librccl.so.1 already mapped by PyTorch
//     (falling back to dlopen), so exactly one RCCL runtime lives in the process.
#include <dlfcn.h>

#include <stdexcept>
#include <string>
#include <vector>

#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "comm_core.h"

extern "C" hipError_t pvr_sum_chunks(float* dst, const float* src, int k, int64_t n, int64_t stride, float scale, hipStream_t s);

namespace pvr_comm {
namespace {

struct Api {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGetVersion) get_version = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  bool ok = false;
  std::string err;
};

template <typename F>
void sym(void* h, const char* name, F& out, std::string& err) {
  out = reinterpret_cast<F>(dlsym(h, name));
  if (!out) err += std::string(" missing ") + name;
}

const Api& api() {
  static Api a = [] {
    Api r;
    // The RCCL torch already mapped: the wheel bundles its own (SONAME librccl.so), a system copy
    // would be a second RCCL runtime in the process (measured 6 % slower steps at world 1 when
    // /opt/rocm's librccl.so.1 was loaded beside torch's)
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      r.err = std::string("cannot load librccl: ") + dlerror();
      return r;
    }
    sym(h, "ncclGetUniqueId", r.get_unique_id, r.err);
    sym(h, "ncclCommInitRank", r.init_rank, r.err);
    sym(h, "ncclCommDestroy", r.destroy, r.err);
    sym(h, "ncclAllReduce", r.all_reduce, r.err);
    sym(h, "ncclBroadcast", r.broadcast, r.err);
    sym(h, "ncclReduceScatter", r.reduce_scatter, r.err);
    sym(h, "ncclAllGather", r.all_gather, r.err);
    sym(h, "ncclGetErrorString", r.error_string, r.err);
    sym(h, "ncclGetVersion", r.get_version, r.err);
    sym(h, "ncclSend", r.send, r.err);
    sym(h, "ncclRecv", r.recv, r.err);
    sym(h, "ncclGroupStart", r.group_start, r.err);
    sym(h, "ncclGroupEnd", r.group_end, r.err);
    r.ok = r.err.empty();
    return r;
  }();
  return a;
}

const Api& need_api() {
  const Api& a = api();
  TORCH_CHECK(a.ok, "RCCL unavailable:", a.err);
  return a;
}

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    const Api& a = api();
    TORCH_CHECK(false, "RCCL ", what, " failed: ", a.error_string ? a.error_string(r) : "?", " (", (int)r, ")");
  }
}

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "HIP ", what, " failed: ", hipGetErrorString(e));
}

ncclDataType_t dtype_of(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kFloat32: return ncclFloat32;
    case torch::kBFloat16: return ncclBfloat16;
    case torch::kFloat16: return ncclFloat16;
    case torch::kFloat64: return ncclFloat64;
    case torch::kInt32: return ncclInt32;
    case torch::kInt64: return ncclInt64;
    case torch::kUInt8: return ncclUint8;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL: ", t.scalar_type());
  }
  return ncclFloat32;
}

// comm_core.h's Transport over RCCL: grouped ncclSend / ncclRecv on the communicator's stream
// (all world-1 peers of a phase at once: every xGMI link busy), local sums by a HIP kernel.
class RcclTransport : public Transport {
 public:
  RcclTransport(ncclComm_t comm, hipStream_t stream, int rank, int world) : comm_(comm), stream_(stream), rank_(rank), world_(world) {}
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void group_start() override { nccl_check(api().group_start(), "ncclGroupStart"); }
  void group_end() override { nccl_check(api().group_end(), "ncclGroupEnd"); }
  void send(const void* buf, size_t bytes, int peer) override {
    nccl_check(api().send(buf, bytes, ncclUint8, peer, comm_, stream_), "ncclSend");
  }
  void recv(void* buf, size_t bytes, int peer) override { nccl_check(api().recv(buf, bytes, ncclUint8, peer, comm_, stream_), "ncclRecv"); }
  void sum_into(float* dst, const float* src, int k, size_t n, size_t stride, float scale) override {
    hip_check(pvr_sum_chunks(dst, src, k, (int64_t)n, (int64_t)stride, scale, stream_), "sum_chunks");
  }

 private:
  ncclComm_t comm_;
  hipStream_t stream_;
  int rank_, world_;
};

}  // namespace

class Communicator {
 public:
  Communicator(const std::string& uid_bytes, int rank, int world, int device)
      : rank_(rank), world_(world), device_(device),
        stream_(c10::hip::getStreamFromPool(/*isHighPriority=*/false, (c10::DeviceIndex)device)) {
    const Api& a = need_api();
    TORCH_CHECK(uid_bytes.size() == sizeof(ncclUniqueId), "bad unique id size ", uid_bytes.size());
    TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "bad rank/world ", rank, "/", world);
    ncclUniqueId uid;
    memcpy(&uid, uid_bytes.data(), sizeof(uid));
    c10::hip::HIPGuard guard((c10::DeviceIndex)device);
    nccl_check(a.init_rank(&comm_, world, uid, rank), "ncclCommInitRank");
    events_.resize(kEvents);
    for (auto& e : events_) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    ready_.resize(kEvents);
    for (auto& e : ready_) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    one_ = torch::ones({1}, torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device));
  }

  ~Communicator() {
    // Communicator teardown at interpreter exit can race the HIP runtime's own teardown: only an
    // explicit destroy() releases the RCCL communicator; events are process-lifetime.
  }

  static std::string unique_id() {
    const Api& a = need_api();
    ncclUniqueId uid;
    nccl_check(a.get_unique_id(&uid), "ncclGetUniqueId");
    return std::string(reinterpret_cast<const char*>(&uid), sizeof(uid));
  }

  static int version() {
    const Api& a = need_api();
    int v = 0;
    nccl_check(a.get_version(&v), "ncclGetVersion");
    return v;
  }

  // Queue an in-place all-reduce of `t` on the comm stream behind everything already queued on the
  // caller's current stream. Returns a handle for wait().
  int64_t all_reduce_async(torch::Tensor t, bool average) {
    live();
    check_tensor(t);
    const int64_t h = gate();
    nccl_check(api().all_reduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), average ? ncclAvg : ncclSum, comm_,
                                stream_.stream()),
               "ncclAllReduce");
    return finish(h);
  }

  // The same all-reduce with the framework's own schedule (comm_core.h mesh: reduce-scatter and
  // all-gather as grouped point-to-point transfers to every peer at once) instead of RCCL's
  // all-reduce algorithm; fp32 only. Its slicing / peer logic is unit-tested on a fake transport
  // (tests/cpp/test_comm_core.cpp).
  int64_t all_reduce_mesh_async(torch::Tensor t, bool average) {
    live();
    check_tensor(t);
    TORCH_CHECK(t.scalar_type() == torch::kFloat32, "mesh all-reduce: fp32 tensors");
    const size_t n = (size_t)t.numel();
    const size_t need = mesh_scratch_elems(n);
    // sized once at setup (reserve_mesh): growing here would need a stream sync mid-backward, since
    // earlier collectives on the in-order comm stream may still read the old scratch
    TORCH_CHECK(need == 0 || (scratch_.defined() && (size_t)scratch_.numel() >= need),
                "mesh all-reduce of ", n, " elements needs reserve_mesh(>= ", n, ") first");
    const int64_t h = gate();
    RcclTransport tr(comm_, stream_.stream(), rank_, world_);
    mesh_all_reduce(tr, t.data_ptr<float>(), n, need ? scratch_.data_ptr<float>() : nullptr, average);
    return finish(h);
  }

  size_t mesh_scratch_elems(size_t n) const { return (size_t)(world_ > 1 ? world_ - 1 : 0) * max_chunk(n, world_); }

  // Allocate the mesh all-reduce scratch for messages of up to max_numel elements (call at setup,
  // before any collective is in flight: no synchronisation is needed then).
  void reserve_mesh(int64_t max_numel) {
    const size_t need = mesh_scratch_elems((size_t)max_numel);
    if (need > 0 && (!scratch_.defined() || (size_t)scratch_.numel() < need)) {
      hip_check(hipStreamSynchronize(stream_.stream()), "hipStreamSynchronize");  // setup only
      scratch_ = torch::empty({(int64_t)need}, torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device_));
    }
  }

  // out[world * n] <- all ranks' in[n] (stream-ordered like all_reduce_async)
  int64_t all_gather_async(torch::Tensor in, torch::Tensor out) {
    live();
    check_tensor(in);
    check_tensor(out);
    TORCH_CHECK(out.numel() == in.numel() * world_ && out.scalar_type() == in.scalar_type(), "all_gather: size/dtype");
    const int64_t h = gate();
    nccl_check(api().all_gather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), dtype_of(in), comm_, stream_.stream()),
               "ncclAllGather");
    return finish(h);
  }

  // out[n] <- reduce(in[world * n]) slice of this rank
  int64_t reduce_scatter_async(torch::Tensor in, torch::Tensor out, bool average) {
    live();
    check_tensor(in);
    check_tensor(out);
    TORCH_CHECK(in.numel() == out.numel() * world_ && out.scalar_type() == in.scalar_type(), "reduce_scatter: size/dtype");
    const int64_t h = gate();
    nccl_check(api().reduce_scatter(in.data_ptr(), out.data_ptr(), (size_t)out.numel(), dtype_of(in), average ? ncclAvg : ncclSum,
                                    comm_, stream_.stream()),
               "ncclReduceScatter");
    return finish(h);
  }

  int64_t broadcast_async(torch::Tensor t, int root) {
    live();
    check_tensor(t);
    const int64_t h = gate();
    nccl_check(api().broadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), root, comm_, stream_.stream()),
               "ncclBroadcast");
    return finish(h);
  }

  // Make the caller's current stream wait for collective `h` (no host synchronisation).
  void wait(int64_t h) {
    TORCH_CHECK(h >= issued_ - kEvents && h < issued_, "stale or unknown collective handle ", h);
    hip_check(hipStreamWaitEvent(caller(), events_[h % kEvents], 0), "hipStreamWaitEvent");
  }

  // Caller's stream waits for every collective issued so far.
  void wait_all() {
    if (issued_ > 0) wait(issued_ - 1);  // the comm stream is in-order
  }

  // Host-blocking barrier: a one-element all-reduce, then synchronise the comm stream.
  void barrier() {
    live();
    const int64_t h = gate();
    nccl_check(api().all_reduce(one_.data_ptr(), one_.data_ptr(), 1, ncclFloat32, ncclMax, comm_, stream_.stream()), "barrier");
    finish(h);
    hip_check(hipStreamSynchronize(stream_.stream()), "hipStreamSynchronize");
  }

  void synchronize() { hip_check(hipStreamSynchronize(stream_.stream()), "hipStreamSynchronize"); }

  void destroy() {
    if (comm_) {
      hip_check(hipStreamSynchronize(stream_.stream()), "hipStreamSynchronize");
      nccl_check(api().destroy(comm_), "ncclCommDestroy");
      comm_ = nullptr;
    }
  }

  int rank() const { return rank_; }
  int world() const { return world_; }
  int64_t issued() const { return issued_; }
  int64_t stream_handle() const { return (int64_t)(intptr_t)stream_.stream(); }

 private:
  static constexpr int kEvents = 256;

  hipStream_t caller() const { return c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream(); }

  void live() const { TORCH_CHECK(comm_ != nullptr, "communicator destroyed"); }

  void check_tensor(const torch::Tensor& t) const {
    TORCH_CHECK(t.is_cuda() && t.get_device() == device_, "collective tensor must live on cuda:", device_);
    TORCH_CHECK(t.is_contiguous(), "collective tensor must be contiguous");
  }

  // comm stream waits for the caller's queued work; returns the handle of the next collective
  int64_t gate() {
    hipEvent_t r = ready_[issued_ % kEvents];
    hip_check(hipEventRecord(r, caller()), "hipEventRecord");
    hip_check(hipStreamWaitEvent(stream_.stream(), r, 0), "hipStreamWaitEvent");
    return issued_;
  }

  int64_t finish(int64_t h) {
    hip_check(hipEventRecord(events_[h % kEvents], stream_.stream()), "hipEventRecord");
    issued_ = h + 1;
    return h;
  }

  int rank_, world_, device_;
  c10::hip::HIPStream stream_;
  ncclComm_t comm_ = nullptr;
  std::vector<hipEvent_t> events_, ready_;
  int64_t issued_ = 0;
  torch::Tensor one_, scratch_;
};

void register_comm(pybind11::module& m) {
  namespace py = pybind11;
  m.def("rccl_available", [] { return api().ok; });
  m.def("rccl_error", [] { return api().err; });
  m.def("rccl_path", [] {  // file the resolved RCCL entry points live in
    Dl_info info;
    const Api& a = api();
    if (a.get_version && dladdr(reinterpret_cast<void*>(a.get_version), &info) && info.dli_fname) return std::string(info.dli_fname);
    return std::string();
  });
  m.def("rccl_version", &Communicator::version);
  m.def("rccl_unique_id", [] { return py::bytes(Communicator::unique_id()); });
  py::class_<Communicator>(m, "Communicator")
      .def(py::init([](py::bytes uid, int rank, int world, int device) {
             return new Communicator(std::string(uid), rank, world, device);
           }),
           py::arg("unique_id"), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def("all_reduce_async", &Communicator::all_reduce_async, py::arg("tensor"), py::arg("average") = true)
      .def("all_reduce_mesh_async", &Communicator::all_reduce_mesh_async, py::arg("tensor"), py::arg("average") = true)
      .def("reserve_mesh", &Communicator::reserve_mesh, py::arg("max_numel"))
      .def("all_gather_async", &Communicator::all_gather_async)
      .def("reduce_scatter_async", &Communicator::reduce_scatter_async, py::arg("input"), py::arg("output"),
           py::arg("average") = true)
      .def("broadcast_async", &Communicator::broadcast_async, py::arg("tensor"), py::arg("root") = 0)
      .def("wait", &Communicator::wait)
      .def("wait_all", &Communicator::wait_all)
      .def("barrier", &Communicator::barrier)
      .def("synchronize", &Communicator::synchronize)
      .def("destroy", &Communicator::destroy)
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("world", &Communicator::world)
      .def_property_readonly("issued", &Communicator::issued)
      .def_property_readonly("stream_handle", &Communicator::stream_handle);
}

}  // namespace pvr_comm
