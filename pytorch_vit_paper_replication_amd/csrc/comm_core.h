// Transport-agnostic collective schedules of the native communicator.
//
// xGMI on an MI355X node is a full mesh of point-to-point links (7 per GPU). A ring all-reduce
// drives one outgoing link per GPU at a time; the "mesh" all-reduce here sends to every peer at
// once instead:
//   reduce-scatter: the buffer is cut into `world` chunks; chunk p goes to rank p from every other
//                   rank (all world-1 sends in one group), rank p sums what it received into its
//                   own chunk (and scales it for an average);
//   all-gather:     every rank sends its reduced chunk to every peer (again one group).
// Each rank moves 2 (W-1)/W of the buffer, the same bytes as a ring, but over all links at once.
//
// The schedule is written against a small Transport interface (grouped point-to-point send/recv
// plus a local "sum k chunks" reduction), so the same code runs on RCCL (ncclSend / ncclRecv on the
// communicator's HIP stream, a HIP reduction kernel; csrc/comm.cpp) and on an in-process fake
// transport of threads and host buffers (tests/cpp/test_comm_core.cpp), which is how the slicing,
// peer and offset logic is unit-tested without a multi-GPU node. No HIP / torch dependencies.
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>

namespace pvr_comm {

// Element range [begin, end) of chunk c when n elements are cut into `world` chunks whose
// boundaries are multiples of `align` elements (the last chunk takes the remainder; chunks may be
// empty when n is small).
struct ChunkRange {
  size_t begin, end;
  size_t size() const { return end - begin; }
};

inline ChunkRange chunk_of(size_t n, int world, int c, size_t align = 64) {
  if (world <= 0 || c < 0 || c >= world) throw std::invalid_argument("chunk_of: bad rank/world");
  const size_t units = (n + align - 1) / align;  // align-sized units, spread as evenly as possible
  const size_t base = units / (size_t)world, extra = units % (size_t)world;
  auto start = [&](int k) {
    const size_t u = (size_t)k * base + ((size_t)k < extra ? (size_t)k : extra);
    const size_t e = u * align;
    return e < n ? e : n;
  };
  return ChunkRange{start(c), start(c + 1)};
}

// Largest chunk (scratch sizing for the reduce-scatter).
inline size_t max_chunk(size_t n, int world, size_t align = 64) {
  size_t m = 0;
  for (int c = 0; c < world; ++c) {
    const size_t s = chunk_of(n, world, c, align).size();
    m = s > m ? s : m;
  }
  return m;
}

// What a collective schedule needs from the wire and the device.
class Transport {
 public:
  virtual ~Transport() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // sends / receives between group_start and group_end are posted together (none blocks the others)
  virtual void group_start() = 0;
  virtual void group_end() = 0;
  virtual void send(const void* buf, size_t bytes, int peer) = 0;
  virtual void recv(void* buf, size_t bytes, int peer) = 0;
  // dst[i] = scale * (dst[i] + sum_{j < k} src[j * stride + i]) for i < n (fp32, in stream order
  // after the group that filled src)
  virtual void sum_into(float* dst, const float* src, int k, size_t n, size_t stride, float scale) = 0;
};

// In-place mesh all-reduce of n fp32 elements. scratch: (world - 1) * max_chunk(n, world) floats.
inline void mesh_all_reduce(Transport& tr, float* buf, size_t n, float* scratch, bool average, size_t align = 64) {
  const int W = tr.world(), r = tr.rank();
  if (W == 1) {
    return;  // nothing to exchange; an average over one rank is the identity
  }
  const ChunkRange mine = chunk_of(n, W, r, align);
  const size_t stride = max_chunk(n, W, align);
  // reduce-scatter: chunk p of my buffer -> rank p; peers' copies of my chunk -> scratch slots
  tr.group_start();
  int slot = 0;
  for (int d = 1; d < W; ++d) {
    const int p = (r + d) % W;  // staggered peer order: every rank starts on a different link
    const ChunkRange cp = chunk_of(n, W, p, align);
    if (cp.size()) tr.send(buf + cp.begin, cp.size() * sizeof(float), p);
    const int q = (r - d + W) % W;
    if (mine.size()) tr.recv(scratch + (size_t)slot * stride, mine.size() * sizeof(float), q);
    ++slot;
  }
  tr.group_end();
  if (mine.size()) tr.sum_into(buf + mine.begin, scratch, W - 1, mine.size(), stride, average ? 1.0f / (float)W : 1.0f);
  // all-gather: my reduced chunk -> every peer; their chunks -> their ranges of my buffer
  tr.group_start();
  for (int d = 1; d < W; ++d) {
    const int p = (r + d) % W;
    if (mine.size()) tr.send(buf + mine.begin, mine.size() * sizeof(float), p);
    const int q = (r - d + W) % W;
    const ChunkRange cq = chunk_of(n, W, q, align);
    if (cq.size()) tr.recv(buf + cq.begin, cq.size() * sizeof(float), q);
  }
  tr.group_end();
}

}  // namespace pvr_comm
