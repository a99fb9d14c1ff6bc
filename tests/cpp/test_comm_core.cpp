// Fake-transport unit test of the native communicator's collective schedule (csrc/comm_core.h):
// W threads, one per "rank", exchange host buffers through an in-process mailbox hub that plays
// the role of RCCL's grouped ncclSend / ncclRecv. Checks the mesh all-reduce (sum and average)
// against a directly computed reference for many world sizes and buffer lengths, including
// lengths that leave chunks empty or uneven, and that every posted receive is matched exactly.
// Built and run by tests/test_comm_fake_transport.py (g++ -pthread, no GPU).
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <thread>
#include <tuple>
#include <vector>

#include "comm_core.h"

namespace {

// Messages are matched in posting order per (src, dst) pair, like RCCL's p2p channels.
struct Hub {
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::pair<int, int>, std::vector<std::vector<char>>> box;  // (src, dst) -> FIFO
  std::map<std::pair<int, int>, size_t> head;
  long sends = 0, recvs = 0;
};

class FakeTransport : public pvr_comm::Transport {
 public:
  FakeTransport(Hub& hub, int rank, int world) : hub_(hub), rank_(rank), world_(world) {}
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void group_start() override {
    if (in_group_) throw std::runtime_error("nested group");
    in_group_ = true;
  }
  void group_end() override {
    if (!in_group_) throw std::runtime_error("group_end without group_start");
    in_group_ = false;
    // sends are buffered at post time; receives complete here (a group never deadlocks)
    for (auto& r : pending_) {
      std::unique_lock<std::mutex> lk(hub_.mu);
      const auto key = std::make_pair(std::get<2>(r), rank_);
      hub_.cv.wait(lk, [&] { return hub_.box[key].size() > hub_.head[key]; });
      const std::vector<char>& m = hub_.box[key][hub_.head[key]++];
      if (m.size() != std::get<1>(r)) throw std::runtime_error("message size mismatch");
      std::memcpy(std::get<0>(r), m.data(), m.size());
      ++hub_.recvs;
    }
    pending_.clear();
  }
  void send(const void* buf, size_t bytes, int peer) override {
    if (!in_group_) throw std::runtime_error("send outside a group");
    if (peer == rank_ || peer < 0 || peer >= world_) throw std::runtime_error("bad peer");
    std::lock_guard<std::mutex> lk(hub_.mu);
    hub_.box[std::make_pair(rank_, peer)].emplace_back((const char*)buf, (const char*)buf + bytes);
    ++hub_.sends;
    hub_.cv.notify_all();
  }
  void recv(void* buf, size_t bytes, int peer) override {
    if (!in_group_) throw std::runtime_error("recv outside a group");
    if (peer == rank_ || peer < 0 || peer >= world_) throw std::runtime_error("bad peer");
    pending_.emplace_back(buf, bytes, peer);
  }
  void sum_into(float* dst, const float* src, int k, size_t n, size_t stride, float scale) override {
    for (size_t i = 0; i < n; ++i) {
      float s = dst[i];
      for (int j = 0; j < k; ++j) s += src[(size_t)j * stride + i];
      dst[i] = s * scale;
    }
  }

 private:
  Hub& hub_;
  int rank_, world_;
  bool in_group_ = false;
  std::vector<std::tuple<void*, size_t, int>> pending_;
};

int run_case(int world, size_t n, bool average, size_t align, unsigned seed) {
  std::mt19937 gen(seed);
  std::uniform_real_distribution<float> dist(-1.f, 1.f);
  std::vector<std::vector<float>> bufs(world, std::vector<float>(n));
  for (auto& b : bufs)
    for (auto& v : b) v = dist(gen);
  std::vector<double> ref(n, 0.0);
  for (int r = 0; r < world; ++r)
    for (size_t i = 0; i < n; ++i) ref[i] += bufs[r][i];
  if (average)
    for (auto& v : ref) v /= world;
  Hub hub;
  std::vector<std::thread> th;
  std::vector<std::string> errs(world);
  for (int r = 0; r < world; ++r) {
    th.emplace_back([&, r] {
      try {
        FakeTransport tr(hub, r, world);
        std::vector<float> scratch((size_t)(world - 1) * pvr_comm::max_chunk(n, world, align) + 1);
        pvr_comm::mesh_all_reduce(tr, bufs[r].data(), n, scratch.data(), average, align);
      } catch (const std::exception& e) {
        errs[r] = e.what();
      }
    });
  }
  for (auto& t : th) t.join();
  for (int r = 0; r < world; ++r)
    if (!errs[r].empty()) {
      std::printf("FAIL world=%d n=%zu rank %d: %s\n", world, n, r, errs[r].c_str());
      return 1;
    }
  double worst = 0.0;
  for (int r = 0; r < world; ++r)
    for (size_t i = 0; i < n; ++i) worst = std::max(worst, std::fabs(bufs[r][i] - ref[i]) / (1.0 + std::fabs(ref[i])));
  // every rank must hold bit-identical results (the all-gather copies one reduced chunk everywhere)
  bool same = true;
  for (int r = 1; r < world; ++r) same = same && bufs[r] == bufs[0];
  // every posted message consumed; exactly 2 (W-1) non-empty transfers per rank per chunk owner
  bool drained = hub.sends == hub.recvs;
  for (auto& kv : hub.box) drained = drained && hub.head[kv.first] == kv.second.size();
  if (worst > 1e-5 || !same || !drained) {
    std::printf("FAIL world=%d n=%zu avg=%d align=%zu: err %.3e same %d drained %d (sends %ld recvs %ld)\n", world, n, (int)average,
                align, worst, (int)same, (int)drained, hub.sends, hub.recvs);
    return 1;
  }
  return 0;
}

int check_chunks() {
  // chunks tile [0, n) exactly, in rank order, on align boundaries
  for (int w : {1, 2, 3, 7, 8})
    for (size_t n : {0ul, 1ul, 63ul, 64ul, 65ul, 500ul, 4096ul, 100003ul}) {
      size_t at = 0;
      for (int c = 0; c < w; ++c) {
        const auto cr = pvr_comm::chunk_of(n, w, c, 64);
        if (cr.begin != at || cr.end < cr.begin || (cr.begin % 64 && cr.begin != n)) {
          std::printf("FAIL chunk_of n=%zu w=%d c=%d [%zu,%zu)\n", n, w, c, cr.begin, cr.end);
          return 1;
        }
        at = cr.end;
      }
      if (at != n) {
        std::printf("FAIL chunk_of n=%zu w=%d covers %zu\n", n, w, at);
        return 1;
      }
    }
  return 0;
}

}  // namespace

int main() {
  int fails = check_chunks();
  int cases = 0;
  unsigned seed = 1;
  for (int world : {1, 2, 3, 4, 7, 8})
    for (size_t n : {1ul, 5ul, 63ul, 64ul, 200ul, 1000ul, 4097ul, 70001ul})
      for (bool avg : {false, true})
        for (size_t align : {1ul, 64ul}) {
          fails += run_case(world, n, avg, align, seed++);
          ++cases;
        }
  if (fails) {
    std::printf("%d of %d cases FAILED\n", fails, cases);
    return 1;
  }
  std::printf("ALL OK: %d mesh all-reduce cases over the fake transport\n", cases);
  return 0;
}
