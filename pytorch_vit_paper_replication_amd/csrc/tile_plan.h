// Grid planning of the GEMM kernels, as plain constexpr C++ (no HIP headers): the kernels call it on
// the device (hipcc treats constexpr functions as host + device) and tests/cpp/test_tile_plan.cpp
// checks it on the host under AddressSanitizer / UndefinedBehaviorSanitizer.
#pragma once

namespace pvr {

// Bijective XCD-aware remap: blocks are dealt round-robin over 8 XCDs (b, b+8 share one); block b
// gets logical id remap(b) so that each XCD owns a contiguous range of logical tiles, i.e. tiles that
// share operand panels share that XCD's L2. Bijective for every n (the n % 8 != 0 case included).
constexpr int xcd_remap_c(int bid, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// Split-K tail of the one-tile-per-workgroup GEMM (see GemmParams::tail_*): with R full dispatch
// rounds of `cus` tiles and rem < cus tiles left over, the leftover tiles' K loops are split into
// `split` parts each. Rules: split <= 4, every part keeps >= 12 K-tiles (the fp32 partial-tile exchange
// costs about one 12-K-tile loop), split * rem <= cus, and split * rem <= max_units when max_units > 0;
// the workspace must hold split * rem partial tiles (65536 floats each) and rem arrival counters.
struct TailPlan {
  int from;   // tiles [0, from) run whole, one per workgroup
  int split;  // K-parts per leftover tile (0: no split)
};

constexpr TailPlan plan_tail_c(int ntiles, int nkt, int cus, long long ws_elems, int cnt_elems, int max_units, int min_kt = 12) {
  TailPlan t{0, 0};
  if (cus <= 0 || ntiles < cus) return t;
  const int rem = ntiles % cus;
  if (rem == 0) return t;
  int s = cus / rem;
  s = s < 4 ? s : 4;
  while (s > 1 && nkt / s < min_kt) --s;
  if (max_units > 0)
    while (s > 1 && rem * s > max_units) --s;
  if (s < 2) return t;
  if ((long long)rem * s * 65536 > ws_elems || rem > cnt_elems) return t;
  t.from = ntiles - rem;
  t.split = s;
  return t;
}

// Workgroups of a split-tail launch: ids [0, from) whole tiles, then units * split K-parts. A part's
// (leftover tile, part) comes from the XCD remap over the units, so the parts of one tile mostly land
// on one XCD. That is a locality hint only: the XCD ranges (units / 8 ids each) do not align with the
// tiles' part groups, so some tiles straddle two XCDs (ViT-B/16 fc2: 79 tiles x 3 parts, counted by
// tests/cpp/test_tile_plan.cpp). The hand-off is correct because the partials are stored and read
// with sc1 (device-coherent, L2-bypassing) accesses and counted by an agent-scope atomic, not because
// the parts share an L2.
constexpr int tail_grid(const TailPlan& t, int ntiles) {
  return t.split > 1 ? t.from + (ntiles - t.from) * t.split : ntiles;
}

struct TailUnit {
  int tile;  // output tile index
  int part;  // K-part (-1: a whole tile)
};

constexpr TailUnit tail_unit_c(const TailPlan& t, int ntiles, int bid) {
  if (t.split > 1 && bid >= t.from) {
    const int units = (ntiles - t.from) * t.split;
    const int u = xcd_remap_c(bid - t.from, units);
    return TailUnit{t.from + u / t.split, u % t.split};
  }
  return TailUnit{xcd_remap_c(bid, t.split > 1 ? t.from : ntiles), -1};
}

// K range [kbeg, kend) (in K-tiles) of part `part` of `split` over nkt K-tiles
constexpr int tail_kbeg(int part, int split, int nkt) { return part * nkt / split; }

}  // namespace pvr
