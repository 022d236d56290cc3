// tests/cpp/test_plan.cpp -- CPU checks of the host-staging plan
// (qsfs-fuse_amd/csrc/qsmd5_plan.h, used by qsmd5_rt_staging.cpp run_batch).
//
// For many length mixes (qsfs part sets, ragged, tiny, one huge chunk), ring
// sizes, slice targets and column widths, the plan must:
//   1. cut the host chunks (lane order, longest first) into contiguous groups;
//   2. stage every byte of every chunk exactly once: the columns of a chunk
//      are [jW, (j+1)W) clipped to its length, for j = 0 .. ncols - 1;
//   3. make each slice's active chunks the prefix of its group still live in
//      that column, with active > 0 (no empty launches);
//   4. fit every slice in one region, and the ring in the staging cap unless a
//      single slice alone is larger (then one region of that size);
//   5. use columns only when some chunk is longer than W; W a multiple of 64,
//      and when automatic a multiple of 64 KiB, >= kColMin, with at most
//      kColMaxPerChunk (+1) columns per chunk;
//   6. number the segment descriptors of multi-column groups densely (nseg);
// the host-ordered staging schedule (pipeline_turn) must respect every
// copy/kernel/region order against simulated engines and never stall;
// and the multi-GPU split (plan_shards) must give contiguous shards, on
// k = min(#GPUs, max(ceil(bytes / shard_bytes), ceil(parts / resident))) GPUs,
// each within one chunk of an equal share of the bytes.
// Prints "plan ok <cases>" and exits 0, or the first violation and exits 1.
#include <stdio.h>
#include <stdlib.h>

#include <cmath>
#include <random>
#include <vector>

#include "../../qsfs-fuse_amd/csrc/qsmd5_plan.h"

using namespace qsmd5;

static int fails = 0;
#define CHECK(cond, ...)                        \
  do {                                          \
    if (!(cond)) {                              \
      if (fails++ < 10) {                       \
        fprintf(stderr, "FAIL %s: ", #cond);    \
        fprintf(stderr, __VA_ARGS__);           \
        fprintf(stderr, "\n");                  \
      }                                         \
    }                                           \
  } while (0)

static void check(const std::vector<uint64_t>& len, uint64_t cap, uint64_t slice, int64_t col,
                  const char* what) {
  const HostPlan P = plan_host(len, cap, slice, col);
  if (len.empty()) {
    CHECK(P.slices.empty() && P.groups.empty(), "%s: empty input", what);
    return;
  }
  const uint64_t longest = len.front();
  // 5. column width
  if (P.W != kNoColumns) {
    CHECK(P.W < longest, "%s: W %llu not below the longest chunk", what, (unsigned long long)P.W);
    CHECK(P.W % 64 == 0, "%s: W %llu not a multiple of 64", what, (unsigned long long)P.W);
    if (col < 0) {
      CHECK(P.W % kColGrain == 0 && P.W >= kColMin, "%s: automatic W %llu", what,
            (unsigned long long)P.W);
      CHECK((longest + P.W - 1) / P.W <= kColMaxPerChunk + 1, "%s: %llu columns per chunk", what,
            (unsigned long long)((longest + P.W - 1) / P.W));
    }
  } else {
    CHECK(col == 0 || (col < 0) || (uint64_t)std::max<int64_t>(64, col & ~63ll) >= longest,
          "%s: no columns although forced width %lld < longest", what, (long long)col);
    for (const Group& g : P.groups) CHECK(g.ncols == 1, "%s: ncols %u without columns", what, g.ncols);
  }
  // 1. groups partition [0, n) contiguously
  size_t next = 0;
  for (const Group& g : P.groups) {
    CHECK(g.first == next && g.count > 0, "%s: group at %zu count %zu, expected start %zu", what,
          g.first, g.count, next);
    next = g.first + g.count;
    const uint64_t want_cols =
        P.W == kNoColumns ? 1 : std::max<uint64_t>(1, (len[g.first] + P.W - 1) / P.W);
    CHECK(g.ncols == want_cols, "%s: group ncols %u, want %llu", what, g.ncols,
          (unsigned long long)want_cols);
  }
  CHECK(next == len.size(), "%s: groups cover %zu of %zu chunks", what, next, len.size());
  // 2, 3, 4, 6 per slice
  std::vector<uint64_t> staged(len.size(), 0);
  std::vector<uint32_t> next_col(P.groups.size(), 0);
  size_t seg = 0;
  uint64_t max_slice_bytes = 0;
  for (const Slice& sl : P.slices) {
    CHECK(sl.group < P.groups.size(), "%s: slice group %zu", what, sl.group);
    const Group& g = P.groups[sl.group];
    CHECK(sl.col == next_col[sl.group], "%s: group %zu column %u out of order", what, sl.group, sl.col);
    next_col[sl.group] = sl.col + 1;
    CHECK(sl.active > 0 && sl.active <= g.count, "%s: active %zu of %zu", what, sl.active, g.count);
    uint64_t bytes = 0;
    for (size_t k = 0; k < g.count; ++k) {
      const uint64_t b = P.col_bytes(len[g.first + k], sl.col);
      if (k < sl.active) {
        CHECK(b > 0, "%s: active chunk %zu has no bytes in column %u", what, g.first + k, sl.col);
        CHECK(b == std::min(P.W == kNoColumns ? len[g.first + k] : P.W,
                            len[g.first + k] - (P.W == kNoColumns ? 0 : (uint64_t)sl.col * P.W)),
              "%s: column bytes", what);
        staged[g.first + k] += b;
        bytes += stage_bytes(b);
      } else {
        CHECK(b == 0, "%s: chunk %zu live in column %u but outside the active prefix", what,
              g.first + k, sl.col);
      }
    }
    CHECK(bytes <= P.region, "%s: slice needs %llu B > region %llu B", what,
          (unsigned long long)bytes, (unsigned long long)P.region);
    max_slice_bytes = std::max(max_slice_bytes, bytes);
    if (g.ncols > 1) {
      CHECK(sl.seg0 == seg, "%s: seg0 %zu, want %zu", what, sl.seg0, seg);
      seg += sl.active;
    }
  }
  for (size_t gi = 0; gi < P.groups.size(); ++gi)
    CHECK(next_col[gi] == P.groups[gi].ncols, "%s: group %zu has %u of %u columns", what, gi,
          next_col[gi], P.groups[gi].ncols);
  CHECK(seg == P.nseg, "%s: nseg %zu, want %zu", what, P.nseg, seg);
  for (size_t i = 0; i < len.size(); ++i)
    CHECK(staged[i] == len[i], "%s: chunk %zu staged %llu of %llu B", what, i,
          (unsigned long long)staged[i], (unsigned long long)len[i]);
  CHECK(P.nregions >= 1 && P.nregions <= P.slices.size(), "%s: nregions %zu", what, P.nregions);
  CHECK(P.nregions * P.region <= std::max(cap, P.region), "%s: ring %llu B over cap %llu B", what,
        (unsigned long long)(P.nregions * P.region), (unsigned long long)cap);
}

static void check_shards(const std::vector<uint64_t>& len, size_t ndev, uint64_t per,
                         const char* what, size_t resident = 32768) {
  size_t k = 0;
  const std::vector<uint32_t> sh = plan_shards(len, ndev, per, &k, resident);
  uint64_t total = 0, longest = 0;
  for (uint64_t L : len) total += L, longest = std::max(longest, L);
  // more GPUs for more bytes (links) or more parts than one GPU keeps resident
  const uint64_t by_parts = (len.size() + resident - 1) / resident;
  const size_t want_k = (size_t)std::min<uint64_t>(
      std::max<size_t>(1, ndev), std::max<uint64_t>({1, (total + per - 1) / per, by_parts}));
  CHECK(k == want_k, "%s: %zu shards, want %zu", what, k, want_k);
  CHECK(sh.size() == len.size(), "%s: shard list size", what);
  std::vector<uint64_t> bytes(k, 0);
  for (size_t i = 0; i < sh.size(); ++i) {
    CHECK(sh[i] < k, "%s: shard %u >= %zu", what, sh[i], k);
    // contiguous ranges; an index may be skipped when one chunk outweighs a share
    if (i) CHECK(sh[i] >= sh[i - 1], "%s: shards not contiguous", what);
    if (sh[i] < k) bytes[sh[i]] += len[i];
  }
  for (size_t d = 0; d < k; ++d)
    CHECK(bytes[d] <= total / k + longest, "%s: shard %zu holds %llu of %llu B", what, d,
          (unsigned long long)bytes[d], (unsigned long long)total);
  bool equal = true;
  for (uint64_t L : len) equal = equal && L == len.front();
  if (equal && !len.empty()) {  // equal parts: every GPU that can get one does
    size_t used = 0;
    for (size_t d = 0; d < k; ++d) used += bytes[d] > 0;
    CHECK(used == std::min(k, len.size()), "%s: %zu of %zu shards used for %zu equal parts", what,
          used, k, len.size());
  }
}

// 2-D copy runs (plan_copy_runs).  `allocs` are disjoint [lo, hi) ranges; a
// span is ok only inside one of them.  The runs must cover rows 0..n-1 once,
// in order; a multi-row run must have equal widths, the constant positive
// stride of its rows, stride >= width, and its whole source span inside ONE
// allocation (the GPUTEST_r01 fault was a span from a pinned pool into a
// pageable one); and a run may not stop where the next row could have joined.
struct Alloc {
  uint64_t lo, hi;
};
static int span_in(const std::vector<Alloc>& a, uint64_t lo, uint64_t hi) {
  for (size_t i = 0; i < a.size(); ++i)
    if (lo >= a[i].lo && lo < a[i].hi) return hi <= a[i].hi ? (int)i : -1;
  return -1;
}
static void check_runs(const std::vector<uint64_t>& src, const std::vector<uint64_t>& w,
                       const std::vector<Alloc>& allocs, const char* what, size_t* multi = nullptr) {
  const size_t n = src.size();
  size_t span_calls = 0;
  const std::vector<CopyRun> runs = plan_copy_runs(
      n, [&](size_t k) { return src[k]; }, [&](size_t k) { return w[k]; },
      [&](uint64_t lo, uint64_t hi) {
        ++span_calls;
        return span_in(allocs, lo, hi) >= 0;
      });
  size_t next = 0;
  for (const CopyRun& r : runs) {
    CHECK(r.first == next && r.rows >= 1, "%s: run at %zu rows %zu, expected start %zu", what,
          r.first, r.rows, next);
    next = r.first + r.rows;
    if (r.rows > 1) {
      if (multi) ++*multi;
      CHECK(r.stride >= w[r.first] && r.stride > 0, "%s: stride %llu < width %llu", what,
            (unsigned long long)r.stride, (unsigned long long)w[r.first]);
      for (size_t j = 1; j < r.rows; ++j) {
        CHECK(w[r.first + j] == w[r.first], "%s: unequal widths in a run", what);
        CHECK(src[r.first + j] == src[r.first] + j * r.stride, "%s: row %zu off the stride", what,
              r.first + j);
      }
      const uint64_t end = src[r.first] + (r.rows - 1) * r.stride + w[r.first];
      CHECK(span_in(allocs, src[r.first], end) >= 0, "%s: run at %zu spans allocations", what,
            r.first);
    } else {
      CHECK(r.stride == 0, "%s: one-row run with a stride", what);
    }
    const size_t nx = r.first + r.rows;  // maximality
    if (nx < n && r.rows >= 1 && w[nx] == w[r.first] && w[nx] > 0 && src[nx] > src[nx - 1]) {
      const uint64_t d = src[nx] - src[nx - 1];
      const bool same = r.rows > 1 ? d == r.stride : d >= w[r.first] && d < (1ull << 40);
      const uint64_t end = src[nx] + w[nx];
      CHECK(!(same && span_in(allocs, src[r.first], end) >= 0), "%s: run at %zu stops early at %zu",
            what, r.first, nx);
    }
  }
  CHECK(next == n, "%s: runs cover %zu of %zu rows", what, next, n);
  CHECK(span_calls <= 2 * runs.size() * 64 + 1, "%s: %zu span checks for %zu runs", what, span_calls,
        runs.size());
}

static int run_copy_run_cases(std::mt19937_64& rng) {
  int cases = 0;
  const uint64_t MiB = 1ull << 20;
  // The seed-0 shape: equal-length chunks, one in a pinned pool, the next in a
  // pageable pool at a higher address with unmapped memory between them, at
  // both orders, and equal-length pairs in two pinned pools.
  for (uint64_t L : {55ull, 88ull, 4095ull, 1ull << 20}) {
    const std::vector<Alloc> two = {{0x10000000, 0x10000000 + 24 * MiB},
                                    {0x7f0000000000, 0x7f0000000000 + 24 * MiB}};
    size_t multi = 0;
    check_runs({two[0].lo + 100, two[1].lo + 100}, {L, L}, two, "pinned -> pageable", &multi);
    check_runs({two[0].lo + 100, two[1].lo + 100, two[1].lo + 100 + (two[1].lo - two[0].lo)}, {L, L, L},
               two, "stride continues past the second pool", &multi);
    CHECK(multi == 0, "cross-allocation pairs merged (L=%llu)", (unsigned long long)L);
    cases += 2;
  }
  {  // a file's parts in one buffer: one run; the same rows split over two
     // adjacent pools (no gap): one run per pool
    std::vector<uint64_t> src, w;
    const std::vector<Alloc> one = {{1 << 30, (1ull << 30) + 64 * 10 * MiB}};
    for (int i = 0; i < 64; ++i) src.push_back(one[0].lo + i * 10 * MiB), w.push_back(10 * MiB);
    size_t multi = 0;
    check_runs(src, w, one, "file parts", &multi);
    CHECK(multi == 1, "file parts: %zu runs, want 1", multi);
    const std::vector<Alloc> split = {{1 << 30, (1ull << 30) + 40 * 10 * MiB},
                                      {(1ull << 30) + 40 * 10 * MiB, (1ull << 30) + 64 * 10 * MiB}};
    multi = 0;
    check_runs(src, w, split, "parts over two adjacent pools", &multi);
    CHECK(multi == 2, "two pools: %zu runs, want 2", multi);
    cases += 2;
  }
  {  // negative, zero and overlapping strides never merge
    const std::vector<Alloc> one = {{4096, 1ull << 32}};
    size_t multi = 0;
    check_runs({1 << 20, (1 << 20) - 4096, (1 << 20) - 8192}, {1000, 1000, 1000}, one, "negative", &multi);
    check_runs({1 << 20, 1 << 20, 1 << 20}, {1000, 1000, 1000}, one, "duplicates", &multi);
    check_runs({1 << 20, (1 << 20) + 500, (1 << 20) + 1000}, {1000, 1000, 1000}, one, "overlap", &multi);
    CHECK(multi == 0, "negative/zero/overlapping strides merged");
    cases += 3;
  }
  for (int t = 0; t < 400; ++t) {  // random pools, positions and widths
    std::vector<Alloc> allocs;
    uint64_t base = 1 << 20;
    const int na = 1 + (int)(rng() % 5);
    for (int a = 0; a < na; ++a) {
      const uint64_t size = (1 + rng() % 64) * 4096;
      if (rng() % 2) base += (1 + rng() % 8) * 4096;  // a gap, or adjacent pools
      allocs.push_back({base, base + size});
      base += size;
    }
    const size_t n = 1 + rng() % 60;
    std::vector<uint64_t> src(n), w(n);
    const uint64_t W = 1 + rng() % 3000;
    const uint64_t stride = W + rng() % 2000;
    uint64_t p = allocs[0].lo + rng() % 512;
    for (size_t k = 0; k < n; ++k) {
      w[k] = rng() % 8 ? W : 1 + rng() % 3000;
      if (rng() % 6 == 0) {  // jump into a random pool
        const Alloc& a = allocs[rng() % allocs.size()];
        p = a.lo + rng() % (a.hi - a.lo);
      }
      src[k] = p;
      p += rng() % 10 ? stride : rng() % 9000;
    }
    check_runs(src, w, allocs, "random");
    ++cases;
  }
  return cases;
}

// The host-ordered staging schedule (pipeline_turn) against simulated
// engines: ncopy copy streams and some compute streams, each running its
// queue in order with random durations; the metadata block lands at a random
// time.  The host calls pipeline_turn; when a turn enqueues nothing, time
// moves to the next completion (no completion pending = a stall).  Checked:
// a slice's copies are enqueued only after the kernel that last used its
// region has finished, and only after the metadata block has landed if the
// slice has gather rows; its kernel only after its copies have landed and the
// metadata block too; kernels in slice order; every slice runs.
static int run_pipeline_cases(std::mt19937_64& rng) {
  int cases = 0;
  for (int t = 0; t < 3000; ++t) {
    const size_t S = 1 + rng() % 120;
    const size_t nregions = 1 + rng() % (S + 2);
    const size_t R = std::min(nregions, S);
    const int ncopy = 1 + (int)(rng() % 4), ncomp = 1 + (int)(rng() % 7);
    std::vector<int> group(S);
    for (size_t si = 0; si < S; ++si) group[si] = (int)(rng() % ncomp);
    std::vector<bool> gathers(S);
    for (size_t si = 0; si < S; ++si) gathers[si] = rng() % 5 == 0;
    const double meta_at = (double)(rng() % 50);
    double now = 0;
    std::vector<double> copy_end(S, -1), kern_end(S, -1);
    std::vector<double> copy_stream_free(ncopy, 0), comp_stream_free(ncomp, 0);
    auto done_by = [&](double end) { return end >= 0 && end <= now; };
    PipelineState st;
    size_t launched_before = 0;
    bool stalled = false;
    for (int turns = 0; st.nk < S; ++turns) {
      const bool meta = now >= meta_at;
      const int r = pipeline_turn(
          S, R, meta, st, [&](size_t si) { return done_by(copy_end[si]) ? 1 : 0; },
          [&](size_t si) { return done_by(kern_end[si]) ? 1 : 0; },
          [&](size_t si) { return gathers[si] ? true : false; },
          [&](size_t si) {
            CHECK(si < R || done_by(kern_end[si - R]),
                  "case %d: copies of slice %zu before the kernel of slice %zu (its region) ended", t, si,
                  si - R);
            CHECK(!gathers[si] || meta, "case %d: gather rows of slice %zu before the metadata", t, si);
            const int cs = (int)(si % ncopy);
            const double start = std::max(now, copy_stream_free[cs]);
            copy_end[si] = copy_stream_free[cs] = start + 1 + (double)(rng() % 20);
            return 0;
          },
          [&](size_t si) {
            CHECK(done_by(copy_end[si]), "case %d: kernel of slice %zu before its copies landed", t, si);
            CHECK(meta, "case %d: kernel of slice %zu before the metadata landed", t, si);
            CHECK(si == launched_before, "case %d: kernel %zu out of order", t, si);
            ++launched_before;
            const int k = group[si];
            const double start = std::max(now, comp_stream_free[k]);
            kern_end[si] = comp_stream_free[k] = start + 1 + (double)(rng() % 30);
            return 0;
          });
      CHECK(r >= 0, "case %d: turn failed", t);
      if (r > 0) continue;
      // the host waits: the next completion (a copy, a kernel, the metadata)
      double next = 1e300;
      for (size_t si = 0; si < S; ++si) {
        if (copy_end[si] > now) next = std::min(next, copy_end[si]);
        if (kern_end[si] > now) next = std::min(next, kern_end[si]);
      }
      if (!meta) next = std::min(next, meta_at);
      if (next == 1e300 || turns > 100000) {
        stalled = true;
        break;
      }
      now = next;
    }
    CHECK(!stalled, "case %d: S=%zu nregions=%zu stalled at nc=%zu nk=%zu", t, S, R, st.nc, st.nk);
    CHECK(st.nc == S && st.nk == S, "case %d: not every slice ran", t);
    ++cases;
  }
  return cases;
}

// Pull-driven batches (plan_read, qsmd5_hash_read): groups cover the lanes in
// order; every byte of every chunk lies in exactly one column window; each
// column's live lanes are a prefix and fit one region (count x stride); W is a
// multiple of 64 (256 for the staged stride), at least kReadColMin unless one
// column holds the group's longest chunk; a group never exceeds kReadMaxRows.
static int check_read(const std::vector<uint64_t>& len, uint64_t staging, const char* what) {
  const ReadPlan P = plan_read(len, staging);
  if (len.empty()) {
    CHECK(P.groups.empty(), "%s: empty input", what);
    return 1;
  }
  size_t next = 0;
  for (const ReadGroup& g : P.groups) {
    CHECK(g.first == next && g.count > 0 && g.count <= kReadMaxRows, "%s: group range", what);
    CHECK(g.W % 64 == 0 && g.W > 0, "%s: W %llu", what, (unsigned long long)g.W);
    CHECK(g.stride == stage_bytes(g.W) && g.count * g.stride <= P.region, "%s: rows do not fit", what);
    const uint64_t L0 = len[g.first];
    CHECK(g.W >= kReadColMin || (uint64_t)g.ncols * g.W >= L0, "%s: narrow W", what);
    CHECK((uint64_t)g.ncols * g.W >= L0 && (g.ncols == 1 || (uint64_t)(g.ncols - 1) * g.W < L0),
          "%s: ncols", what);
    for (uint32_t j = 0; j < g.ncols; ++j) {
      const size_t a = ReadPlan::active(len, g, j);
      CHECK(a >= 1 && a <= g.count, "%s: empty column %u", what, j);
      for (size_t k = 0; k < g.count; ++k) {
        const uint64_t b = ReadPlan::col_bytes(g, len[g.first + k], j);
        CHECK((k < a) == (b > 0 || j == 0), "%s: live lanes not a prefix (col %u lane %zu)", what, j, k);
      }
    }
    for (size_t k = 0; k < g.count; ++k) {  // the windows tile each chunk exactly
      uint64_t sum = 0;
      for (uint32_t j = 0; j < g.ncols; ++j) sum += ReadPlan::col_bytes(g, len[g.first + k], j);
      CHECK(sum == len[g.first + k], "%s: lane %zu covered %llu of %llu bytes", what, g.first + k,
            (unsigned long long)sum, (unsigned long long)len[g.first + k]);
    }
    next += g.count;
  }
  CHECK(next == len.size(), "%s: lanes not all grouped", what);
  CHECK(P.region >= staging / 2 && (P.region <= staging / 2 || P.region == stage_bytes(kReadColMin)),
        "%s: region", what);
  return 1;
}

static int run_read_cases(std::mt19937_64& rng) {
  const uint64_t KiB = 1024, MiB = 1ull << 20, GiB = 1ull << 30;
  int cases = 0;
  std::vector<std::vector<uint64_t>> sets = {
      {}, {0}, {1}, {64}, {10 * MiB}, std::vector<uint64_t>(128, 10 * MiB),
      std::vector<uint64_t>(512, 10 * MiB), std::vector<uint64_t>(10000, 10 * MiB),
      std::vector<uint64_t>(65535, 10 * MiB), {3 * GiB, 1, 0, 0}};
  {
    std::vector<uint64_t> v(10, 10 * MiB);  // PrepareUpload's averaged tail pair
    v.push_back(5 * MiB + 6172);
    v.push_back(5 * MiB + 6173);
    sets.push_back(v);
  }
  for (int t = 0; t < 30; ++t) {
    std::vector<uint64_t> v(1 + rng() % 2000);
    for (auto& L : v) L = rng() % (1 + (rng() % 3 == 0 ? 64 * MiB : 300 * KiB));
    sets.push_back(v);
  }
  for (auto& v : sets) {
    std::sort(v.begin(), v.end(), [](uint64_t a, uint64_t b) { return a > b; });
    for (uint64_t staging : {(uint64_t)0, 1 * MiB, 64 * MiB, 256 * MiB, 1 * GiB, 8 * GiB})
      cases += check_read(v, staging, "read plan");
  }
  {  // the shapes the design promises (qsmd5_hash_read)
    std::vector<uint64_t> v(512, 10 * MiB);
    const ReadPlan P = plan_read(v, 512 * MiB);  // 256 MiB regions: 512 rows of 508 KiB
    CHECK(P.groups.size() == 1 && P.groups[0].ncols == 21 && P.groups[0].W == 519936,
          "512 x 10 MiB through 512 MiB: %zu groups, %u columns of %llu", P.groups.size(),
          P.groups.empty() ? 0 : P.groups[0].ncols,
          (unsigned long long)(P.groups.empty() ? 0 : P.groups[0].W));
    std::vector<uint64_t> w(10000, 10 * MiB);  // rows of 64 KiB + skew: 3840 per region
    const ReadPlan Q = plan_read(w, 512 * MiB);
    CHECK(Q.groups.size() == 3 && Q.groups[0].count == 3840 && Q.groups[2].count == 2320,
          "10000 parts through 512 MiB: %zu groups of %zu", Q.groups.size(),
          Q.groups.empty() ? (size_t)0 : Q.groups[0].count);
    ++cases;
  }
  return cases;
}

int main() {
  const uint64_t MiB = 1ull << 20, GiB = 1ull << 30;
  std::mt19937_64 rng(1234);
  int cases = 0;
  auto run = [&](std::vector<uint64_t> len, const char* what) {
    std::sort(len.begin(), len.end(), [](uint64_t a, uint64_t b) { return a > b; });
    for (uint64_t cap : {256 * MiB, 2 * GiB, 16 * GiB})
      for (uint64_t slice : {(uint64_t)0, 64 * MiB, 1 * GiB})
        for (int64_t col : {(int64_t)-1, (int64_t)0, (int64_t)64, (int64_t)192, (int64_t)4160,
                            (int64_t)1 << 20, (int64_t)3000}) {
          // forced tiny columns on long chunks: millions of slices; keep the
          // checker's work (columns x chunks) bounded
          if (col > 0 && !len.empty() &&
              (double)(len.front() / (uint64_t)std::max<int64_t>(64, col) + 1) * len.size() > 3e6)
            continue;
          check(len, cap, slice, col, what);
          ++cases;
        }
  };
  run({}, "empty");
  run({1}, "one byte");
  run({10 * MiB}, "one part");
  run(std::vector<uint64_t>(512, 10 * MiB), "512 x 10 MiB");
  run(std::vector<uint64_t>(4096, 10 * MiB), "4096 x 10 MiB");
  {
    std::vector<uint64_t> v(10, 10 * MiB);  // PrepareUpload of 100 MiB + 12345 B: averaged pair
    v.push_back(5 * MiB + 6172);
    v.push_back(5 * MiB + 6173);
    run(v, "file parts with averaged tail");
  }
  {
    std::vector<uint64_t> v;
    for (int i = 0; i < 700; ++i) {  // log-uniform 8 KiB .. 64 MiB, as the ragged fixture
      const double e = 13.0 + (26.0 - 13.0) * (double)(rng() % 100000) / 100000.0;
      v.push_back((uint64_t)std::max(1.0, std::exp2(e)) + rng() % 97);
    }
    run(v, "ragged 8 KiB..64 MiB");
  }
  {
    std::vector<uint64_t> v;
    for (int i = 0; i < 3000; ++i) v.push_back(1 + rng() % 5000);
    run(v, "3000 tiny");
  }
  {
    std::vector<uint64_t> v(200, 64 * MiB);
    v.push_back(3 * GiB);  // one chunk much longer than the rest
    run(v, "one huge chunk");
  }
  for (int t = 0; t < 40; ++t) {
    std::vector<uint64_t> v(1 + rng() % 300);
    for (auto& L : v) L = 1 + rng() % (1 + (rng() % 4 == 0 ? 200 * MiB : 3 * MiB));
    run(v, "random mix");
  }
  {  // multi-GPU split
    std::vector<std::vector<uint64_t>> sets = {
        {}, {1}, std::vector<uint64_t>(4096, 10 * MiB), std::vector<uint64_t>(10000, 10 * MiB),
        std::vector<uint64_t>(3, 20 * GiB)};
    std::vector<uint64_t> mix;
    for (int i = 0; i < 5000; ++i) mix.push_back(1 + rng() % (64 * MiB));
    sets.push_back(mix);
    sets.push_back(std::vector<uint64_t>(100000, 1024));  // many small objects: 98 MiB, 100 K parts
    for (const auto& v : sets)
      for (size_t nd : {(size_t)1, (size_t)2, (size_t)3, (size_t)8})
        for (uint64_t per : {(uint64_t)1, 1 * GiB, 4 * GiB, 64 * GiB}) {
          check_shards(v, nd, per, "shards");
          check_shards(v, nd, per, "shards by part count", 1000);
          cases += 2;
        }
  }
  cases += run_copy_run_cases(rng);
  cases += run_pipeline_cases(rng);
  cases += run_read_cases(rng);
  printf("plan %s %d cases\n", fails ? "FAIL" : "ok", cases);
  return fails ? 1 : 0;
}
