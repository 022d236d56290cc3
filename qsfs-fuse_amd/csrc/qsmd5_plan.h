// qsfs-fuse_amd/csrc/qsmd5_plan.h -- the staging plan for host-resident chunks.
//
// Pure host logic (no HIP), shared by the runtime (qsmd5_rt_staging.cpp run_batch)
// and the CPU tests (tests/cpp/test_plan.cpp), which check its invariants.
//
// Host-resident chunks (the qsfs case: parts in pooled host buffers,
// ResourceManager.cpp:53-77) are staged into a device ring in SLICES.  The
// chunks, sorted by length (descending), form GROUPS that fit one ring region;
// a group is cut into COLUMNS of width W: column j of a group is bytes
// [jW, (j+1)W) of each of its chunks still that long.  One slice = one
// (group, column): one H2D transfer into a region, then one kernel launch that
// resumes each chain from its parked state.  Columns let every chain start as
// soon as the first column lands, so the serial chain of the LAST chunk copied
// no longer trails the transfer: only its last column (~2 ms at W = 256 KiB)
// does.  W = kNoColumns (chunks no longer than a column) degenerates to
// whole-chunk row slices.
//
// Staged segments are packed at 256-B alignment, segments of 16 KiB and more
// plus a 4 KiB + 256 B skew, so that equal-size parts never sit at a
// power-of-two stride (the lanes of a wave walk their chunks in lockstep; a
// power-of-two stride sends every lane's request to the same HBM channel).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <vector>

namespace qsmd5 {

constexpr uint64_t kSliceMin = 512ull << 20;  // automatic slice target bounds
constexpr uint64_t kSliceMax = 4ull << 30;
constexpr uint64_t kAlign = 256;
constexpr uint64_t kSkew = 4096 + 256;
constexpr uint64_t kColGrain = 64ull << 10;  // automatic column widths are multiples of this
constexpr uint64_t kColMin = 256ull << 10;   // ... and at least this: 2-D copies keep the link
                                             // rate down to 256 KiB rows, and 128 KiB loses 2%
constexpr uint64_t kColMaxPerChunk = 1024;   // automatic columns per chunk (launches per group)
constexpr uint64_t kNoColumns = ~0ull;

constexpr uint64_t kSkewFrom = 16ull << 10;  // segments this long or longer get the skew

// Bytes one staged segment of L message bytes occupies in a region.  The skew
// is for long equal segments, whose lanes walk in lockstep at a power-of-two
// stride; short ones (a wave's 64 lanes inside 1 MiB) spread over the channels
// anyway (1 M x 1 KiB device-resident at an exact stride: 58.6% of HBM peak,
// profiles/r01_saturation_tiny.jsonl), and skewing them would stage 1 KiB
// objects at 5.25 KiB each.
inline uint64_t stage_bytes(uint64_t L) {
  return ((L + kAlign - 1) & ~(kAlign - 1)) + (L >= kSkewFrom ? kSkew : 0);
}

struct Group {
  size_t first, count;  // range in the host lane order
  uint32_t ncols;
};

struct Slice {
  size_t group;
  uint32_t col;
  size_t active;  // chunks of the group still live in this column (a prefix)
  size_t seg0;    // first entry in the segment/order arrays (multi-column groups)
};

struct HostPlan {
  uint64_t W = kNoColumns;  // column width, or kNoColumns
  uint64_t slice_target = 0;
  uint64_t region = 0;      // bytes of one ring region
  size_t nregions = 0;      // regions in the ring (slice s uses region s % nregions)
  size_t nseg = 0;          // segment descriptors of multi-column groups
  std::vector<Group> groups;
  std::vector<Slice> slices;

  // Message bytes of a chunk of length L in column j.
  uint64_t col_bytes(uint64_t L, uint32_t j) const {
    if (W == kNoColumns) return j == 0 ? L : 0;
    const uint64_t o = (uint64_t)j * W;
    return L > o ? std::min(W, L - o) : 0;
  }
};

// host_len: lengths (>= 1) of the host chunks in lane order, longest first.
// staging_cap: bytes of device memory the ring may use.
// slice_bytes: slice target, 0 = automatic (a quarter of the batch, clamped to
//   [kSliceMin, kSliceMax]).
// column_bytes: < 0 automatic: kColMin, or longest / kColMaxPerChunk for
//   chunks over 256 MiB, a multiple of kColGrain.  Narrow columns shorten the
//   tail: the chain of the last column starts only when its bytes have landed
//   (1024 x 10 MiB pageable: 2.5 MiB columns 48.5 GiB/s, 256 KiB 52.4;
//   profiles/r01_config3_column_width.jsonl).  0 = whole chunks; > 0 forced
//   (rounded down to a multiple of 64, at least 64).
inline HostPlan plan_host(const std::vector<uint64_t>& host_len, uint64_t staging_cap,
                          uint64_t slice_bytes, int64_t column_bytes) {
  HostPlan P;
  if (host_len.empty()) return P;
  uint64_t host_total = 0;
  const uint64_t max_host = host_len.front();
  for (uint64_t L : host_len) host_total += stage_bytes(L);
  P.slice_target =
      slice_bytes ? slice_bytes : std::min(kSliceMax, std::max(kSliceMin, host_total / 4));
  uint64_t w;
  if (column_bytes < 0) {
    const uint64_t per = (max_host + kColMaxPerChunk - 1) / kColMaxPerChunk;
    w = std::max(kColMin, (per + kColGrain - 1) / kColGrain * kColGrain);
  } else if (column_bytes == 0) {
    w = kNoColumns;
  } else {
    w = std::max<uint64_t>(64, (uint64_t)column_bytes & ~63ull);
  }
  if (w < max_host) P.W = w;
  // A region holds one column of a whole group.  When the column width sits
  // at its floor (kColMin) the chunks' first columns may overshoot the slice
  // target slightly; grow the region (up to half the ring) rather than split
  // off a small second group whose columns would all trail the first.
  uint64_t first_cols = 0;
  for (uint64_t L : host_len) first_cols += stage_bytes(P.col_bytes(L, 0));
  P.region = std::max<uint64_t>({P.slice_target, stage_bytes(P.col_bytes(max_host, 0)),
                                 P.W == kNoColumns ? 0 : std::min<uint64_t>(first_cols, staging_cap / 2)});
  for (size_t k = 0; k < host_len.size();) {
    Group g{k, 0, 1};
    uint64_t bytes = 0;
    while (k < host_len.size()) {
      const uint64_t b = stage_bytes(P.col_bytes(host_len[k], 0));
      if (g.count > 0 && bytes + b > P.region) break;
      bytes += b;
      ++g.count;
      ++k;
    }
    const uint64_t longest = host_len[g.first];
    if (P.W != kNoColumns) g.ncols = (uint32_t)std::max<uint64_t>(1, (longest + P.W - 1) / P.W);
    P.groups.push_back(g);
  }
  for (size_t gi = 0; gi < P.groups.size(); ++gi) {
    const Group& g = P.groups[gi];
    for (uint32_t j = 0; j < g.ncols; ++j) {
      size_t act = 0;
      while (act < g.count && P.col_bytes(host_len[g.first + act], j) > 0) ++act;
      P.slices.push_back(Slice{gi, j, act, P.nseg});
      if (g.ncols > 1) P.nseg += act;
    }
  }
  // Groups are formed; shrink the region to the largest slice actually
  // planned, so that small batches get many regions and their copies run ahead
  // of the kernels instead of waiting for the one region to free up (one
  // 10 MiB part: 40 columns in 40 regions, not 1).
  uint64_t need = 0;
  for (const Slice& sl : P.slices) {
    const Group& g = P.groups[sl.group];
    uint64_t b = 0;
    for (size_t k = 0; k < sl.active; ++k) b += stage_bytes(P.col_bytes(host_len[g.first + k], sl.col));
    need = std::max(need, b);
  }
  P.region = std::max<uint64_t>(need, kAlign);
  const uint64_t cap = std::min<uint64_t>(staging_cap, host_total + P.region);
  P.nregions = (size_t)std::max<uint64_t>(1, cap / P.region);
  P.nregions = std::min(P.nregions, P.slices.size());
  return P;
}

// H2D copy runs of one slice (qsmd5_rt_staging.cpp run_batch).  Rows k .. k+rows-1
// of a slice's active chunks go as ONE hipMemcpy2DAsync when they have equal
// widths, a constant source stride >= the width (and < 2^40), AND their whole
// source span [src(k), src(k + rows - 1) + w) lies inside one allocation or
// mapping (span_ok).  A 2-D copy reads its source as that span: across two
// allocations it touches memory the caller never passed in.  With a pinned
// first row HIP reads the span by DMA, and the bytes past the allocation were
// a GPU page fault (GPUTEST_r01.json, test_gpu_fuzz seed 0: equal-length
// chunks in a pinned pool and a pageable numpy pool).  A run whose span leaves
// its first row's allocation is cut at the longest prefix that stays inside it
// (span_ok is monotone in the span's end), and the rest start a new run.
// Negative, zero (duplicates) and overlapping (< w) strides never merge.
struct CopyRun {
  size_t first, rows;  // rows [first, first + rows) of the slice's active chunks
  uint64_t stride;     // source pitch of a multi-row run (0 for one row)
};

// src(k): source address of row k (column offset included); w(k): its bytes;
// span_ok(lo, hi): [lo, hi) lies in ONE allocation or mapping.
template <class Src, class Width, class SpanOk>
inline std::vector<CopyRun> plan_copy_runs(size_t n, Src&& src, Width&& w, SpanOk&& span_ok) {
  std::vector<CopyRun> runs;
  constexpr uint64_t kMaxStride = 1ull << 40;
  for (size_t k = 0; k < n;) {
    const uint64_t w0 = w(k), s0 = src(k);
    size_t rows = 1;
    uint64_t stride = 0;
    if (k + 1 < n && w0 > 0 && w(k + 1) == w0 && src(k + 1) > s0) {
      const uint64_t d = src(k + 1) - s0;
      if (d >= w0 && d < kMaxStride) {
        rows = 2;
        while (k + rows < n && w(k + rows) == w0 && src(k + rows) > src(k + rows - 1) &&
               src(k + rows) - src(k + rows - 1) == d)
          ++rows;
        auto fits = [&](size_t r) { return span_ok(s0, s0 + (uint64_t)(r - 1) * d + w0); };
        if (!fits(rows)) {
          size_t good = 1, bad = rows;  // fits(1) holds: one row is the caller's own bytes
          while (bad - good > 1) {
            const size_t mid = good + (bad - good) / 2;
            (fits(mid) ? good : bad) = mid;
          }
          rows = good;
        }
        if (rows > 1) stride = d;
      }
    }
    runs.push_back(CopyRun{k, rows, stride});
    k += rows;
  }
  return runs;
}

// Multi-GPU split of host chunks (qsmd5_rt_staging.cpp run_sharded).  North star:
// shard "only when one file's part count exceeds a single GPU's batch"; and
// host data is bound by each GPU's own PCIe link, so large host batches gain
// from more links.  The chunks (in caller order, lengths host_len) go in
// contiguous, byte-balanced ranges to
//   k = min(ndev, max(ceil(total / shard_bytes), ceil(n / resident)))
// GPUs: `resident` is the most chains one GPU keeps resident in one launch
// (32 768, the 64 KiB-ring latency kernel), and shard_bytes the host bytes
// worth one more link (4 GiB: ~80 ms of PCIe, one 10 MiB chain's time).  A
// small batch stays on one GPU: a chain costs ~85 ms per 10 MiB on any number
// of GPUs.  Returns the shard index of each chunk (0 .. k-1), and k in *nshards.
inline std::vector<uint32_t> plan_shards(const std::vector<uint64_t>& host_len, size_t ndev,
                                         uint64_t shard_bytes, size_t* nshards,
                                         size_t resident = 32768) {
  uint64_t total = 0;
  for (uint64_t L : host_len) total += L;
  const uint64_t per = std::max<uint64_t>(1, shard_bytes);
  const uint64_t by_parts = (host_len.size() + std::max<size_t>(1, resident) - 1) / std::max<size_t>(1, resident);
  const size_t k = (size_t)std::min<uint64_t>(
      std::max<size_t>(1, ndev), std::max<uint64_t>({1, (total + per - 1) / per, by_parts}));
  std::vector<uint32_t> shard(host_len.size(), 0);
  uint64_t cum = 0;
  size_t sh = 0;
  for (size_t i = 0; i < host_len.size(); ++i) {
    // shard sh takes chunks while the bytes before them are below its share
    while (sh + 1 < k && cum >= total / k * (sh + 1)) ++sh;
    shard[i] = (uint32_t)sh;
    cum += host_len[i];
  }
  if (nshards) *nshards = k;
  return shard;
}

// The host-ordered staging schedule (qsmd5_rt_staging.cpp run_batch): S slices,
// nregions ring regions (slice si fills region si % nregions), the copies of
// slice si enqueued at most after the host has seen the kernel of slice
// si - nregions finish (its region is then free), the kernel of slice si
// launched only after the host has seen slice si's copies land, and slices
// with gather rows (read from the metadata block) copied only once that
// block has landed (`meta`).  pipeline_turn runs one turn: the copies of at
// most one slice (a pageable copy is staged by HIP on the calling thread, so
// kernels go out between copies), then every kernel that is ready, in slice
// order.  Returns 1 if anything was enqueued, 0 if the host must wait, -1 if
// a callback failed.  Callbacks:
//   copy_landed(si) / kernel_done(si): 1 yes, 0 not yet, -1 error;
//   needs_meta(si): the slice has gather rows;
//   enqueue_copies(si) / launch(si): 0 or an error code.
// tests/cpp/test_plan.cpp drives it against simulated engines with random
// completion times: every order is respected, every slice runs, no stall.
struct PipelineState {
  size_t nc = 0;  // slices whose copies are enqueued
  size_t nk = 0;  // slices whose kernels are launched
  int err = 0;    // the failing callback's code, when a turn returns -1
};

template <class CopyLanded, class KernelDone, class NeedsMeta, class EnqueueCopies, class Launch>
inline int pipeline_turn(size_t S, size_t nregions, bool meta, PipelineState& st,
                         CopyLanded&& copy_landed, KernelDone&& kernel_done, NeedsMeta&& needs_meta,
                         EnqueueCopies&& enqueue_copies, Launch&& launch) {
  bool moved = false;
  if (st.nc < S) {
    bool ok = true;
    if (st.nc >= nregions) {  // its region: free once the host saw the last user's kernel end
      if (st.nc - nregions >= st.nk) {
        ok = false;  // that kernel is not even launched yet
      } else {
        const int q = kernel_done(st.nc - nregions);
        if (q < 0) return -1;
        ok = q == 1;
      }
    }
    if (ok && needs_meta(st.nc) && !meta) ok = false;
    if (ok) {
      if (int rc = enqueue_copies(st.nc)) {
        st.err = rc;
        return -1;
      }
      ++st.nc;
      moved = true;
    }
  }
  while (st.nk < st.nc && meta) {
    const int q = copy_landed(st.nk);
    if (q < 0) return -1;
    if (!q) break;
    if (int rc = launch(st.nk)) {
      st.err = rc;
      return -1;
    }
    ++st.nk;
    moved = true;
  }
  return moved ? 1 : 0;
}

// ---- pull-driven batches (qsmd5_hash_read, qsmd5_rt_read.cpp) -----------------
// The chunks are not in memory as whole buffers (a qsfs file's parts live in
// its page cache, File::ReadNoLoad gathers them, File.cpp:308-375): the
// library asks for them in COLUMN WINDOWS and hashes each window as it lands,
// every chain parking its state between windows.  The staging budget B is
// split into two host regions (the reader fills one while the other is copied
// to the GPU; the GPU path passes 2B / R to split it into R,
// qsmd5_rt_read.cpp read_regions) and as many device regions; a region holds
// one column of a GROUP of up to `rows_max` chunks, row k at stride
// stage_bytes(W).  So the GPU's width
// (one chain per chunk in a group) depends on the budget only through the
// column width W, never on how many whole chunks fit: 512 x 10 MiB parts go in
// ONE group of 512 chains through 512 MiB of staging (21 columns of 508 KiB),
// and a 100 GB object never stages more than B.
constexpr uint64_t kReadColMin = 64ull << 10;   // narrowest column: ~1 K blocks per launch
constexpr uint64_t kReadColsTarget = 8;         // columns per group when the budget allows
constexpr size_t kReadMaxRows = 32768;          // one resident round of the column kernels

struct ReadGroup {
  size_t first, count;  // lanes [first, first + count) of the longest-first order
  uint64_t W;           // column width (a multiple of 64)
  uint64_t stride;      // row pitch in a region: stage_bytes(W)
  uint32_t ncols;
};

struct ReadPlan {
  uint64_t region = 0;  // bytes of one staging region
  std::vector<ReadGroup> groups;
  // Lanes of group g live in column j: a prefix (lengths are longest first);
  // column 0 holds every lane, empty chunks included (they finish there).
  static size_t active(const std::vector<uint64_t>& len, const ReadGroup& g, uint32_t j) {
    if (j == 0) return g.count;
    size_t a = 0;
    while (a < g.count && len[g.first + a] > (uint64_t)j * g.W) ++a;
    return a;
  }
  // Bytes of lane k's chunk (length L) in column j of its group.
  static uint64_t col_bytes(const ReadGroup& g, uint64_t L, uint32_t j) {
    const uint64_t o = (uint64_t)j * g.W;
    return L > o ? std::min(g.W, L - o) : 0;
  }
};

// len: chunk lengths in lane order, longest first.  staging: the budget B.
inline ReadPlan plan_read(const std::vector<uint64_t>& len, uint64_t staging) {
  ReadPlan P;
  if (len.empty()) return P;
  const uint64_t min_row = stage_bytes(kReadColMin);
  P.region = std::max<uint64_t>(staging / 2, min_row);
  const size_t rows_max =
      (size_t)std::max<uint64_t>(1, std::min<uint64_t>(kReadMaxRows, P.region / min_row));
  for (size_t k = 0; k < len.size();) {
    ReadGroup g{k, std::min(rows_max, len.size() - k), 0, 0, 1};
    const uint64_t L0 = len[k];
    // the widest W whose rows all fit one region: count x (W + kSkew) <= region
    const uint64_t per = P.region / g.count;  // >= min_row
    const uint64_t w_budget = (per - kSkew) / kAlign * kAlign;
    const uint64_t per_col = (L0 + kReadColsTarget - 1) / kReadColsTarget;
    const uint64_t w_target = std::max(kReadColMin, (per_col + kColGrain - 1) / kColGrain * kColGrain);
    uint64_t W = std::min(w_budget, w_target);
    const uint64_t whole = std::max<uint64_t>(kAlign, (L0 + kAlign - 1) / kAlign * kAlign);
    if (whole < W) W = whole;  // short chunks: one column
    g.W = W;
    g.stride = stage_bytes(W);
    g.ncols = (uint32_t)std::max<uint64_t>(1, (L0 + W - 1) / W);
    P.groups.push_back(g);
    k += g.count;
  }
  return P;
}

}  // namespace qsmd5
