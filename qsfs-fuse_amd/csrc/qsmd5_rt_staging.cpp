// qsfs-fuse_amd/csrc/qsmd5_rt_staging.cpp -- one synchronous batch on one GPU (the host-ordered
// staging pipeline), the multi-GPU split, the sleeping wait, chain-rate samples
// (the runtime's units: qsmd5_rt.h).
#include "qsmd5_rt.h"

namespace qsmd5 {
namespace rt {

// Cache policy of the latency kernels' producer loads for a device batch whose
// longest chunk is `longest` bytes: QSMD5_LOAD_NT=1 / 0 forces nt / default.
static bool load_nt_for(uint64_t longest) {
  const char* e = getenv("QSMD5_LOAD_NT");
  if (e && *e) return strcmp(e, "0") != 0;
  (void)longest;
  return false;
}

// Chains per workgroup of the latency kernel for a device batch of n chunks
// whose longest has `longest` bytes.  64 lanes of a wave reading 64 long
// chunks in lockstep run ~7% slower once the parts reach 64 MiB (and at exact
// 32 MiB strides): 1293-1300 cycles per block from the first block on, at an
// unchanged 2.40 GHz, against 1225 for 56 MiB parts
// (profiles/r02_plateau_lanes.log, ubench ptrace).  Half a wave per CU --
// half the address span per CU -- brings them back to 1235-1242.  The chains
// then occupy twice the CUs, so only while one round still holds the batch
// (256 CUs x 32 lanes).  QSMD5_PC_LANES overrides (1..64).
static uint32_t pc_lanes_for(size_t n, uint64_t longest) {
  const uint64_t forced = env_u64("QSMD5_PC_LANES", 0);
  if (forced >= 1 && forced <= 64) return (uint32_t)forced;
  constexpr uint64_t kLongPart = 32ull << 20;  // the skewed regime (kSkewMinBlocks blocks)
  if (longest >= kLongPart && n <= qsmd5::kLatencyKernelResident / 2) return 32;
  return 64;
}

using qsmd5::kNoColumns;
using qsmd5::stage_bytes;

// The GPU chain rate averaged over timed batches (double bits; 0 = none yet),
// for the routing cost model (qsmd5_rt_route.cpp).  Only a batch that ran
// as ONE latency-kernel launch (<= 16 384 chunks, one chain per lane) with a
// longest chunk of >= 4 MiB measures a chain: its kernel time is that chain's.
std::atomic<uint64_t> g_gpu_chain_bits{0};

// One outlier must not steer routing: the first qualifying batch
// of each bound GPU is not used (deferred code-object loading and clock
// ramp-up can fall inside its window), a sample outside [0.03, 0.6] GiB/s --
// the ~1190 cycles per 64-B block expected at 2.4 GHz is 0.12 -- is not a
// chain-bound launch, and the rest are folded into an average (new samples
// weigh 1/4), so one slow launch on a shared GPU moves it by a quarter at most.
void note_gpu_chain(std::atomic<uint32_t>& dev_samples, uint64_t longest, size_t n, unsigned launches,
                    double kernel_ms) {
  if (launches != 1 || n > qsmd5::kLatencyKernelResident || longest < (4ull << 20) || kernel_ms <= 0)
    return;
  if (dev_samples.fetch_add(1, std::memory_order_relaxed) == 0) return;  // this GPU's first
  const double gibs = (double)longest / (kernel_ms * 1e-3) / 1073741824.0;
  if (gibs < 0.03 || gibs > 0.6) return;
  uint64_t old = g_gpu_chain_bits.load(std::memory_order_relaxed), bits;
  do {
    double avg = gibs;
    if (old) {
      memcpy(&avg, &old, sizeof(avg));
      avg = 0.75 * avg + 0.25 * gibs;
    }
    memcpy(&bits, &avg, sizeof(bits));
  } while (!g_gpu_chain_bits.compare_exchange_weak(old, bits, std::memory_order_relaxed));
}

// How the calling thread waits for a synchronous batch.  hipStreamSynchronize
// spins a host core for the whole batch, and so does hipEventSynchronize even
// on a hipEventBlockingSync event (ubench/thread_cpu_probe.hip: 80 ms waits
// cost the caller 80 ms of CPU in all three forms).  A GPU batch of 10 MiB
// parts is one ~85 ms chain, so a daemon that sends waves to the GPU to keep
// its cores for itself would lose one core per waiting thread.  A batch the
// cost model expects to take >= 1 ms therefore sleeps through 90% of that
// estimate and then checks an event every 100 us (QSMD5_WAIT=poll; the
// route sweep's 32 GPU waves of 8 parts: the caller's CPU went from 2.7 s to
// ~0, same wall time, profiles/r04_wait_ab.log); shorter batches keep the
// spin, which wakes faster (a 1 KiB call stays at ~39 us).
// QSMD5_WAIT=spin / block / poll forces one form for every batch.
int wait_mode() {  // 0 auto, 1 block, 2 spin, 3 poll
  static const int mode = [] {
    const char* e = getenv("QSMD5_WAIT");
    return !e || !*e || !strcmp(e, "auto") ? 0 : !strcmp(e, "block") ? 1 : !strcmp(e, "poll") ? 3 : 2;
  }();
  return mode;
}

// Wait for everything enqueued on stream s of GPU d (caller holds d.mu).
hipError_t wait_stream(Dev& d, hipStream_t s, double est_ms) {
  const int mode = wait_mode();
  if (mode == 2 || (mode == 0 && est_ms < 1.0)) return hipStreamSynchronize(s);
  hipError_t e = hipEventRecord(d.ev_done, s);
  if (e != hipSuccess) return e;
  if (mode == 1) return hipEventSynchronize(d.ev_done);
  // poll: sleep through most of the expected time (est_ms is the batch's
  // shortest plausible time, gpu_wait_est_ms), then check every 100 us
  // (every 1 ms once a batch runs 2 s past its start: a shared or slow GPU)
  auto t0 = std::chrono::steady_clock::now();
  if (est_ms > 0) std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(est_ms * 900.0)));
  for (;;) {
    e = hipEventQuery(d.ev_done);
    if (e != hipErrorNotReady) return e;
    std::this_thread::sleep_for(std::chrono::microseconds(
        std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2) ? 1000 : 100));
  }
}

// The synchronous batch on one GPU: device chunks in one launch; host chunks
// staged in slices with copy/compute overlap.  Caller holds r.mu and has made
// r.device current.  Device chunks must live on r.device: a kernel reading
// another GPU's memory would fault unless peer access happens to be enabled.
int run_batch(Dev& r, const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags) {
  auto t0 = std::chrono::steady_clock::now();
  if (n > 0xffffffffull) return fail(-EINVAL, "qsmd5: too many chunks");

  std::vector<uint64_t> len(n);
  std::vector<MemKind> kind(n);
  std::vector<uint8_t> hipk(n, 0);  // Classifier::operator() *hip of each chunk
  Classifier cls(flags, n);
  for (size_t i = 0; i < n; ++i) {
    uint64_t L = chunks[i].len;
    if (flags & QSMD5_FLAG_REF_TRUNCATE32) L &= 0xffffffffull;
    if (L >= kMaxChunkLen) return fail(-EINVAL, "qsmd5: chunk longer than 2^38 bytes");
    if (L > 0 && !chunks[i].ptr) return fail(-EINVAL, "qsmd5: NULL ptr with non-zero len");
    len[i] = L;
    int owner = -1;
    kind[i] = L ? cls(chunks[i].ptr, &owner, &hipk[i]) : kDeviceMem;  // empty chunks read nothing
    if (L && kind[i] == kDeviceMem && owner != r.device)
      return fail(-EINVAL, "qsmd5: chunk lives on GPU " + std::to_string(owner) +
                               ", not on a bound GPU (QSMD5_DEVICE/QSMD5_DEVICES)");
    if (L && kind[i] == kDeviceMem && cls.overruns_allocation(reinterpret_cast<uintptr_t>(chunks[i].ptr), L))
      return fail(-EINVAL, "qsmd5: device chunk " + std::to_string(i) + " (" + std::to_string(L) +
                               " bytes) runs past the end of its allocation");
  }

  const auto t_classified = std::chrono::steady_clock::now();
  // Lane order: device chunks first, then host chunks; each group sorted by
  // length (descending) so the lanes of a wavefront finish together.  Device
  // chunks of equal length are ordered by address: a wave's lanes then read
  // neighbouring buffers, which spread evenly over the HBM channels, whatever
  // order a buffer pool handed them out in (512 x 10 MiB pool buffers in
  // shuffled order: 50.8 -> 59.3 GiB/s, profiles/r01_config_pool.jsonl).
  // Host chunks are staged in lane order into our own skewed layout; equal
  // lengths go by address too, so a pool's buffers handed out in any order
  // (and glibc's downward-growing mmaps, which the kernel merges into one VMA)
  // line up as ascending constant-stride rows: one 2-D copy per column where
  // they share a mapping (qsmd5_plan.h plan_copy_runs).
  std::vector<uint32_t> dev_idx, host_idx;
  for (size_t i = 0; i < n; ++i) (kind[i] == kDeviceMem ? dev_idx : host_idx).push_back((uint32_t)i);
  auto by_len_addr = [&](uint32_t a, uint32_t b) {
    if (len[a] != len[b]) return len[a] > len[b];
    const uintptr_t pa = reinterpret_cast<uintptr_t>(chunks[a].ptr);
    const uintptr_t pb = reinterpret_cast<uintptr_t>(chunks[b].ptr);
    return pa < pb || (pa == pb && a < b);
  };
  // A file's parts or a pool's buffers usually arrive in order already (1 M
  // chunks: 7.7 ms to sort, ~1 ms to check)
  if (!std::is_sorted(dev_idx.begin(), dev_idx.end(), by_len_addr))
    std::sort(dev_idx.begin(), dev_idx.end(), by_len_addr);
  if (!std::is_sorted(host_idx.begin(), host_idx.end(), by_len_addr))
    std::sort(host_idx.begin(), host_idx.end(), by_len_addr);

  const auto t_sorted = std::chrono::steady_clock::now();
  // Staging plan for the host chunks (qsmd5_plan.h; its invariants are tested
  // on the CPU by tests/cpp/test_plan.cpp).
  std::vector<uint64_t> host_len(host_idx.size());
  for (size_t k = 0; k < host_idx.size(); ++k) host_len[k] = len[host_idx[k]];
  int64_t column_bytes = -1;  // automatic
  if (const char* ev = getenv("QSMD5_COLUMN_BYTES"); ev && *ev)
    column_bytes = (int64_t)env_u64("QSMD5_COLUMN_BYTES", 0);  // 0 = whole chunks
  // read per batch (tests shrink the ring to one region to drive region reuse)
  r.staging_cap = env_u64("QSMD5_STAGING_BYTES", kDefaultStaging);
  const qsmd5::HostPlan plan =
      qsmd5::plan_host(host_len, r.staging_cap, env_u64("QSMD5_SLICE_BYTES", 0), column_bytes);
  const auto t_hostplan = std::chrono::steady_clock::now();
  const uint64_t W = plan.W, region = plan.region;
  const std::vector<qsmd5::Group>& groups = plan.groups;
  const std::vector<qsmd5::Slice>& slices = plan.slices;
  const size_t nseg = plan.nseg, nregions = plan.nregions;
  auto col_bytes = [&](uint64_t L, uint32_t j) { return plan.col_bytes(L, j); };
  // Tiny host batches ride inline: the CPU copies their bytes into the pinned
  // metadata block, so descriptors, lane orders and data go to the GPU in ONE
  // copy, and copy, kernel and digests stay on one stream (profiles/
  // r01_small_call_latency.log).  Only for chunks the runtime classified
  // itself: under QSMD5_FLAG_HOST a caller's stray device pointer must not
  // reach a CPU memcpy.
  uint64_t inline_bytes = 0;
  bool inline_data = slices.size() == 1 && !(flags & QSMD5_FLAG_HOST) && groups[0].ncols == 1;
  if (inline_data) {
    for (uint64_t L : host_len) inline_bytes += stage_bytes(L);
    inline_data = inline_bytes <= kInlineBytes;
  }
  if (!inline_data) inline_bytes = 0;
  if (!slices.empty() && !inline_data)
    if (int rc = r.d_staging.reserve(nregions * region)) return rc;

  // H2D copies of each slice (qsmd5_plan.h plan_copy_runs): runs of rows in one
  // allocation at a constant stride go as one 2-D copy.  Rows left on their
  // own that sit in a pinned or registered host allocation (a pool of pinned
  // buffers, each its own allocation) are gathered by ONE qsmd5_gather_kernel
  // launch per slice instead of one hipMemcpyAsync each (QSMD5_GATHER=0: off).
  std::vector<std::vector<qsmd5::CopyRun>> slice_runs(inline_data ? 0 : slices.size());
  std::vector<uintptr_t> gather_dev(inline_data ? 0 : host_idx.size(), 0);  // 0: not gatherable
  if (!inline_data && !slices.empty()) {
    for (size_t si = 0; si < slices.size(); ++si) {
      const qsmd5::Slice& sl = slices[si];
      const qsmd5::Group& g = groups[sl.group];
      const uint64_t col_off = W == kNoColumns ? 0 : (uint64_t)sl.col * W;
      slice_runs[si] = qsmd5::plan_copy_runs(
          sl.active,
          [&](size_t k) {
            return (uint64_t)reinterpret_cast<uintptr_t>(chunks[host_idx[g.first + k]].ptr) + col_off;
          },
          [&](size_t k) { return col_bytes(len[host_idx[g.first + k]], sl.col); },
          [&](uint64_t lo, uint64_t hi) { return cls.span_in_one(lo, hi); });
    }
    // Gather candidates: rows left on their own (a file's parts or one pool
    // slab form 2-D runs and never get here), in HIP-known or unclassified
    // memory, 16-B aligned, the whole chunk in one pinned/registered host
    // allocation.  Checked once per chunk.
    if (env_u64("QSMD5_GATHER", 1)) {
      std::vector<uint8_t> seen(host_idx.size(), 0);
      for (size_t si = 0; si < slices.size(); ++si) {
        const qsmd5::Group& g = groups[slices[si].group];
        for (const qsmd5::CopyRun& run : slice_runs[si]) {
          const size_t k = g.first + run.first;
          if (run.rows != 1 || seen[k]) continue;
          seen[k] = 1;
          const uint32_t ci = host_idx[k];
          const uintptr_t p = reinterpret_cast<uintptr_t>(chunks[ci].ptr);
          uintptr_t dev = 0;
          if (hipk[ci] != 0 && (p & 15u) == 0 && cls.hip_host_range(p, p + host_len[k], &dev))
            gather_dev[k] = dev;
        }
      }
    }
  }
  auto gathered = [&](const qsmd5::Slice& sl, const qsmd5::CopyRun& run) {
    return run.rows == 1 && gather_dev[groups[sl.group].first + run.first] != 0;
  };
  size_t ngather = 0;
  for (size_t si = 0; si < slice_runs.size(); ++si)
    for (const qsmd5::CopyRun& run : slice_runs[si]) ngather += gathered(slices[si], run);

  const auto t_runs = std::chrono::steady_clock::now();
  // One metadata block: descriptors (device pointers) for every chunk, then
  // segment descriptors of the multi-column slices; the lane->chunk maps; the
  // gather rows; the inline data.
  const size_t meta_bytes = n * sizeof(qsmd5_chunk) + nseg * sizeof(qsmd5_chunk);
  const size_t order_words = n + nseg;
  const size_t desc_span = (meta_bytes + 255) & ~size_t(255);
  const size_t order_span = (order_words * sizeof(uint32_t) + 255) & ~size_t(255);
  const size_t gather_off = desc_span + order_span;
  const size_t gather_span = (ngather * qsmd5::kGatherRowBytes + 255) & ~size_t(255);
  const size_t data_off = gather_off + gather_span;
  const size_t block_bytes = data_off + inline_bytes;
  if (int rc = r.h_meta.reserve(block_bytes + 256)) return rc;
  if (int rc = r.d_meta.reserve(block_bytes + 256)) return rc;
  if (int rc = r.h_dig.reserve(n * 16 + 16)) return rc;
  if (int rc = r.d_dig.reserve(n * 16 + 16)) return rc;
  if (nseg)
    if (int rc = r.d_state.reserve(n * 16 + 16)) return rc;
  uint8_t* hm = static_cast<uint8_t*>(r.h_meta.p);
  uint8_t* dm = static_cast<uint8_t*>(r.d_meta.p);
  qsmd5_chunk* hd = reinterpret_cast<qsmd5_chunk*>(hm);
  qsmd5_chunk* hseg = hd + n;
  uint32_t* ho = reinterpret_cast<uint32_t*>(hm + desc_span);
  uint32_t* hso = ho + n;
  for (size_t i = 0; i < n; ++i) hd[i] = {len[i] ? chunks[i].ptr : nullptr, len[i]};
  uint8_t* stage = inline_data ? dm + data_off : static_cast<uint8_t*>(r.d_staging.p);
  size_t ngather_filled = 0;
  std::vector<uint8_t*> slice_base(slices.size());
  std::vector<size_t> row_off;  // staged offset of each active row of the slice
  for (size_t si = 0; si < slices.size(); ++si) {
    const qsmd5::Slice& sl = slices[si];
    const qsmd5::Group& g = groups[sl.group];
    uint8_t* base = stage + (si % nregions) * region;
    slice_base[si] = base;
    uint64_t off = 0;
    bool any_gather = false;
    if (!inline_data)
      for (const qsmd5::CopyRun& run : slice_runs[si]) any_gather = any_gather || gathered(sl, run);
    if (any_gather) row_off.resize(sl.active);
    for (size_t k = 0; k < sl.active; ++k) {
      const uint32_t ci = host_idx[g.first + k];
      if (g.ncols > 1) {
        hseg[sl.seg0 + k] = {base + off, len[ci]};
        hso[sl.seg0 + k] = ci;
      } else {
        hd[ci].ptr = base + off;
      }
      if (inline_data) memcpy(hm + data_off + off, chunks[ci].ptr, len[ci]);
      if (any_gather) row_off[k] = off;
      off += stage_bytes(col_bytes(len[ci], sl.col));
    }
    if (!any_gather) continue;
    const uint64_t col_off = W == kNoColumns ? 0 : (uint64_t)sl.col * W;
    for (const qsmd5::CopyRun& run : slice_runs[si]) {
      if (!gathered(sl, run)) continue;
      const size_t k = run.first;
      uint64_t* gr = reinterpret_cast<uint64_t*>(hm + gather_off) + 3 * ngather_filled;
      gr[0] = gather_dev[g.first + k] + col_off;
      gr[1] = reinterpret_cast<uint64_t>(base + row_off[k]);
      gr[2] = col_bytes(len[host_idx[g.first + k]], sl.col);
      ++ngather_filled;
    }
  }
  size_t pos = 0;
  for (uint32_t ci : dev_idx) ho[pos++] = ci;
  for (uint32_t ci : host_idx) ho[pos++] = ci;

  const auto t_planned = std::chrono::steady_clock::now();
  hipStream_t s0 = r.compute[0];
  EventSet events;
  // On any failure after work was enqueued, wait for it before returning: an
  // H2D copy may still be reading the caller's buffers.
  auto drain = [&](int code) {
    for (int k = 0; k < r.ncopy; ++k) (void)hipStreamSynchronize(r.copy[k]);
    for (hipStream_t s : r.compute) (void)hipStreamSynchronize(s);
    return code;
  };
  QS_HIP(hipMemcpyAsync(dm, hm, block_bytes, hipMemcpyHostToDevice, s0));
  // A single slice runs entirely on s0 (copy, then kernel: stream order, no
  // events); several slices overlap copies and kernels over the streams.
  const bool one_stream = slices.size() <= 1;
  if (!one_stream) QS_HIP(hipEventRecord(r.ev_meta, s0));
  // QSMD5_TRACE=1: per-slice copy/kernel timeline on stderr (diagnostics).
  const bool trace = env_u64("QSMD5_TRACE", 0) != 0;
  std::vector<hipEvent_t> tr(trace ? 4 * slices.size() + 1 : 0, nullptr);
  for (auto& ev : tr)
    if (int rc = events.make(&ev, hipEventDefault)) return drain(rc);
  if (trace) QS_HIP(hipEventRecord(tr.back(), s0));
  const uint32_t* d_order = reinterpret_cast<const uint32_t*>(dm + desc_span);
  const qsmd5_chunk* d_desc = reinterpret_cast<const qsmd5_chunk*>(dm);
  const qsmd5_chunk* d_seg = d_desc + n;
  uint32_t* d_dig = static_cast<uint32_t*>(r.d_dig.p);
  bool first_kernel = true;
  unsigned launches = 0;   // hashing launches (a chain-rate sample needs exactly one)
  unsigned used = 0;  // compute streams (1..) that ran work: joined into s0 at the end
  auto mark_first = [&](hipStream_t s) -> int {
    if (first_kernel) {
      QS_HIP(hipEventRecord(r.ev_first, s));
      first_kernel = false;
    }
    return 0;
  };
  auto launch = [&](hipStream_t s, const uint32_t* ord, size_t cnt, bool aligned16,
                    uint64_t longest) -> int {
    if (int rc = mark_first(s)) return rc;
    ++launches;
    static const uint32_t skew = (uint32_t)env_u64("QSMD5_SKEW_BLOCKS", qsmd5::kPcSkewBlocks);
    hipError_t e = qsmd5::launch_batch(d_desc, ord, (uint32_t)cnt, d_dig,
                                       kernel_choice(cnt, aligned16), s, skew,
                                       load_nt_for(longest), pc_lanes_for(cnt, longest));
    if (e != hipSuccess) return hip_fail(e, "qsmd5 kernel launch");
    return 0;
  };

  // Device-resident chunks: one launch.
  if (!dev_idx.empty()) {
    bool aligned16 = true;
    for (uint32_t ci : dev_idx)
      aligned16 = aligned16 && (reinterpret_cast<uintptr_t>(hd[ci].ptr) & 15u) == 0;
    if (int rc = launch(s0, d_order, dev_idx.size(), aligned16, len[dev_idx[0]])) return drain(rc);
  }
  // Host-resident slices: H2D on a copy stream into the slice's ring region
  // (after the kernel that last used the region), then a launch on its group's
  // compute stream (so a group's columns run in order) once the copy and the
  // descriptors have landed.  Runs of equal-length chunks at a constant host
  // stride inside one allocation (a file's parts) go as one 2-D copy per column.
  //
  // The order between copy and compute streams is kept by THIS thread, not by
  // hipStreamWaitEvent: while a stream holds a wait on another stream's
  // pending event, HIP keeps one of its own threads polling for the whole
  // batch -- a host core per batch (ubench/thread_cpu_probe.hip: 40 column
  // slices ordered by stream waits, 0.91 cores; the same slices ordered by the
  // host, 0; equal wall time).  So a slice's copies are enqueued once the host
  // has seen the kernel that last used its region finish, and its kernel is
  // launched once the host has seen its copies land; the thread sleeps between
  // checks (20 us, backing off to 200 us while nothing moves).  Copies run
  // nregions slices ahead and kernels queue behind each other, so neither
  // engine idles on the host's latency.  A single slice needs no ordering: its
  // copy and kernel run on s0 in stream order.
  const size_t S = slices.size();
  std::vector<hipEvent_t> copied(one_stream ? 0 : S, nullptr), done(one_stream ? 0 : S, nullptr);
  std::vector<size_t> gather_first(S + 1, 0);  // gather rows of slice si: [first[si], first[si + 1])
  for (size_t si = 0; si < S; ++si) {
    size_t k = 0;
    if (!inline_data)
      for (const qsmd5::CopyRun& run : slice_runs[si]) k += gathered(slices[si], run) ? 1 : 0;
    gather_first[si + 1] = gather_first[si] + k;
  }
  auto slice_gathers = [&](size_t si) { return gather_first[si + 1] - gather_first[si]; };
  // The slice's copies (planned above): 2-D runs and single rows by DMA,
  // gathered rows by one kernel launch; then `copied[si]` on the copy stream.
  auto enqueue_copies = [&](size_t si, hipStream_t cp) -> int {
    const qsmd5::Slice& sl = slices[si];
    const qsmd5::Group& g = groups[sl.group];
    const uint64_t col_off = W == kNoColumns ? 0 : (uint64_t)sl.col * W;
    uint8_t* dst = slice_base[si];
    if (trace) QS_HIP(hipEventRecord(tr[4 * si], cp));
    size_t slice_gather = 0;
    static const std::vector<qsmd5::CopyRun> kNoRuns;  // inline data: already in the meta copy
    const std::vector<qsmd5::CopyRun>& runs = inline_data ? kNoRuns : slice_runs[si];
    for (const qsmd5::CopyRun& run : runs) {
      const uint32_t ci = host_idx[g.first + run.first];
      const uint64_t w = col_bytes(len[ci], sl.col);
      if (gathered(sl, run)) {
        ++slice_gather;
        dst += stage_bytes(w);
        continue;
      }
      const uint8_t* src = static_cast<const uint8_t*>(chunks[ci].ptr) + col_off;
      hipError_t e = hipSuccess;
      if (run.rows > 1) {
        e = hipMemcpy2DAsync(dst, stage_bytes(w), src, (size_t)run.stride, w, run.rows,
                             hipMemcpyHostToDevice, cp);
        // Belt and braces: should HIP still refuse a span inside one allocation
        // (nothing is enqueued then), copy the rows one by one.
        if (e == hipErrorInvalidValue) {
          (void)hipGetLastError();
          e = hipSuccess;
          for (size_t j = 0; j < run.rows && e == hipSuccess; ++j)
            e = hipMemcpyAsync(dst + j * stage_bytes(w), src + j * run.stride, w,
                               hipMemcpyHostToDevice, cp);
        }
      } else {
        e = hipMemcpyAsync(dst, src, w, hipMemcpyHostToDevice, cp);
      }
      if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync H2D");
      dst += run.rows * stage_bytes(w);
    }
    if (slice_gather) {  // the gather rows live in the metadata block (landed: see below)
      hipError_t e = qsmd5::launch_gather(dm + gather_off + gather_first[si] * qsmd5::kGatherRowBytes,
                                          (uint32_t)slice_gather, cp,
                                          (uint32_t)env_u64("QSMD5_GATHER_GROUPS", 8));
      if (e != hipSuccess) return hip_fail(e, "qsmd5 gather launch");
    }
    if (trace) QS_HIP(hipEventRecord(tr[4 * si + 1], cp));
    if (!one_stream) {
      if (int rc = events.make(&copied[si], hipEventDisableTiming)) return rc;
      QS_HIP(hipEventRecord(copied[si], cp));
    }
    return 0;
  };
  // The slice's kernel on its compute stream; then `done[si]` if a later
  // slice reuses the region.
  auto launch_slice = [&](size_t si, hipStream_t cs) -> int {
    const qsmd5::Slice& sl = slices[si];
    const qsmd5::Group& g = groups[sl.group];
    const uint64_t col_off = W == kNoColumns ? 0 : (uint64_t)sl.col * W;
    if (trace) QS_HIP(hipEventRecord(tr[4 * si + 2], cs));
    if (g.ncols > 1) {
      if (int rc = mark_first(cs)) return rc;
      ++launches;
      hipError_t e = qsmd5::launch_column(d_seg + sl.seg0, d_order + n + sl.seg0, (uint32_t)sl.active,
                                          d_dig, col_off, W, static_cast<uint32_t*>(r.d_state.p), cs);
      if (e != hipSuccess) return hip_fail(e, "qsmd5 column kernel launch");
    } else {
      // staged chunks sit at 256-B-aligned offsets plus a 16-B-multiple skew
      if (int rc = launch(cs, d_order + dev_idx.size() + g.first, sl.active, true, 0)) return rc;
    }
    if (!one_stream && si + nregions < S) {  // a later slice reuses this region
      if (int rc = events.make(&done[si], hipEventDisableTiming)) return rc;
      QS_HIP(hipEventRecord(done[si], cs));
    }
    if (trace) QS_HIP(hipEventRecord(tr[4 * si + 3], cs));
    return 0;
  };
  auto compute_stream_of = [&](size_t si) {
    return one_stream ? 0 : 1 + (int)(slices[si].group % (kComputeStreams - 1));
  };
  // 1 = complete, 0 = pending, -1 = error (t_last_error set)
  auto landed = [&](hipEvent_t ev) -> int {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 1;
    if (q == hipErrorNotReady) return 0;
    (void)hip_fail(q, "waiting for a staging step");
    return -1;
  };
  if (one_stream) {
    if (S) {
      used |= 1u;
      if (int rc = enqueue_copies(0, s0)) return drain(rc);
      if (int rc = launch_slice(0, s0)) return drain(rc);
    }
  } else {
    qsmd5::PipelineState st;
    bool meta = false;  // the metadata block (descriptors, gather rows) has landed
    int idle_us = 20;
    while (st.nk < S) {
      if (!meta) {
        const int q = landed(r.ev_meta);
        if (q < 0) return drain(-EIO);
        meta = q == 1;
      }
      const int t = qsmd5::pipeline_turn(
          S, nregions, meta, st, [&](size_t si) { return landed(copied[si]); },
          [&](size_t si) { return landed(done[si]); },
          [&](size_t si) { return slice_gathers(si) != 0; },
          [&](size_t si) { return enqueue_copies(si, r.copy[si % r.ncopy]); },
          [&](size_t si) {
            const int csi = compute_stream_of(si);
            used |= 1u << csi;
            return launch_slice(si, r.compute[csi]);
          });
      if (t < 0) return drain(st.err ? st.err : -EIO);
      if (st.nk == S) break;
      if (t > 0) {
        idle_us = 20;
      } else {
        std::this_thread::sleep_for(std::chrono::microseconds(idle_us));
        idle_us = std::min(200, idle_us * 2);
      }
    }
  }
  // Every kernel is enqueued.  The compute streams that ran slices end with a
  // timing event each; the host sees them all complete before the digests
  // come back on s0 (after s0's own device-chunk kernel, in stream order).
  std::vector<hipEvent_t> tails;
  for (int k = 1; k < kComputeStreams; ++k) {
    if (!(used & (1u << k))) continue;
    hipEvent_t t = nullptr;
    if (int rc = events.make(&t, hipEventDefault)) return drain(rc);
    // from here on copies of the caller's buffers may be in flight: every
    // failure drains before it returns
    if (hipError_t e = hipEventRecord(t, r.compute[k]); e != hipSuccess)
      return drain(hip_fail(e, "hipEventRecord"));
    tails.push_back(t);
  }
  if (!first_kernel)
    if (hipError_t e = hipEventRecord(r.ev_last, s0); e != hipSuccess)
      return drain(hip_fail(e, "hipEventRecord"));
  uint64_t longest_len = 0, host_bytes = 0;
  for (size_t i = 0; i < n; ++i) longest_len = std::max(longest_len, len[i]);
  for (uint64_t L : host_len) host_bytes += L;
  // The compute streams' queued kernels: how much is left is not known here
  // (a group's columns run one after another behind its copies), so the host
  // keeps polling, backing off from 20 us to 500 us.
  for (hipEvent_t t : tails) {
    if (wait_mode() == 1 || wait_mode() == 2) {  // QSMD5_WAIT=block / spin: HIP's own wait
      const hipError_t e = hipEventSynchronize(t);
      if (e != hipSuccess) return drain(hip_fail(e, "waiting for the batch"));
      continue;
    }
    int idle_us = 20;
    for (;;) {
      const int q = landed(t);
      if (q < 0) return drain(-EIO);
      if (q) break;
      std::this_thread::sleep_for(std::chrono::microseconds(idle_us));
      idle_us = std::min(500, idle_us * 2);
    }
  }
  if (hipError_t e = hipMemcpyAsync(r.h_dig.p, d_dig, n * 16, hipMemcpyDeviceToHost, s0); e != hipSuccess)
    return drain(hip_fail(e, "hipMemcpyAsync D2H"));
  // one stream (a single slice, or device chunks only): copy and kernel in
  // stream order, so the cost model's copy + chain is what is left to wait
  const double est_ms = tails.empty() ? gpu_wait_est_ms(longest_len, host_bytes) : 0.0;
  hipError_t e = wait_stream(r, s0, est_ms);
  if (e != hipSuccess) return drain(hip_fail(e, "waiting for the batch"));
  memcpy(digests, r.h_dig.p, n * 16);
  if (trace) {
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t_end = std::chrono::steady_clock::now();
    fprintf(stderr, "qsmd5 trace: %zu chunks: classify %.2f ms, sort %.2f ms, plan %.2f ms "
            "(staging plan %.2f, copy runs + gather rows %.2f, descriptors %.2f), "
            "enqueue+run %.2f ms\n", n, ms(t0, t_classified), ms(t_classified, t_sorted),
            ms(t_sorted, t_planned), ms(t_sorted, t_hostplan), ms(t_hostplan, t_runs),
            ms(t_runs, t_planned), ms(t_planned, t_end));
    fprintf(stderr, "qsmd5 trace: %zu slices, column width %llu, %zu groups, %zu regions, "
            "%zu gathered rows\n", slices.size(), (unsigned long long)(W == kNoColumns ? 0 : W),
            groups.size(), nregions, ngather);
    for (size_t si = 0; si < slices.size(); ++si) {
      float t[4] = {0, 0, 0, 0};
      for (int k = 0; k < 4; ++k) (void)hipEventElapsedTime(&t[k], tr.back(), tr[4 * si + k]);
      fprintf(stderr, "  slice %zu g%zu c%u n=%zu copy %.2f..%.2f ms kernel %.2f..%.2f ms\n", si,
              slices[si].group, slices[si].col, slices[si].active, t[0], t[1], t[2], t[3]);
    }
  }
  float kms = 0;
  r.last_kernel_ms =
      (!first_kernel && hipEventElapsedTime(&kms, r.ev_first, r.ev_last) == hipSuccess) ? kms : 0.0;
  for (hipEvent_t t : tails)  // slices on the other compute streams
    if (!first_kernel && hipEventElapsedTime(&kms, r.ev_first, t) == hipSuccess)
      r.last_kernel_ms = std::max(r.last_kernel_ms, (double)kms);
  {
    uint64_t longest = 0;
    for (uint64_t L : len) longest = std::max(longest, L);
    note_gpu_chain(r.chain_samples, longest, n, launches, r.last_kernel_ms);
  }
  r.last_wall_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

// Multi-GPU batch (QSMD5_DEVICES binds more than one GPU).
// Device chunks run on the GPU that holds them.  Host chunks (the qsfs case)
// are cut into contiguous, byte-balanced ranges over k = min(#GPUs,
// ceil(host bytes / QSMD5_SHARD_BYTES)) GPUs: host data is bound by each GPU's
// own PCIe link, so shards add ingest bandwidth, while a small batch stays on
// one GPU (a chain costs ~85 ms per 10 MiB on any number of GPUs).  One thread
// per GPU runs run_batch on its shard, and the digests are scattered back by
// chunk index.  In one process there is no collective: every shard's digests
// land in host memory.  (One process per GPU is qsmd5/parallel.py: RCCL.)
int run_sharded(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags,
                double* kernel_ms, double* wall_ms) {
  Runtime& R = rt();
  auto t0 = std::chrono::steady_clock::now();
  const size_t nd = R.devs.size();
  std::vector<std::vector<uint32_t>> part(nd);
  std::vector<uint32_t> host;
  if (n > 0xffffffffull) return fail(-EINVAL, "qsmd5: too many chunks");
  Classifier cls(flags, n);
  for (size_t i = 0; i < n; ++i) {
    uint64_t L = chunks[i].len;
    if (flags & QSMD5_FLAG_REF_TRUNCATE32) L &= 0xffffffffull;
    int owner = -1;
    if (L && chunks[i].ptr && cls(chunks[i].ptr, &owner) == kDeviceMem) {
      size_t d = 0;
      while (d < nd && R.devs[d]->device != owner) ++d;
      if (d == nd)
        return fail(-EINVAL, "qsmd5: chunk lives on GPU " + std::to_string(owner) +
                                 ", not on a bound GPU (QSMD5_DEVICES)");
      part[d].push_back((uint32_t)i);
    } else {
      host.push_back((uint32_t)i);
    }
  }
  std::vector<uint64_t> host_len(host.size());
  for (size_t j = 0; j < host.size(); ++j) {
    uint64_t L = chunks[host[j]].len;
    if (flags & QSMD5_FLAG_REF_TRUNCATE32) L &= 0xffffffffull;
    host_len[j] = L;
  }
  size_t k = 1;
  const std::vector<uint32_t> shard = qsmd5::plan_shards(host_len, nd, R.shard_bytes, &k, qsmd5::kLatency2KernelResident);
  for (size_t j = 0; j < host.size(); ++j) part[shard[j]].push_back(host[j]);
  if (env_u64("QSMD5_TRACE", 0)) {
    for (size_t d = 0; d < nd; ++d)
      fprintf(stderr, "qsmd5 shard: context %zu (GPU %d) takes %zu chunks\n", d, R.devs[d]->device,
              part[d].size());
  }
  std::vector<int> rc(nd, 0);
  std::vector<std::string> err(nd);
  std::vector<double> kms(nd, 0.0);
  auto work = [&](size_t d) {
    try {
      const std::vector<uint32_t>& idx = part[d];
      std::vector<qsmd5_chunk> sub(idx.size());
      for (size_t j = 0; j < idx.size(); ++j) sub[j] = chunks[idx[j]];
      std::vector<uint8_t> dig(16 * idx.size());
      Dev& dv = *R.devs[d];
      hipError_t e = hipSetDevice(dv.device);
      if (e != hipSuccess) {
        rc[d] = hip_fail(e, "hipSetDevice");
      } else {
        std::lock_guard<std::mutex> lk(dv.mu);
        rc[d] = run_batch(dv, sub.data(), sub.size(), reinterpret_cast<uint8_t(*)[16]>(dig.data()),
                          flags);
        kms[d] = dv.last_kernel_ms;
      }
      if (rc[d] == 0)
        for (size_t j = 0; j < idx.size(); ++j) memcpy(digests[idx[j]], &dig[16 * j], 16);
    } catch (const std::bad_alloc&) {
      rc[d] = fail(-ENOMEM, "qsmd5: host allocation failed");
    } catch (...) {
      rc[d] = fail(-EIO, "qsmd5: internal error");
    }
    if (rc[d]) err[d] = t_last_error;  // thread_local: carry it to the caller
  };
  std::vector<std::thread> th;
  size_t mine = nd;
  for (size_t d = 0; d < nd; ++d) {
    if (part[d].empty()) continue;
    if (mine == nd) {
      mine = d;  // the calling thread takes the first shard
      continue;
    }
    try {
      th.emplace_back(work, d);
    } catch (...) {
      work(d);  // no thread available: run it here
    }
  }
  if (mine != nd) work(mine);
  for (auto& t : th) t.join();
  (void)hipSetDevice(R.devs[0]->device);
  for (size_t d = 0; d < nd; ++d)
    if (rc[d]) return fail(rc[d], err[d]);
  *kernel_ms = *std::max_element(kms.begin(), kms.end());
  *wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

}  // namespace rt
}  // namespace qsmd5
