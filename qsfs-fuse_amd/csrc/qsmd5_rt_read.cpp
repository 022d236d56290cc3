// qsfs-fuse_amd/csrc/qsmd5_rt_read.cpp -- pull-driven batches (qsmd5_hash_read): a
// file's parts read by the caller in column windows into the library's pinned
// staging and hashed as the windows land (the runtime's units: qsmd5_rt.h).
//
// Why: inside qsfs, DoMultiPartUpload reads each part into
// a pooled transfer buffer (QSTransferManager.cpp:611-623) and the pool holds
// -n buffers (TransferManager.h:74-86), so a batch over pool buffers is at most
// -n parts wide -- 5 at qsfs's default, far below the width at which a GPU
// batch pays (it costs one chain time, ~85 ms per 10 MiB part, whatever its
// width).  Here the library owns the staging and asks for the bytes window by
// window (File::ReadNoLoad, File.cpp:308-375, gathers any byte range of a
// loaded file), and every part of the file is its own chain, parked between
// windows: the batch is as wide as the file, the staging stays bounded.
//
// Schedule on the GPU (the job's read slot: its own streams and buffers, up to
// QSMD5_READ_SLOTS jobs side by side, qsmd5_rt.h ReadSlot; qsmd5_plan.h
// plan_read): step s = (group, column).  The budget is split into R staging
// regions (read_regions below).  The calling thread fills host region s % R
// through the caller's reads and enqueues its H2D copy into device region
// s % R on the copy stream; the column kernel that hashes it goes on the
// kernel stream once the host has seen that copy land (gpu_read).  So the
// reads of window s + 1 run while window s copies and window s - 1 hashes.
// With one reader the reads are the bound: a column kernel of 512 chains x
// 252 KiB runs in ~2 ms, its copy in ~2.5 ms, while one thread gathers the
// 127 MiB window in ~7 ms (the page cache's memset + memcpy, as ReadNoLoad).
#include <array>
#include <deque>
#include <functional>

#include "qsmd5_rt.h"

namespace qsmd5 {
namespace rt {

namespace {

// Threads kept for the length of one call: the window loops hand
// each window's shares to them instead of starting threads per window (a
// 100 GB file at the default staging is ~800 windows).  A crew thread runs
// with its call depth raised, so a read callback that calls back into the
// library on it is a nested call, exactly as on the calling thread: it skips
// the shutdown gate and the shared lock that the outer call already holds
// (an outermost call there could wait at the gate of a shutdown
// that in turn waits for the outer call).
class Crew {
 public:
  explicit Crew(size_t want) {
    for (size_t k = 0; k < want; ++k) {
      try {
        th_.emplace_back([this, k] { loop(k); });
      } catch (...) {
        break;  // fewer helpers: wait() runs the other shares on the caller
      }
    }
  }
  ~Crew() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    go_.notify_all();
    for (auto& t : th_) t.join();
  }
  Crew(const Crew&) = delete;
  Crew& operator=(const Crew&) = delete;
  // Shares [0, T) of f: share t runs on helper t if there is one.  Every
  // start() is followed by wait() before the next.
  void start(std::function<void(size_t)> f, size_t T) {
    std::lock_guard<std::mutex> lk(mu_);
    f_ = std::move(f);
    T_ = T;
    pending_ = std::min(T, th_.size());
    ++gen_;
    go_.notify_all();
  }
  // Runs the shares no helper took, then waits for the helpers' shares.
  void wait() {
    for (size_t t = th_.size(); t < T_; ++t) f_(t);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
    T_ = 0;
  }

 private:
  void loop(size_t k) {
    ++t_call_depth;  // this thread's calls into the library are nested calls
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      go_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      if (k >= T_) continue;
      lk.unlock();
      f_(k);  // f_ is replaced only after wait() saw this share done
      lk.lock();
      if (--pending_ == 0) done_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable go_, done_;
  std::vector<std::thread> th_;
  std::function<void(size_t)> f_;
  size_t T_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct ReadJob {
  qsmd5_read_fn read;
  void* user;
  std::vector<uint64_t> len;     // hashed length of each chunk (REF_TRUNCATE32 applied)
  std::vector<uint32_t> order;   // lane -> chunk, longest first (ties by index)
  std::vector<uint64_t> sorted;  // len[order[k]]
  uint64_t total = 0;
  bool short_read = false;       // the caller's read came back short: not a GPU failure
  bool nested = false;           // called from inside another qsmd5 call (a read callback)
  double read_s = 0;             // time in the caller's reads
  // The read-rate samples (routing, below): windows read while no CPU worker
  // hashed ("clean": every window of a GPU job, the first of a CPU job) and
  // windows read while the CPU workers hashed the one before ("busy").
  double clean_read_s = 0, busy_read_s = 0;
  uint64_t clean_bytes = 0, busy_bytes = 0;
  size_t readers = 1;            // threads calling read at once (QSMD5_FLAG_READ_PARALLEL)
  std::unique_ptr<Crew> reader_crew;  // readers - 1 helpers, made with the job
  // Where a call's time goes (QSMD5_TRACE=1 prints it):
  // waiting for a read slot, reserving buffers and sending the descriptors,
  // waiting for a staging region (its last copy, or its last kernel), and
  // from the last window's copy to the digests on the host.
  double slot_s = 0, setup_s = 0, region_wait_s = 0, tail_s = 0;
  double kernel_wait_s = 0;  // the part of region_wait_s spent on a device region's last kernel
};

// The window of column j of group g for its `active` live lanes, lane k at
// dst + k * stride.  A count other than asked fails the job (-EIO), as a short
// ReadNoLoad stops the reference's upload (QSTransferManager.cpp:625-643).
// With QSMD5_FLAG_READ_PARALLEL the window's rows are read by J.readers
// threads at once (row k on thread k % readers: this one and the job's reader
// crew); the first short read stops them all and is reported from this thread
// (fail() keeps its message per thread).
int fill_window(ReadJob& J, const ReadGroup& g, uint32_t j, size_t active, uint8_t* dst,
                uint64_t* bytes = nullptr) {
  const uint64_t off = (uint64_t)j * g.W;
  if (bytes) {
    *bytes = 0;
    for (size_t k = 0; k < active; ++k) *bytes += ReadPlan::col_bytes(g, J.len[J.order[g.first + k]], j);
  }
  struct Short {
    std::atomic<bool> hit{false};
    std::mutex mu;
    uint32_t c = 0;
    uint64_t got = 0, want = 0;
  } bad;
  auto rows = [&](size_t first, size_t step) noexcept {
    for (size_t k = first; k < active && !bad.hit.load(std::memory_order_relaxed); k += step) {
      const uint32_t c = J.order[g.first + k];
      const uint64_t w = ReadPlan::col_bytes(g, J.len[c], j);
      if (!w) continue;
      const uint64_t got = J.read(J.user, c, off, w, dst + k * g.stride);
      if (got != w) {
        std::lock_guard<std::mutex> lk(bad.mu);
        if (!bad.hit.load()) {
          bad.c = c;
          bad.got = got;
          bad.want = w;
          bad.hit.store(true);
        }
        return;
      }
    }
  };
  const size_t T = J.reader_crew ? std::min(J.readers, std::max<size_t>(active, 1)) : 1;
  if (T > 1) {
    J.reader_crew->start([&](size_t t) { rows(t + 1, T); }, T - 1);
    rows(0, T);
    J.reader_crew->wait();
  } else {
    rows(0, 1);
  }
  if (bad.hit.load()) {
    J.short_read = true;
    return fail(-EIO, "qsmd5_hash_read: short read of chunk " + std::to_string(bad.c) + " at offset " +
                          std::to_string(off) + ": " + std::to_string(bad.got) + " of " +
                          std::to_string(bad.want) + " bytes");
  }
  return 0;
}

// Wait for `ev` without holding a core: poll, sleeping 20 us backing off to 500 us.
int poll_event(hipEvent_t ev, const char* what) {
  int idle_us = 20;
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return hip_fail(q, what);
    std::this_thread::sleep_for(std::chrono::microseconds(idle_us));
    idle_us = std::min(500, idle_us * 2);
  }
}

// A read slot for this job (qsmd5_rt.h ReadSlot) and the bound GPU it is on.
// With several GPUs bound (QSMD5_DEVICES), the job goes to the one with the
// fewest jobs in flight for its slots (the first on a tie), so files flushed
// at once spread over the node's GPUs and one file at a time stays on the
// primary.  The GPU and slot are taken together under that GPU's lock, so two
// jobs starting at once never both pick a GPU whose last slot only one of
// them can have; when every slot is busy, the job waits on the least-loaded
// GPU -- unless it may not wait (a nested call, made from a read callback of
// a job that holds a slot itself: ADVICE r05), which then gets no slot (r
// stays null).  The slot's streams and events are made on first use.
struct SlotLease {
  Dev* r = nullptr;
  int k = -1;
  size_t index = 0;  // the GPU's place in rt().devs
  explicit SlotLease(bool may_wait) {
    Runtime& R = rt();
    const size_t n = R.devs.size();
    std::vector<std::pair<double, size_t>> by_load(n);
    for (size_t i = 0; i < n; ++i) {
      Dev* d = R.devs[i];
      std::lock_guard<std::mutex> lk(d->read_mu);
      by_load[i] = {(double)__builtin_popcount(d->read_busy) / (double)std::max(1, d->nread_slots), i};
    }
    std::stable_sort(by_load.begin(), by_load.end(),
                     [](const std::pair<double, size_t>& x, const std::pair<double, size_t>& y) {
                       return x.first < y.first;
                     });
    for (const auto& c : by_load)
      if (take(*R.devs[c.second], c.second, false)) return;
    if (may_wait) take(*R.devs[by_load[0].second], by_load[0].second, true);
  }
  // A free slot of d (waiting for one if `wait`); false if none was free.
  bool take(Dev& d, size_t i, bool wait) {
    std::unique_lock<std::mutex> lk(d.read_mu);
    auto free_slot = [&] {
      for (int s = 0; s < d.nread_slots; ++s)
        if (!(d.read_busy & (1u << s))) {
          k = s;
          return true;
        }
      return false;
    };
    if (wait) d.read_cv.wait(lk, free_slot);
    else if (!free_slot()) return false;
    d.read_busy |= 1u << k;
    r = &d;
    index = i;
    return true;
  }
  ~SlotLease() {
    if (!r) return;
    {
      std::lock_guard<std::mutex> lk(r->read_mu);
      r->read_busy &= ~(1u << k);
    }
    r->read_cv.notify_one();
  }
  SlotLease(const SlotLease&) = delete;
  SlotLease& operator=(const SlotLease&) = delete;
  // The slot on its GPU (made current: the streams and buffers live there).
  int ready(ReadSlot** out) {
    hipError_t e = hipSetDevice(r->device);  // guarded() restores the caller's device
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    if (rt().devs.size() > 1 && env_u64("QSMD5_TRACE", 0))  // diagnostics (tests/test_gpu_multi.py)
      fprintf(stderr, "qsmd5 read: job on context %zu (GPU %d)\n", index, r->device);
    ReadSlot& rs = r->read_slot[k];
    for (hipStream_t* s : {&rs.stream, &rs.copy})
      if (!*s && (e = hipStreamCreateWithFlags(s, hipStreamNonBlocking)) != hipSuccess) {
        *s = nullptr;
        return hip_fail(e, "hipStreamCreate");
      }
    for (hipEvent_t* ev : rs.events())
      if (!*ev && (e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) {
        *ev = nullptr;
        return hip_fail(e, "hipEventCreate");
      }
    *out = &rs;
    return 0;
  }
};

// Staging regions per job on the GPU path (QSMD5_READ_REGIONS, 2..4): the
// budget is split into that many host regions (and as many device regions
// with the overlap), so a window is budget / regions wide and up to
// regions - 1 windows are in flight behind the one being read.  By default 2
// for a job read on one thread and 4 for one read by parallel readers: on the
// MI355X box (profiles/r06_flush_sweep_tree.jsonl, 512 x 10 MiB) 4 readers
// ran at 48 GiB/s with 4 regions, steadily, against 46 at best and 34-42
// often with 2, while one reader ran at 21 GiB/s with 2 regions and 13-17
// with 4 (narrower windows of page-cache gathers).  Either way the budget's
// bytes are the same, so read slot 0's pre-allocation fits both.
int read_regions(size_t readers) {
  const uint64_t dflt = readers > 1 ? 4 : 2;
  return (int)std::min<uint64_t>(kMaxReadRegions, std::max<uint64_t>(2, env_u64("QSMD5_READ_REGIONS", dflt)));
}

// Metadata bytes of a job of n chunks over `dregions` device regions: one
// descriptor set per region, then the lane orders.
size_t read_desc_span(size_t n) { return (n * sizeof(qsmd5_chunk) + 255) & ~size_t(255); }
size_t read_meta_bytes(size_t n, int dregions) { return dregions * read_desc_span(n) + n * sizeof(uint32_t); }

// 1 = complete, 0 = pending, < 0 = a HIP failure (t_last_error set).
int event_state(hipEvent_t ev, const char* what) {
  const hipError_t q = hipEventQuery(ev);
  if (q == hipSuccess) return 1;
  if (q == hipErrorNotReady) return 0;
  return hip_fail(q, what);
}

// The GPU backend of a pull-driven batch.  Step s = (group, column) of the
// plan: the calling thread fills host region s % R through the caller's
// reads, then enqueues its H2D copy on the slot's copy stream into device
// region s % R; the column kernel that hashes it goes on the slot's kernel
// stream once the host has seen that copy land (the kernels of a group run in
// column order on that one stream: each resumes the chains the last one
// parked).  The order between the two streams is kept by this thread, not by
// hipStreamWaitEvent (which keeps a HIP thread polling for the whole batch:
// DESIGN.md §5, "Host CPU of a GPU wave"), as run_batch does:
//   - host region s % R is refilled once the copy that last read it (step
//     s - R) has landed;
//   - device region s % R is overwritten once the kernel that last read it
//     (step s - R) has finished;
//   - kernel s is launched at the first check after copy s has landed (before
//     and after each window's reads, and right after a host region's wait).
// So the copy of window s and the kernel of window s - 1 run while the caller
// reads window s + 1 (with one stream, copy s + 1 queued
// behind kernel s, ~27 GiB/s of copy + kernel, once parallel readers outran
// it).  QSMD5_READ_OVERLAP=0 keeps the round-5 order: copy and kernel on one
// stream into one device region.
int gpu_read(ReadJob& J, uint64_t staging, uint8_t (*digests)[16]) {
  using clock = std::chrono::steady_clock;
  auto secs = [](clock::time_point a, clock::time_point b) { return std::chrono::duration<double>(b - a).count(); };
  const auto t_lease = clock::now();
  SlotLease lease(!J.nested);
  if (!lease.r)
    return fail(-EDEADLK, "qsmd5_hash_read: a nested call (from a read callback) found no free read slot "
                          "under QSMD5_FLAG_GPU_ONLY; every slot is held by calls waiting on their reads");
  J.slot_s = secs(t_lease, clock::now());
  const auto t_setup = clock::now();
  ReadSlot* slot = nullptr;
  if (int rc = lease.ready(&slot)) return rc;
  ReadSlot& rs = *slot;
  const bool overlap = env_u64("QSMD5_READ_OVERLAP", 1) != 0;
  const int R = read_regions(J.readers);
  const int dregions = overlap ? R : 1;
  const size_t n = J.len.size();
  const ReadPlan P = plan_read(J.sorted, 2 * staging / R);  // regions of staging / R
  uint64_t region = 0;
  for (const ReadGroup& g : P.groups) region = std::max<uint64_t>(region, g.count * g.stride);
  // metadata: one descriptor set per device region, then the lane orders
  const size_t desc_span = read_desc_span(n);
  const size_t meta_bytes = read_meta_bytes(n, dregions);
  if (int rc = rs.h_read.reserve(R * region)) return rc;
  if (int rc = rs.d_read.reserve(dregions * region)) return rc;
  if (int rc = rs.h_meta.reserve(std::max<size_t>(meta_bytes, 16 * n))) return rc;
  if (int rc = rs.d_meta.reserve(meta_bytes)) return rc;
  if (int rc = rs.d_state.reserve(16 * n)) return rc;
  if (int rc = rs.d_dig.reserve(16 * n)) return rc;
  uint8_t* hm = static_cast<uint8_t*>(rs.h_meta.p);
  uint8_t* dm = static_cast<uint8_t*>(rs.d_meta.p);
  uint8_t* dstage = static_cast<uint8_t*>(rs.d_read.p);
  // Lane k of group g reads its window from row k of the device region; the
  // descriptor carries the chunk's whole length (the column kernel's segment
  // form: it finishes the chain in the column that holds the chunk's end).
  uint32_t* ho = reinterpret_cast<uint32_t*>(hm + dregions * desc_span);
  for (int d = 0; d < dregions; ++d) {
    qsmd5_chunk* hd = reinterpret_cast<qsmd5_chunk*>(hm + d * desc_span);
    for (const ReadGroup& g : P.groups)
      for (size_t k = 0; k < g.count; ++k) {
        const uint32_t c = J.order[g.first + k];
        hd[g.first + k] = qsmd5_chunk{dstage + d * region + k * g.stride, J.len[c]};
        ho[g.first + k] = c;
      }
  }
  const hipStream_t ks = rs.stream, cs = overlap ? rs.copy : rs.stream;
  // After a failure, let everything enqueued finish before returning: a copy
  // may still be reading a host region the next call refills.
  auto drain = [&](int rc) {
    (void)hipStreamSynchronize(cs);
    (void)hipStreamSynchronize(ks);
    return rc;
  };
  auto hip = [&](hipError_t e, const char* what) { return e == hipSuccess ? 0 : hip_fail(e, what); };
  if (int rc = hip(hipMemcpyAsync(dm, hm, meta_bytes, hipMemcpyHostToDevice, ks), "hipMemcpyAsync H2D"))
    return drain(rc);
  const uint32_t* d_ord = reinterpret_cast<const uint32_t*>(dm + dregions * desc_span);
  uint32_t* d_dig = static_cast<uint32_t*>(rs.d_dig.p);
  uint32_t* d_state = static_cast<uint32_t*>(rs.d_state.p);
  uint8_t* hstage = static_cast<uint8_t*>(rs.h_read.p);
  J.setup_s = secs(t_setup, clock::now());
  // Windows whose copies are enqueued and whose kernels are not (overlap), in step order.
  struct Pending {
    const ReadGroup* g;
    uint32_t j;
    size_t act;
    int reg;
  };
  std::deque<Pending> pend;
  auto launch_kernel = [&](const Pending& p) -> int {
    const qsmd5_chunk* d_desc = reinterpret_cast<const qsmd5_chunk*>(dm + (overlap ? p.reg : 0) * desc_span);
    if (int rc = hip(qsmd5::launch_column(d_desc + p.g->first, d_ord + p.g->first, (uint32_t)p.act, d_dig,
                                          (uint64_t)p.j * p.g->W, p.g->W, d_state, ks),
                     "qsmd5 column kernel launch"))
      return rc;
    return overlap ? hip(hipEventRecord(rs.hashed[p.reg], ks), "hipEventRecord") : 0;
  };
  // Launch the pending kernels whose copies have landed, in order; with
  // `until` >= 0, wait (sleeping) until the one of step `until` is launched.
  auto advance = [&](long long until, size_t first_step) -> int {
    int idle_us = 20;
    size_t s = first_step;
    while (!pend.empty()) {
      const int q = event_state(rs.copied[pend.front().reg], "qsmd5_hash_read: staging copy");
      if (q < 0) return q;
      if (q == 0) {
        if (until < (long long)s) return 0;
        std::this_thread::sleep_for(std::chrono::microseconds(idle_us));
        idle_us = std::min(500, idle_us * 2);
        continue;
      }
      if (int rc = launch_kernel(pend.front())) return rc;
      pend.pop_front();
      ++s;
    }
    return 0;
  };
  auto timed_poll = [&](hipEvent_t ev, const char* what, double* also = nullptr) {
    const auto w0 = clock::now();
    const int rc = poll_event(ev, what);
    const double w = secs(w0, clock::now());
    J.region_wait_s += w;
    if (also) *also += w;
    return rc;
  };
  size_t step = 0, launched = 0;  // launched: steps whose kernels are enqueued
  for (const ReadGroup& g : P.groups)
    for (uint32_t j = 0; j < g.ncols; ++j, ++step) {
      const int reg = (int)(step % R);
      uint8_t* host = hstage + reg * region;
      if (overlap) {
        const size_t before = pend.size();
        if (int rc = advance(-1, launched)) return drain(rc);
        launched += before - pend.size();
      }
      if (step >= (size_t)R) {  // the copy that last read this host region (step - R) has landed
        if (int rc = timed_poll(rs.copied[reg], "qsmd5_hash_read: staging copy")) return drain(rc);
        if (overlap) {  // ... so its kernel goes now, and runs while this window is read
          const size_t before = pend.size();
          if (int rc = advance(-1, launched)) return drain(rc);
          launched += before - pend.size();
        }
      }
      const size_t act = ReadPlan::active(J.sorted, g, j);
      const auto r0 = clock::now();
      uint64_t wbytes = 0;
      const int frc = fill_window(J, g, j, act, host, &wbytes);
      const double rs_s = secs(r0, clock::now());
      J.read_s += rs_s;
      J.clean_read_s += rs_s;
      J.clean_bytes += wbytes;
      if (frc) return drain(frc);
      if (overlap) {
        // device region `reg` is free once the kernel of step - R has run:
        // launch it first if it is still pending (its copy has landed: see above)
        const size_t before = pend.size();
        if (int rc = advance(step >= (size_t)R ? (long long)(step - R) : -1, launched)) return drain(rc);
        launched += before - pend.size();
        if (step >= (size_t)R)
          if (int rc = timed_poll(rs.hashed[reg], "qsmd5_hash_read: column kernel", &J.kernel_wait_s))
            return drain(rc);
      }
      uint8_t* dst = dstage + (overlap ? reg : 0) * region;
      if (int rc = hip(hipMemcpyAsync(dst, host, act * g.stride, hipMemcpyHostToDevice, cs), "hipMemcpyAsync H2D"))
        return drain(rc);
      if (int rc = hip(hipEventRecord(rs.copied[reg], cs), "hipEventRecord")) return drain(rc);
      const Pending p{&g, j, act, reg};
      if (overlap) {
        pend.push_back(p);
      } else {
        if (int rc = launch_kernel(p)) return drain(rc);  // stream order after its copy
        ++launched;
      }
    }
  const auto t_tail = clock::now();
  if (overlap)
    if (int rc = advance((long long)step, launched)) return drain(rc);
  // the metadata's H2D ran first on the kernel stream: its host block is free for the digests
  if (int rc = hip(hipMemcpyAsync(hm, d_dig, 16 * n, hipMemcpyDeviceToHost, ks), "hipMemcpyAsync D2H"))
    return drain(rc);
  if (int rc = hip(hipEventRecord(rs.done, ks), "hipEventRecord")) return drain(rc);
  if (int rc = poll_event(rs.done, "qsmd5_hash_read: waiting for the batch")) return drain(rc);
  memcpy(digests, hm, 16 * n);
  J.tail_s = secs(t_tail, clock::now());
  return 0;
}

// The CPU path's pageable staging, kept between calls (up to
// QSMD5_READ_SLOTS buffers; released by qsmd5_shutdown).  A fresh 256 MiB
// buffer per call page-faulted on its first two windows' reads -- ~40 ms of
// a 128 x 10 MiB pre-hash on the MI355X box's host (profiles/r06_rate_sweep.jsonl:
// the CPU path's reads at 11 GiB/s against the GPU path's 19 into its
// pinned staging) -- and those slow first reads were the "clean" read-rate
// sample routing priced the GPU path with.
struct CpuStagingCache {
  std::mutex mu;
  std::vector<std::pair<size_t, uint8_t*>> free;  // (bytes, buffer)
};
// Constructed when the library loads, not at first use: a function-local
// static's lazy initialisation is published by an inline guard check that a
// ThreadSanitizer build of a caller cannot see inside this (uninstrumented)
// library, which then reports the first two callers' use of the mutex as a
// race (tests/test_multipart_cpu.py, staged flow under TSan).
CpuStagingCache g_cpu_staging_cache;
CpuStagingCache& cpu_staging_cache() { return g_cpu_staging_cache; }

class CpuStaging {
 public:
  explicit CpuStaging(size_t bytes) {
    CpuStagingCache& c = cpu_staging_cache();
    {
      std::lock_guard<std::mutex> lk(c.mu);
      size_t best = c.free.size();
      for (size_t i = 0; i < c.free.size(); ++i)
        if (c.free[i].first >= bytes && (best == c.free.size() || c.free[i].first < c.free[best].first)) best = i;
      if (best < c.free.size()) {
        bytes_ = c.free[best].first;
        p_ = c.free[best].second;
        c.free.erase(c.free.begin() + best);
        return;
      }
    }
    p_ = new (std::nothrow) uint8_t[bytes];
    bytes_ = p_ ? bytes : 0;
    if (p_) memset(p_, 0, bytes);  // fault the pages in here, not inside the timed first reads
  }
  ~CpuStaging() {
    if (!p_) return;
    CpuStagingCache& c = cpu_staging_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    c.free.emplace_back(bytes_, p_);
    const size_t keep = (size_t)std::max<uint64_t>(1, env_u64("QSMD5_READ_SLOTS", 4));
    while (c.free.size() > keep) {  // drop the smallest
      auto it = std::min_element(c.free.begin(), c.free.end());
      delete[] it->second;
      c.free.erase(it);
    }
  }
  CpuStaging(const CpuStaging&) = delete;
  CpuStaging& operator=(const CpuStaging&) = delete;
  uint8_t* get() const { return p_; }

 private:
  uint8_t* p_ = nullptr;
  size_t bytes_ = 0;
};

// Whether the CPU backend runs a window of `act` rows on T threads in the
// AVX-512 lanes (md5_mb16_blocks): as cpu_batch decides, at least 2 rows per
// thread (a lane's chain runs at ~0.6x a scalar chain), QSMD5_CPU_MB=0: never.
bool read_lanes(size_t act, size_t T) {
  return act >= 2 * T && env_u64("QSMD5_CPU_MB", 1) && qsmd5::cpu::mb16_available();
}

// The CPU backend of a pull-driven batch: the same windows, double-buffered
// like the GPU's: the calling thread reads window s + 1 (the caller's reads
// stay on its thread, or its reader threads with QSMD5_FLAG_READ_PARALLEL)
// while worker threads fold window s's rows into their
// chunks' running contexts (md5_cpu.h Ctx) -- 16 rows at a time per thread in
// the AVX-512 lanes where read_lanes says so (the rows' whole blocks continue
// their chunks' states; a final column's last len % 64 bytes go through the
// Ctx), else one row at a time.  *hash_ms: the workers' wall time, for the
// load feedback.
int cpu_read(ReadJob& J, uint64_t staging, uint8_t (*digests)[16], double* hash_ms) {
  using clock = std::chrono::steady_clock;
  const size_t n = J.len.size();
  const ReadPlan P = plan_read(J.sorted, staging);
  uint64_t region = 0;
  for (const ReadGroup& g : P.groups) region = std::max<uint64_t>(region, g.count * g.stride);
  CpuStaging buf(2 * std::max<uint64_t>(region, 1));
  if (!buf.get()) return fail(-ENOMEM, "qsmd5_hash_read: host staging allocation failed");
  std::vector<qsmd5::cpu::Ctx> ctx(n);

  // One window's hashing: rows [0, act) of group g, column j, at `base`.
  struct Window {
    const ReadGroup* g = nullptr;
    uint32_t j = 0;
    size_t act = 0, T = 1;
    bool lanes = false;
    const uint8_t* base = nullptr;
  };
  auto row_scalar = [&](const Window& w, size_t k) {
    const uint32_t c = J.order[w.g->first + k];
    const uint64_t b = ReadPlan::col_bytes(*w.g, J.len[c], w.j);
    if (b) ctx[c].update(w.base + k * w.g->stride, b);
  };
  // lanes: thread t takes rows t, t + T, ... (lengths fall with k, so each
  // thread gets a like share of long and short rows)
  auto rows_lanes = [&](const Window& w, size_t t) {
    std::vector<std::array<uint32_t, 4>> st;
    std::vector<const uint8_t*> ptr;
    std::vector<uint64_t> nb;
    std::vector<size_t> rows;
    for (size_t k = t; k < w.act; k += w.T) {
      const uint32_t c = J.order[w.g->first + k];
      const uint64_t b = ReadPlan::col_bytes(*w.g, J.len[c], w.j);
      if (!b) continue;
      if (ctx[c].tail_len || b < 64) {  // a partial block pending: the Ctx's own path
        ctx[c].update(w.base + k * w.g->stride, b);
        continue;
      }
      st.push_back({ctx[c].h[0], ctx[c].h[1], ctx[c].h[2], ctx[c].h[3]});
      ptr.push_back(w.base + k * w.g->stride);
      nb.push_back(b >> 6);
      rows.push_back(k);
    }
    if (!rows.empty())
      qsmd5::cpu::md5_mb16_blocks(reinterpret_cast<uint32_t(*)[4]>(st.data()), ptr.data(), nb.data(),
                                  rows.size());
    for (size_t r = 0; r < rows.size(); ++r) {
      const size_t k = rows[r];
      const uint32_t c = J.order[w.g->first + k];
      const uint64_t b = ReadPlan::col_bytes(*w.g, J.len[c], w.j);
      for (int q = 0; q < 4; ++q) ctx[c].h[q] = st[r][q];
      ctx[c].total += nb[r] << 6;
      if (b & 63) ctx[c].update(w.base + k * w.g->stride + (nb[r] << 6), b & 63);
    }
  };
  // The window in flight on the workers (a crew kept for the call, made at the
  // first window); finish() waits for them (and runs on this thread any share
  // a worker could not be started for).
  Window cur;
  std::atomic<size_t> next{0};
  // the hashing's own wall time (not the wait for the next window's reads):
  // launch to the last worker's end
  clock::time_point t_start;
  std::atomic<int64_t> t_end_ns{0};
  auto stamp_end = [&] {
    const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(clock::now() - t_start).count();
    int64_t cur_ns = t_end_ns.load();
    while (ns > cur_ns && !t_end_ns.compare_exchange_weak(cur_ns, ns)) {
    }
  };
  auto work = [&](const Window& w, size_t t) noexcept {
    if (w.lanes) rows_lanes(w, t);
    else
      for (size_t k; (k = next.fetch_add(1)) < w.act;) row_scalar(w, k);
    stamp_end();
  };
  std::unique_ptr<Crew> crew;  // declared after everything its threads touch
  auto finish = [&] {
    if (!cur.g) return;
    crew->wait();
    *hash_ms += (double)t_end_ns.load() * 1e-6;
    cur = Window();
  };
  auto launch = [&](const Window& w) {
    if (!crew) crew.reset(new Crew(cpu_threads()));
    cur = w;
    next.store(0);
    t_end_ns.store(0);
    t_start = clock::now();
    crew->start([&](size_t t) { work(cur, t); }, w.T);
  };
  size_t step = 0;
  for (const ReadGroup& g : P.groups)
    for (uint32_t j = 0; j < g.ncols; ++j, ++step) {
      uint8_t* host = buf.get() + (step & 1) * region;
      const size_t act = ReadPlan::active(J.sorted, g, j);
      // this region was last hashed two steps back, and finish() below waited for it
      const auto r0 = clock::now();
      uint64_t wbytes = 0;
      const int rc = fill_window(J, g, j, act, host, &wbytes);
      const double rs_s = std::chrono::duration<double>(clock::now() - r0).count();
      J.read_s += rs_s;
      (cur.g ? J.busy_read_s : J.clean_read_s) += rs_s;  // read while the workers hashed, or alone
      (cur.g ? J.busy_bytes : J.clean_bytes) += wbytes;
      finish();  // window s - 1: its rows are folded, its region is free
      if (rc) return rc;
      Window w;
      w.g = &g;
      w.j = j;
      w.act = act;
      w.T = std::min<size_t>({cpu_threads(), act, (size_t)std::max<uint64_t>(1, act * g.W >> 20)});
      w.lanes = read_lanes(act, w.T);
      w.base = host;
      launch(w);
    }
  finish();
  for (size_t c = 0; c < n; ++c) ctx[c].final(digests[c]);
  return 0;
}

// The caller's read rates (bytes per second of its read callbacks), for
// routing.  Both backends overlap the reads with the hashing, but not alike
// (profiles/r06_flush_sweep.jsonl): on the GPU path the
// host only reads, while on the CPU path the reads share the host with the
// workers hashing the window before -- 128 x 10 MiB from qsfs-like pages read
// at ~19 GiB/s alone and ~12.5 GiB/s beside the hashing on the MI355X box.
// So two rates are kept, each averaged over recent jobs (a new sample weighs
// 1/2; samples of >= 32 MiB): "clean" from windows read with no CPU worker
// running (a GPU job's windows, a CPU job's first) and "busy" from windows
// read beside the workers.  Before a first sample the clean rate is 12 GiB/s
// (one thread's memcpy out of a page cache, as qsfs's ReadNoLoad) and the busy
// rate the clean one; QSMD5_READ_GIBS overrides both.
std::atomic<uint64_t> g_read_clean_bits{0}, g_read_busy_bits{0};

double load_gibs(const std::atomic<uint64_t>& a) {
  const uint64_t bits = a.load(std::memory_order_relaxed);
  if (!bits) return 0;
  double v;
  memcpy(&v, &bits, sizeof(v));
  return v;
}

double read_gibs_clean() {
  const double env = env_gibs("QSMD5_READ_GIBS");
  if (env > 0) return env;
  const double v = load_gibs(g_read_clean_bits);
  return v > 0 ? v : 12.0;
}

double read_gibs_busy() {
  const double env = env_gibs("QSMD5_READ_GIBS");
  if (env > 0) return env;
  const double v = load_gibs(g_read_busy_bits);
  return v > 0 ? v : read_gibs_clean();
}

void fold_rate(std::atomic<uint64_t>& a, uint64_t bytes, double secs) {
  if (bytes < (32ull << 20) || secs <= 0) return;
  const double sample = (double)bytes / secs / kGiB;
  const double old = load_gibs(a);
  const double v = old > 0 ? 0.5 * old + 0.5 * sample : sample;
  uint64_t bits;
  memcpy(&bits, &v, sizeof(bits));
  a.store(bits, std::memory_order_relaxed);
}

void note_read_rate(const ReadJob& J) {
  fold_rate(g_read_clean_bits, J.clean_bytes, J.clean_read_s);
  fold_rate(g_read_busy_bits, J.busy_bytes, J.busy_read_s);
}

// The GPU path's wall time for this job: the reads and the chains overlap,
// window by window, so it is the longer of the two plus what cannot overlap --
// the last window's copy and column kernel after its read.  Chains of one
// group run as long as its longest chunk; groups run one after another.
double gpu_read_est_ms(const ReadJob& J, uint64_t staging, double read_ms) {
  const ReadPlan P = plan_read(J.sorted, 2 * staging / read_regions(J.readers));
  const double chain = gpu_chain_gibs();
  double chain_ms = 0, tail_ms = 0;
  for (const ReadGroup& g : P.groups) {
    chain_ms += 1e3 * (double)J.sorted[g.first] / kGiB / chain;
    tail_ms = 1e3 * ((double)std::min<uint64_t>(g.W, J.sorted[g.first]) / chain +
                     (double)(g.count * g.stride) / link_gibs()) / kGiB;
  }
  return kGpuCallMs + std::max(read_ms, chain_ms) + tail_ms;
}

void log_read(const char* backend, const char* reason, const ReadJob& J) {
  if (!log_wanted(QSMD5_LOG_INFO)) return;
  log_msg(QSMD5_LOG_INFO, "qsmd5: backend=%s reason=%s chunks=%zu bytes=%llu (read)", backend, reason,
          J.len.size(), (unsigned long long)J.total);
}

}  // namespace

void release_read_cache() {
  CpuStagingCache& c = cpu_staging_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  for (auto& b : c.free) delete[] b.second;
  c.free.clear();
}

// do_init (qsmd5_rt_device.cpp) calls this for the primary GPU: read slot 0's
// streams, events and buffers for a job at the default staging budget of up
// to 4096 chunks, made at start-up rather than inside the first pull-driven
// call.  VERDICT r05 item 2: they took 65-80 ms of pinned and device
// allocation in the first GPU job, and under auto routing the first GPU job
// often comes after CPU-routed ones (profiles/r06_flush_sweep.jsonl).
// QSMD5_READ_PREWARM=0 skips it; a failure here is not an init failure (the
// first job then allocates what it needs, as before).
void prewarm_read_slot(Dev& d) {
  if (!env_u64("QSMD5_READ_PREWARM", 1)) return;
  ReadSlot& rs = d.read_slot[0];
  hipError_t e = hipSuccess;
  for (hipStream_t* s : {&rs.stream, &rs.copy})
    if (!*s && (e = hipStreamCreateWithFlags(s, hipStreamNonBlocking)) != hipSuccess) *s = nullptr;
  for (hipEvent_t* ev : rs.events())
    if (!*ev && (e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) *ev = nullptr;
  const uint64_t staging = env_u64("QSMD5_READ_STAGING_BYTES", kDefaultReadStaging);
  const int R = read_regions(1);
  const uint64_t region = std::max<uint64_t>(staging / R, stage_bytes(kReadColMin));  // gpu_read's plan
  const int dregions = env_u64("QSMD5_READ_OVERLAP", 1) ? R : 1;
  constexpr size_t n = 4096;
  const size_t meta = read_meta_bytes(n, dregions);
  const bool ok = e == hipSuccess && rs.h_read.reserve(R * region) == 0 &&
                  rs.d_read.reserve(dregions * region) == 0 && rs.h_meta.reserve(std::max<size_t>(meta, 16 * n)) == 0 &&
                  rs.d_meta.reserve(meta) == 0 && rs.d_state.reserve(16 * n) == 0 && rs.d_dig.reserve(16 * n) == 0;
  if (!ok) {
    (void)hipGetLastError();
    log_msg(QSMD5_LOG_INFO, "qsmd5: read slot not pre-allocated (%s); the first pull-driven job allocates it",
            t_last_error.c_str());
  }
}

int hash_read_routed(const uint64_t* lens, size_t n, qsmd5_read_fn read, void* user,
                     uint64_t staging_bytes, uint8_t (*digests)[16], int flags) {
  using clock = std::chrono::steady_clock;
  const auto t_entry = clock::now();
  if (n == 0) return 0;
  if (!lens || !read || !digests) return fail(-EINVAL, "qsmd5_hash_read: NULL lens/read/digests");
  if (n > 0xffffffffull) return fail(-EINVAL, "qsmd5: too many chunks");
  Backend b = kAuto;
  if (int rc = requested_backend(flags, &b)) return rc;
  ReadJob J;
  J.read = read;
  J.user = user;
  // Called from a read callback of another qsmd5 call (on its thread or a
  // reader-crew thread: both run at depth >= 1 before this call's own scope).
  J.nested = t_call_depth > 1;
  if (flags & QSMD5_FLAG_READ_PARALLEL)
    J.readers = (size_t)std::min<uint64_t>(16, std::max<uint64_t>(1, env_u64("QSMD5_READ_THREADS", 4)));
  J.len.resize(n);
  uint64_t longest = 0;
  for (size_t i = 0; i < n; ++i) {
    uint64_t L = lens[i];
    if (flags & QSMD5_FLAG_REF_TRUNCATE32) L &= 0xffffffffull;
    if (L >= kMaxChunkLen) return fail(-EINVAL, "qsmd5: chunk longer than 2^38 bytes");
    J.len[i] = L;
    J.total += L;
    longest = std::max(longest, L);
  }
  J.order.resize(n);
  std::iota(J.order.begin(), J.order.end(), 0u);
  std::stable_sort(J.order.begin(), J.order.end(),
                   [&](uint32_t a, uint32_t c) { return J.len[a] > J.len[c]; });
  J.sorted.resize(n);
  for (size_t k = 0; k < n; ++k) J.sorted[k] = J.len[J.order[k]];
  if (J.readers > 1 && n > 1) J.reader_crew.reset(new Crew(J.readers - 1));
  const uint64_t staging = staging_bytes ? staging_bytes
                                         : env_u64("QSMD5_READ_STAGING_BYTES", kDefaultReadStaging);
  // QSMD5_TRACE=1: one line per call on stderr with where its time went.
  const char* reason = "";
  double init_s = 0, cpu_hash_ms = 0;
  clock::time_point t_backend = t_entry;
  struct Trace {
    const ReadJob& J;
    const char*& reason;
    double& init_s;
    double& cpu_hash_ms;
    clock::time_point& t_backend;
    clock::time_point t_entry;
    ~Trace() {
      if (!env_u64("QSMD5_TRACE", 0)) return;
      const auto now = clock::now();
      auto ms = [](clock::time_point a, clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
      };
      fprintf(stderr, "qsmd5 read trace: {\"backend\": \"%s\", \"reason\": \"%s\", \"chunks\": %zu, "
              "\"bytes\": %llu, \"readers\": %zu, \"nested\": %d, \"route_ms\": %.3f, \"init_ms\": %.3f, "
              "\"slot_ms\": %.3f, \"setup_ms\": %.3f, \"read_ms\": %.3f, \"region_wait_ms\": %.3f, "
              "\"kernel_wait_ms\": %.3f, \"tail_ms\": %.3f, \"cpu_hash_ms\": %.3f, \"total_ms\": %.3f}\n",
              t_last_backend == QSMD5_BACKEND_GPU ? "gpu" : "cpu", reason, J.len.size(),
              (unsigned long long)J.total, J.readers, J.nested ? 1 : 0, ms(t_entry, t_backend),
              1e3 * init_s, 1e3 * J.slot_s, 1e3 * J.setup_s, 1e3 * J.read_s, 1e3 * J.region_wait_s,
              1e3 * J.kernel_wait_s, 1e3 * J.tail_s, cpu_hash_ms, ms(t_entry, now));
    }
  } trace{J, reason, init_s, cpu_hash_ms, t_backend, t_entry};
  // idle-host CPU time of this batch: 16 lanes per thread where cpu_read will
  // use them and they are priced, else scalar chains
  auto cpu_read_model_ms = [&]() {
    const double lanes = read_lanes_model_ms(longest, J.total, n);
    return lanes >= 0 ? lanes : cpu_model_ms(longest, J.total);
  };
  auto on_cpu = [&](const char* why) {
    reason = why;
    t_backend = clock::now();
    log_read("cpu", why, J);
    double hash_ms = 0;
    const int rc = cpu_read(J, staging, digests, &hash_ms);
    cpu_hash_ms += hash_ms;
    if (rc == 0) {
      t_last_backend = QSMD5_BACKEND_CPU;
      g_cpu_batches.fetch_add(1);
      g_cpu_chunks.fetch_add(n);
      note_cpu_batch(cpu_read_model_ms(), hash_ms);  // as cpu_read runs them
      note_read_rate(J);
    }
    return rc;
  };
  if (b == kCpu) return on_cpu("forced");
  const bool background = b == kAuto && (flags & QSMD5_FLAG_BACKGROUND) && qsmd5_device_count() > 0;
  if (b == kAuto && g_gpu_lost.load()) return on_cpu("gpu-lost");
  // A nested call: the outer call holds a read slot through its
  // read callbacks, so under auto routing a nested batch takes the CPU path,
  // which needs no slot; forced onto the GPU it takes a slot only if one is
  // free (gpu_read: -EDEADLK otherwise).
  if (b == kAuto && J.nested) return on_cpu("nested");
  if (b == kAuto && !background) {
    // Wall time on each backend (reads and hashing overlap on both, at the
    // read rate each backend's reads get); the GPU also when it is within 5%
    // of the CPU: its hashing leaves the host's cores to the daemon.
    const double gib = (double)J.total / kGiB;
    const double cpu_ms = std::max(1e3 * gib / read_gibs_busy(), cpu_read_model_ms() / cpu_efficiency());
    const double gpu_ms = gpu_read_est_ms(J, staging, 1e3 * gib / read_gibs_clean());
    if (cpu_ms * 1.05 < gpu_ms) return on_cpu("size");
  }
  reason = b == kGpu ? "forced" : background ? "background" : "size";
  log_read("gpu", reason, J);
  const auto t_init = clock::now();
  int rc = ensure_init();
  t_backend = clock::now();
  init_s = std::chrono::duration<double>(t_backend - t_init).count();
  bool sticky = false;
  if (rc == 0) {
    const char* inj = getenv("QSMD5_INJECT_GPU_FAULT");
    if (inj && *inj && strcmp(inj, "0")) {
      sticky = !strcmp(inj, "sticky");
      rc = fail(-EIO, "qsmd5: injected GPU fault (QSMD5_INJECT_GPU_FAULT)");
    } else {
      rc = gpu_read(J, staging, digests);
    }
  }
  if (rc == 0) {
    t_last_backend = QSMD5_BACKEND_GPU;
    g_gpu_batches.fetch_add(1);
    g_gpu_chunks.fetch_add(n);
    note_read_rate(J);
    return 0;
  }
  // Forced GPU: no fallback.  A short read or -EINVAL is the caller's, not the GPU's,
  // and so is a nested call that found no slot.
  if (b == kGpu || rc == -EINVAL || rc == -EDEADLK || J.short_read) return rc;
  note_gpu_failure(rc, sticky);
  const std::string gpu_err = t_last_error;
  if (rc != -ENODEV)
    log_msg(QSMD5_LOG_WARN, "qsmd5: GPU read batch of %zu chunks failed (%s); re-reading and hashing "
            "it on the CPU", n, gpu_err.c_str());
  J.short_read = false;
  J.read_s = J.clean_read_s = J.busy_read_s = 0;  // the CPU run's own reads only
  J.clean_bytes = J.busy_bytes = 0;
  const int rc2 = on_cpu("fallback");
  if (rc2) return fail(rc2, t_last_error + " (after GPU failure: " + gpu_err + ")");
  g_fallbacks.fetch_add(1);
  return 0;
}

}  // namespace rt
}  // namespace qsmd5
