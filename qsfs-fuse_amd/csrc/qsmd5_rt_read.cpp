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
// Schedule on the GPU (the job's read slot: its own stream and buffers, up to
// QSMD5_READ_SLOTS jobs side by side, qsmd5_rt.h ReadSlot; qsmd5_plan.h
// plan_read): step s = (group,
// column).  The calling thread fills host region s % 2 through the caller's
// reads, then enqueues its H2D copy into the one device region and the column
// kernel that hashes it.  Stream order keeps the device region safe (copy s+1
// runs after kernel s); the host waits only before refilling a host region, for
// the copy that last read it (two steps back), so the reads of step s+1 run
// while step s copies and hashes.  The reads are the bound: a column kernel of
// 512 chains x 508 KiB runs in ~4 ms, the copy in ~5 ms, while one thread
// gathers the 254 MiB in ~20 ms (the page cache's memcpy).
#include <array>

#include "qsmd5_rt.h"

namespace qsmd5 {
namespace rt {

namespace {

struct ReadJob {
  qsmd5_read_fn read;
  void* user;
  std::vector<uint64_t> len;     // hashed length of each chunk (REF_TRUNCATE32 applied)
  std::vector<uint32_t> order;   // lane -> chunk, longest first (ties by index)
  std::vector<uint64_t> sorted;  // len[order[k]]
  uint64_t total = 0;
  bool short_read = false;       // the caller's read came back short: not a GPU failure
  double read_s = 0;             // time in the caller's reads (the read-rate estimate)
  size_t readers = 1;            // threads calling read at once (QSMD5_FLAG_READ_PARALLEL)
};

// The window of column j of group g for its `active` live lanes, lane k at
// dst + k * stride.  A count other than asked fails the job (-EIO), as a short
// ReadNoLoad stops the reference's upload (QSTransferManager.cpp:625-643).
// With QSMD5_FLAG_READ_PARALLEL the window's rows are read by J.readers
// threads at once (row k on thread k % readers); the first short read stops
// them all and is reported from this thread (fail() keeps its message per
// thread).
int fill_window(ReadJob& J, const ReadGroup& g, uint32_t j, size_t active, uint8_t* dst) {
  const uint64_t off = (uint64_t)j * g.W;
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
  const size_t T = std::min(J.readers, std::max<size_t>(active, 1));
  std::vector<std::thread> th;
  for (size_t t = 1; t < T; ++t) {
    try {
      th.emplace_back(rows, t, T);
    } catch (...) {  // no thread: this one reads that share too
      rows(t, T);
    }
  }
  rows(0, T);
  for (auto& t : th) t.join();
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
// GPU.  The slot's stream and events are made on first use.
struct SlotLease {
  Dev* r = nullptr;
  int k = -1;
  size_t index = 0;  // the GPU's place in rt().devs
  SlotLease() {
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
    take(*R.devs[by_load[0].second], by_load[0].second, true);
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
    {
      std::lock_guard<std::mutex> lk(r->read_mu);
      r->read_busy &= ~(1u << k);
    }
    r->read_cv.notify_one();
  }
  SlotLease(const SlotLease&) = delete;
  SlotLease& operator=(const SlotLease&) = delete;
  // The slot on its GPU (made current: the stream and buffers live there).
  int ready(ReadSlot** out) {
    hipError_t e = hipSetDevice(r->device);  // guarded() restores the caller's device
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    if (rt().devs.size() > 1 && env_u64("QSMD5_TRACE", 0))  // diagnostics (tests/test_gpu_multi.py)
      fprintf(stderr, "qsmd5 read: job on context %zu (GPU %d)\n", index, r->device);
    ReadSlot& rs = r->read_slot[k];
    if (!rs.stream && (e = hipStreamCreateWithFlags(&rs.stream, hipStreamNonBlocking)) != hipSuccess) {
      rs.stream = nullptr;
      return hip_fail(e, "hipStreamCreate");
    }
    for (hipEvent_t* ev : {&rs.copied[0], &rs.copied[1], &rs.done})
      if (!*ev && (e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) {
        *ev = nullptr;
        return hip_fail(e, "hipEventCreate");
      }
    *out = &rs;
    return 0;
  }
};

int gpu_read(ReadJob& J, uint64_t staging, uint8_t (*digests)[16]) {
  SlotLease lease;
  ReadSlot* slot = nullptr;
  if (int rc = lease.ready(&slot)) return rc;
  ReadSlot& rs = *slot;
  const size_t n = J.len.size();
  const ReadPlan P = plan_read(J.sorted, staging);
  uint64_t region = 0;
  for (const ReadGroup& g : P.groups) region = std::max<uint64_t>(region, g.count * g.stride);
  const size_t desc_span = (n * sizeof(qsmd5_chunk) + 255) & ~size_t(255);
  const size_t meta_bytes = desc_span + n * sizeof(uint32_t);
  if (int rc = rs.h_read.reserve(2 * region)) return rc;
  if (int rc = rs.d_read.reserve(region)) return rc;
  if (int rc = rs.h_meta.reserve(std::max<size_t>(meta_bytes, 16 * n))) return rc;
  if (int rc = rs.d_meta.reserve(meta_bytes)) return rc;
  if (int rc = rs.d_state.reserve(16 * n)) return rc;
  if (int rc = rs.d_dig.reserve(16 * n)) return rc;
  uint8_t* hm = static_cast<uint8_t*>(rs.h_meta.p);
  uint8_t* dm = static_cast<uint8_t*>(rs.d_meta.p);
  uint8_t* dstage = static_cast<uint8_t*>(rs.d_read.p);
  // Lane k of group g reads its window from the device region's row k; the
  // descriptor carries the chunk's whole length (the column kernel's segment
  // form: it finishes the chain in the column that holds the chunk's end).
  qsmd5_chunk* hd = reinterpret_cast<qsmd5_chunk*>(hm);
  uint32_t* ho = reinterpret_cast<uint32_t*>(hm + desc_span);
  for (const ReadGroup& g : P.groups)
    for (size_t k = 0; k < g.count; ++k) {
      const uint32_t c = J.order[g.first + k];
      hd[g.first + k] = qsmd5_chunk{dstage + k * g.stride, J.len[c]};
      ho[g.first + k] = c;
    }
  const hipStream_t s = rs.stream;
  // After a failure, let everything enqueued finish before returning: a copy
  // may still be reading a host region the next call refills.
  auto drain = [&](int rc) {
    (void)hipStreamSynchronize(s);
    return rc;
  };
  auto hip = [&](hipError_t e, const char* what) { return e == hipSuccess ? 0 : hip_fail(e, what); };
  if (int rc = hip(hipMemcpyAsync(dm, hm, meta_bytes, hipMemcpyHostToDevice, s), "hipMemcpyAsync H2D"))
    return drain(rc);
  const qsmd5_chunk* d_desc = reinterpret_cast<const qsmd5_chunk*>(dm);
  const uint32_t* d_ord = reinterpret_cast<const uint32_t*>(dm + desc_span);
  uint32_t* d_dig = static_cast<uint32_t*>(rs.d_dig.p);
  uint32_t* d_state = static_cast<uint32_t*>(rs.d_state.p);
  uint8_t* hstage = static_cast<uint8_t*>(rs.h_read.p);
  size_t step = 0;
  for (const ReadGroup& g : P.groups)
    for (uint32_t j = 0; j < g.ncols; ++j, ++step) {
      const int reg = (int)(step & 1);
      uint8_t* host = hstage + reg * region;
      if (step >= 2)  // the copy that last read this region (step - 2) has finished
        if (int rc = poll_event(rs.copied[reg], "qsmd5_hash_read: staging copy")) return drain(rc);
      const size_t act = ReadPlan::active(J.sorted, g, j);
      const auto r0 = std::chrono::steady_clock::now();
      const int frc = fill_window(J, g, j, act, host);
      J.read_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - r0).count();
      if (frc) return drain(frc);
      if (int rc = hip(hipMemcpyAsync(dstage, host, act * g.stride, hipMemcpyHostToDevice, s),
                       "hipMemcpyAsync H2D"))
        return drain(rc);
      if (int rc = hip(hipEventRecord(rs.copied[reg], s), "hipEventRecord")) return drain(rc);
      if (int rc = hip(qsmd5::launch_column(d_desc + g.first, d_ord + g.first, (uint32_t)act, d_dig,
                                            (uint64_t)j * g.W, g.W, d_state, s),
                       "qsmd5 column kernel launch"))
        return drain(rc);
    }
  // the metadata's H2D ran first on this stream: its host block is free for the digests
  if (int rc = hip(hipMemcpyAsync(hm, d_dig, 16 * n, hipMemcpyDeviceToHost, s), "hipMemcpyAsync D2H"))
    return drain(rc);
  if (int rc = hip(hipEventRecord(rs.done, s), "hipEventRecord")) return drain(rc);
  if (int rc = poll_event(rs.done, "qsmd5_hash_read: waiting for the batch")) return drain(rc);
  memcpy(digests, hm, 16 * n);
  return 0;
}

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
  std::unique_ptr<uint8_t[]> buf(new (std::nothrow) uint8_t[2 * std::max<uint64_t>(region, 1)]);
  if (!buf) return fail(-ENOMEM, "qsmd5_hash_read: host staging allocation failed");
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
  // The window in flight on the workers; finish() joins them (and runs on
  // this thread any share a worker could not be started for).
  Window cur;
  std::vector<std::thread> th;
  std::vector<uint8_t> started;  // per worker slot: a thread runs it
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
  auto finish = [&] {
    for (auto& t : th) t.join();
    th.clear();
    if (cur.g) {
      for (size_t t = 0; t < cur.T; ++t)
        if (!started[t]) work(cur, t);
      *hash_ms += (double)t_end_ns.load() * 1e-6;
    }
    cur = Window();
  };
  auto launch = [&](const Window& w) {
    cur = w;
    next.store(0);
    t_end_ns.store(0);
    started.assign(w.T, 0);
    t_start = clock::now();
    for (size_t t = 0; t < w.T; ++t) {
      try {
        th.emplace_back(work, std::cref(cur), t);
        started[t] = 1;
      } catch (...) {
        break;  // finish() runs the rest on this thread
      }
    }
  };
  size_t step = 0;
  for (const ReadGroup& g : P.groups)
    for (uint32_t j = 0; j < g.ncols; ++j, ++step) {
      uint8_t* host = buf.get() + (step & 1) * region;
      const size_t act = ReadPlan::active(J.sorted, g, j);
      // this region was last hashed two steps back, and finish() below waited for it
      const auto r0 = clock::now();
      const int rc = fill_window(J, g, j, act, host);
      J.read_s += std::chrono::duration<double>(clock::now() - r0).count();
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

// The caller's read rate (bytes per second of its read callbacks), averaged
// over recent jobs of >= 64 MiB (a new job weighs 1/2); before the first such
// job, QSMD5_READ_GIBS or 12 GiB/s (one thread's memcpy out of a page cache,
// as qsfs's ReadNoLoad).  Both backends overlap the reads with the hashing,
// so a job's wall time is about max(reads, hashing): routing compares the two
// backends on that, and a tie goes to the GPU (the CPU's threads are busy for
// it, the GPU's not).
std::atomic<uint64_t> g_read_gibs_bits{0};

double read_gibs() {
  const double env = env_gibs("QSMD5_READ_GIBS");
  if (env > 0) return env;
  const uint64_t bits = g_read_gibs_bits.load(std::memory_order_relaxed);
  if (!bits) return 12.0;
  double v;
  memcpy(&v, &bits, sizeof(v));
  return v;
}

void note_read_rate(const ReadJob& J) {
  if (J.total < (64ull << 20) || J.read_s <= 0) return;
  const double sample = (double)J.total / J.read_s / kGiB;
  const uint64_t old_bits = g_read_gibs_bits.load(std::memory_order_relaxed);
  double v = sample;
  if (old_bits) {
    double old;
    memcpy(&old, &old_bits, sizeof(old));
    v = 0.5 * old + 0.5 * sample;
  }
  uint64_t bits;
  memcpy(&bits, &v, sizeof(bits));
  g_read_gibs_bits.store(bits, std::memory_order_relaxed);
}

void log_read(const char* backend, const char* reason, const ReadJob& J) {
  if (!log_wanted(QSMD5_LOG_INFO)) return;
  log_msg(QSMD5_LOG_INFO, "qsmd5: backend=%s reason=%s chunks=%zu bytes=%llu (read)", backend, reason,
          J.len.size(), (unsigned long long)J.total);
}

}  // namespace

int hash_read_routed(const uint64_t* lens, size_t n, qsmd5_read_fn read, void* user,
                     uint64_t staging_bytes, uint8_t (*digests)[16], int flags) {
  if (n == 0) return 0;
  if (!lens || !read || !digests) return fail(-EINVAL, "qsmd5_hash_read: NULL lens/read/digests");
  if (n > 0xffffffffull) return fail(-EINVAL, "qsmd5: too many chunks");
  Backend b = kAuto;
  if (int rc = requested_backend(flags, &b)) return rc;
  ReadJob J;
  J.read = read;
  J.user = user;
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
  const uint64_t staging = staging_bytes ? staging_bytes
                                         : env_u64("QSMD5_READ_STAGING_BYTES", kDefaultReadStaging);
  // idle-host CPU time of this batch: 16 lanes per thread where cpu_read will
  // use them and they are priced, else scalar chains
  auto cpu_read_model_ms = [&]() {
    const double lanes = read_lanes_model_ms(longest, J.total, n);
    return lanes >= 0 ? lanes : cpu_model_ms(longest, J.total);
  };
  auto on_cpu = [&](const char* reason) {
    log_read("cpu", reason, J);
    double hash_ms = 0;
    const int rc = cpu_read(J, staging, digests, &hash_ms);
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
  if (b == kAuto && !background) {
    // price the hashing as for a batch of host chunks of these lengths
    const double read_ms = 1e3 * (double)J.total / kGiB / read_gibs();
    if (std::max(read_ms, cpu_read_model_ms() / cpu_efficiency()) <
        std::max(read_ms, gpu_est_ms(longest, J.total)))
      return on_cpu("size");
  }
  log_read("gpu", b == kGpu ? "forced" : background ? "background" : "size", J);
  int rc = ensure_init();
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
  // Forced GPU: no fallback.  A short read or -EINVAL is the caller's, not the GPU's.
  if (b == kGpu || rc == -EINVAL || J.short_read) return rc;
  note_gpu_failure(rc, sticky);
  const std::string gpu_err = t_last_error;
  if (rc != -ENODEV)
    log_msg(QSMD5_LOG_WARN, "qsmd5: GPU read batch of %zu chunks failed (%s); re-reading and hashing "
            "it on the CPU", n, gpu_err.c_str());
  J.short_read = false;
  const int rc2 = on_cpu("fallback");
  if (rc2) return fail(rc2, t_last_error + " (after GPU failure: " + gpu_err + ")");
  g_fallbacks.fetch_add(1);
  return 0;
}

}  // namespace rt
}  // namespace qsmd5
