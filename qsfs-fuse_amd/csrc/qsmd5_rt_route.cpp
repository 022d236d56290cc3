// qsfs-fuse_amd/csrc/qsmd5_rt_route.cpp -- group commit of concurrent callers, backend
// routing and its cost model, the CPU backend, split batches, GPU-failure fallback
// (the runtime's units: qsmd5_rt.h).
#include <cmath>

#include "qsmd5_rt.h"

namespace qsmd5 {
namespace rt {

// Calls in flight against qsmd5_shutdown: CallScope (qsmd5_rt.h).
std::shared_mutex g_calls;
thread_local int t_call_depth = 0;
std::atomic<int> g_shutdown_pending{0};
std::mutex g_gate_mu;
std::condition_variable g_gate_cv;

// ---- group commit ------------------------------------------------------------
// qsfs hashes parts from up to numtransfer executor threads at once
// (TransferManager.cpp:55-60) plus FUSE threads, each call a batch of its own
// (often one part).  A batch costs one chain time (~85 ms per 10 MiB) whatever
// its width, so concurrent calls are merged: a caller that finds the GPU idle
// becomes the leader and runs every queued request as ONE batch; callers that
// arrive meanwhile queue and are taken by the next leader.  Five concurrent
// one-part calls then cost two chain times instead of five.  A merged batch
// that fails (one caller's bad pointer, an allocation too large for the merged
// size) is re-run request by request, so each caller gets its own result.
struct Request {
  const qsmd5_chunk* chunks;
  size_t n;
  uint8_t (*digests)[16];
  int flags;
  int rc = 0;
  std::string err;
  bool done = false;
  Request* next = nullptr;  // intrusive FIFO: queueing and taking never allocate
};

struct Coalescer {
  std::mutex mu;
  std::condition_variable cv;
  Request* head = nullptr;
  Request* tail = nullptr;
  size_t queued = 0;      // requests in the list
  size_t prev_group = 0;  // requests the previous leader ran
  bool busy = false;
};

static Coalescer& coalescer() {
  static Coalescer* c = new Coalescer;  // leaked, as rt()
  return *c;
}

constexpr size_t kMaxGroupChunks = 1u << 24;

// One batch on the bound GPU(s); timings go to the runtime's last_* fields.
static int run_any(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags) {
  Runtime& R = rt();
  int rc = 0;
  double kernel_ms = 0, wall_ms = 0;
  if (R.devs.size() == 1) {
    Dev& d = primary();
    std::lock_guard<std::mutex> lk(d.mu);
    rc = run_batch(d, chunks, n, digests, flags);
    kernel_ms = d.last_kernel_ms;
    wall_ms = d.last_wall_ms;
  } else {
    rc = run_sharded(chunks, n, digests, flags, &kernel_ms, &wall_ms);
  }
  if (rc == 0) {
    std::lock_guard<std::mutex> lk(R.timing_mu);
    R.last_kernel_ms = kernel_ms;
    R.last_wall_ms = wall_ms;
  }
  return rc;
}

// Runs the requests first, first->next, ... (nothing may escape: the leader
// must always get back to clearing `busy` in group_commit).
static void run_group(Request* first) noexcept {
  auto run_one = [](Request* q) {
    const char* what = nullptr;
    try {
      q->rc = run_any(q->chunks, q->n, q->digests, q->flags);
    } catch (const std::bad_alloc&) {
      q->rc = -ENOMEM;
      what = "qsmd5: host allocation failed";
    } catch (...) {
      q->rc = -EIO;
      what = "qsmd5: internal error";
    }
    if (q->rc) {
      try {
        q->err = what ? std::string(what) : t_last_error;
      } catch (...) {
      }
    }
  };
  if (!first->next) {
    run_one(first);
    return;
  }
  int rc = 0;
  try {
    size_t total = 0;
    int all_host = QSMD5_FLAG_HOST;  // kept only if every merged caller vouches for its chunks
    for (Request* q = first; q; q = q->next) {
      total += q->n;
      all_host &= q->flags;
    }
    std::vector<qsmd5_chunk> merged;
    merged.reserve(total);
    for (Request* q = first; q; q = q->next)
      for (size_t i = 0; i < q->n; ++i) {
        qsmd5_chunk c = q->chunks[i];
        if (q->flags & QSMD5_FLAG_REF_TRUNCATE32) c.len &= 0xffffffffull;  // per caller
        merged.push_back(c);
      }
    std::vector<uint8_t> dig(16 * total);
    rc = run_any(merged.data(), total, reinterpret_cast<uint8_t(*)[16]>(dig.data()), all_host);
    if (rc == 0) {
      size_t off = 0;
      for (Request* q = first; q; q = q->next) {
        memcpy(q->digests, &dig[16 * off], 16 * q->n);
        off += q->n;
      }
      return;
    }
  } catch (...) {
    // fall through: re-run one by one
  }
  for (Request* q = first; q; q = q->next) run_one(q);  // each caller gets its own result
}

static int group_commit(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags) {
  if (env_u64("QSMD5_NO_COALESCE", 0)) return run_any(chunks, n, digests, flags);
  Coalescer& co = coalescer();
  Request req{chunks, n, digests, flags, 0, std::string(), false, nullptr};
  // Linger: callers released by the previous launch usually re-submit within
  // microseconds (a worker loop hashing part after part).  A new leader waits
  // up to this long for as many requests as the previous group held, so they
  // ride in this launch instead of the next one; a lone caller never waits.
  static const std::chrono::microseconds linger(env_u64("QSMD5_COALESCE_LINGER_US", 300));
  std::unique_lock<std::mutex> lk(co.mu);
  if (co.tail) co.tail->next = &req;
  else co.head = &req;
  co.tail = &req;
  ++co.queued;
  co.cv.notify_all();  // a lingering leader counts arrivals
  while (!req.done) {
    if (co.busy) {
      co.cv.wait(lk);
      continue;
    }
    co.busy = true;
    if (co.prev_group > 1 && co.queued < co.prev_group && linger.count() > 0) {
      const size_t want = co.prev_group;
      co.cv.wait_for(lk, linger, [&] { return co.queued >= want; });
    }
    // Lead: take the queue's head requests (FIFO) up to kMaxGroupChunks, at least one.
    Request* first = co.head;
    Request* last = first;
    size_t total = first->n, taken = 1;
    while (last->next && total + last->next->n <= kMaxGroupChunks) {
      last = last->next;
      total += last->n;
      ++taken;
    }
    co.head = last->next;
    if (!co.head) co.tail = nullptr;
    last->next = nullptr;
    co.queued -= taken;
    co.prev_group = taken;
    lk.unlock();
    run_group(first);
    lk.lock();
    // Waiters read `done` only under the lock, so a request stays alive here.
    for (Request* q = first; q;) {
      Request* nx = q->next;
      q->done = true;
      q = nx;
    }
    co.busy = false;
    co.cv.notify_all();
  }
  if (req.rc) t_last_error = req.err;  // the leader's thread ran it
  return req.rc;
}




// ---- backend routing ---------------------------------------------------------
// "The backend is chosen by size: CPU below a threshold, GPU
// above" and "GPU failure falls back to CPU and returns the same digest"; §5:
// log the backend; an env knob selects auto/cpu/gpu.
//
// A GPU batch costs one chain time for its longest chunk whatever its width
// (r_gpu per chain: the latency kernel's ~1190 cycles per 64 B at 2.4 GHz =
// 0.12 GiB/s), plus its host bytes over the link (53.7 GiB/s measured) and
// ~30 us of calls.  The CPU hashes each chunk as one chain too, several times
// faster per chain (r_cpu, md5_cpu.h), but only T = QSMD5_CPU_THREADS chains
// at a time, and a device-resident chunk must first come back over the link.
// So a lone part (the reference's unchanged per-part md5() call site,
// QSClient.cpp:369-371) is always faster on the CPU.  Equal host parts of size
// S break even at
//   n* = (S / r_gpu + call) / (S / (T r_cpu) - S / r_link)
// -- ~25 parts of 10 MiB at T = 4 and r_cpu = 0.7 GiB/s.  Above that the
// gfx950 kernels win, by 20-70x on whole files (batch pre-hash, §8f row 1).
//
// The rates are this host's, not constants: r_cpu is
// timed once, at the first routing decision, on a 128 KiB buffer (~0.2 ms;
// best of 3), and so is one thread's 16-lane AVX-512 group when the host has
// it; r_gpu is averaged over the kernel times of single-launch GPU batches
// of <= 16 384 chunks whose longest chunk is >= 4 MiB (one chain per lane:
// the regime the estimate describes; each GPU's first such batch is skipped,
// note_gpu_chain), and is 0.119 GiB/s until then.
// QSMD5_CPU_GIBS / QSMD5_GPU_CHAIN_GIBS / QSMD5_LINK_GIBS override them;
// QSMD5_CALIBRATE=0 keeps the defaults.  qsmd5_get_rates reports what is used.

std::atomic<uint64_t> g_gpu_batches{0}, g_cpu_batches{0}, g_fallbacks{0};
std::atomic<uint64_t> g_gpu_chunks{0}, g_cpu_chunks{0};
std::atomic<bool> g_gpu_lost{false};
thread_local int t_last_backend = 0;

int requested_backend(int flags, Backend* b) {
  if ((flags & QSMD5_FLAG_GPU_ONLY) && (flags & QSMD5_FLAG_CPU_ONLY))
    return fail(-EINVAL, "qsmd5: QSMD5_FLAG_GPU_ONLY and QSMD5_FLAG_CPU_ONLY together");
  if (flags & QSMD5_FLAG_GPU_ONLY) {
    *b = kGpu;
    return 0;
  }
  if (flags & QSMD5_FLAG_CPU_ONLY) {
    *b = kCpu;
    return 0;
  }
  const char* e = getenv("QSMD5_BACKEND");
  *b = (e && !strcmp(e, "gpu")) ? kGpu : (e && !strcmp(e, "cpu")) ? kCpu : kAuto;
  if (e && *e && *b == kAuto && strcmp(e, "auto"))
    return fail(-EINVAL, "qsmd5: QSMD5_BACKEND must be auto, gpu or cpu");
  return 0;
}

size_t cpu_threads() {
  const uint64_t hw = std::max(1u, std::thread::hardware_concurrency());
  return (size_t)std::max<uint64_t>(1, std::min<uint64_t>(hw, env_u64("QSMD5_CPU_THREADS", 4)));
}

double env_gibs(const char* name) {
  const char* e = getenv(name);
  const double v = e && *e ? atof(e) : 0.0;
  return v > 0 ? v : 0.0;
}



static CpuRates measure_cpu_rates() {
  CpuRates r;
  if (!env_u64("QSMD5_CALIBRATE", 1)) return r;
  constexpr size_t kBytes = 128u << 10;
  std::unique_ptr<uint8_t[]> buf(new (std::nothrow) uint8_t[kBytes]);
  if (!buf) return r;
  for (size_t i = 0; i < kBytes; ++i) buf[i] = (uint8_t)(i * 131u + (i >> 9));
  auto best_of_3 = [](auto&& f) {
    double best = 1e30;
    for (int k = 0; k < 3; ++k) {  // the first pass also wakes an idle core
      const auto t0 = std::chrono::steady_clock::now();
      f();
      best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    return best;
  };
  uint8_t d[16];
  const double t_chain = best_of_3([&] { qsmd5::cpu::md5(buf.get(), kBytes, d); });
  if (t_chain > 0) {
    r.chain = (double)kBytes / t_chain / kGiB;
    r.measured = true;
  }
  if (env_u64("QSMD5_CPU_MB", 1) && qsmd5::cpu::mb16_available()) {
    // 16 messages of kBytes / 16 (8 KiB), one per lane, run together
    constexpr uint32_t kLanes = 16;
    const uint8_t* ptrs[kLanes];
    uint64_t lens[kLanes];
    uint8_t out[kLanes][16];
    for (uint32_t i = 0; i < kLanes; ++i) {
      ptrs[i] = buf.get() + i * (kBytes / kLanes);
      lens[i] = kBytes / kLanes;
    }
    struct Pull {
      uint32_t next = 0;
      static bool take(void* ctx, uint32_t* i) {
        Pull* p = static_cast<Pull*>(ctx);
        if (p->next >= kLanes) return false;
        *i = p->next++;
        return true;
      }
    };
    const double t_mb = best_of_3([&] {
      Pull p;
      qsmd5::cpu::md5_mb16(ptrs, lens, out, Pull::take, &p);
    });
    if (t_mb > 0) r.lane_thread = r.lane16 = (double)kBytes / t_mb / kGiB;
    // 32 messages of 4 KiB in two interleaved 16-lane groups: whether this
    // core's vector pipes run two groups faster than one (QSMD5_CPU_MB_GROUPS
    // = 1 / 2 forces the choice)
    constexpr uint32_t kLanes2 = 32;
    const uint8_t* ptrs2[kLanes2];
    uint64_t lens2[kLanes2];
    uint8_t out2[kLanes2][16];
    for (uint32_t i = 0; i < kLanes2; ++i) {
      ptrs2[i] = buf.get() + i * (kBytes / kLanes2);
      lens2[i] = kBytes / kLanes2;
    }
    struct Pull2 {
      uint32_t next = 0;
      static bool take(void* ctx, uint32_t* i) {
        Pull2* p = static_cast<Pull2*>(ctx);
        if (p->next >= kLanes2) return false;
        *i = p->next++;
        return true;
      }
    };
    const double t_mb2 = best_of_3([&] {
      Pull2 p;
      qsmd5::cpu::md5_mb32(ptrs2, lens2, out2, Pull2::take, &p);
    });
    if (t_mb2 > 0) r.lane32 = (double)kBytes / t_mb2 / kGiB;
    const uint64_t forced = env_u64("QSMD5_CPU_MB_GROUPS", 0);
    if (forced == 1) r.lane32 = 0;  // never two groups
    const bool two = forced ? forced == 2 : (r.lane32 > 0 && r.lane16 > 0 && r.lane32 > 1.05 * r.lane16);
    if (two) {
      r.mb_groups = 2;
      if (r.lane32 > 0) r.lane_thread = r.lane32;
    } else {
      r.lane32 = 0;
    }
  }
  return r;
}

const CpuRates& cpu_rates() {
  static const CpuRates r = measure_cpu_rates();  // thread-safe, once per process
  return r;
}

double cpu_gibs_per_thread() {
  const double v = env_gibs("QSMD5_CPU_GIBS");
  return v > 0 ? v : cpu_rates().chain;
}

double gpu_chain_gibs(bool* measured) {
  const double v = env_gibs("QSMD5_GPU_CHAIN_GIBS");
  if (measured) *measured = false;
  if (v > 0) return v;
  const uint64_t bits = g_gpu_chain_bits.load(std::memory_order_relaxed);
  if (!bits) return kGpuChainGiBs;
  double g;
  memcpy(&g, &bits, sizeof(g));
  if (measured) *measured = true;
  return g;
}

double link_gibs() {
  const double v = env_gibs("QSMD5_LINK_GIBS");
  return v > 0 ? v : kLinkGiBs;
}

// Estimated wall time (ms) on each backend of a batch whose longest chunk is
// `longest` bytes: the GPU moves `host_bytes` over the link, the CPU hashes
// `total` bytes of which `d2h_bytes` must first be read back from a GPU.
double gpu_est_ms(uint64_t longest, uint64_t host_bytes) {
  return kGpuCallMs + 1e3 * ((double)longest / gpu_chain_gibs() + (double)host_bytes / link_gibs()) / kGiB;
}
// The shortest time the same batch can plausibly take, for how long a waiting
// thread may sleep before it starts polling (wait_stream): a measured chain
// rate pulled down by a slow sample (a shared GPU) must not make the caller
// oversleep, so the chain is priced at the faster of the measured and the
// nominal rate.
double gpu_wait_est_ms(uint64_t longest, uint64_t host_bytes) {
  const double chain = std::max(gpu_chain_gibs(), kGpuChainGiBs);
  return 1e3 * ((double)longest / chain + (double)host_bytes / link_gibs()) / kGiB;
}
// ---- the CPU backend under load --------------------------
// The CPU estimates assume that each of the T backend threads gets a core.  A
// qsfs daemon's own workers and FUSE threads (or other tenants) may hold those
// cores; then a CPU batch takes longer than priced, and the GPU -- which
// leaves the cores alone -- becomes the faster route.  So every CPU batch
// priced at >= 2 ms is timed, and efficiency = priced / measured (at most 1)
// is folded into an average (a new sample weighs 1/2); the CPU estimates are
// divided by it.  Without a new sample it relaxes back to 1 with a 10 s time
// constant (QSMD5_CPU_EFF_DECAY_S), so a load that has gone does not keep
// batches off the CPU for good: the next CPU batch measures again.
// QSMD5_CPU_LOAD_FEEDBACK=0 prices the idle host always; qsmd5_get_cpu_efficiency
// reports the current value.
static std::atomic<uint64_t> g_cpu_eff_bits{0};  // double; 0 = no sample yet
static std::atomic<int64_t> g_cpu_eff_at{0};     // steady_clock ns of the last sample

static int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

double cpu_efficiency() {
  if (!env_u64("QSMD5_CPU_LOAD_FEEDBACK", 1)) return 1.0;
  const uint64_t bits = g_cpu_eff_bits.load(std::memory_order_relaxed);
  if (!bits) return 1.0;
  double e;
  memcpy(&e, &bits, sizeof(e));
  const double tau = std::max<double>(0.001, (double)env_u64("QSMD5_CPU_EFF_DECAY_S", 10));
  const double dt = std::max<double>(0.0, (now_ns() - g_cpu_eff_at.load(std::memory_order_relaxed)) * 1e-9);
  return 1.0 - (1.0 - e) * std::exp(-dt / tau);
}

void note_cpu_batch(double priced_ms, double measured_ms) {
  if (priced_ms < 2.0 || measured_ms <= 0) return;
  const double sample = std::min(1.0, std::max(0.02, priced_ms / measured_ms));
  const double cur = cpu_efficiency();
  const double e = g_cpu_eff_bits.load(std::memory_order_relaxed) ? 0.5 * cur + 0.5 * sample : sample;
  uint64_t bits;
  memcpy(&bits, &e, sizeof(bits));
  g_cpu_eff_bits.store(bits, std::memory_order_relaxed);
  g_cpu_eff_at.store(now_ns(), std::memory_order_relaxed);
}

// The idle-host model (no load factor): the longest chain on one thread, or all
// bytes over T threads.
double cpu_model_ms(uint64_t longest, uint64_t total) {
  const double T = (double)cpu_threads(), rc = cpu_gibs_per_thread();
  return 1e3 * std::max((double)longest / rc, (double)total / (T * rc)) / kGiB;
}

double cpu_est_ms(uint64_t longest, uint64_t total, uint64_t d2h_bytes) {
  return cpu_model_ms(longest, total) / cpu_efficiency() + 1e3 * (double)d2h_bytes / kD2HGiBs / kGiB;
}

static uint64_t routed_len(const qsmd5_chunk& c, int flags) {
  return (flags & QSMD5_FLAG_REF_TRUNCATE32) ? (c.len & 0xffffffffull) : c.len;
}

// Price the CPU backend's multi-buffer lanes (cpu_batch, md5_cpu_mb.cpp) for
// batches that will run on them -- AVX-512F, at least 2 chunks per thread,
// every chunk in host memory -- at this host's measured 16-lane rate (a lane's
// chain = 1/16 of it).  On by default since round 5: on the
// MI355X box's EPYC 9575F the lanes beat a pool-bound GPU wave by ~3x up to
// ~240 parts of 10 MiB on an idle host, and when qsfs's own
// threads hold those cores the load feedback above (cpu_efficiency) sees the
// lanes slow down and moves the batches to the GPU.  QSMD5_ROUTE_LANES=0
// prices the scalar chains only (the round 1-4 default).
static bool lanes_priced(const qsmd5_chunk* chunks, size_t n, int flags) {
  if (!env_u64("QSMD5_ROUTE_LANES", 1) || !env_u64("QSMD5_CPU_MB", 1) ||
      !qsmd5::cpu::mb16_available() || n < 2 * std::min<size_t>(cpu_threads(), n) ||
      cpu_rates().lane_thread <= 0)
    return false;
  if ((flags & QSMD5_FLAG_HOST) || qsmd5_device_count() <= 0) return true;
  Classifier cls(flags, n);
  for (size_t i = 0; i < n; ++i) {
    int owner = -1;
    if (chunks[i].len && cls(chunks[i].ptr, &owner) == kDeviceMem) return false;
  }
  return true;
}

// The lanes' idle-host model: the longest chain in one lane, or all bytes over
// T threads' lanes together -- with the lane count cpu_batch will run: two
// groups (32 lanes, lane32) only where this core timed them faster AND the
// batch fills 32 lanes on every thread AND they come out ahead, else one
// (16 lanes, lane16).  Pricing a half-filled batch at 32 lanes' chain rate
// would double its estimate.
static double lanes_est_ms(double rate, double lanes, uint64_t longest, uint64_t total, double T) {
  return 1e3 * std::max((double)longest / (rate / lanes), (double)total / (T * rate)) / kGiB;
}
// The pull-driven CPU path (qsmd5_rt_read.cpp cpu_read) runs 16 lanes per
// thread where it has at least 2 rows per thread: its idle-host model, or a
// negative value where the lanes are not priced (QSMD5_ROUTE_LANES=0), not
// available, or the batch too narrow for them.
double read_lanes_model_ms(uint64_t longest, uint64_t total, size_t n) {
  const size_t T = std::min<size_t>(cpu_threads(), std::max<size_t>(n, 1));
  if (!env_u64("QSMD5_ROUTE_LANES", 1) || !env_u64("QSMD5_CPU_MB", 1) || !qsmd5::cpu::mb16_available() ||
      n < 2 * T)
    return -1.0;
  const CpuRates& c = cpu_rates();
  const double r16 = c.lane16 > 0 ? c.lane16 : c.lane_thread;
  if (r16 <= 0) return -1.0;
  return 1e3 * std::max((double)longest / (r16 / 16.0), (double)total / ((double)T * r16)) / kGiB;
}

static double lanes_model_ms(uint64_t longest, uint64_t total, size_t n) {
  const CpuRates& c = cpu_rates();
  const double T = (double)std::min<size_t>(cpu_threads(), std::max<size_t>(n, 1));
  const double r16 = c.lane16 > 0 ? c.lane16 : c.lane_thread;
  double ms = lanes_est_ms(r16, 16.0, longest, total, T);
  if (c.mb_groups == 2 && c.lane32 > 0 && (double)n >= 32.0 * T)
    ms = std::min(ms, lanes_est_ms(c.lane32, 32.0, longest, total, T));
  return ms;
}

// True when the CPU is expected to finish this batch first (see above).  The
// estimates first take every chunk as host memory (the GPU's upper bound, the
// CPU's lower one); only if the CPU still looks faster are the pointers
// classified, so that device-resident chunks charge the CPU their read-back
// and the GPU no link time.
bool cpu_is_faster(const qsmd5_chunk* chunks, size_t n, int flags) {
  uint64_t total = 0, longest = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t L = routed_len(chunks[i], flags);
    total += L;
    longest = std::max(longest, L);
  }
  const bool lanes = lanes_priced(chunks, n, flags);  // only for all-host batches
  auto cpu_ms_of = [&](uint64_t d2h) {
    if (!lanes) return cpu_est_ms(longest, total, d2h);
    return lanes_model_ms(longest, total, n) / cpu_efficiency();
  };
  if (!(cpu_ms_of(0) < gpu_est_ms(longest, total))) return false;
  if (lanes || (flags & QSMD5_FLAG_HOST) || qsmd5_device_count() <= 0) return true;
  uint64_t dev_bytes = 0;
  Classifier cls(flags, n);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t L = routed_len(chunks[i], flags);
    int owner = -1;
    if (L && cls(chunks[i].ptr, &owner) == kDeviceMem) dev_bytes += L;
  }
  return cpu_ms_of(dev_bytes) < gpu_est_ms(longest, total - dev_bytes);
}

// What the idle-host model prices a CPU batch of these (host) chunks at, for
// the load feedback: the lanes where cpu_batch will run them, else scalar
// chains.  Batches under 1 MiB are not worth a sample (0).
double cpu_priced_ms(const qsmd5_chunk* chunks, size_t n, int flags) {
  uint64_t total = 0, longest = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t L = routed_len(chunks[i], flags);
    total += L;
    longest = std::max(longest, L);
  }
  if (total < (1u << 20)) return 0.0;
  if (!(flags & QSMD5_FLAG_HOST) && qsmd5_device_count() > 0) {  // device chunks: D2H-bound, no sample
    Classifier cls(flags, n);
    for (size_t i = 0; i < n; ++i) {
      int owner = -1;
      if (chunks[i].len && cls(chunks[i].ptr, &owner) == kDeviceMem) return 0.0;
    }
  }
  const bool mb = env_u64("QSMD5_CPU_MB", 1) && qsmd5::cpu::mb16_available() &&
                  cpu_rates().lane_thread > 0 && n >= 2 * std::min<size_t>(cpu_threads(), n);
  return mb ? lanes_model_ms(longest, total, n) : cpu_model_ms(longest, total);
}

// Ragged batches (qsfs -b sweeps, a file's parts plus small files): the GPU's
// time is its longest chain, which a host core runs ~6x faster.  So the
// longest host chunks go to the CPU threads while the GPU hashes the rest,
// when that cuts the estimated time by at least 10% (QSMD5_SPLIT=0: never).
// E.g. BASELINE config 4 (659 chunks, 8 KiB-64 MiB): the GPU alone needs one
// 64 MiB chain, ~0.53 s.  A device-resident chunk can go too: the CPU share
// then pays its copy to the host (kD2HGiBs, the CPU backend's 8 MiB pieces),
// ~5 ms for 64 MiB against the ~0.45 s its chain takes on the GPU.  Returns
// the chunks for the CPU, longest first, or an empty list.
std::vector<uint32_t> plan_split(const qsmd5_chunk* chunks, size_t n, int flags) {
  std::vector<uint32_t> none;
  if (n < 2 || !env_u64("QSMD5_SPLIT", 1)) return none;
  uint64_t total = 0, longest = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t L = routed_len(chunks[i], flags);
    total += L;
    longest = std::max(longest, L);
  }
  const double gpu_all = gpu_est_ms(longest, total);
  // only where one chain, not the link, sets the GPU's time
  const double chain_ms = 1e3 * (double)longest / gpu_chain_gibs() / kGiB;
  if (chain_ms < 0.5 * gpu_all) return none;
  const size_t K = std::min<size_t>(n - 1, std::max<size_t>(64, 64 * cpu_threads()));
  std::vector<uint32_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0u);
  auto longer = [&](uint32_t a, uint32_t b) {
    const uint64_t la = routed_len(chunks[a], flags), lb = routed_len(chunks[b], flags);
    return la != lb ? la > lb : a < b;
  };
  std::partial_sort(idx.begin(), idx.begin() + (K + 1), idx.end(), longer);
  const bool classify_ptrs = !(flags & QSMD5_FLAG_HOST) && qsmd5_device_count() > 0;
  std::unique_ptr<Classifier> cls(classify_ptrs ? new Classifier(flags, K) : nullptr);
  double best = gpu_all;
  size_t best_k = 0;
  uint64_t cpu_bytes = 0, d2h_bytes = 0;
  for (size_t k = 1; k <= K; ++k) {
    const uint32_t i = idx[k - 1];
    const uint64_t L = routed_len(chunks[i], flags);
    int owner = -1;
    if (cls && L && (*cls)(chunks[i].ptr, &owner) == kDeviceMem) d2h_bytes += L;
    cpu_bytes += L;
    const double copy_ms = 1e3 * (double)d2h_bytes / kD2HGiBs / 1073741824.0;
    const double t = std::max(cpu_est_ms(routed_len(chunks[idx[0]], flags), cpu_bytes) + copy_ms,
                              gpu_est_ms(routed_len(chunks[idx[k]], flags), total - cpu_bytes));
    if (t < best) {
      best = t;
      best_k = k;
    }
  }
  if (best_k == 0 || best > 0.9 * gpu_all) return none;
  idx.resize(best_k);
  return idx;
}

// The multi-buffer queue of cpu_batch: host chunks go to the AVX-512 lanes,
// device chunks met on the way are hashed by the calling thread right there.
struct MbQueue {
  std::atomic<size_t>* next;
  size_t n;
  const uint32_t* order;
  const uint8_t* on_dev;
  std::atomic<int>* hip_err;
  bool (*device_chunk)(void* self, uint32_t i);
  void* self;
};

static bool mb_pull(void* ctx, uint32_t* out) {
  MbQueue* q = static_cast<MbQueue*>(ctx);
  for (size_t k; (k = q->next->fetch_add(1)) < q->n && q->hip_err->load() == (int)hipSuccess;) {
    const uint32_t i = q->order[k];
    if (!q->on_dev[i]) {
      *out = i;
      return true;
    }
    if (!q->device_chunk(q->self, i)) return false;
  }
  return false;
}

// The CPU backend: every chunk on up to cpu_threads() host threads (longest
// first, taken from a shared counter).  With AVX-512 (QSMD5_CPU_MB=0: never)
// and at least 2 host chunks per thread, each thread runs 16 host chunks at
// once, one per vector lane (md5_cpu_mb.cpp): 7-10x the scalar rate per
// thread (ubench/cpu_mb_rate.py); the routing cost model prices them
// (lanes_priced, QSMD5_ROUTE_LANES=0: scalar chains only).  A device-resident chunk is read through
// the thread's own 8 MiB host buffer, piece by piece, so a fallback over a large
// device batch holds at most 8 MiB per thread of host memory; that needs a
// working HIP context.
int cpu_batch(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags,
              bool allow_mb) {
  std::vector<uint64_t> len(n);
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) {
    len[i] = chunks[i].len;
    if (flags & QSMD5_FLAG_REF_TRUNCATE32) len[i] &= 0xffffffffull;
    if (len[i] >= kMaxChunkLen) return fail(-EINVAL, "qsmd5: chunk longer than 2^38 bytes");
    if (len[i] && !chunks[i].ptr) return fail(-EINVAL, "qsmd5: NULL ptr with non-zero len");
    total += len[i];
  }
  // Device memory cannot be read by a host core: find it (only where HIP has
  // devices at all, and not when the caller vouches for host memory).
  std::vector<uint8_t> on_dev(n, 0);
  if (!(flags & QSMD5_FLAG_HOST) && qsmd5_device_count() > 0) {
    Classifier cls(flags, n);
    for (size_t i = 0; i < n; ++i) {
      int owner = -1;
      if (!len[i] || cls(chunks[i].ptr, &owner) != kDeviceMem) continue;
      if (g_gpu_lost.load())
        return fail(-EIO, "qsmd5: the GPU context is lost; a device-resident chunk cannot be read");
      // its read-back copy would run past the allocation on the GPU too
      if (cls.overruns_allocation(reinterpret_cast<uintptr_t>(chunks[i].ptr), len[i]))
        return fail(-EINVAL, "qsmd5: device chunk " + std::to_string(i) + " (" + std::to_string(len[i]) +
                                 " bytes) runs past the end of its allocation");
      on_dev[i] = 1;
    }
  }
  std::vector<uint32_t> order(n);
  std::iota(order.begin(), order.end(), 0u);
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return len[a] > len[b]; });
  std::atomic<size_t> next{0};
  std::atomic<int> hip_err{(int)hipSuccess};
  size_t n_host = 0;
  for (size_t i = 0; i < n; ++i) n_host += !on_dev[i];
  // A lane's chain runs at ~0.6x a scalar chain (the 16 lanes share the
  // vector pipes), so the lanes pay once a thread has 2 or more chunks.
  const bool mb = allow_mb && n_host >= 2 * std::min<size_t>(cpu_threads(), n) &&
                  env_u64("QSMD5_CPU_MB", 1) && qsmd5::cpu::mb16_available();
  // Two interleaved 16-lane groups per thread where this core runs them
  // faster (timed once, CpuRates) and the batch fills 32 lanes on every
  // thread -- and only if the estimate says so: a lane of 32 runs its chain
  // slower than a lane of 16 (EPYC 9575F: 10.2 GiB/s over 32 lanes against
  // 6.7 over 16 per thread), so a batch dominated by one long chunk (config
  // 4's 64 MiB) is faster on 16 (profiles/r04_cpu_mb_groups.log).
  bool mb32 = false;
  if (mb && cpu_rates().mb_groups == 2 && cpu_rates().lane32 > 0 && cpu_rates().lane16 > 0) {
    const double T = (double)std::min<size_t>(cpu_threads(), n);
    if ((double)n_host >= 32.0 * T) {
      uint64_t longest = 0, host_total = 0;
      for (size_t i = 0; i < n; ++i)
        if (!on_dev[i]) {
          longest = std::max(longest, len[i]);
          host_total += len[i];
        }
      auto est = [&](double rate, double lanes) {
        return std::max((double)longest / (rate / lanes), (double)host_total / (T * rate));
      };
      static const bool forced2 = env_u64("QSMD5_CPU_MB_GROUPS", 0) == 2;  // tests: always
      mb32 = forced2 || est(cpu_rates().lane32, 32.0) < est(cpu_rates().lane16, 16.0);
    }
  }
  std::vector<const uint8_t*> ptrs;
  if (mb) {
    ptrs.resize(n);
    for (size_t i = 0; i < n; ++i) ptrs[i] = static_cast<const uint8_t*>(chunks[i].ptr);
  }
  struct Worker {
    const qsmd5_chunk* chunks;
    const uint64_t* len;
    uint8_t (*digests)[16];
    std::atomic<int>* hip_err;
    std::unique_ptr<uint8_t[]> bounce;
    // a device chunk through the thread's 8 MiB host buffer; false on a HIP error
    bool device_chunk(uint32_t i) {
      constexpr uint64_t kPiece = 8ull << 20;
      const uint8_t* p = static_cast<const uint8_t*>(chunks[i].ptr);
      if (!bounce) bounce.reset(new (std::nothrow) uint8_t[kPiece]);
      if (!bounce) return set_err(hipErrorOutOfMemory);
      qsmd5::cpu::Ctx c;
      for (uint64_t off = 0; off < len[i]; off += kPiece) {
        const uint64_t m = std::min(kPiece, len[i] - off);
        const hipError_t e = hipMemcpy(bounce.get(), p + off, m, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return set_err(e);
        c.update(bounce.get(), m);
      }
      c.final(digests[i]);
      return true;
    }
    bool set_err(hipError_t e) {
      int ok = (int)hipSuccess;
      hip_err->compare_exchange_strong(ok, (int)e);
      return false;
    }
  };
  auto work = [&]() noexcept {
    Worker w{chunks, len.data(), digests, &hip_err, nullptr};
    if (mb) {
      MbQueue q{&next, n, order.data(), on_dev.data(), &hip_err,
                [](void* self, uint32_t i) { return static_cast<Worker*>(self)->device_chunk(i); },
                &w};
      if (mb32) qsmd5::cpu::md5_mb32(ptrs.data(), len.data(), digests, mb_pull, &q);
      else qsmd5::cpu::md5_mb16(ptrs.data(), len.data(), digests, mb_pull, &q);
      return;
    }
    for (size_t k; (k = next.fetch_add(1)) < n && hip_err.load() == (int)hipSuccess;) {
      const uint32_t i = order[k];
      if (!on_dev[i]) {
        qsmd5::cpu::md5(chunks[i].ptr, len[i], digests[i]);
        continue;
      }
      if (!w.device_chunk(i)) return;
    }
  };
  // Threads only where they pay (a thread start costs ~20-50 us): >= 1 MiB
  // of work per thread.
  const size_t T = std::min<size_t>({cpu_threads(), n, (size_t)std::max<uint64_t>(1, total >> 20)});
  std::vector<std::thread> th;
  for (size_t t = 1; t < T; ++t) {
    try {
      th.emplace_back(work);
    } catch (...) {
      break;  // fewer helpers: the calling thread still takes every chunk left
    }
  }
  work();
  for (auto& t : th) t.join();
  if (hip_err.load() != (int)hipSuccess)
    return hip_fail((hipError_t)hip_err.load(), "qsmd5 CPU backend: reading a device chunk (8 MiB "
                                                "host buffer or hipMemcpy D2H)");
  return 0;
}

static void log_call(const char* backend, const char* reason, size_t n, const qsmd5_chunk* chunks) {
  if (!log_wanted(QSMD5_LOG_INFO)) return;
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += chunks[i].len;
  log_msg(QSMD5_LOG_INFO, "qsmd5: backend=%s reason=%s chunks=%zu bytes=%llu", backend, reason, n,
       (unsigned long long)total);
}

// After a failed GPU batch: is the HIP context gone for good (a sticky error
// such as an illegal address)?  Then every later call goes to the CPU; the
// daemon keeps producing Content-MD5s until it is restarted.
void note_gpu_failure(int rc, bool injected_sticky) {
  if (g_gpu_lost.load()) return;
  bool lost = injected_sticky;
  std::string why = injected_sticky ? "injected sticky fault (QSMD5_INJECT_GPU_FAULT=sticky)" : "";
  if (!lost && rc == -EIO && rt().ready) {
    hipError_t e = hipStreamQuery(primary().compute[0]);
    if (e != hipSuccess && e != hipErrorNotReady) {
      lost = true;
      why = hipGetErrorString(e);
    }
  }
  if (lost && !g_gpu_lost.exchange(true))
    log_msg(QSMD5_LOG_ERROR, "qsmd5: GPU context lost (%s); hashing on the CPU from now on -- restart "
         "the process to use the GPU again", why.c_str());
}

// One GPU attempt, with the test-only fault injection (QSMD5_INJECT_GPU_FAULT:
// "1" fails every GPU batch as a HIP error would, "sticky" also marks the
// context lost).
static int gpu_attempt(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int gflags,
                bool* sticky) {
  *sticky = false;
  int rc = ensure_init();
  if (rc) return rc;
  const char* inj = getenv("QSMD5_INJECT_GPU_FAULT");
  if (inj && *inj && strcmp(inj, "0")) {
    *sticky = !strcmp(inj, "sticky");
    return fail(-EIO, "qsmd5: injected GPU fault (QSMD5_INJECT_GPU_FAULT)");
  }
  return group_commit(chunks, n, digests, gflags);
}

// plan_split's batch: the CPU chunks on the CPU backend's threads, started
// first, while this thread runs the rest through the GPU path.  A GPU failure
// falls back to the CPU for the GPU's share (auto mode only reaches here).
static int run_split(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int gflags,
              const std::vector<uint32_t>& to_cpu) {
  std::vector<uint8_t> on_cpu(n, 0);
  for (uint32_t i : to_cpu) on_cpu[i] = 1;
  std::vector<qsmd5_chunk> cc, gc;
  std::vector<uint32_t> cmap, gmap;
  cc.reserve(to_cpu.size());
  gc.reserve(n - to_cpu.size());
  for (size_t i = 0; i < n; ++i) {
    (on_cpu[i] ? cc : gc).push_back(chunks[i]);
    (on_cpu[i] ? cmap : gmap).push_back((uint32_t)i);
  }
  std::vector<uint8_t> cd(16 * cc.size()), gd(16 * gc.size());
  auto* cdig = reinterpret_cast<uint8_t(*)[16]>(cd.data());
  auto* gdig = reinterpret_cast<uint8_t(*)[16]>(gd.data());
  int rc_cpu = 0;
  std::string cpu_err;
  auto cpu_side = [&]() noexcept {
    try {
      // the longest chunks, few per thread: their chains set the time, and a
      // scalar chain is the faster one (no multi-buffer lanes)
      rc_cpu = cpu_batch(cc.data(), cc.size(), cdig, gflags, false);
    } catch (...) {
      rc_cpu = fail(-ENOMEM, "qsmd5: CPU share of a split batch failed");
    }
    if (rc_cpu) cpu_err = t_last_error;
  };
  log_call("gpu+cpu", "split", n, chunks);
  std::thread th;
  bool threaded = true;
  try {
    th = std::thread(cpu_side);
  } catch (...) {
    threaded = false;  // no thread: the CPU share runs after the GPU's
  }
  struct JoinOnExit {  // an exception from the GPU share must not leave `th` joinable
    std::thread& t;
    ~JoinOnExit() {
      if (t.joinable()) t.join();
    }
  } join_on_exit{th};
  bool sticky = false;
  int rc = gpu_attempt(gc.data(), gc.size(), gdig, gflags, &sticky);
  if (threaded) th.join(); else cpu_side();
  bool gpu_failed = false;
  if (rc) {
    if (rc == -EINVAL) return rc;
    note_gpu_failure(rc, sticky);
    const std::string gpu_err = t_last_error;
    if (rc != -ENODEV)
      log_msg(QSMD5_LOG_WARN, "qsmd5: GPU share (%zu chunks) of a split batch failed (%s); "
              "re-hashing it on the CPU", gc.size(), gpu_err.c_str());
    if (int rc2 = cpu_batch(gc.data(), gc.size(), gdig, gflags))
      return fail(rc2, t_last_error + " (after GPU failure: " + gpu_err + ")");
    g_fallbacks.fetch_add(1);
    gpu_failed = true;
  }
  if (rc_cpu) return fail(rc_cpu, cpu_err);
  for (size_t k = 0; k < cc.size(); ++k) memcpy(digests[cmap[k]], cdig[k], 16);
  for (size_t k = 0; k < gc.size(); ++k) memcpy(digests[gmap[k]], gdig[k], 16);
  g_cpu_batches.fetch_add(1);
  if (gpu_failed) {
    g_cpu_chunks.fetch_add(n);
    t_last_backend = QSMD5_BACKEND_CPU;
  } else {
    g_gpu_batches.fetch_add(1);
    g_cpu_chunks.fetch_add(cc.size());
    g_gpu_chunks.fetch_add(gc.size());
    t_last_backend = QSMD5_BACKEND_SPLIT;
  }
  return 0;
}

int hash_routed(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags) {
  Backend b = kAuto;
  if (int rc = requested_backend(flags, &b)) return rc;
  const int gflags = flags & ~(QSMD5_FLAG_GPU_ONLY | QSMD5_FLAG_CPU_ONLY);
  auto on_cpu = [&](const char* reason) {
    log_call("cpu", reason, n, chunks);
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = cpu_batch(chunks, n, digests, gflags);
    if (rc == 0) {
      t_last_backend = QSMD5_BACKEND_CPU;
      g_cpu_batches.fetch_add(1);
      g_cpu_chunks.fetch_add(n);
      note_cpu_batch(cpu_priced_ms(chunks, n, gflags),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    return rc;
  };
  if (b == kCpu) return on_cpu("forced");
  const bool background = b == kAuto && (gflags & QSMD5_FLAG_BACKGROUND) && qsmd5_device_count() > 0;
  if (b == kAuto && !background) {
    if (g_gpu_lost.load()) return on_cpu("gpu-lost");
    if (cpu_is_faster(chunks, n, gflags)) return on_cpu("size");
    const std::vector<uint32_t> to_cpu = plan_split(chunks, n, gflags);
    if (!to_cpu.empty()) return run_split(chunks, n, digests, gflags, to_cpu);
  }
  if (background && g_gpu_lost.load()) return on_cpu("gpu-lost");
  log_call("gpu", b == kGpu ? "forced" : background ? "background" : "size", n, chunks);
  bool sticky = false;
  int rc = gpu_attempt(chunks, n, digests, gflags, &sticky);
  if (rc == 0) {
    t_last_backend = QSMD5_BACKEND_GPU;
    g_gpu_batches.fetch_add(1);
    g_gpu_chunks.fetch_add(n);
    return 0;
  }
  // Forced GPU: no fallback.  -EINVAL is the caller's error, not the GPU's.
  if (b == kGpu || rc == -EINVAL) return rc;
  note_gpu_failure(rc, sticky);
  const std::string gpu_err = t_last_error;
  if (rc != -ENODEV)  // no usable GPU at all was logged once, at the failed initialisation
    log_msg(QSMD5_LOG_WARN, "qsmd5: GPU batch of %zu chunks failed (%s); re-hashing it on the CPU",
            n, gpu_err.c_str());
  const int rc2 = on_cpu("fallback");
  if (rc2) return fail(rc2, t_last_error + " (after GPU failure: " + gpu_err + ")");
  g_fallbacks.fetch_add(1);
  return 0;
}

}  // namespace rt
}  // namespace qsmd5
