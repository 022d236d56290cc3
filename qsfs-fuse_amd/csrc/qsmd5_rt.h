// qsfs-fuse_amd/csrc/qsmd5_rt.h -- the host runtime's internal interface,
// shared by its translation units (not installed; the product interface is
// include/qsmd5.h, whose entry points qsmd5_runtime.cpp implements).
//
//   qsmd5_rt_device.cpp   errors and the log sink; binding the GPU(s), lazy
//                         init and fork awareness; memory classification;
//                         the kernel choice
//   qsmd5_rt_staging.cpp  one synchronous batch on one GPU (run_batch: the
//                         host-ordered staging pipeline), the multi-GPU split
//                         (run_sharded), the sleeping wait, chain-rate samples
//   qsmd5_rt_route.cpp    group commit of concurrent callers, backend routing
//                         and its cost model, the CPU backend, split batches,
//                         the fallback after a GPU failure
//   qsmd5_rt_read.cpp     pull-driven batches (qsmd5_hash_read): the caller's
//                         reads in column windows through pinned staging
//   qsmd5_runtime.cpp     the extern "C" entry points and the streaming context
//
// Everything here lives in qsmd5::rt and is hidden from the shared library's
// dynamic symbol table (-fvisibility=hidden): only the C-ABI is exported.
#ifndef QSFS_AMD_QSMD5_RT_H_
#define QSFS_AMD_QSMD5_RT_H_

#include <errno.h>
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/qsmd5.h"
#include "md5_cpu.h"
#include "md5_launch.h"
#include "qsmd5_plan.h"
#include "qsmd5_vma.h"

namespace qsmd5 {
namespace rt {

using qsmd5::kKernelCoalesced;
using qsmd5::kKernelLatency;
using qsmd5::kKernelLatency2;
using qsmd5::kKernelThroughput;

constexpr uint64_t kMaxChunkLen = 1ull << 38;
constexpr int kComputeStreams = 8;
constexpr int kMaxCopyStreams = 4;
constexpr uint64_t kDefaultStaging = 16ull << 30;   // device staging ring
constexpr uint64_t kInlineBytes = 256ull << 10;     // staged bytes a batch may carry inline

// ---- errors, log sink, environment (qsmd5_rt_device.cpp) ----------------------
extern thread_local std::string t_last_error;  // qsmd5_last_error()
int fail(int code, const std::string& what);   // sets t_last_error, returns code

struct LogSink {
  qsmd5_log_fn fn;
  void* user;
};
extern std::atomic<const LogSink*> g_log_sink;
bool log_wanted(int level);
__attribute__((format(printf, 2, 3))) void log_msg(int level, const char* fmt, ...);

int hip_fail(hipError_t e, const char* what);  // -ENOMEM or -EIO, with HIP's message

#define QS_HIP(call)                                  \
  do {                                                \
    hipError_t e_ = (call);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #call); \
  } while (0)

uint64_t env_u64(const char* name, uint64_t dflt);
double env_gibs(const char* name);  // a positive rate in GiB/s, else 0

// ---- ThreadSanitizer: the pinned allocator's hand-off --------------------------
// HIP's pinned allocator is not instrumented (host-sanitizer builds,
// scripts/build_sanitized.sh, instrument only this library): a block one
// thread frees and another is handed next carries no happens-before TSan can
// see, and a GPU-box run reported the second owner's first write as racing
// the first owner's last read.  Every pinned allocation the library makes or
// hands out acquires one sync object and every free releases it, as the
// allocator's own lock does.  No code in other builds.
#if defined(__has_feature)
#if __has_feature(thread_sanitizer)
#include <sanitizer/tsan_interface.h>
#define QSMD5_TSAN 1
#endif
#endif
extern char g_pinned_sync;
inline void pinned_handed_out() {
#ifdef QSMD5_TSAN
  __tsan_acquire(&g_pinned_sync);
#endif
}
inline void pinned_handed_back() {
#ifdef QSMD5_TSAN
  __tsan_release(&g_pinned_sync);
#endif
}

// ---- bound GPUs and lifetime (qsmd5_rt_device.cpp) ---------------------------
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int reserve(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) {
      (void)hipFree(p);
      p = nullptr;
      cap = 0;
    }
    size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      p = nullptr;
      return hip_fail(e, "hipMalloc");
    }
    cap = want;
    return 0;
  }
};

struct HostPinned {
  void* p = nullptr;
  size_t cap = 0;
  int reserve(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) {
      pinned_handed_back();
      (void)hipHostFree(p);
      p = nullptr;
      cap = 0;
    }
    size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      p = nullptr;
      return hip_fail(e, "hipHostMalloc");
    }
    pinned_handed_out();
    cap = want;
    return 0;
  }
};

// Events of one batch, destroyed together when the batch returns.
struct EventSet {
  std::vector<hipEvent_t> ev;
  EventSet() = default;
  EventSet(const EventSet&) = delete;
  EventSet& operator=(const EventSet&) = delete;
  ~EventSet() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
  int make(hipEvent_t* out, unsigned flags) {
    hipError_t e = hipEventCreateWithFlags(out, flags);
    if (e != hipSuccess) return hip_fail(e, "hipEventCreate");
    ev.push_back(*out);
    return 0;
  }
};

// One pull-driven batch in flight (qsmd5_hash_read, qsmd5_rt_read.cpp): its
// stream, events and buffers.  A job runs for as long as the caller's reads
// take, so it must not hold Dev::mu (every other batch on this GPU) meanwhile;
// and jobs of different files (qsfs flushes files from several FUSE threads at
// once) each read on their own thread, so a GPU keeps up to
// QSMD5_READ_SLOTS (default 4, at most kMaxReadSlots) of them running side
// by side.  The stream and events are made on first use, the buffers grow
// with the jobs (HostPinned / DevBuf reserve).
constexpr int kMaxReadSlots = 8;
constexpr int kMaxReadRegions = 4;  // staging regions per job (QSMD5_READ_REGIONS, default 2)
struct ReadSlot {
  hipStream_t stream = nullptr;  // kernels (and, with QSMD5_READ_OVERLAP=0, the copies too)
  hipStream_t copy = nullptr;    // window copies into the device regions
  hipEvent_t copied[kMaxReadRegions] = {};  // the last H2D copy out of host region k (into device region k)
  hipEvent_t hashed[kMaxReadRegions] = {};  // the last column kernel over device region k
  hipEvent_t done = nullptr;
  // every event above, for creation and release
  std::vector<hipEvent_t*> events() {
    std::vector<hipEvent_t*> v = {&done};
    for (int k = 0; k < kMaxReadRegions; ++k) {
      v.push_back(&copied[k]);
      v.push_back(&hashed[k]);
    }
    return v;
  }
  HostPinned h_read, h_meta;  // the staging regions; descriptors + orders, then digests
  DevBuf d_read, d_meta, d_state, d_dig;
};

// One bound GPU: its streams, scratch and staging ring.  Batches on one Dev are
// serialised by its mutex; different Devs run concurrently (multi-GPU shards).
struct Dev {
  std::mutex mu;
  int device = -1;
  hipStream_t copy[kMaxCopyStreams] = {};
  int ncopy = 2;  // H2D streams (QSMD5_COPY_STREAMS), slices alternate over them
  hipStream_t compute[kComputeStreams] = {};
  // d_meta / h_meta: one block [chunk + segment descriptors | lane orders |
  // inline host data of tiny batches], so one H2D copy carries them all.
  DevBuf d_meta, d_dig, d_staging, d_state;
  HostPinned h_meta, h_dig;
  // Per-batch events, reused (batches on one Dev are serialised by mu).
  hipEvent_t ev_meta = nullptr, ev_first = nullptr, ev_last = nullptr;
  hipEvent_t ev_done = nullptr;  // end of a batch, polled by a sleeping caller (wait_stream)
  uint64_t staging_cap = kDefaultStaging;
  double last_wall_ms = 0, last_kernel_ms = 0;
  std::atomic<uint32_t> chain_samples{0};  // batches that qualified as a chain-rate sample
  // Pull-driven batches: slots taken under read_mu, a job waits on read_cv
  // while all nread_slots are busy (qsmd5_rt_read.cpp).
  std::mutex read_mu;
  std::condition_variable read_cv;
  uint32_t read_busy = 0;  // bit k: slot k has a job
  int nread_slots = 4;
  ReadSlot read_slot[kMaxReadSlots];
};

struct Runtime {
  bool ready = false;
  int init_rc = 0;
  std::string init_msg;         // why init failed, for callers on other threads
  std::vector<Dev*> devs;       // devs[0] = primary (ctx, device-async, fill)
  uint64_t shard_bytes = 0;     // host bytes per extra GPU before a batch is sharded
  std::mutex timing_mu;
  double last_wall_ms = 0, last_kernel_ms = 0;
};

Runtime& rt();
Dev& primary();

// Lazy initialisation, undone by qsmd5_shutdown.  g_init_state: 0 = not yet
// (or shut down), 1 = ready, 2 = failed (sticky until a shutdown).  The fast
// path is one acquire load; init and shutdown serialise on g_init_mu.
extern std::mutex g_init_mu;
extern std::atomic<int> g_init_state;
extern pid_t g_init_pid;                     // the process that owns the HIP state
extern std::atomic<bool> g_forked_child;     // set in a child forked after init
extern std::atomic<int> g_inits;             // do_init runs (qsmd5_stats.inits)
int ensure_init();
int release_dev(Dev& d);

// ---- memory classification (qsmd5_rt_device.cpp) -----------------------------
enum MemKind { kHostMem = 0, kDeviceMem = 1 };

// Device memory reports its GPU ordinal in *owner (host memory: -1).
// *hip_known: HIP knows the pointer (device, pinned or registered host memory).
MemKind classify(const void* p, int* owner = nullptr, bool* hip_known = nullptr);

// Classifies the chunk pointers of one batch.  classify()'s query costs ~30 ns
// for HIP memory and 70-260 ns for pageable memory.  It is serialised inside
// HIP, so host threads make it slower, not faster
// (profiles/r01_ubench_classify.log).  Two exact range caches avoid it:
// - A HIP allocation (device, pinned or registered host) found once is
//   remembered by its exact range (hipMemGetAddressRange).  Every byte of one
//   allocation has the same kind and owner.
// - A pointer HIP does not know (pageable) is remembered by the VMA that holds
//   it (/proc/self/maps, read once per batch after QSMD5_MAPS_AFTER = 2048
//   pageable queries), if that VMA is readable and
//   anonymous or a regular file.  Device memory never lives in such a VMA:
//   VRAM is an unreadable reservation or a mapping of a /dev file, and VMAs of
//   different backing or permissions never merge.  This cache only ever
//   answers "host", so it can never send a host pointer to a kernel.
// A batch's chunks mostly sit in a few allocations (a pool, a file buffer,
// torch's caching allocator).  QSMD5_FLAG_HOST skips all queries.
// Host ranges registered through qsmd5_register_host, widened to whole pages
// (a malloc'd vector<char> starts 16 B into its mapping).  HIP's
// hipMemGetAddressRange does not describe registered memory, so the
// classifier takes their exact extent from here (leaked, as rt()).
struct Registry {
  std::mutex mu;
  std::map<uintptr_t, uintptr_t> base_of;  // user pointer -> page-aligned base
  std::map<uintptr_t, uintptr_t> end_of;   // page-aligned base -> end
  // The registered range holding p, if any: [*lo, *hi).
  bool find(uintptr_t p, uintptr_t* lo, uintptr_t* hi) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = end_of.upper_bound(p);
    if (it == end_of.begin()) return false;
    --it;
    if (p >= it->second) return false;
    *lo = it->first;
    *hi = it->second;
    return true;
  }
};
Registry& registry();

class Classifier {
 public:
  Classifier(int flags, size_t n)
      : all_host_(flags & QSMD5_FLAG_HOST),
        maps_after_(n >= 2 ? env_u64("QSMD5_MAPS_AFTER", kMapsAfter) : ~0ull) {}
  // *hip (optional): 1 = HIP-known memory (device, pinned, registered); 0 =
  // pageable as far as the caches tell (a registered subrange of a cached VMA
  // reads as 0: it then just misses the gather kernel); 2 = not classified
  // (QSMD5_FLAG_HOST).
  MemKind operator()(const void* p, int* owner, uint8_t* hip = nullptr) {
    *owner = -1;
    if (hip) *hip = all_host_ ? 2 : 0;
    if (all_host_ || !p) return kHostMem;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    for (int k = 0; k < used_; ++k) {
      const Range& r = ranges_[(next_ + kRanges - 1 - k) % kRanges];  // newest first
      if (a - r.lo < r.size) {
        *owner = r.owner;
        if (hip) *hip = r.hip ? 1 : 0;
        return r.kind;
      }
    }
    bool hip_known = false;
    const MemKind kind = classify(p, owner, &hip_known);
    if (hip) *hip = hip_known ? 1 : 0;
    if (hip_known) {
      uintptr_t lo = 0;
      size_t size = 0;
      if (hip_range(a, *owner, &lo, &size)) remember(lo, size, kind, *owner, true);
    } else if (kind == kHostMem && ++pageable_queries_ >= maps_after_) {
      if (!maps_read_) read_maps();
      auto it = std::upper_bound(vmas_.begin(), vmas_.end(), a,
                                 [](uintptr_t x, const Vma& v) { return x < v.lo; });
      if (it != vmas_.begin() && a - (it - 1)->lo < (it - 1)->hi - (it - 1)->lo)
        remember((it - 1)->lo, (it - 1)->hi - (it - 1)->lo, kHostMem, -1, false);
    }
    return kind;
  }

  // Does [lo, hi) lie inside ONE allocation or mapping?  Decides whether rows
  // of host chunks may go as one 2-D copy (qsmd5_plan.h plan_copy_runs), so it
  // is exact and ignores QSMD5_FLAG_HOST: a HIP-known first row (pinned or
  // registered) needs the span inside its exact HIP allocation, which HIP then
  // reads by DMA; a pageable first row needs the span inside one host VMA, which
  // HIP reads with the CPU.  The VMA cache of operator() is not used here: a
  // registered subrange of a pageable VMA is HIP memory with a smaller range.
  // Does [lo, lo + len) run past the end of the HIP allocation that holds lo,
  // as far as the cache knows it (operator() just remembered the range of a
  // HIP-known pointer)?  A device chunk that does would send the kernel past
  // the allocation -- a GPU memory fault, not just a wrong digest -- so the
  // batch is refused instead.  An allocation whose extent HIP does not report
  // (no cached range) is let through, as before.
  bool overruns_allocation(uintptr_t lo, uint64_t len) const {
    for (int k = 0; k < used_; ++k) {
      const Range& r = ranges_[(next_ + kRanges - 1 - k) % kRanges];
      if (r.hip && lo - r.lo < r.size) return len > r.size - (lo - r.lo);
    }
    return false;
  }

  bool span_in_one(uintptr_t lo, uintptr_t hi) {
    if (hi <= lo) return true;
    for (int k = 0; k < used_; ++k) {
      const Range& r = ranges_[(next_ + kRanges - 1 - k) % kRanges];
      if (r.hip && lo - r.lo < r.size) return hi - r.lo <= r.size;
    }
    int owner = -1;
    bool hip_known = false;
    (void)classify(reinterpret_cast<const void*>(lo), &owner, &hip_known);
    if (hip_known) {
      uintptr_t b = 0;
      size_t size = 0;
      if (!hip_range(lo, owner, &b, &size)) return false;
      remember(b, size, owner >= 0 ? kDeviceMem : kHostMem, owner, true);
      return hi - b <= size;
    }
    if (!maps_read_) read_maps();
    auto it = std::upper_bound(vmas_.begin(), vmas_.end(), lo,
                               [](uintptr_t x, const Vma& v) { return x < v.lo; });
    return it != vmas_.begin() && lo < (it - 1)->hi && hi <= (it - 1)->hi;
  }

  // The exact allocation holding HIP-known address a: hipMemGetAddressRange
  // for HIP allocations, the library's registry for memory registered through
  // qsmd5_register_host (which hipMemGetAddressRange does not describe).
  static bool hip_range(uintptr_t a, int owner, uintptr_t* lo, size_t* size) {
    hipDeviceptr_t base = nullptr;
    size_t sz = 0;
    if (hipMemGetAddressRange(&base, &sz, reinterpret_cast<void*>(a)) == hipSuccess && sz &&
        a - reinterpret_cast<uintptr_t>(base) < sz) {
      *lo = reinterpret_cast<uintptr_t>(base);
      *size = sz;
      return true;
    }
    (void)hipGetLastError();
    uintptr_t rlo = 0, rhi = 0;
    if (owner >= 0 || !registry().find(a, &rlo, &rhi)) return false;
    *lo = rlo;
    *size = rhi - rlo;
    return true;
  }

  // Does [lo, hi) lie inside ONE pinned or registered host allocation?  Then a
  // kernel may read it over PCIe (qsmd5_gather_kernel); *dev is the
  // device-visible address of lo.  Exact, like span_in_one, and independent of
  // QSMD5_FLAG_HOST: a device pointer or pageable memory answers false.
  bool hip_host_range(uintptr_t lo, uintptr_t hi, uintptr_t* dev) {
    if (hi <= lo || !span_in_one(lo, hi)) return false;
    for (int k = 0; k < used_; ++k) {
      Range& r = ranges_[(next_ + kRanges - 1 - k) % kRanges];
      if (!r.hip || lo - r.lo >= r.size) continue;
      if (r.kind != kHostMem) return false;
      if (!r.dev) {
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, reinterpret_cast<void*>(r.lo), 0) != hipSuccess || !d) {
          (void)hipGetLastError();
          return false;
        }
        r.dev = reinterpret_cast<uintptr_t>(d);
      }
      *dev = r.dev + (lo - r.lo);
      return true;
    }
    return false;  // pageable: span_in_one found it in a host VMA
  }

 private:
  // Parse the maps only after this many pageable queries in one batch: by then
  // the queries have cost (70-260 ns each) about what one parse of a large
  // process's maps does, so a batch never pays much more than twice the better.
  static constexpr uint64_t kMapsAfter = 2048;
  struct Vma {
    uintptr_t lo, hi;
  };
  void remember(uintptr_t lo, size_t size, MemKind kind, int owner, bool hip) {
    ranges_[next_] = Range{lo, size, kind, owner, hip, 0};
    next_ = (next_ + 1) % kRanges;
    used_ = used_ < kRanges ? used_ + 1 : kRanges;
  }
  // The VMAs qsmd5_vma.h lets us cache as host memory; anything else (device
  // files, dma-bufs, anon inodes) is left to the per-pointer query.
  void read_maps() {
    maps_read_ = true;
    FILE* f = fopen("/proc/self/maps", "r");
    if (!f) return;
    char line[4096];
    uint64_t lo = 0, hi = 0;
    while (fgets(line, sizeof(line), f))
      if (qsmd5::host_vma_from_maps_line(line, &lo, &hi)) vmas_.push_back(Vma{(uintptr_t)lo, (uintptr_t)hi});
    fclose(f);
  }
  struct Range {
    uintptr_t lo;
    size_t size;
    MemKind kind;
    int owner;
    bool hip;        // an exact HIP allocation (else a host VMA)
    uintptr_t dev;   // pinned/registered host allocation: device-visible address of lo (0: unknown)
  };
  static constexpr int kRanges = 8;
  Range ranges_[kRanges] = {};
  int used_ = 0, next_ = 0;
  bool all_host_;
  uint64_t maps_after_;
  uint64_t pageable_queries_ = 0;
  bool maps_read_ = false;
  std::vector<Vma> vmas_;  // sorted: /proc/self/maps lists VMAs in address order
};

int kernel_choice(size_t n, bool aligned16);

// ---- one batch on the GPU(s) (qsmd5_rt_staging.cpp) --------------------------
// The GPU chain rate averaged over timed batches (double bits; 0 = none yet).
extern std::atomic<uint64_t> g_gpu_chain_bits;
int wait_mode();  // QSMD5_WAIT: 0 auto, 1 block, 2 spin, 3 poll
hipError_t wait_stream(Dev& d, hipStream_t s, double est_ms);
int run_batch(Dev& r, const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags);
int run_sharded(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags,
                double* kernel_ms, double* wall_ms);

// ---- pull-driven batches (qsmd5_rt_read.cpp) -------------------------------------
constexpr uint64_t kDefaultReadStaging = 256ull << 20;  // QSMD5_READ_STAGING_BYTES
void prewarm_read_slot(Dev& d);  // read slot 0's buffers at init (QSMD5_READ_PREWARM)
void release_read_cache();       // the CPU path's cached staging (qsmd5_shutdown)
int hash_read_routed(const uint64_t* lens, size_t n, qsmd5_read_fn read, void* user,
                     uint64_t staging_bytes, uint8_t (*digests)[16], int flags);

// ---- entry-point scope (every extern "C" call that may reach the runtime) -----
// Entry points leave the calling thread's current HIP device as they found
// it: the runtime makes its own GPU current, and a torch or HIP thread working
// on another GPU must not come back on ours.
struct DeviceRestore {
  int prev = -1;
  DeviceRestore() {
    if (g_forked_child.load(std::memory_order_relaxed)) return;  // not our HIP state
    if (hipGetDevice(&prev) != hipSuccess) {
      prev = -1;
      (void)hipGetLastError();
    }
  }
  ~DeviceRestore() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Calls in flight against qsmd5_shutdown: every entry point
// that may reach the runtime holds g_calls shared for its whole duration (the
// outermost one on a thread; entry points call each other), and shutdown takes
// it exclusively, so it waits for every call in flight -- the group-commit
// leader's merged batch, a split batch's CPU thread, a sharded batch's threads
// all run inside some caller's call -- and calls that arrive meanwhile wait
// for it, then initialise afresh.  A child forked after init takes no lock: a
// parent thread may have held it at fork(), and the child never touches the
// parent's HIP state anyway.
//
// glibc's rwlock prefers readers: while any call holds g_calls shared, a new
// lock_shared succeeds even with shutdown waiting for the exclusive lock, so
// calls that keep overlapping (executor + FUSE threads) could starve shutdown
// forever (tests/cpp/shutdown_starvation.cpp: 20 s and counting
// before this gate).  So a shutdown first raises g_shutdown_pending, and a new
// OUTERMOST call waits at the gate until no shutdown is pending; calls
// already in flight finish, and the exclusive lock comes free.
extern std::shared_mutex g_calls;
extern thread_local int t_call_depth;
extern std::atomic<int> g_shutdown_pending;  // shutdowns waiting for or holding g_calls
extern std::mutex g_gate_mu;
extern std::condition_variable g_gate_cv;

struct CallScope {
  bool locked = false;
  CallScope() {
    if (t_call_depth++ == 0 && !g_forked_child.load(std::memory_order_relaxed)) {
      if (g_shutdown_pending.load(std::memory_order_acquire) > 0) {
        std::unique_lock<std::mutex> lk(g_gate_mu);
        g_gate_cv.wait(lk, [] { return g_shutdown_pending.load() == 0; });
      }
      g_calls.lock_shared();
      locked = true;
    }
  }
  ~CallScope() {
    --t_call_depth;
    if (locked) g_calls.unlock_shared();
  }
  CallScope(const CallScope&) = delete;
  CallScope& operator=(const CallScope&) = delete;
};

template <class F>
int guarded(F&& f) {
  CallScope call;
  DeviceRestore keep;
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return fail(-ENOMEM, "qsmd5: host allocation failed");
  } catch (...) {
    return fail(-EIO, "qsmd5: internal error");
  }
}

// ---- routing, cost model, CPU backend (qsmd5_rt_route.cpp) -------------------
constexpr double kGpuChainGiBs = 0.119;  // until a batch has been timed on this GPU
constexpr double kLinkGiBs = 53.7;
constexpr double kGpuCallMs = 0.03;
constexpr double kD2HGiBs = 10.0;  // device chunk read back by the CPU backend (8 MiB pieces)
constexpr double kCpuChainGiBs = 0.7;  // QSMD5_CALIBRATE=0, or a timer that failed
constexpr double kGiB = 1073741824.0;

enum Backend { kAuto = 0, kGpu = 1, kCpu = 2 };

extern std::atomic<uint64_t> g_gpu_batches, g_cpu_batches, g_fallbacks;
extern std::atomic<uint64_t> g_gpu_chunks, g_cpu_chunks;
extern std::atomic<bool> g_gpu_lost;     // a sticky GPU fault: every later call hashes on the CPU
extern thread_local int t_last_backend;  // qsmd5_last_backend()

int requested_backend(int flags, Backend* b);
size_t cpu_threads();
// This host's CPU MD5 rates, timed once (qsmd5_rt_route.cpp, "backend routing").
struct CpuRates {
  double chain = kCpuChainGiBs;  // one thread, one scalar chain
  double lane_thread = 0;        // one thread, its AVX-512 lanes together (0: no AVX-512F)
  int mb_groups = 1;             // 16-lane groups per thread that timed faster (1 or 2)
  double lane16 = 0, lane32 = 0;  // one thread's rate with 16 / 32 lanes busy
  bool measured = false;
};
const CpuRates& cpu_rates();
double cpu_gibs_per_thread();
double gpu_chain_gibs(bool* measured = nullptr);
double link_gibs();
// Estimated wall time (ms) on each backend (see qsmd5_rt_route.cpp).
double gpu_est_ms(uint64_t longest, uint64_t host_bytes);
double gpu_wait_est_ms(uint64_t longest, uint64_t host_bytes);  // its lower bound, for sleeping
double cpu_est_ms(uint64_t longest, uint64_t total, uint64_t d2h_bytes = 0);
// Load feedback (qsmd5_rt_route.cpp): the share of its priced rate the CPU
// backend got lately (1 = as priced); note_cpu_batch adds a timed batch.
double cpu_efficiency();
void note_cpu_batch(double priced_ms, double measured_ms);
double cpu_priced_ms(const qsmd5_chunk* chunks, size_t n, int flags);
double cpu_model_ms(uint64_t longest, uint64_t total);  // scalar chains, idle host
double read_lanes_model_ms(uint64_t longest, uint64_t total, size_t n);  // < 0: not priced
bool cpu_is_faster(const qsmd5_chunk* chunks, size_t n, int flags);
std::vector<uint32_t> plan_split(const qsmd5_chunk* chunks, size_t n, int flags);
int cpu_batch(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags,
              bool allow_mb = true);
int hash_routed(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags);
// After a failed GPU batch: marks the context lost on a sticky HIP error.
void note_gpu_failure(int rc, bool injected_sticky);

}  // namespace rt
}  // namespace qsmd5

#endif  // QSFS_AMD_QSMD5_RT_H_
