// qsfs-fuse_amd/csrc/qsmd5_runtime.cpp -- host runtime behind include/qsmd5.h.
//
// Owns the device, streams, descriptor/digest scratch and the host->device
// staging ring.  Every entry point is extern "C", catches everything, and
// reports failure as a negative errno (never an empty digest).  Hashing runs on
// the gfx950 kernels (md5_kernels.hip) or on the library's own CPU MD5
// (md5_cpu.h), chosen per call by size, with a CPU fallback when the GPU fails
// ("backend routing" below).
//
// Host-resident batches (the qsfs case: parts sit in pooled host buffers,
// ResourceManager.cpp:53-77) are cut into slices (a quarter of the batch,
// clamped to [512 MiB, 4 GiB]); each slice is copied H2D into a ring region on
// the copy stream and hashed by its own launch on one of kComputeStreams
// streams, so PCIe transfer of slice k+1 overlaps hashing of slice k.  A slice
// launch takes one chain time (~85 ms for 10 MiB parts) whatever its size and
// only ~4 hardware queues run kernels concurrently, so slices are kept large
// enough that the copy, not kernel concurrency, is the bound.  Staged chunks
// are packed with a 4 KiB + 256 B skew so that equal-size parts never sit at a
// power-of-two stride (lanes walk their chunks in lockstep; a power-of-two
// stride sends every lane's request to the same HBM channel).
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
#include <mutex>
#include <memory>
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

namespace {

using qsmd5::kKernelCoalesced;
using qsmd5::kKernelLatency;
using qsmd5::kKernelLatency2;
using qsmd5::kKernelThroughput;

constexpr uint64_t kMaxChunkLen = 1ull << 38;
constexpr int kComputeStreams = 8;
constexpr int kMaxCopyStreams = 4;
constexpr uint64_t kDefaultStaging = 16ull << 30;   // device staging ring
constexpr uint64_t kInlineBytes = 256ull << 10;     // staged bytes a batch may carry inline


thread_local std::string t_last_error;

int fail(int code, const std::string& what) {
  t_last_error = what;
  return code;
}

// ---- log sink -----------------------------------------------------------------
// qsfs logs through glog macros (base/LogMacros.h) and
// should see the digest backend and batch size at DebugInfo, next to its
// upload lines (QSClient.cpp:378-380).  A FUSE daemon's stderr is usually
// gone, so qsmd5_set_log_callback hands every line to the host's logger
// instead; levels are qsfs's LogLevel::Value (base/LogLevel.h:27).  Without a
// sink, warnings and errors go to stderr, and Info lines only under QSMD5_LOG=1.
struct LogSink {
  qsmd5_log_fn fn;
  void* user;
};
std::atomic<const LogSink*> g_log_sink{nullptr};  // replaced sinks are leaked: a logger
                                                  // thread may still be reading one

bool log_wanted(int level) {
  static const bool env_on = getenv("QSMD5_LOG") && strcmp(getenv("QSMD5_LOG"), "0") != 0;
  return g_log_sink.load(std::memory_order_acquire) != nullptr || level >= QSMD5_LOG_WARN || env_on;
}

__attribute__((format(printf, 2, 3))) void log_msg(int level, const char* fmt, ...) {
  if (!log_wanted(level)) return;
  char line[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(line, sizeof(line), fmt, ap);
  va_end(ap);
  if (const LogSink* s = g_log_sink.load(std::memory_order_acquire)) {
    s->fn(level, line, s->user);
    return;
  }
  fprintf(stderr, "%s\n", line);
}

int hip_fail(hipError_t e, const char* what) {
  std::string s = std::string(what) + ": " + hipGetErrorString(e);
  return fail(e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation ? -ENOMEM : -EIO, s);
}

#define QS_HIP(call)                                  \
  do {                                                \
    hipError_t e_ = (call);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #call); \
  } while (0)

uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  unsigned long long x = strtoull(v, &end, 0);
  return (end && *end == 0) ? (uint64_t)x : dflt;
}

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

Runtime& rt() {
  static Runtime* r = new Runtime;  // intentionally leaked: no teardown order issues
  return *r;
}

Dev& primary() { return *rt().devs[0]; }

// Lazy initialisation, undone by qsmd5_shutdown.  g_init_state: 0 = not yet
// (or shut down), 1 = ready, 2 = failed (sticky until a shutdown).  The fast
// path is one acquire load; init and shutdown serialise on g_init_mu.
std::mutex g_init_mu;
std::atomic<int> g_init_state{0};
pid_t g_init_pid = 0;                     // the process that owns the HIP state
std::atomic<bool> g_forked_child{false};  // set in a child forked after init

void on_fork_child() {
  // HIP state does not survive fork(): a child of a process in which this
  // library ever initialised HIP (even if it shut its own runtime down since:
  // HIP itself stays up) must not touch the GPU (it hashes on the CPU under
  // auto routing, see ensure_init).  Registered at the first init.
  if (g_init_pid != 0) g_forked_child.store(true);
}

// Devices to bind: QSMD5_DEVICES = "all" or a comma list of ordinals (an
// ordinal may repeat: two contexts on one GPU, used by the tests to exercise
// sharding on a one-GPU box); otherwise the single QSMD5_DEVICE / current one.
int parse_devices(int n, std::vector<int>* out) {
  const char* ev = getenv("QSMD5_DEVICES");
  if (ev && *ev) {
    if (!strcmp(ev, "all")) {
      for (int d = 0; d < n; ++d) out->push_back(d);
      return 0;
    }
    const char* p = ev;
    while (*p) {
      char* end = nullptr;
      long d = strtol(p, &end, 10);
      if (end == p) return fail(-EINVAL, "qsmd5: QSMD5_DEVICES is not a comma list of ordinals");
      if (d < 0 || d >= n) return fail(-ENODEV, "qsmd5: QSMD5_DEVICES names a missing GPU");
      out->push_back((int)d);
      p = end;
      if (*p == ',') ++p;
      else if (*p) return fail(-EINVAL, "qsmd5: QSMD5_DEVICES is not a comma list of ordinals");
    }
    if (out->empty() || out->size() > 64) return fail(-EINVAL, "qsmd5: QSMD5_DEVICES needs 1..64 ordinals");
    return 0;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const char* ed = getenv("QSMD5_DEVICE");
  if (ed && *ed) dev = atoi(ed);
  if (dev < 0 || dev >= n) return fail(-ENODEV, "qsmd5: QSMD5_DEVICE out of range");
  out->push_back(dev);
  return 0;
}

int init_dev(Dev& d, int device) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  d.device = device;
  d.ncopy = (int)std::min<uint64_t>(kMaxCopyStreams,
                                     std::max<uint64_t>(1, env_u64("QSMD5_COPY_STREAMS", 2)));
  for (int k = 0; k < d.ncopy; ++k)
    if ((e = hipStreamCreateWithFlags(&d.copy[k], hipStreamNonBlocking)) != hipSuccess)
      return hip_fail(e, "hipStreamCreate");
  for (auto& s : d.compute)
    if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess)
      return hip_fail(e, "hipStreamCreate");
  d.staging_cap = env_u64("QSMD5_STAGING_BYTES", kDefaultStaging);
  if ((e = hipEventCreateWithFlags(&d.ev_meta, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&d.ev_first, hipEventDefault)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&d.ev_last, hipEventDefault)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&d.ev_done, hipEventBlockingSync | hipEventDisableTiming)) !=
          hipSuccess)
    return hip_fail(e, "hipEventCreate");
  if ((e = qsmd5::warm_up(d.compute[0])) != hipSuccess ||
      (e = hipStreamSynchronize(d.compute[0])) != hipSuccess)
    return hip_fail(e, "qsmd5: kernel warm-up (is this a gfx950 GPU?)");
  return 0;
}

// Everything init_dev and run_batch allocated for one GPU: wait for its
// streams, then destroy events and streams and free scratch, staging and the
// pinned metadata (qsmd5_shutdown).  Every handle is tried even if one fails.
int release_dev(Dev& d) {
  if (d.device < 0) return 0;
  int bad = 0;
  auto chk = [&](hipError_t e) {
    if (e != hipSuccess) {
      (void)hipGetLastError();
      bad = 1;
    }
  };
  chk(hipSetDevice(d.device));
  for (int k = 0; k < kMaxCopyStreams; ++k)
    if (d.copy[k]) {
      chk(hipStreamSynchronize(d.copy[k]));
      chk(hipStreamDestroy(d.copy[k]));
      d.copy[k] = nullptr;
    }
  for (auto& s : d.compute)
    if (s) {
      chk(hipStreamSynchronize(s));
      chk(hipStreamDestroy(s));
      s = nullptr;
    }
  for (hipEvent_t* e : {&d.ev_meta, &d.ev_first, &d.ev_last, &d.ev_done})
    if (*e) {
      chk(hipEventDestroy(*e));
      *e = nullptr;
    }
  for (DevBuf* b : {&d.d_meta, &d.d_dig, &d.d_staging, &d.d_state})
    if (b->p) {
      chk(hipFree(b->p));
      b->p = nullptr;
      b->cap = 0;
    }
  for (HostPinned* b : {&d.h_meta, &d.h_dig})
    if (b->p) {
      chk(hipHostFree(b->p));
      b->p = nullptr;
      b->cap = 0;
    }
  d.device = -1;
  return bad;
}

std::atomic<int> g_inits{0};  // do_init runs (qsmd5_stats.inits)

void do_init() {
  g_inits.fetch_add(1);
  Runtime& r = rt();
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) {
    r.init_rc = fail(-ENODEV, "qsmd5: no usable GPU (hipGetDeviceCount)");
    r.init_msg = t_last_error;
    return;
  }
  std::vector<int> ords;
  if (int rc = parse_devices(n, &ords)) {
    r.init_rc = rc;
    r.init_msg = t_last_error;
    return;
  }
  for (int o : ords) {
    Dev* d = new Dev;
    r.devs.push_back(d);  // kept even if half built: qsmd5_shutdown releases it
    if (int rc = init_dev(*d, o)) {
      r.init_rc = rc;
      r.init_msg = t_last_error;
      return;
    }
  }
  r.shard_bytes = env_u64("QSMD5_SHARD_BYTES", 4ull << 30);
  (void)hipSetDevice(r.devs[0]->device);
  r.ready = true;
  r.init_rc = 0;
  if (log_wanted(QSMD5_LOG_INFO))
    for (const Dev* d : r.devs) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, d->device) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      log_msg(QSMD5_LOG_INFO, "qsmd5: bound GPU %d (%s, %d CUs), staging ring up to %llu MiB", d->device,
           p.gcnArchName, p.multiProcessorCount, (unsigned long long)(d->staging_cap >> 20));
    }
}

int ensure_init() {
  // A forked child first: no HIP call at all, not even a (re-)initialisation
  // after the parent or the child itself shut the runtime down.
  if (g_forked_child.load(std::memory_order_relaxed))
    return fail(-ENODEV, "qsmd5: the GPU runtime was initialised before fork(); a forked child "
                         "cannot use it (initialise after the fork, as qsfs does)");
  if (g_init_state.load(std::memory_order_acquire) == 0) {
    std::lock_guard<std::mutex> lk(g_init_mu);
    if (g_init_state.load() == 0) {
      static std::once_flag atfork_once;
      std::call_once(atfork_once, [] { pthread_atfork(nullptr, nullptr, on_fork_child); });
      g_init_pid = getpid();
      do_init();
      g_init_state.store(rt().ready ? 1 : 2, std::memory_order_release);
      if (!rt().ready)
        log_msg(QSMD5_LOG_WARN, "qsmd5: GPU runtime not available (%s); %s", rt().init_msg.c_str(),
             getenv("QSMD5_BACKEND") && !strcmp(getenv("QSMD5_BACKEND"), "gpu")
                 ? "QSMD5_BACKEND=gpu: hashing calls fail"
                 : "hashing on the CPU");
    }
  }
  Runtime& r = rt();
  if (!r.ready) return fail(r.init_rc ? r.init_rc : -ENODEV, r.init_msg);
  // Calls may come from threads whose current device differs.
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != r.devs[0]->device) {
    hipError_t e = hipSetDevice(r.devs[0]->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  }
  return 0;
}

enum MemKind { kHostMem = 0, kDeviceMem = 1 };

// Device memory reports its GPU ordinal in *owner (host memory: -1).
// *hip_known: HIP knows the pointer (device, pinned or registered host memory).
MemKind classify(const void* p, int* owner = nullptr, bool* hip_known = nullptr) {
  if (owner) *owner = -1;
  if (hip_known) *hip_known = false;
  if (!p) return kHostMem;
  hipPointerAttribute_t a;
  memset(&a, 0, sizeof(a));
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // pageable host memory: clear the sticky error
    return kHostMem;
  }
  // pageable memory either fails the query or reports "unregistered"
  if (hip_known) *hip_known = a.type != hipMemoryTypeUnregistered;
  if (a.type != hipMemoryTypeDevice) return kHostMem;
  if (owner) *owner = a.device;
  return kDeviceMem;
}

// Classifies the chunk pointers of one batch.  The query above costs ~30 ns
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
Registry& registry() {
  static Registry* r = new Registry;
  return *r;
}

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

int kernel_choice(size_t n, bool aligned16) {
  const char* k = getenv("QSMD5_KERNEL");
  if (k && !strcmp(k, "pc")) return kKernelLatency;
  if (k && !strcmp(k, "pc2")) return kKernelLatency2;
  if (k && !strcmp(k, "v1")) return kKernelThroughput;
  if (k && !strcmp(k, "coal")) return aligned16 ? kKernelCoalesced : kKernelThroughput;
  // The latency kernel wins while every chunk has its own chain lane in one
  // resident round (one 128 KiB-LDS workgroup per CU); its 64 KiB-ring variant
  // doubles the round (two workgroups per CU) at ~3% per chain, which still
  // beats the throughput kernels up to 32 768 chunks (+16% at 20-24 K, +6% at
  // 32 K; profiles/r01_ubench_cross2.log).  Beyond that the throughput kernels
  // keep 2+ waves per SIMD and the bound moves to VALU x clock and HBM, where
  // coalesced LDS-DMA staging beats per-lane loads (16-B-aligned chunks).
  if (n <= qsmd5::kLatencyKernelResident) return kKernelLatency;
  if (n <= qsmd5::kLatency2KernelResident) return kKernelLatency2;
  return aligned16 ? kKernelCoalesced : kKernelThroughput;
}

// Cache policy of the latency kernels' producer loads for a device batch whose
// longest chunk is `longest` bytes: QSMD5_LOAD_NT=1 / 0 forces nt / default.
bool load_nt_for(uint64_t longest) {
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
uint32_t pc_lanes_for(size_t n, uint64_t longest) {
  const uint64_t forced = env_u64("QSMD5_PC_LANES", 0);
  if (forced >= 1 && forced <= 64) return (uint32_t)forced;
  constexpr uint64_t kLongPart = 32ull << 20;  // the skewed regime (kSkewMinBlocks blocks)
  if (longest >= kLongPart && n <= qsmd5::kLatencyKernelResident / 2) return 32;
  return 64;
}

using qsmd5::kNoColumns;
using qsmd5::stage_bytes;

// The GPU chain rate averaged over timed batches (double bits; 0 = none yet),
// for the routing cost model ("backend routing" below).  Only a batch that ran
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

double gpu_est_ms(uint64_t longest, uint64_t host_bytes);       // routing cost model, below
double gpu_wait_est_ms(uint64_t longest, uint64_t host_bytes);  // its lower bound, for sleeping

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
    QS_HIP(hipEventRecord(t, r.compute[k]));
    tails.push_back(t);
  }
  if (!first_kernel) QS_HIP(hipEventRecord(r.ev_last, s0));
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
  QS_HIP(hipMemcpyAsync(r.h_dig.p, d_dig, n * 16, hipMemcpyDeviceToHost, s0));
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

Coalescer& coalescer() {
  static Coalescer* c = new Coalescer;  // leaked, as rt()
  return *c;
}

constexpr size_t kMaxGroupChunks = 1u << 24;

// One batch on the bound GPU(s); timings go to the runtime's last_* fields.
int run_any(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags) {
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
void run_group(Request* first) noexcept {
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

int group_commit(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags) {
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
std::shared_mutex g_calls;
thread_local int t_call_depth = 0;

struct CallScope {
  bool locked = false;
  CallScope() {
    if (t_call_depth++ == 0 && !g_forked_child.load(std::memory_order_relaxed)) {
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
constexpr double kGpuChainGiBs = 0.119;  // until a batch has been timed on this GPU
constexpr double kLinkGiBs = 53.7;
constexpr double kGpuCallMs = 0.03;
constexpr double kD2HGiBs = 10.0;  // device chunk read back by the CPU backend (8 MiB pieces)
constexpr double kCpuChainGiBs = 0.7;  // QSMD5_CALIBRATE=0, or a timer that failed
constexpr double kGiB = 1073741824.0;

enum Backend { kAuto = 0, kGpu = 1, kCpu = 2 };

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

// This host's CPU MD5 rates, timed once (see above).
struct CpuRates {
  double chain = kCpuChainGiBs;  // one thread, one scalar chain
  double lane_thread = 0;        // one thread, its AVX-512 lanes together (0: no AVX-512F)
  int mb_groups = 1;             // 16-lane groups per thread that timed faster (1 or 2)
  double lane16 = 0, lane32 = 0;  // one thread's rate with 16 / 32 lanes busy
  bool measured = false;
};

CpuRates measure_cpu_rates() {
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

double gpu_chain_gibs(bool* measured = nullptr) {
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
double cpu_est_ms(uint64_t longest, uint64_t total, uint64_t d2h_bytes = 0) {
  const double T = (double)cpu_threads(), rc = cpu_gibs_per_thread();
  return 1e3 * (std::max((double)longest / rc, (double)total / (T * rc)) + (double)d2h_bytes / kD2HGiBs) / kGiB;
}

uint64_t routed_len(const qsmd5_chunk& c, int flags) {
  return (flags & QSMD5_FLAG_REF_TRUNCATE32) ? (c.len & 0xffffffffull) : c.len;
}

// Opt-in (QSMD5_ROUTE_LANES=1): price the CPU backend's multi-buffer lanes
// (cpu_batch, md5_cpu_mb.cpp) for batches that will run on them -- AVX-512F,
// at least 2 chunks per thread, every chunk in host memory -- at this host's
// measured 16-lane rate (a lane's chain = 1/16 of it).  Off by default (DESIGN.md
// §1): the lanes are faster than the GPU below ~240 parts of 10 MiB at T = 4
// on the MI355X box's EPYC 9575F (6.9 GiB/s per thread), but they hold T cores
// at full AVX-512 load for the batch, and a qsfs daemon runs its transfer
// workers and FUSE threads on those cores; the GPU leaves them free.
bool lanes_priced(const qsmd5_chunk* chunks, size_t n, int flags) {
  if (!env_u64("QSMD5_ROUTE_LANES", 0) || !env_u64("QSMD5_CPU_MB", 1) ||
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
    const double lt = cpu_rates().lane_thread;  // a lane's chain: 1/(16 x groups) of it
    const double lanes_per_thread = 16.0 * cpu_rates().mb_groups;
    return 1e3 * std::max((double)longest / (lt / lanes_per_thread),
                          (double)total / ((double)cpu_threads() * lt)) / kGiB;
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

bool mb_pull(void* ctx, uint32_t* out) {
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
// thread (ubench/cpu_mb_rate.py).  The routing cost model above still prices
// the scalar path, so a batch is never sent to the CPU on the strength of it.  A device-resident chunk is read through
// the thread's own 8 MiB host buffer, piece by piece, so a fallback over a large
// device batch holds at most 8 MiB per thread of host memory; that needs a
// working HIP context.
int cpu_batch(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags,
              bool allow_mb = true) {
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

void log_call(const char* backend, const char* reason, size_t n, const qsmd5_chunk* chunks) {
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
int gpu_attempt(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int gflags,
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
int run_split(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int gflags,
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
    const int rc = cpu_batch(chunks, n, digests, gflags);
    if (rc == 0) {
      t_last_backend = QSMD5_BACKEND_CPU;
      g_cpu_batches.fetch_add(1);
      g_cpu_chunks.fetch_add(n);
    }
    return rc;
  };
  if (b == kCpu) return on_cpu("forced");
  if (b == kAuto) {
    if (g_gpu_lost.load()) return on_cpu("gpu-lost");
    if (cpu_is_faster(chunks, n, gflags)) return on_cpu("size");
    const std::vector<uint32_t> to_cpu = plan_split(chunks, n, gflags);
    if (!to_cpu.empty()) return run_split(chunks, n, digests, gflags, to_cpu);
  }
  log_call("gpu", b == kGpu ? "forced" : "size", n, chunks);
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

}  // namespace

// ----------------------------------------------------------------------------
// Streaming context (MD5 class).  One stream is one serial chain, which a host
// core runs ~6x faster than one GPU lane (the routing rule above), so under
// QSMD5_BACKEND=auto or cpu the context hashes on the CPU (md5_cpu.h; device
// pieces are copied to the host first).  Under QSMD5_BACKEND=gpu the state
// stays on the device between updates; bytes that do not fill a 64-byte block
// wait in `tail` on the host (MD5::buffer, MD5.h:79).  A GPU update that fails
// leaves the context failed: later update/final calls return -EIO rather than
// hash a stream with a hole in it.
struct qsmd5_ctx {
  bool on_cpu = false;
  bool failed = false;
  qsmd5::cpu::Ctx cpu;
  uint32_t* d_state = nullptr;  // 4 words
  uint8_t* d_tail = nullptr;    // 64 bytes
  uint8_t* d_seg = nullptr;     // 64 bytes: column segment descriptor, lane order {0}, spare
  uint8_t* d_stage = nullptr;   // staging for host updates
  size_t stage_cap = 0;
  uint64_t hashed = 0;          // bytes folded into d_state (whole blocks)
  uint8_t tail[64];
  uint32_t tail_len = 0;
  uint64_t total = 0;
  bool finalized = false;
  uint8_t digest[16];
};

extern "C" {

int qsmd5_init(int flags) {
  (void)flags;
  return guarded([] { return ensure_init(); });
}

int qsmd5_shutdown(void) {
  // In a child forked after init the HIP handles are the parent's: drop them
  // without a HIP call and without taking a lock another parent thread may
  // have held at fork() (the Dev objects and their memory are leaked; they go
  // with the child's exit).  Later calls in the child hash on the CPU.
  if (g_forked_child.load()) {
    g_init_state.store(0, std::memory_order_release);
    return 0;
  }
  if (t_call_depth > 0)
    return fail(-EINVAL, "qsmd5_shutdown: called from inside a qsmd5 call on this thread");
  try {
    std::unique_lock<std::shared_mutex> calls(g_calls);  // every call in flight has returned
    std::lock_guard<std::mutex> lk(g_init_mu);
    Runtime& r = rt();
    const bool own_hip = g_init_pid == getpid();
    int prev = -1;
    if (own_hip && !r.devs.empty() && hipGetDevice(&prev) != hipSuccess) {
      prev = -1;
      (void)hipGetLastError();
    }
    int rc = 0;
    for (Dev* d : r.devs) {  // no call is in flight: nothing else can hold d->mu
      if (own_hip && release_dev(*d) != 0 && rc == 0) rc = -EIO;
      delete d;
    }
    g_gpu_chain_bits.store(0, std::memory_order_relaxed);  // a re-init times its GPU afresh
    r.devs.clear();
    {
      Registry& R = registry();
      std::lock_guard<std::mutex> rl(R.mu);
      if (own_hip)
        for (const auto& kv : R.end_of)
          if (hipHostUnregister(reinterpret_cast<void*>(kv.first)) != hipSuccess) {
            (void)hipGetLastError();
            if (rc == 0) rc = -EIO;
          }
      R.base_of.clear();
      R.end_of.clear();
    }
    if (own_hip && prev >= 0) (void)hipSetDevice(prev);
    r.ready = false;
    r.init_rc = 0;
    r.init_msg.clear();
    r.shard_bytes = 0;
    g_init_state.store(0, std::memory_order_release);  // a forked child stays CPU-only
    if (rc) return fail(rc, "qsmd5_shutdown: a HIP release call failed (resources dropped anyway)");
    return 0;
  } catch (...) {
    return fail(-EIO, "qsmd5: internal error");
  }
}

int qsmd5_abi_version(void) { return QSMD5_ABI_VERSION; }

int qsmd5_set_log_callback(qsmd5_log_fn fn, void* user) {
  const LogSink* s = nullptr;
  if (fn) {
    s = new (std::nothrow) LogSink{fn, user};
    if (!s) return fail(-ENOMEM, "qsmd5: host allocation failed");
  }
  g_log_sink.store(s, std::memory_order_release);
  return 0;
}

int qsmd5_device_count(void) {
  if (g_forked_child.load(std::memory_order_relaxed)) return 0;  // the parent's HIP state
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

const char* qsmd5_strerror(int err) {
  switch (err) {
    case 0: return "success";
    case -EINVAL: return "invalid argument";
    case -ENODEV: return "no usable GPU";
    case -ENOMEM: return "out of memory";
    case -EIO: return "GPU runtime error";
    default: return "unknown error";
  }
}

const char* qsmd5_last_error(void) { return t_last_error.c_str(); }

void qsmd5_hex(const uint8_t digest[16], char out[33]) {
  static const char kHex[] = "0123456789abcdef";
  for (int i = 0; i < 16; ++i) {
    out[2 * i] = kHex[digest[i] >> 4];
    out[2 * i + 1] = kHex[digest[i] & 15];
  }
  out[32] = 0;
}

void qsmd5_base64(const uint8_t digest[16], char out[25]) {
  static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  char* o = out;
  for (int i = 0; i < 15; i += 3) {  // 5 full groups of 3 bytes
    const uint32_t v = (uint32_t)digest[i] << 16 | (uint32_t)digest[i + 1] << 8 | digest[i + 2];
    *o++ = kB64[v >> 18];
    *o++ = kB64[(v >> 12) & 63];
    *o++ = kB64[(v >> 6) & 63];
    *o++ = kB64[v & 63];
  }
  const uint32_t last = digest[15];  // 1 trailing byte -> 2 chars + "=="
  *o++ = kB64[last >> 2];
  *o++ = kB64[(last & 3) << 4];
  *o++ = '=';
  *o++ = '=';
  *o = 0;
}

int qsmd5_hash_batch_ex(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags) {
  return guarded([&] {
    if (n == 0) return 0;
    if (!chunks || !digests) return fail(-EINVAL, "qsmd5: NULL chunks/digests");
    if (n > 0xffffffffull) return fail(-EINVAL, "qsmd5: too many chunks");
    return hash_routed(chunks, n, digests, flags);
  });
}

int qsmd5_hash_batch(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16]) {
  return qsmd5_hash_batch_ex(chunks, n, digests, 0);
}

int qsmd5_hash_one(const void* ptr, uint64_t len, uint8_t digest[16]) {
  if (!digest) return fail(-EINVAL, "qsmd5: NULL digest");
  qsmd5_chunk c = {ptr, len};
  return qsmd5_hash_batch_ex(&c, 1, reinterpret_cast<uint8_t(*)[16]>(digest), 0);
}

int qsmd5_kernel_choice(size_t n) { return kernel_choice(n, false); }

int qsmd5_kernel_choice_ex(size_t n, int flags) {
  return kernel_choice(n, (flags & QSMD5_FLAG_ALIGNED16) != 0);
}

int qsmd5_hash_batch_device_async(const qsmd5_chunk* d_chunks, const uint32_t* d_order, size_t n,
                                  uint8_t (*d_digests)[16], void* hip_stream) {
  return qsmd5_hash_batch_device_async_ex(d_chunks, d_order, n, d_digests, hip_stream, 0);
}

int qsmd5_hash_batch_device_async_ex(const qsmd5_chunk* d_chunks, const uint32_t* d_order,
                                     size_t n, uint8_t (*d_digests)[16], void* hip_stream,
                                     int flags) {
  return guarded([&] {
    if (n == 0) return 0;
    if (!d_chunks || !d_digests) return fail(-EINVAL, "qsmd5: NULL device arrays");
    if (n > 0xffffffffull) return fail(-EINVAL, "qsmd5: too many chunks");
    if (int rc = ensure_init()) return rc;
    hipError_t e = qsmd5::launch_batch(
        d_chunks, d_order, (uint32_t)n, reinterpret_cast<uint32_t*>(d_digests),
        kernel_choice(n, (flags & QSMD5_FLAG_ALIGNED16) != 0), static_cast<hipStream_t>(hip_stream));
    if (e != hipSuccess) return hip_fail(e, "qsmd5 kernel launch");
    return 0;
  });
}

int qsmd5_alloc_pinned(size_t bytes, void** out) {
  return guarded([&] {
    if (!out) return fail(-EINVAL, "qsmd5: NULL out");
    *out = nullptr;
    if (int rc = ensure_init()) return rc;
    QS_HIP(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return 0;
  });
}

int qsmd5_free_pinned(void* ptr) {
  return guarded([&] {
    if (!ptr) return 0;
    if (int rc = ensure_init()) return rc;
    QS_HIP(hipHostFree(ptr));
    return 0;
  });
}


int qsmd5_register_host(void* ptr, size_t bytes) {
  return guarded([&] {
    if (!ptr || !bytes) return fail(-EINVAL, "qsmd5: NULL or empty range to register");
    if (int rc = ensure_init()) return rc;
    const uintptr_t page = 4096, u = reinterpret_cast<uintptr_t>(ptr);
    const uintptr_t lo = u & ~(page - 1), hi = (u + bytes + page - 1) & ~(page - 1);
    Registry& R = registry();
    std::lock_guard<std::mutex> lk(R.mu);
    if (R.base_of.count(u) || R.end_of.count(lo))
      return fail(-EINVAL, "qsmd5: range already registered, or starts in the first page of "
                           "one (registration covers whole 4 KiB pages)");
    // Heap buffers often share a boundary page with a neighbour (glibc hands
    // out adjacent chunks once its mmap threshold has grown), and a pool
    // registers them one by one.  HIP locks a page that is already locked
    // again; if it refuses, say why instead of a generic -EIO.
    auto it = R.end_of.lower_bound(hi);
    const bool overlaps = it != R.end_of.begin() && std::prev(it)->second > lo;
    const hipError_t e = hipHostRegister(reinterpret_cast<void*>(lo), hi - lo, hipHostRegisterDefault);
    if (e != hipSuccess) {
      if (!overlaps) return hip_fail(e, "hipHostRegister");
      (void)hipGetLastError();
      return fail(-EINVAL, std::string("qsmd5: range shares a page with a range already registered, "
                                       "and HIP refused it: ") + hipGetErrorString(e));
    }
    R.base_of[u] = lo;
    R.end_of[lo] = hi;
    return 0;
  });
}

int qsmd5_unregister_host(void* ptr) {
  return guarded([&] {
    if (!ptr) return fail(-EINVAL, "qsmd5: NULL pointer to unregister");
    if (int rc = ensure_init()) return rc;
    Registry& R = registry();
    std::lock_guard<std::mutex> lk(R.mu);
    auto it = R.base_of.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == R.base_of.end())
      return fail(-EINVAL, "qsmd5: pointer was not registered by qsmd5_register_host");
    const uintptr_t base = it->second;
    R.base_of.erase(it);
    R.end_of.erase(base);
    QS_HIP(hipHostUnregister(reinterpret_cast<void*>(base)));
    return 0;
  });
}

constexpr size_t kMaxRefPartId = 65535;  // uint16_t part ids, TransferHandle.h:50

int qsmd5_plan_parts(uint64_t file_size, uint64_t buf_size, uint64_t min_part, uint64_t threshold,
                     uint64_t range_begin, qsmd5_part* parts, size_t cap, size_t* nparts) {
  if (!nparts) return fail(-EINVAL, "qsmd5: NULL nparts");
  if (buf_size == 0) return fail(-EINVAL, "qsmd5: buffer size must be > 0");
  std::vector<qsmd5_part> v;
  auto add = [&](uint64_t id, uint64_t off, uint64_t sz) {
    qsmd5_part p;
    p.part_number = (uint32_t)id;
    p.reserved = 0;
    p.offset = range_begin + off;
    p.size = sz;
    v.push_back(p);
  };
  // The reference's part id is uint16_t (Part, TransferHandle.h:50,86; the
  // PartIdToPartMap key, :45): part 65 536 narrows to id 0, part 65 537 to
  // id 1, whose map insert then fails (TransferHandle.cpp:252-256) and that
  // part is silently dropped from the upload.  No numbering can reproduce
  // such an upload, so a plan of more than 65 535 parts is refused (before it
  // is built) with the count reported in *nparts.
  if (file_size >= threshold) {
    const uint64_t count = file_size / buf_size + (file_size % buf_size ? 1 : 0);
    if (count > kMaxRefPartId) {
      *nparts = (size_t)count;
      return fail(-EINVAL, "qsmd5: " + std::to_string(count) + " parts: the reference numbers "
                           "parts with uint16_t ids (TransferHandle.h:50), so parts above 65535 "
                           "would wrap and collide; use a larger buffer size");
    }
  }
  try {
    if (file_size < threshold) {
      add(1, 0, file_size);  // single PutObject (QSTransferManager.cpp:543-546)
    } else {
      const uint64_t count = file_size / buf_size + (file_size % buf_size ? 1 : 0);
      const uint64_t last = file_size - (count - 1) * buf_size;
      // Averaging needs a previous full part to merge with.
      const bool avg = last < min_part && count >= 2;
      const uint64_t full = avg ? count - 1 : count;
      for (uint64_t i = 1; i < full; ++i) add(i, (i - 1) * buf_size, buf_size);
      if (!avg) {
        add(count, (count - 1) * buf_size, last);
      } else {
        const uint64_t sz1 = (last + buf_size) / 2;
        const uint64_t sz2 = last + buf_size - sz1;
        add(full, (full - 1) * buf_size, sz1);
        add(count, (full - 1) * buf_size + sz1, sz2);
      }
    }
  } catch (...) {
    return fail(-ENOMEM, "qsmd5: host allocation failed");
  }
  *nparts = v.size();
  if (parts && cap) memcpy(parts, v.data(), std::min(cap, v.size()) * sizeof(qsmd5_part));
  return cap && cap < v.size() ? fail(-EINVAL, "qsmd5: parts capacity too small") : 0;
}

int qsmd5_hash_parts(const void* file, const qsmd5_part* parts, size_t n, uint8_t (*digests)[16]) {
  return guarded([&] {
    if (n == 0) return 0;
    if (!parts || !digests) return fail(-EINVAL, "qsmd5: NULL parts/digests");
    std::vector<qsmd5_chunk> c(n);
    const uint64_t base = parts[0].offset;
    for (size_t i = 0; i < n; ++i) {
      if (parts[i].offset < base) return fail(-EINVAL, "qsmd5: part offset before parts[0]");
      c[i].ptr = static_cast<const uint8_t*>(file) + (parts[i].offset - base);
      c[i].len = parts[i].size;
    }
    return qsmd5_hash_batch_ex(c.data(), n, digests, 0);
  });
}

int qsmd5_etag_matches(const uint8_t digest[16], const char* etag) {
  if (!digest || !etag) return fail(-EINVAL, "qsmd5: NULL digest/etag");
  size_t n = strlen(etag);
  const char* p = etag;
  if (n >= 2 && p[0] == '"' && p[n - 1] == '"') {
    ++p;
    n -= 2;
  }
  if (n != 32) return fail(-EINVAL, "qsmd5: ETag is not a 32-hex-digit MD5");
  auto nib = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  int match = 1;
  for (int i = 0; i < 16; ++i) {
    const int hi = nib(p[2 * i]), lo = nib(p[2 * i + 1]);
    if (hi < 0 || lo < 0) return fail(-EINVAL, "qsmd5: ETag is not a 32-hex-digit MD5");
    if (((hi << 4) | lo) != digest[i]) match = 0;
  }
  return match;
}

int qsmd5_verify_etag(const void* ptr, uint64_t len, const char* etag) {
  // validate the ETag's form before spending a GPU pass on it
  uint8_t d[16] = {0};
  if (int rc = qsmd5_etag_matches(d, etag); rc < 0) return rc;
  if (int rc = qsmd5_hash_one(ptr, len, d)) return rc;
  return qsmd5_etag_matches(d, etag);
}

int qsmd5_last_backend(void) { return t_last_backend; }

int qsmd5_route(const qsmd5_chunk* chunks, size_t n, int flags) {
  if (n && !chunks) return fail(-EINVAL, "qsmd5: NULL chunks");
  return guarded([&] {
    if (cpu_is_faster(chunks, n, flags)) return QSMD5_BACKEND_CPU;
    return plan_split(chunks, n, flags).empty() ? QSMD5_BACKEND_GPU : QSMD5_BACKEND_SPLIT;
  });
}

int qsmd5_get_rates(qsmd5_rates* out) {
  if (!out) return fail(-EINVAL, "qsmd5: NULL rates");
  return guarded([&] {
    memset(out, 0, sizeof(*out));
    const CpuRates& c = cpu_rates();
    const bool cpu_env = env_gibs("QSMD5_CPU_GIBS") > 0;
    bool gpu_measured = false;
    out->gpu_chain_gibs = gpu_chain_gibs(&gpu_measured);
    out->cpu_chain_gibs = cpu_gibs_per_thread();
    out->cpu_lane_thread_gibs = c.lane_thread;
    out->link_gibs = link_gibs();
    out->d2h_gibs = kD2HGiBs;
    out->gpu_call_ms = kGpuCallMs;
    out->cpu_threads = (int)cpu_threads();
    out->source = (c.measured ? QSMD5_RATE_CPU_MEASURED : 0) | (cpu_env ? QSMD5_RATE_CPU_ENV : 0) |
                  (gpu_measured ? QSMD5_RATE_GPU_MEASURED : 0) |
                  (env_gibs("QSMD5_GPU_CHAIN_GIBS") > 0 ? QSMD5_RATE_GPU_ENV : 0);
    return 0;
  });
}

int qsmd5_get_stats(qsmd5_stats* out) {
  if (!out) return fail(-EINVAL, "qsmd5: NULL stats");
  memset(out, 0, sizeof(*out));
  out->gpu_batches = g_gpu_batches.load();
  out->cpu_batches = g_cpu_batches.load();
  out->fallbacks = g_fallbacks.load();
  out->gpu_chunks = g_gpu_chunks.load();
  out->cpu_chunks = g_cpu_chunks.load();
  out->gpu_lost = g_gpu_lost.load() ? 1 : 0;
  out->inits = g_inits.load();
  return 0;
}

int qsmd5_last_timing(double* wall_ms, double* kernel_ms) {
  Runtime& r = rt();
  std::lock_guard<std::mutex> lk(r.timing_mu);
  if (wall_ms) *wall_ms = r.last_wall_ms;
  if (kernel_ms) *kernel_ms = r.last_kernel_ms;
  return 0;
}

int qsmd5_synth_fill_lcg(void* d_base, uint64_t stride, uint64_t len, uint32_t seed0,
                         uint32_t nchunks, void* hip_stream) {
  return guarded([&] {
    if (!d_base && len && nchunks) return fail(-EINVAL, "qsmd5: NULL base");
    if (int rc = ensure_init()) return rc;
    hipError_t e = qsmd5::launch_lcg_fill(static_cast<uint8_t*>(d_base), stride, len, seed0,
                                          nchunks, static_cast<hipStream_t>(hip_stream));
    if (e != hipSuccess) return hip_fail(e, "qsmd5 fill launch");
    return 0;
  });
}

// ---- streaming context -------------------------------------------------------

int qsmd5_ctx_create(qsmd5_ctx** out) {
  return guarded([&] {
    if (!out) return fail(-EINVAL, "qsmd5: NULL out");
    *out = nullptr;
    Backend b = kAuto;
    if (int rc = requested_backend(0, &b)) return rc;
    if (b != kGpu) {
      qsmd5_ctx* c = new qsmd5_ctx;
      c->on_cpu = true;
      *out = c;
      return 0;
    }
    if (int rc = ensure_init()) return rc;
    qsmd5_ctx* c = new qsmd5_ctx;
    const uint32_t init[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    hipError_t e = hipMalloc(&c->d_state, 16);
    if (e == hipSuccess) e = hipMalloc(&c->d_tail, 64);
    if (e == hipSuccess) e = hipMalloc(&c->d_seg, 64);
    if (e == hipSuccess) e = hipMemset(c->d_seg, 0, 64);  // lane order word = chunk 0
    if (e == hipSuccess) e = hipMemcpy(c->d_state, init, 16, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      qsmd5_ctx_destroy(c);
      return hip_fail(e, "qsmd5_ctx_create");
    }
    *out = c;
    return 0;
  });
}

// The reference MD5 is a value type (MD5.h:51-93 declares no copy members, and
// operator<< takes it by value, MD5.h:61): a copy carries the running state,
// and the two then hash on independently.  A GPU context's state is copied
// device to device; its pending tail bytes live on the host.
int qsmd5_ctx_copy(const qsmd5_ctx* src, qsmd5_ctx** out) {
  return guarded([&] {
    if (!src || !out) return fail(-EINVAL, "qsmd5: NULL ctx/out");
    *out = nullptr;
    qsmd5_ctx* c = new qsmd5_ctx;
    c->on_cpu = src->on_cpu;
    c->failed = src->failed;
    c->cpu = src->cpu;
    c->hashed = src->hashed;
    memcpy(c->tail, src->tail, sizeof c->tail);
    c->tail_len = src->tail_len;
    c->total = src->total;
    c->finalized = src->finalized;
    memcpy(c->digest, src->digest, sizeof c->digest);
    if (src->on_cpu) {
      *out = c;
      return 0;
    }
    if (int rc = ensure_init()) {
      delete c;
      return rc;
    }
    std::lock_guard<std::mutex> lk(primary().mu);  // src's updates run under it
    hipStream_t s = primary().compute[0];
    hipError_t e = hipMalloc(&c->d_state, 16);
    if (e == hipSuccess) e = hipMalloc(&c->d_tail, 64);
    if (e == hipSuccess) e = hipMalloc(&c->d_seg, 64);
    if (e == hipSuccess) e = hipMemsetAsync(c->d_seg, 0, 64, s);
    if (e == hipSuccess) e = hipMemcpyAsync(c->d_state, src->d_state, 16, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      qsmd5_ctx_destroy(c);
      return hip_fail(e, "qsmd5_ctx_copy");
    }
    *out = c;
    return 0;
  });
}

void qsmd5_ctx_destroy(qsmd5_ctx* c) {
  if (!c) return;
  CallScope call;  // its device buffers are freed before a shutdown tears HIP down
  if (c->d_state) (void)hipFree(c->d_state);
  if (c->d_tail) (void)hipFree(c->d_tail);
  if (c->d_seg) (void)hipFree(c->d_seg);
  if (c->d_stage) (void)hipFree(c->d_stage);
  delete c;
}

static int ctx_blocks(qsmd5_ctx* c, const uint8_t* p, uint64_t nblk, bool on_device) {
  Dev& r = primary();
  hipStream_t s = r.compute[0];
  const uint8_t* src = p;
  if (!on_device) {
    const uint64_t bytes = nblk * 64;
    if (bytes > c->stage_cap) {
      if (c->d_stage) (void)hipFree(c->d_stage);
      c->d_stage = nullptr;
      c->stage_cap = 0;
      QS_HIP(hipMalloc(&c->d_stage, bytes));
      c->stage_cap = bytes;
    }
    QS_HIP(hipMemcpyAsync(c->d_stage, p, bytes, hipMemcpyHostToDevice, s));
    src = c->d_stage;
  }
  // The blocks run as one column of a one-lane column batch: the latency
  // kernel's producer/consumer chain (~1207 cycles/block) instead of a lone
  // lane doing its own loads (64 MiB in 1 MiB updates: 1.0 s -> see
  // profiles/r01_stream_ctx_rate.log).  The segment's total length is set one
  // block past the update, so the chain always parks its state in d_state and
  // never finalises; qsmd5_ctx_final runs the tail.
  while (nblk) {
    const uint64_t step = std::min<uint64_t>(nblk, 0x40000000ull);
    const qsmd5_chunk seg = {src, c->hashed + step * 64 + 64};
    QS_HIP(hipMemcpyAsync(c->d_seg, &seg, sizeof(seg), hipMemcpyHostToDevice, s));
    QS_HIP(qsmd5::launch_column(c->d_seg, reinterpret_cast<const uint32_t*>(c->d_seg + 16), 1,
                                reinterpret_cast<uint32_t*>(c->d_seg + 32), c->hashed, step * 64,
                                c->d_state, s));
    QS_HIP(wait_stream(r, s, gpu_wait_est_ms(step * 64, on_device ? 0 : step * 64)));  // seg lives on this frame
    src += step * 64;
    c->hashed += step * 64;
    nblk -= step;
  }
  return 0;
}

// CPU context: host pieces directly; device pieces through a bounded host copy.
static int ctx_update_cpu(qsmd5_ctx* c, const void* ptr, uint64_t len) {
  int owner = -1;
  if (qsmd5_device_count() > 0 && classify(ptr, &owner) == kDeviceMem) {
    if (g_gpu_lost.load())
      return fail(-EIO, "qsmd5: the GPU context is lost; a device-resident piece cannot be read");
    constexpr uint64_t kPiece = 8ull << 20;
    std::vector<uint8_t> buf((size_t)std::min(len, kPiece));
    for (uint64_t off = 0; off < len; off += kPiece) {
      const uint64_t k = std::min(kPiece, len - off);
      QS_HIP(hipMemcpy(buf.data(), static_cast<const uint8_t*>(ptr) + off, k, hipMemcpyDeviceToHost));
      c->cpu.update(buf.data(), k);
    }
    return 0;
  }
  c->cpu.update(ptr, len);
  return 0;
}

int qsmd5_ctx_update(qsmd5_ctx* c, const void* ptr, uint64_t len) {
  return guarded([&] {
    if (!c) return fail(-EINVAL, "qsmd5: NULL ctx");
    if (c->finalized) return fail(-EINVAL, "qsmd5: update after final");
    if (c->failed) return fail(-EIO, "qsmd5: an earlier update of this context failed");
    if (len == 0) return 0;
    if (!ptr) return fail(-EINVAL, "qsmd5: NULL ptr with non-zero len");
    if (c->on_cpu) {
      // a device piece copied only in part would leave a hole: fail the context
      const int rc = ctx_update_cpu(c, ptr, len);
      if (rc) c->failed = true;
      return rc;
    }
    if (int rc = ensure_init()) return rc;
    std::lock_guard<std::mutex> lk(primary().mu);
    int owner = -1;
    const bool dev = classify(ptr, &owner) == kDeviceMem;
    if (dev && owner != primary().device)
      return fail(-EINVAL, "qsmd5: update data lives on GPU " + std::to_string(owner) +
                               ", not on the primary bound GPU");
    const uint8_t* p = static_cast<const uint8_t*>(ptr);
    uint64_t left = len;
    // From here a failure leaves d_state, tail and total out of step: mark the
    // context failed (every exit below that returns nonzero passes here).
    struct FailOnError {
      qsmd5_ctx* c;
      bool ok = false;
      ~FailOnError() {
        if (!ok) c->failed = true;
      }
    } guard{c};
    c->total += len;
    if (c->tail_len) {
      const uint32_t take = (uint32_t)std::min<uint64_t>(64 - c->tail_len, left);
      if (dev) {
        QS_HIP(hipMemcpy(c->tail + c->tail_len, p, take, hipMemcpyDeviceToHost));
      } else {
        memcpy(c->tail + c->tail_len, p, take);
      }
      c->tail_len += take;
      p += take;
      left -= take;
      if (c->tail_len == 64) {
        if (int rc = ctx_blocks(c, c->tail, 1, false)) return rc;
        c->tail_len = 0;
      }
    }
    const uint64_t nblk = left / 64;
    if (nblk) {
      if (int rc = ctx_blocks(c, p, nblk, dev)) return rc;
      p += nblk * 64;
      left -= nblk * 64;
    }
    if (left) {
      if (dev) {
        QS_HIP(hipMemcpy(c->tail, p, left, hipMemcpyDeviceToHost));
      } else {
        memcpy(c->tail, p, left);
      }
      c->tail_len = (uint32_t)left;
    }
    guard.ok = true;
    return 0;
  });
}

int qsmd5_ctx_final(qsmd5_ctx* c, uint8_t digest[16]) {
  return guarded([&] {
    if (!c || !digest) return fail(-EINVAL, "qsmd5: NULL ctx/digest");
    if (c->failed) return fail(-EIO, "qsmd5: an earlier update of this context failed");
    if (!c->finalized && c->on_cpu) {
      c->cpu.final(c->digest);
      c->finalized = true;
    }
    if (!c->finalized) {
      if (int rc = ensure_init()) return rc;
      std::lock_guard<std::mutex> lk(primary().mu);
      hipStream_t s = primary().compute[0];
      QS_HIP(hipMemcpyAsync(c->d_tail, c->tail, 64, hipMemcpyHostToDevice, s));
      QS_HIP(qsmd5::launch_final(c->d_state, c->d_tail, c->tail_len, c->total, s));
      QS_HIP(hipMemcpyAsync(c->digest, c->d_state, 16, hipMemcpyDeviceToHost, s));
      QS_HIP(hipStreamSynchronize(s));
      c->finalized = true;
    }
    memcpy(digest, c->digest, 16);
    return 0;
  });
}

}  // extern "C"
