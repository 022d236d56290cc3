// qsfs-fuse_amd/csrc/qsmd5_rt_device.cpp -- errors and the log sink, binding the GPU(s),
// lazy init and fork awareness, memory classification, the kernel choice
// (the runtime's units: qsmd5_rt.h).
#include "qsmd5_rt.h"

namespace qsmd5 {
namespace rt {

thread_local std::string t_last_error;
char g_pinned_sync;

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
  (void)hipGetLastError();  // consumed here: a later launch's status must be its own
  std::string s = std::string(what) + ": " + hipGetErrorString(e);
  return fail(e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation ? -ENOMEM : -EIO, s);
}


uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  unsigned long long x = strtoull(v, &end, 0);
  return (end && *end == 0) ? (uint64_t)x : dflt;
}


Runtime& rt() {
  static Runtime* r = new Runtime;  // intentionally leaked: no teardown order issues
  return *r;
}

Dev& primary() { return *rt().devs[0]; }

// Lazy-init state (qsmd5_rt.h).
std::mutex g_init_mu;
std::atomic<int> g_init_state{0};
pid_t g_init_pid = 0;                     // the process that owns the HIP state
std::atomic<bool> g_forked_child{false};  // set in a child forked after init

static void on_fork_child() {
  // HIP state does not survive fork(): a child of a process in which this
  // library ever initialised HIP (even if it shut its own runtime down since:
  // HIP itself stays up) must not touch the GPU (it hashes on the CPU under
  // auto routing, see ensure_init).  Registered at the first init.
  if (g_init_pid != 0) g_forked_child.store(true);
}

// Devices to bind: QSMD5_DEVICES = "all" or a comma list of ordinals (an
// ordinal may repeat: two contexts on one GPU, used by the tests to exercise
// sharding on a one-GPU box); otherwise the single QSMD5_DEVICE / current one.
static int parse_devices(int n, std::vector<int>* out) {
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

static int init_dev(Dev& d, int device) {
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
  d.nread_slots = (int)std::min<uint64_t>(kMaxReadSlots, std::max<uint64_t>(1, env_u64("QSMD5_READ_SLOTS", 4)));
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
  for (ReadSlot& rs : d.read_slot) {
    for (hipStream_t* s : {&rs.stream, &rs.copy})
      if (*s) {
        chk(hipStreamSynchronize(*s));
        chk(hipStreamDestroy(*s));
        *s = nullptr;
      }
    for (hipEvent_t* e : rs.events())
      if (*e) {
        chk(hipEventDestroy(*e));
        *e = nullptr;
      }
  }
  for (hipEvent_t* e : {&d.ev_meta, &d.ev_first, &d.ev_last, &d.ev_done})
    if (*e) {
      chk(hipEventDestroy(*e));
      *e = nullptr;
    }
  std::vector<DevBuf*> dbufs = {&d.d_meta, &d.d_dig, &d.d_staging, &d.d_state};
  std::vector<HostPinned*> hbufs = {&d.h_meta, &d.h_dig};
  for (ReadSlot& rs : d.read_slot) {
    for (DevBuf* b : {&rs.d_read, &rs.d_meta, &rs.d_state, &rs.d_dig}) dbufs.push_back(b);
    for (HostPinned* b : {&rs.h_read, &rs.h_meta}) hbufs.push_back(b);
  }
  for (DevBuf* b : dbufs)
    if (b->p) {
      chk(hipFree(b->p));
      b->p = nullptr;
      b->cap = 0;
    }
  for (HostPinned* b : hbufs)
    if (b->p) {
      chk(hipHostFree(b->p));
      b->p = nullptr;
      b->cap = 0;
    }
  d.read_busy = 0;
  d.device = -1;
  return bad;
}

std::atomic<int> g_inits{0};  // do_init runs (qsmd5_stats.inits)

static void do_init() {
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
  prewarm_read_slot(*r.devs[0]);
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


// Device memory reports its GPU ordinal in *owner (host memory: -1).
// *hip_known: HIP knows the pointer (device, pinned or registered host memory).
MemKind classify(const void* p, int* owner, bool* hip_known) {
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


Registry& registry() {
  static Registry* r = new Registry;
  return *r;
}


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

}  // namespace rt
}  // namespace qsmd5
