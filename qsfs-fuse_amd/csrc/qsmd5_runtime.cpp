// qsfs-fuse_amd/csrc/qsmd5_runtime.cpp -- the C-ABI of include/qsmd5.h.
//
// Every entry point is extern "C", catches everything, and reports failure as
// a negative errno (never an empty digest).  Hashing runs on the gfx950
// kernels (md5_kernels.hip) or on the library's own CPU MD5 (md5_cpu.h),
// chosen per call by size, with a CPU fallback when the GPU fails (SURVEY.md
// §8b, §5).  The runtime behind these entry points is in the qsmd5_rt_*.cpp
// units (their interface: qsmd5_rt.h):
//   - qsmd5_rt_device.cpp: the bound GPU(s), their streams, scratch and
//     staging ring; lazy, fork-aware init; which memory a pointer is;
//   - qsmd5_rt_staging.cpp: one batch on one GPU.  Host-resident batches (the
//     qsfs case: parts in pooled host buffers, ResourceManager.cpp:53-77) are
//     cut into slices, copied H2D into ring regions on copy streams and hashed
//     by launches on compute streams, the order kept by the calling thread;
//     staged chunks are packed with a 4 KiB + 256 B skew so that equal-size
//     parts never sit at a power-of-two stride (a power-of-two stride sends
//     every lane's request to the same HBM channel);
//   - qsmd5_rt_route.cpp: group commit of concurrent callers, the backend
//     routing and its cost model, the CPU backend, split batches.
// This file holds the entry points and the streaming context (MD5 class).
#include "qsmd5_rt.h"

using namespace qsmd5::rt;

// ----------------------------------------------------------------------------
// Streaming context (MD5 class).  One stream is one serial chain, which a host
// core runs ~6x faster than one GPU lane (the routing rule, qsmd5_rt_route.cpp), so under
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
    // New calls wait at the gate (CallScope) from here until this returns, so
    // calls that keep overlapping cannot starve the exclusive lock below.
    {
      std::lock_guard<std::mutex> gl(g_gate_mu);
      g_shutdown_pending.fetch_add(1);
    }
    struct Reopen {
      ~Reopen() {
        {
          std::lock_guard<std::mutex> gl(g_gate_mu);
          g_shutdown_pending.fetch_sub(1);
        }
        g_gate_cv.notify_all();
      }
    } reopen;
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
    release_read_cache();
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
    pinned_handed_out();
    return 0;
  });
}

int qsmd5_free_pinned(void* ptr) {
  return guarded([&] {
    if (!ptr) return 0;
    if (int rc = ensure_init()) return rc;
    pinned_handed_back();
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

int qsmd5_hash_read(const uint64_t* lens, size_t n, qsmd5_read_fn read, void* user, uint64_t staging_bytes,
                    uint8_t (*digests)[16], int flags) {
  return guarded([&] { return hash_read_routed(lens, n, read, user, staging_bytes, digests, flags); });
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
    if ((flags & QSMD5_FLAG_BACKGROUND) && qsmd5_device_count() > 0 && !g_gpu_lost.load())
      return QSMD5_BACKEND_GPU;  // latency hidden: the cores stay the daemon's
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

int qsmd5_get_cpu_efficiency(double* out) {
  if (!out) return fail(-EINVAL, "qsmd5: NULL out");
  *out = cpu_efficiency();
  return 0;
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

// A device piece longer than what is left of its HIP allocation: reading it
// (kernel or read-back copy) would fault the GPU (Classifier::overruns_allocation).
static bool device_piece_overruns(const void* ptr, uint64_t len, int owner) {
  uintptr_t lo = 0;
  size_t size = 0;
  const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
  return Classifier::hip_range(a, owner, &lo, &size) && len > size - (a - lo);
}

// CPU context: host pieces directly; device pieces through a bounded host copy.
static int ctx_update_cpu(qsmd5_ctx* c, const void* ptr, uint64_t len) {
  int owner = -1;
  if (qsmd5_device_count() > 0 && classify(ptr, &owner) == kDeviceMem) {
    if (g_gpu_lost.load())
      return fail(-EIO, "qsmd5: the GPU context is lost; a device-resident piece cannot be read");
    if (device_piece_overruns(ptr, len, owner))
      return fail(-EINVAL, "qsmd5: device piece runs past the end of its allocation");
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
      // a device piece copied only in part would leave a hole: fail the
      // context (a piece refused up front, -EINVAL, changed nothing)
      const int rc = ctx_update_cpu(c, ptr, len);
      if (rc && rc != -EINVAL) c->failed = true;
      return rc;
    }
    if (int rc = ensure_init()) return rc;
    std::lock_guard<std::mutex> lk(primary().mu);
    int owner = -1;
    const bool dev = classify(ptr, &owner) == kDeviceMem;
    if (dev && owner != primary().device)
      return fail(-EINVAL, "qsmd5: update data lives on GPU " + std::to_string(owner) +
                               ", not on the primary bound GPU");
    if (dev && device_piece_overruns(ptr, len, owner))
      return fail(-EINVAL, "qsmd5: device piece runs past the end of its allocation");
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
