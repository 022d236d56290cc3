// tests/cpp/multipart_harness.cpp -- QSTransferManager::DoMultiPartUpload with
// the batch pre-hash, end to end.
//
// Builds a file the way qsfs holds one after File::Flush loaded it: its bytes
// live in many separately allocated pages of assorted sizes (Page,
// src/data/Page.h; qsfs pages follow the FUSE write sizes), keyed by offset.
// Then it runs the reference's upload loop through the drop-in helper
// qsmd5::upload_parts_prehashed (qsfs-fuse_amd/host/qsfs_multipart.hpp):
//   - parts sliced as PrepareUpload does (qsmd5_plan_parts, QSTransferManager.cpp:475-550);
//   - a blocking pool of transfer buffers (ResourceManager, ResourceManager.cpp:53-77:
//     -n buffers of -b MiB, TransferManager.h:74-86; qsfs's default is 5 x 10 MiB);
//   - each part gathered from the pages into a pool buffer by a ReadNoLoad
//     restatement (File.cpp:308-375: the pages intersecting [off, off + len),
//     copied piece by piece; bytes no page holds are a short read);
//   - one qsmd5_hash_batch_ex(QSMD5_FLAG_HOST) per wave;
//   - each part's hex digest handed to the "uploader" (UploadMultipart's
//     SetContentMD5, QSClient.cpp:369-371), which records it, optionally after
//     a simulated network time (--upload-ms), on this thread (the reference's
//     sync path, File::Flush -> UploadFile(async = false)) or on an executor
//     (--async=E threads: its async path, QSTransferManager.cpp:654-659).
// --files=F flushes F files at once from F threads through ONE shared pool,
// as qsfs's FUSE threads do; a watchdog reports a deadlock (every waiter
// blocked and no pool or upload progress for --deadlock-s seconds) and exits
// with status 3.  --naive-wave=W replaces the helper with the hold-and-wait
// flow round 3's INTEGRATION.md sketched (W blocking Acquire calls before the
// wave is hashed): the negative control that deadlocks under the same load.
// --staged replaces the waves with the pool-free pre-hash:
// qsmd5::upload_parts_staged pulls every part through qsmd5_hash_read in column
// windows (--staging=BYTES budget, --wave-parts=W parts per call, default the
// whole file), then runs the reference's loop one pool buffer at a time.
// --reference-loop replaces all of it with the reference's own flush loop, the
// baseline the staged binding is timed against: per part,
// Acquire one pool buffer (blocking), ReadNoLoad into it, md5() of the
// IOStream over its first part.size bytes with the REFERENCE's MD5.cpp
// (oracle/_ref/libref_md5.so, ref_md5_iostream = md5(shared_ptr<iostream>),
// MD5.cpp:341-349 -- test infrastructure, dlopen'd only in this mode), then the
// upload; on this thread (File::Flush's async = false) or, with --async=E, md5
// and upload both on the executor, as UploadMultipart computes the digest
// inside MultipleUploadWrapper (QSTransferManager.cpp:602-673, QSClient.cpp:369-371).
// --backends=B1,B2,..: pass k runs under QSMD5_BACKEND = B(k mod n), so the
// backends are compared within one process.
// --read-parallel: the pre-hash's reads on QSMD5_READ_THREADS library threads
// (QSMD5_FLAG_READ_PARALLEL; this file's page gather is thread-safe).
// File content: part-aligned mode (--aligned) makes part i = LCG(12345 + i),
// the parts of tests/golden/batch_10MiB.json, for every file; otherwise file f
// is one LCG(seed + f) stream.  Prints one JSON object with the digests in
// part order and where the time went; tests/test_gpu_multipart.py and
// tests/test_multipart_cpu.py check the digests.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <dirent.h>
#include <dlfcn.h>
#include <limits.h>
#include <pthread.h>
#include <sched.h>
#include <sys/resource.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../qsfs-fuse_amd/host/qsfs_multipart.hpp"

namespace {

using clock_type = std::chrono::steady_clock;

void lcg(uint32_t seed, uint8_t* out, uint64_t n) {
  uint32_t x = seed;
  for (uint64_t i = 0; i < n; ++i) {
    x = x * 1103515245u + 12345u;
    out[i] = (uint8_t)((x >> 16) & 0xff);
  }
}

// The file's pages: offset -> bytes (each its own heap allocation).
struct PagedFile {
  std::map<uint64_t, std::vector<char>> pages;
  uint64_t size = 0;

  // File::ReadNoLoad: gather [off, off + len) into buf; returns bytes found.
  size_t read(uint64_t off, size_t len, char* buf) const {
    memset(buf, 0, len);
    size_t got = 0;
    auto it = pages.upper_bound(off);
    if (it != pages.begin()) --it;
    uint64_t pos = off;
    const uint64_t end = off + len;
    for (; it != pages.end() && pos < end; ++it) {
      const uint64_t po = it->first, pe = po + it->second.size();
      if (pe <= pos) continue;
      if (po > pos) break;  // a hole: the rest is unloaded
      const uint64_t take = std::min(pe, end) - pos;
      memcpy(buf + (pos - off), it->second.data() + (pos - po), take);
      got += take;
      pos += take;
    }
    return got;
  }
};

void build_file(PagedFile* file, uint64_t size, bool aligned, uint64_t buf, uint32_t seed) {
  file->size = size;
  std::vector<uint8_t> all(size);
  if (aligned) {  // parts are independent: fill them on up to 16 threads
    const uint64_t nparts = (size + buf - 1) / buf;
    const unsigned nt = (unsigned)std::min<uint64_t>(nparts, std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        for (uint64_t p = t; p < nparts; p += nt)
          lcg(12345u + (uint32_t)p, all.data() + p * buf, std::min(buf, size - p * buf));
      });
    for (auto& x : th) x.join();
  } else {
    lcg(seed, all.data(), size);
  }
  std::mt19937_64 rng(seed);
  for (uint64_t off = 0; off < size;) {
    const uint64_t len = std::min<uint64_t>(size - off, 1024 + rng() % (3u << 20));
    file->pages.emplace(off, std::vector<char>(all.begin() + off, all.begin() + off + len));
    off += len;
  }
}

std::atomic<int64_t> g_progress_ns{0};  // last pool or upload event (watchdog)
void progress() {
  g_progress_ns.store(clock_type::now().time_since_epoch().count(), std::memory_order_relaxed);
}

// ResourceManager restated with a watchdog's view: BlockingPool (blocking
// acquire, try_acquire, release) plus a count of threads blocked in acquire.
class WatchedPool {
 public:
  typedef qsmd5::PoolBuffer buffer_type;
  explicit WatchedPool(std::vector<qsmd5::PoolBuffer> b) : pool_(std::move(b)) {}
  buffer_type acquire() {
    buffer_type b;
    if (pool_.try_acquire(&b)) {
      progress();
      return b;
    }
    waiting_.fetch_add(1);
    b = pool_.acquire();
    waiting_.fetch_sub(1);
    progress();
    return b;
  }
  bool try_acquire(buffer_type* out) {
    const bool ok = pool_.try_acquire(out);
    if (ok) progress();
    return ok;
  }
  void release(const buffer_type& b) {
    pool_.release(b);
    if (b.data) progress();
  }
  void shutdown() { pool_.shutdown(); }
  int waiting() const { return waiting_.load(); }
  size_t free_count() { return pool_.free_count(); }
  static char* data(const buffer_type& b) { return b.data; }
  static size_t size(const buffer_type& b) { return b.size; }

 private:
  qsmd5::BlockingPool pool_;
  std::atomic<int> waiting_{0};
};

// The transfer manager's executor (ThreadPool, TransferManager.cpp:55-60):
// E threads running submitted upload tasks in order.
class Executor {
 public:
  explicit Executor(int n) {
    for (int i = 0; i < n; ++i)
      th_.emplace_back([this] {
        pthread_setname_np(pthread_self(), "executor");
        loop();
      });
  }
  ~Executor() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> th_;
  bool stop_ = false;
};

// Parts of one file still being uploaded on the executor.
struct InFlight {
  std::mutex mu;
  std::condition_variable cv;
  size_t n = 0;
  void add() {
    std::lock_guard<std::mutex> lk(mu);
    ++n;
  }
  void done() {
    // notify under the lock: the waiter may destroy this object as soon as it
    // sees n == 0 (TSan caught the notify racing the destructor)
    std::lock_guard<std::mutex> lk(mu);
    --n;
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return n == 0; });
  }
};

// CPU seconds (user + system) this process has used so far, all threads.
double cpu_seconds() {
  struct rusage ru;
  getrusage(RUSAGE_SELF, &ru);
  return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
}

// Busy threads of this process so far: "name:cpu_s" for each thread that
// used more than 50 ms (/proc/self/task/*/stat utime + stime), to see which
// thread a backend keeps busy (the runtime's caller, HIP's own threads).
std::string busy_threads() {
  std::string out;
  const long hz = sysconf(_SC_CLK_TCK);
  DIR* dir = opendir("/proc/self/task");
  if (!dir) return out;
  while (struct dirent* de = readdir(dir)) {
    if (de->d_name[0] < '0' || de->d_name[0] > '9') continue;
    const std::string path = std::string("/proc/self/task/") + de->d_name + "/stat";
    FILE* f = fopen(path.c_str(), "r");
    if (!f) continue;
    char buf[1024];
    const size_t got = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[got] = 0;
    const char* l = strchr(buf, '(');
    const char* r = strrchr(buf, ')');
    if (!l || !r) continue;
    const std::string comm(l + 1, r);
    unsigned long ut = 0, st = 0;
    // after ") ": state ppid pgrp session tty tpgid flags minflt cminflt majflt cmajflt utime stime
    if (sscanf(r + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %lu %lu", &ut, &st) != 2) continue;
    const double cs = (double)(ut + st) / hz;
    if (cs < 0.05) continue;
    out += std::string(out.empty() ? "" : ", ") + "\"" + comm + ":" + de->d_name + "\": " +
           std::to_string(cs);
  }
  closedir(dir);
  return out;
}

void sleep_ms(double ms) {
  if (ms > 0) std::this_thread::sleep_for(std::chrono::duration<double, std::milli>(ms));
}

// The hold-and-wait flow (negative control): W blocking acquires, one part
// gathered after each, before the wave is hashed and uploaded.
qsmd5::WaveStats naive_upload(const std::vector<qsmd5_part>& parts, WatchedPool& pool,
                              const PagedFile& file, size_t W, double upload_ms,
                              std::vector<std::string>* md5) {
  qsmd5::WaveStats st;
  for (size_t first = 0; first < parts.size(); first += W) {
    const size_t n = std::min(W, parts.size() - first);
    std::vector<qsmd5::PoolBuffer> held;
    std::vector<qsmd5_chunk> ch;
    for (size_t k = 0; k < n; ++k) {
      held.push_back(pool.acquire());  // blocks while holding the buffers taken so far
      const qsmd5_part& p = parts[first + k];
      file.read(p.offset, p.size, held.back().data);
      ch.push_back(qsmd5_chunk{held.back().data, p.size});
      sleep_ms(1);
    }
    std::vector<uint8_t> dig(16 * n);
    qsmd5::detail::check(qsmd5_hash_batch_ex(ch.data(), n, reinterpret_cast<uint8_t(*)[16]>(dig.data()),
                                             QSMD5_FLAG_HOST),
                         "qsmd5_hash_batch_ex");
    for (size_t k = 0; k < n; ++k) {
      sleep_ms(upload_ms);
      (*md5)[parts[first + k].part_number - 1] = qsmd5::detail::hex(&dig[16 * k]);
      pool.release(held[k]);
    }
    ++st.waves;
    st.parts += n;
  }
  return st;
}

// The reference's md5(shared_ptr<iostream>) from oracle/_ref/libref_md5.so
// (built from /root/reference/src/base/MD5.cpp by oracle/build_ref.sh), found
// next to this binary's tree.
typedef void (*ref_md5_fn)(const char* p, uint64_t len, char out[33]);
ref_md5_fn load_reference_md5() {
  char exe[PATH_MAX];
  const ssize_t m = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
  if (m <= 0) return nullptr;
  exe[m] = 0;
  std::string dir(exe);
  dir = dir.substr(0, dir.rfind('/'));  // tests/cpp
  const std::string so = dir + "/../../oracle/_ref/libref_md5.so";
  void* h = dlopen(so.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "--reference-loop: %s\n", dlerror());
    return nullptr;
  }
  return reinterpret_cast<ref_md5_fn>(dlsym(h, "ref_md5_iostream"));
}

// QSTransferManager::DoMultiPartUpload with -m, as the reference runs it.
// Sync: acquire, read, md5, upload, release per part on this thread.  Async:
// acquire and read here, then the executor runs md5 + upload and releases.
template <class Upload>
qsmd5::WaveStats reference_upload(const std::vector<qsmd5_part>& parts, WatchedPool& pool,
                                  const PagedFile& file, ref_md5_fn ref_md5, bool async,
                                  std::atomic<double>* exec_hash_s, Upload&& upload) {
  using clock = clock_type;
  auto secs = [](clock::time_point a, clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
  };
  qsmd5::WaveStats st;
  st.waves = st.parts = parts.size();
  st.cpu_waves = parts.size();
  for (const qsmd5_part& p : parts) {
    const auto a0 = clock::now();
    qsmd5::PoolBuffer b = pool.acquire();
    const auto a1 = clock::now();
    st.acquire_s += secs(a0, a1);
    if (!b.data) throw std::runtime_error("transfer buffer pool is shut down: upload stopped");
    const size_t got = file.read(p.offset, p.size, b.data);
    const auto a2 = clock::now();
    st.loop_read_s += secs(a1, a2);
    if (got != p.size) {
      pool.release(b);
      throw std::runtime_error("short read of part " + std::to_string(p.part_number));
    }
    if (!async) {
      char hex[33];
      ref_md5(b.data, p.size, hex);
      const auto a3 = clock::now();
      st.hash_s += secs(a2, a3);
      upload(p, b, std::string(hex), false);
      st.upload_call_s += secs(a3, clock::now());
      pool.release(b);
    } else {
      upload(p, b, std::string(), true);  // the executor hashes, uploads, releases
      st.upload_call_s += secs(a2, clock::now());
    }
    ++st.uploaded;
  }
  (void)exec_hash_s;
  return st;
}

}  // namespace

int main(int argc, char** argv) {
  uint64_t size = 64ull * 10 * 1024 * 1024;
  size_t pool_n = 5, files = 1, naive_wave = 0, max_wave = 0;
  bool aligned = false, pinned = false, slab = false, reg = false, pipeline = true, staged = false;
  bool foreground = false;  // --foreground: StagedOptions::background_waves = false
  bool reference_loop = false, read_ahead = true;
  bool read_parallel = false;  // --read-parallel: the pre-hash's reads on QSMD5_READ_THREADS threads
  std::vector<std::string> pass_backends;  // --backends=gpu,cpu,auto: alternate the backend per pass
  uint64_t staging = 0;
  size_t wave_parts = 0, first_wave = 0;
  size_t cpus = 0, load_threads = 0;  // --cpus: the process's cores; --load: spinning threads on them
  uint32_t seed = 12345;
  uint64_t buf = 10ull << 20;
  int repeat = 1, async_threads = 0;
  double upload_ms = 0, deadlock_s = 20;
  uint32_t short_read_part = 0, fail_upload_part = 0;  // fault injection (1-based part numbers)
  size_t cancel_after = SIZE_MAX;  // each file's transfer is cancelled once it handed this many parts on
  size_t check_throws_after = SIZE_MAX;  // fault injection: should_continue() throws from then on
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* key) { return a.rfind(key, 0) == 0 ? a.c_str() + strlen(key) : nullptr; };
    if (const char* v = val("--size=")) size = strtoull(v, nullptr, 0);
    else if (const char* v = val("--pool=")) pool_n = strtoull(v, nullptr, 0);
    else if (const char* v = val("--seed=")) seed = (uint32_t)strtoul(v, nullptr, 0);
    else if (const char* v = val("--buf=")) buf = strtoull(v, nullptr, 0);
    else if (const char* v = val("--repeat=")) repeat = std::max(1, atoi(v));
    else if (const char* v = val("--backends=")) {  // pass k runs under QSMD5_BACKEND = list[k % size]
      std::string list = v;
      for (size_t pos = 0; pos <= list.size();) {
        const size_t c = list.find(',', pos);
        const std::string b = list.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
        if (!b.empty()) pass_backends.push_back(b);
        if (c == std::string::npos) break;
        pos = c + 1;
      }
    }
    else if (const char* v = val("--files=")) files = std::max<size_t>(1, strtoull(v, nullptr, 0));
    else if (const char* v = val("--upload-ms=")) upload_ms = atof(v);
    else if (const char* v = val("--async=")) async_threads = atoi(v);
    else if (const char* v = val("--naive-wave=")) naive_wave = strtoull(v, nullptr, 0);
    else if (const char* v = val("--max-wave=")) max_wave = strtoull(v, nullptr, 0);
    else if (const char* v = val("--deadlock-s=")) deadlock_s = atof(v);
    else if (const char* v = val("--short-read-part=")) short_read_part = (uint32_t)strtoul(v, nullptr, 0);
    else if (const char* v = val("--fail-upload-part=")) fail_upload_part = (uint32_t)strtoul(v, nullptr, 0);
    else if (const char* v = val("--cancel-after=")) cancel_after = strtoull(v, nullptr, 0);
    else if (const char* v = val("--check-throws-after=")) check_throws_after = strtoull(v, nullptr, 0);
    else if (const char* v = val("--staging=")) staging = strtoull(v, nullptr, 0);
    else if (const char* v = val("--wave-parts=")) wave_parts = strtoull(v, nullptr, 0);
    else if (const char* v = val("--first-wave=")) first_wave = strtoull(v, nullptr, 0);
    else if (const char* v = val("--cpus=")) cpus = strtoull(v, nullptr, 0);
    else if (const char* v = val("--load=")) load_threads = strtoull(v, nullptr, 0);
    else if (a == "--staged") staged = true;
    else if (a == "--reference-loop") reference_loop = true;
    else if (a == "--no-read-ahead") read_ahead = false;
    else if (a == "--read-parallel") read_parallel = true;
    else if (a == "--foreground") foreground = true;
    else if (a == "--aligned") aligned = true;
    else if (a == "--pinned") pinned = true;
    else if (a == "--slab") slab = true;
    else if (a == "--register") reg = true;
    else if (a == "--no-pipeline") pipeline = false;
    else {
      fprintf(stderr, "unknown argument %s\n", argv[i]);
      return 2;
    }
  }
  if (pool_n < 1) {
    fprintf(stderr, "--pool must be >= 1\n");
    return 2;
  }
  ref_md5_fn ref_md5 = nullptr;
  if (reference_loop && !(ref_md5 = load_reference_md5())) {
    fprintf(stderr, "--reference-loop needs oracle/_ref/libref_md5.so (oracle/build_ref.sh)\n");
    return 2;
  }
  std::atomic<double> exec_hash_s{0};  // --reference-loop --async: md5 time on the executor
  // --cpus=C: a daemon held to C cores (the first C of its allowed set), set
  // before any thread -- the library's and HIP's included -- is created, so
  // every thread inherits it.
  if (cpus) {
    cpu_set_t allowed, use;
    CPU_ZERO(&use);
    if (sched_getaffinity(0, sizeof(allowed), &allowed)) return 1;
    size_t taken = 0;
    for (int c = 0; c < CPU_SETSIZE && taken < cpus; ++c)
      if (CPU_ISSET(c, &allowed)) {
        CPU_SET(c, &use);
        ++taken;
      }
    if (sched_setaffinity(0, sizeof(use), &use)) return 1;
  }
  // The files' bytes, cut into pages of 1 KiB .. 3 MiB (aligned: one shared
  // file, every part golden; otherwise file f = LCG(seed + f)).
  std::vector<PagedFile> file(aligned ? 1 : files);
  for (size_t f = 0; f < file.size(); ++f) build_file(&file[f], size, aligned, buf, seed + (uint32_t)f);
  size_t n = 0;
  if (qsmd5_plan_parts(size, buf, 4ull << 20, 20ull << 20, 0, nullptr, 0, &n)) return 1;
  std::vector<qsmd5_part> parts(n);
  if (qsmd5_plan_parts(size, buf, 4ull << 20, 20ull << 20, 0, parts.data(), n, &n)) return 1;
  uint64_t largest = 0;
  for (const qsmd5_part& p : parts) largest = std::max(largest, p.size);
  // The transfer buffer pool: one allocation per buffer, as ResourceManager's
  // vector<char>(bufSize) each (TransferManager.cpp:103-108), or --slab: one
  // allocation carved into the buffers (qsmd5::BufferSlab).
  std::vector<std::unique_ptr<std::vector<char>>> owned;
  std::vector<qsmd5::PoolBuffer> pool;
  std::unique_ptr<qsmd5::BufferSlab> slab_pool;
  if (slab) {
    try {
      slab_pool.reset(new qsmd5::BufferSlab(pool_n, largest, pinned));
    } catch (const std::exception& e) {
      fprintf(stderr, "slab: %s\n", e.what());
      return 1;
    }
    pool = slab_pool->buffers();
  }
  for (size_t k = 0; k < pool_n && !slab; ++k) {
    if (pinned) {
      void* p = nullptr;
      if (qsmd5_alloc_pinned(largest, &p)) {
        fprintf(stderr, "qsmd5_alloc_pinned: %s\n", qsmd5_last_error());
        return 1;
      }
      pool.push_back({static_cast<char*>(p), largest});
    } else {
      owned.emplace_back(new std::vector<char>(largest));
      pool.push_back({owned.back()->data(), largest});
    }
  }
  (void)qsmd5_init(0);  // runtime start-up outside the timed uploads (-ENODEV without a GPU)
  // --register: lock the pageable pool's pages once, as a daemon would at start-up
  double register_s = 0;
  if (reg && !pinned) {
    const auto r0 = clock_type::now();
    // one registration per allocation: the slab at once, else each buffer
    std::vector<qsmd5::PoolBuffer> regs =
        slab ? std::vector<qsmd5::PoolBuffer>{{slab_pool->data(), slab_pool->bytes()}} : pool;
    for (auto& b : regs)
      if (qsmd5_register_host(b.data, b.size)) {
        fprintf(stderr, "qsmd5_register_host: %s\n", qsmd5_last_error());
        return 1;
      }
    register_s = std::chrono::duration<double>(clock_type::now() - r0).count();
  }
  // --load=K: K threads spinning on the process's cores for the whole run,
  // standing in for qsfs's own transfer workers and FUSE threads.  The
  // library's host rates are measured first, on the idle host, as a daemon's
  // start-up would.
  qsmd5_rates rates0;
  (void)qsmd5_get_rates(&rates0);
  std::atomic<bool> load_stop{false};
  std::vector<std::thread> load;
  for (size_t k = 0; k < load_threads; ++k)
    load.emplace_back([&] {
      pthread_setname_np(pthread_self(), "load");
      volatile uint64_t x = 0;
      while (!load_stop.load(std::memory_order_relaxed))
        for (int i = 0; i < 4096; ++i) x = x * 6364136223846793005ull + 1;
    });
  // The scheduler gives threads it has just started less than their share
  // for a while (the first pass of a --load run hashed as fast as an idle
  // one, later passes half as fast): let the load settle before timing.
  if (load_threads) std::this_thread::sleep_for(std::chrono::seconds(1));
  WatchedPool shared(pool);
  std::unique_ptr<Executor> exec(async_threads > 0 ? new Executor(async_threads) : nullptr);
  // Watchdog: a thread blocked in acquire, and nothing moved for deadlock_s.
  std::atomic<bool> finished{false};
  progress();
  std::thread watchdog([&] {
    pthread_setname_np(pthread_self(), "watchdog");
    while (!finished.load()) {
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
      const double idle = (clock_type::now().time_since_epoch().count() - g_progress_ns.load()) * 1e-9;
      if (shared.waiting() > 0 && idle > deadlock_s) {
        printf("{\"deadlock\": true, \"waiting\": %d, \"free\": %zu, \"idle_s\": %.1f}\n", shared.waiting(),
               shared.free_count(), idle);
        fflush(stdout);
        fprintf(stderr, "deadlock: %d thread(s) blocked in acquire, %zu buffer(s) free, no progress "
                "for %.1f s\n", shared.waiting(), shared.free_count(), idle);
        _exit(3);
      }
    }
  });
  // --repeat: upload the files again through the same pool, as a daemon reuses
  // its buffers; the first pass pays HIP's first-touch locking of pageable pages.
  std::vector<std::vector<std::string>> md5(files, std::vector<std::string>(n));
  std::vector<std::vector<std::string>> first_md5;
  int pass_mismatch = 0;  // passes whose digests differ from the first pass's
  std::vector<double> hash_runs, wall_runs, cpu_runs;
  std::vector<qsmd5::WaveStats> st(files);
  std::vector<std::string> errors(files);
  double total = 0;
  for (int rep = 0; rep < repeat; ++rep) {
    // --backends: the library reads QSMD5_BACKEND at each call, and no call is
    // in flight between passes, so passes under different backends interleave
    // in one process (same pages, same NUMA placement, same GPU clock history)
    if (!pass_backends.empty()) setenv("QSMD5_BACKEND", pass_backends[rep % pass_backends.size()].c_str(), 1);
    exec_hash_s.store(0);  // per pass, as st[] below
    for (auto& v : md5) std::fill(v.begin(), v.end(), std::string());  // this pass's digests only
    const auto t0 = clock_type::now();
    const double c0 = cpu_seconds();
    std::vector<std::thread> th;
    for (size_t f = 0; f < files; ++f) {
      th.emplace_back([&, f] {
        pthread_setname_np(pthread_self(), ("flush-" + std::to_string(f)).c_str());
        const PagedFile& pf = file[aligned ? 0 : f];
        try {
          if (naive_wave) {
            st[f] = naive_upload(parts, shared, pf, naive_wave, upload_ms, &md5[f]);
            return;
          }
          if (reference_loop) {
            InFlight inflight;
            auto up = [&](const qsmd5_part& p, const qsmd5::PoolBuffer& b, const std::string& hex, bool async) {
              if (!async) {
                sleep_ms(upload_ms);
                md5[f][p.part_number - 1] = hex;
                progress();
                return;
              }
              inflight.add();
              exec->submit([&, p, b] {
                char h[33];
                const auto h0 = clock_type::now();
                ref_md5(b.data, p.size, h);  // md5(buffer) inside UploadMultipart
                double cur = exec_hash_s.load();
                const double d = std::chrono::duration<double>(clock_type::now() - h0).count();
                while (!exec_hash_s.compare_exchange_weak(cur, cur + d)) {
                }
                sleep_ms(upload_ms);
                md5[f][p.part_number - 1] = h;
                shared.release(b);
                inflight.done();
              });
            };
            try {
              st[f] = reference_upload(parts, shared, pf, ref_md5, exec != nullptr, &exec_hash_s, up);
            } catch (...) {
              inflight.wait();
              throw;
            }
            inflight.wait();
            return;
          }
          qsmd5::PrehashOptions opt;
          opt.pipeline = pipeline;
          opt.max_wave = max_wave;
          opt.upload_releases = exec != nullptr;
          // --cancel-after: TransferHandle::Cancel from another thread once K parts went out
          std::atomic<size_t> handed{0};
          if (cancel_after != SIZE_MAX) opt.should_continue = [&] { return handed.load() < cancel_after; };
          if (check_throws_after != SIZE_MAX)
            opt.should_continue = [&] {
              if (handed.load() >= check_throws_after) throw std::runtime_error("injected should_continue failure");
              return true;
            };
          InFlight inflight;
          auto read = [&](const qsmd5_part& p, char* dst) {
            const size_t got = pf.read(p.offset, p.size, dst);
            return p.part_number == short_read_part ? got / 2 : got;  // File::ReadNoLoad found a hole
          };
          auto upload = [&](const qsmd5_part& p, const qsmd5::PoolBuffer& b, const std::string& hex) {
            if (p.part_number == fail_upload_part) throw std::runtime_error("injected upload failure");
            ++handed;
            if (!exec) {  // sync: UploadMultipart on this thread, the buffer released after it
              sleep_ms(upload_ms);
              md5[f][p.part_number - 1] = hex;
              progress();
              return;
            }
            inflight.add();  // async: the executor uploads, its handler releases the buffer
            exec->submit([&, p, b, hex] {
              sleep_ms(upload_ms);
              md5[f][p.part_number - 1] = hex;
              shared.release(b);
              inflight.done();
            });
          };
          // --staged: File::ReadNoLoad over any byte range of the file (the short-read
          // fault hits any window inside the chosen part)
          auto read_range = [&](uint64_t off, size_t len, char* dst) {
            const size_t got = pf.read(off, len, dst);
            if (short_read_part) {
              const qsmd5_part& sp = parts[short_read_part - 1];
              if (off >= sp.offset && off < sp.offset + sp.size) return got / 2;
            }
            return got;
          };
          try {
            if (staged) {
              qsmd5::StagedOptions so;
              so.staging_bytes = staging;
              so.wave_parts = wave_parts;
              so.first_wave_parts = first_wave;
              so.background_waves = !foreground;
              so.pipeline = pipeline;
              so.upload_releases = opt.upload_releases;
              so.should_continue = opt.should_continue;
              so.read_ahead = read_ahead;
              if (read_parallel) so.flags |= QSMD5_FLAG_READ_PARALLEL;  // PagedFile::read is const: thread-safe
              st[f] = qsmd5::upload_parts_staged(parts, shared, read_range, upload, so);
            } else {
              st[f] = qsmd5::upload_parts_prehashed(parts, shared, read, upload, opt);
            }
          } catch (...) {
            inflight.wait();  // parts handed over before the failure are still uploading
            throw;
          }
          inflight.wait();
          if (st[f].uploaded != handed.load()) errors[f] = "stats.uploaded disagrees with the parts uploaded";
        } catch (const std::exception& e) {
          errors[f] = e.what();
        }
      });
    }
    for (auto& t : th) t.join();
    total = std::chrono::duration<double>(clock_type::now() - t0).count();
    // every pass must hand on the same digests as the first (the last pass's
    // are the ones reported and checked against the golden table)
    if (rep == 0) first_md5 = md5;
    else if (md5 != first_md5) ++pass_mismatch;
    double h = 0;
    for (auto& s : st) h += s.hash_s;
    hash_runs.push_back(h);
    wall_runs.push_back(total);
    cpu_runs.push_back(cpu_seconds() - c0);
  }
  finished.store(true);
  watchdog.join();
  load_stop.store(true);
  for (auto& t : load) t.join();
  double cpu_eff = 0;
  (void)qsmd5_get_cpu_efficiency(&cpu_eff);
  const bool injected = short_read_part || fail_upload_part || check_throws_after != SIZE_MAX;
  for (size_t f = 0; f < files; ++f)
    if (!errors[f].empty()) {
      fprintf(stderr, "upload of file %zu failed: %s\n", f, errors[f].c_str());
      if (!injected) return 1;
    }
  // After an injected failure: which parts reached the uploader, and whether
  // every buffer is back in the pool (nothing leaked by the helper thread).
  size_t uploaded = 0;
  for (const auto& v : md5)
    for (const auto& h : v) uploaded += !h.empty();
  const size_t pool_free_after = shared.free_count();
  if (pinned && !slab)
    for (auto& b : pool) qsmd5_free_pinned(b.data);
  if (reg && !pinned) {
    if (slab) qsmd5_unregister_host(slab_pool->data());
    else
      for (auto& b : pool) qsmd5_unregister_host(b.data);
  }
  qsmd5::WaveStats sum;
  size_t stopped = 0;
  for (const auto& s : st) {
    stopped += s.stopped;
    sum.uploaded += s.uploaded;
    sum.waves += s.waves;
    sum.parts += s.parts;
    sum.gpu_waves += s.gpu_waves;
    sum.cpu_waves += s.cpu_waves;
    sum.split_waves += s.split_waves;
    sum.rehashed += s.rehashed;
    sum.widest_wave = std::max(sum.widest_wave, s.widest_wave);
    sum.gather_s += s.gather_s;
    sum.hash_s += s.hash_s;
    sum.upload_s += s.upload_s;
    sum.wait_s += s.wait_s;
    sum.acquire_s += s.acquire_s;
    sum.loop_read_s += s.loop_read_s;
    sum.upload_call_s += s.upload_call_s;
    sum.read_ahead += s.read_ahead;
  }
  if (reference_loop && exec) sum.hash_s += exec_hash_s.load();
  auto md5_list = [&](const std::vector<std::string>& v) {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); ++i) s += std::string(i ? ", " : "") + "\"" + v[i] + "\"";
    return s + "]";
  };
  printf("{\"deadlock\": false, \"error\": \"%s\", \"uploaded\": %zu, \"stats_uploaded\": %zu, \"stopped\": %zu, \"pool_free_after\": %zu, \"size\": %llu, \"parts\": %zu, \"files\": %zu, \"pages\": %zu, \"pool\": %zu, "
         "\"pinned\": %s, \"slab\": %s, \"registered\": %s, \"pipeline\": %s, \"staged\": %s, \"staging\": %llu, \"async_threads\": %d, "
         "\"naive_wave\": %zu, \"upload_ms\": %.3f, \"register_s\": %.6f, \"waves\": %zu, "
         "\"widest_wave\": %zu, \"gpu_waves\": %zu, \"cpu_waves\": %zu, \"split_waves\": %zu, "
         "\"seconds\": %.6f, \"gather_s\": %.6f, \"hash_s\": %.6f, \"upload_s\": %.6f, \"wait_s\": %.6f, "
         "\"part_sizes\": [",
         errors[0].c_str(), uploaded, sum.uploaded, stopped, pool_free_after, (unsigned long long)size, n, files, file[0].pages.size(), pool_n, pinned ? "true" : "false",
         slab ? "true" : "false", reg && !pinned ? "true" : "false", pipeline ? "true" : "false",
         staged ? "true" : "false", (unsigned long long)staging, async_threads, naive_wave, upload_ms, register_s, sum.waves, sum.widest_wave, sum.gpu_waves,
         sum.cpu_waves, sum.split_waves, total, sum.gather_s, sum.hash_s, sum.upload_s, sum.wait_s);
  for (size_t i = 0; i < n; ++i) printf("%s%llu", i ? ", " : "", (unsigned long long)parts[i].size);
  printf("], \"hash_s_runs\": [");
  for (size_t i = 0; i < hash_runs.size(); ++i) printf("%s%.6f", i ? ", " : "", hash_runs[i]);
  printf("], \"wall_s_runs\": [");
  for (size_t i = 0; i < wall_runs.size(); ++i) printf("%s%.6f", i ? ", " : "", wall_runs[i]);
  printf("], \"cpus\": %zu, \"load_threads\": %zu, \"cpu_efficiency\": %.4f, \"wave_parts\": %zu, \"first_wave\": %zu, "
         "\"background_waves\": %s, \"rehashed\": %zu",
         cpus, load_threads, cpu_eff, wave_parts, first_wave, foreground ? "false" : "true", sum.rehashed);
  printf(", \"pass_mismatch\": %d", pass_mismatch);
  printf(", \"reference_loop\": %s, \"read_ahead\": %zu, \"acquire_s\": %.6f, \"loop_read_s\": %.6f, "
         "\"upload_call_s\": %.6f", reference_loop ? "true" : "false", sum.read_ahead, sum.acquire_s,
         sum.loop_read_s, sum.upload_call_s);
  printf(", \"busy_threads\": {%s}, \"cpu_s_runs\": [", busy_threads().c_str());
  for (size_t i = 0; i < cpu_runs.size(); ++i) printf("%s%.6f", i ? ", " : "", cpu_runs[i]);
  printf("], \"md5\": %s, \"md5_files\": [", md5_list(md5[0]).c_str());
  for (size_t f = 0; f < files; ++f) printf("%s%s", f ? ", " : "", md5_list(md5[f]).c_str());
  printf("]}\n");
  return 0;
}
