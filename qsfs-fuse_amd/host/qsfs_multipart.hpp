// qsfs-fuse_amd/host/qsfs_multipart.hpp -- the batch pre-hash inside qsfs's
// multipart upload loop.
//
// The reference uploads a file's parts in QSTransferManager::DoMultiPartUpload
// (src/client/QSTransferManager.cpp:602-673): for each queued part it acquires
// a pooled transfer buffer (ResourceManager::Acquire, ResourceManager.cpp:53-67,
// which BLOCKS until a buffer is free), gathers the part's bytes from the
// file's pages into it (File::ReadNoLoad, src/data/File.cpp:308-375), wraps it
// in an IOStream of the part's size, and hands it to UploadMultipart, which
// computes md5(stream) for the Content-MD5 (QSClient.cpp:369-371).  The buffer
// goes back to the pool when the part's upload returns
// (ReceivedHandlerMultipleUpload, QSTransferManager.cpp:215-220).  One buffer,
// one serial hash, at a time; a flushing thread never holds more than one
// buffer while it waits for another.
//
// upload_parts_prehashed() keeps that buffer discipline and hashes in waves:
//   - a wave blocks in acquire() for its FIRST buffer only, while it holds no
//     buffer of its own, and then takes just the buffers free at that moment
//     (try_acquire(), which never blocks).  So no thread ever waits for a
//     buffer while holding one that only it would release, and any number of
//     files flushing at once through one blocking pool cannot deadlock (the
//     hold-and-wait condition never holds);
//   - the wave's parts are gathered (read) and hashed with ONE
//     qsmd5_hash_batch_ex(QSMD5_FLAG_HOST) call, routed by size like any call
//     (few parts: the library's CPU MD5; many: the gfx950 kernels);
//   - each part, its buffer and its hex digest go to the caller's upload,
//     and the buffer is released as soon as that part's upload returns;
//   - with `pipeline` (default), the next wave is gathered and hashed on a
//     helper thread while this thread uploads the current one, so the hash
//     time hides behind the upload (the overlap the reference's async
//     handler has, QSTransferManager.cpp:654-659);
//   - the transfer's cancel flag (opt.should_continue, the reference's
//     handle->ShouldContinue() at QSTransferManager.cpp:608 and 646) is asked
//     before a wave takes buffers and before each part's upload; a cancelled
//     upload returns every buffer it did not hand over and reports how many
//     parts it uploaded, so the caller marks the rest failed (:669-671).
//
// The pool holds `-n` (numtransfer) buffers of `-b` MiB: the transfer
// manager's heap is bufSize x maxParallelTransfers (TransferManager.h:74-86,
// constructed with defaults at Drive.cpp:124), shared by every file upload.
// Waves are therefore at most -n parts: qsfs's default -n 5 keeps them below
// the GPU break-even and on the CPU; on the MI355X box auto routing first
// sends waves to the GPU at -n 64 (the break-even, priced at the host's
// measured CPU rate, lies between 33 and 64 parts of 10 MiB there;
// INTEGRATION.md §3, profiles/r04_pool_sweep.jsonl).
//
// Header-only over the C-ABI (include/qsmd5.h).  Throws qsmd5::Error on a
// hashing failure and std::runtime_error on a short read or a shut-down pool,
// as the reference stops the upload there (QSTransferManager.cpp:611-643).
#ifndef QSFS_AMD_QSFS_MULTIPART_HPP_
#define QSFS_AMD_QSFS_MULTIPART_HPP_

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <condition_variable>
#include <exception>
#include <functional>
#include <future>
#include <mutex>
#include <stdexcept>
#include <string>
#include <system_error>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "qsfs_md5.hpp"

namespace qsmd5 {

// One pooled transfer buffer (ResourceManager's vector<char>(bufSize)).
struct PoolBuffer {
  char* data;
  size_t size;
};

// A transfer-buffer pool carved from ONE allocation (pageable, or pinned
// through qsmd5_alloc_pinned).  The reference allocates each pool buffer on
// its own (TransferManager.cpp:103-108); buffers in one allocation at a
// constant stride let the library move a wave's columns to the GPU as one 2-D
// copy each instead of one copy per buffer (qsmd5_plan.h plan_copy_runs).
class BufferSlab {
 public:
  BufferSlab(size_t count, size_t size, bool pinned) : count_(count), size_(size), pinned_(pinned) {
    const size_t bytes = count * size;
    if (pinned_) {
      void* p = nullptr;
      detail::check(qsmd5_alloc_pinned(bytes ? bytes : 1, &p), "qsmd5_alloc_pinned");
      base_ = static_cast<char*>(p);
    } else {
      heap_.resize(bytes ? bytes : 1);
      base_ = heap_.data();
    }
  }
  ~BufferSlab() {
    if (pinned_) qsmd5_free_pinned(base_);
  }
  BufferSlab(const BufferSlab&) = delete;
  BufferSlab& operator=(const BufferSlab&) = delete;
  char* data() const { return base_; }
  size_t bytes() const { return count_ * size_; }
  std::vector<PoolBuffer> buffers() const {
    std::vector<PoolBuffer> v;
    for (size_t k = 0; k < count_; ++k) v.push_back(PoolBuffer{base_ + k * size_, size_});
    return v;
  }

 private:
  size_t count_, size_;
  bool pinned_;
  char* base_ = nullptr;
  std::vector<char> heap_;
};

// The pool interface upload_parts_prehashed needs -- ResourceManager's
// Acquire / Release (ResourceManager.cpp:53-77) plus a non-blocking
// try_acquire -- restated over PoolBuffers.  A qsfs binding adapts the real
// ResourceManager instead; any type with the same members
// works:
//   typedef ... buffer_type;                       copyable handle
//   buffer_type acquire();                         blocks; a null handle = shut down
//   bool try_acquire(buffer_type* out);            never blocks; false = none free
//   void release(const buffer_type& b);
//   static char* data(const buffer_type& b);       nullptr for a null handle
//   static size_t size(const buffer_type& b);
class BlockingPool {
 public:
  typedef PoolBuffer buffer_type;
  explicit BlockingPool(std::vector<PoolBuffer> buffers) : free_(std::move(buffers)) {}
  buffer_type acquire() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return shutdown_ || !free_.empty(); });
    if (shutdown_) return PoolBuffer{nullptr, 0};
    const PoolBuffer b = free_.back();
    free_.pop_back();
    return b;
  }
  bool try_acquire(buffer_type* out) {
    std::lock_guard<std::mutex> lk(mu_);
    if (shutdown_ || free_.empty()) return false;
    *out = free_.back();
    free_.pop_back();
    return true;
  }
  void release(const buffer_type& b) {
    if (!b.data) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      free_.push_back(b);
    }
    cv_.notify_one();
  }
  void shutdown() {  // ResourceManager::ShutdownAndWait's flag: acquire() stops blocking
    {
      std::lock_guard<std::mutex> lk(mu_);
      shutdown_ = true;
    }
    cv_.notify_all();
  }
  size_t free_count() {
    std::lock_guard<std::mutex> lk(mu_);
    return free_.size();
  }
  static char* data(const buffer_type& b) { return b.data; }
  static size_t size(const buffer_type& b) { return b.size; }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<PoolBuffer> free_;
  bool shutdown_ = false;
};

// What the upload did: parts hashed, which backend the library picked for
// each wave, and the time in each phase.  gather_s and hash_s are summed over
// waves wherever they ran (with `pipeline`, mostly on the helper thread,
// overlapped with upload_s); wait_s is the time the uploading thread spent
// waiting for the next wave to be ready, i.e. hashing NOT hidden.
struct WaveStats {
  size_t waves = 0, parts = 0;
  size_t uploaded = 0;   // parts handed to upload(), in part order: parts[0, uploaded)
  bool stopped = false;  // should_continue() said stop (TransferHandle::ShouldContinue)
  size_t gpu_waves = 0, cpu_waves = 0, split_waves = 0;  // by qsmd5_last_backend of each wave
  size_t widest_wave = 0;
  size_t rehashed = 0;   // upload_parts_staged: parts re-hashed from their buffer (source_changed)
  double gather_s = 0, hash_s = 0, upload_s = 0, wait_s = 0, wall_s = 0;
  // upload_parts_staged's upload loop, on the calling thread (VERDICT r05 item
  // 3): blocked in the pool's acquire(); in the loop's own read of a part into
  // its buffer, or waiting for that part's read-ahead; inside upload().
  // read_ahead = parts whose read ran behind the previous part's upload.
  double acquire_s = 0, loop_read_s = 0, upload_call_s = 0;
  size_t read_ahead = 0;
};

struct PrehashOptions {
  // Gather + hash the next wave on a helper thread while this one uploads.
  // The helper calls read(), so read() must not wait for a lock the calling
  // thread holds: a synchronous File::Flush keeps the file's recursive_mutex
  // through the upload (File.cpp:619, 641-643) and every ReadNoLoad takes it
  // (File.cpp:310) -- pass false there ("The file's lock").
  bool pipeline = true;
  size_t max_wave = 0;         // parts per wave at most (0: as many as free buffers)
  bool upload_releases = false;  // true: a buffer is upload()'s once upload() returns, and
                                 // its completion handler releases it (an async
                                 // executor); false: released when upload() returns
  // The transfer's cancel flag (TransferHandle::ShouldContinue, TransferHandle.h:159-162),
  // asked where the reference's loop asks it (QSTransferManager.cpp:608, 646): before a
  // wave takes buffers and before each part is handed to upload().  Once it says
  // false, no further part is uploaded, every buffer not handed over goes back
  // to the pool, and the call returns with stats.stopped; the caller marks
  // parts [stats.uploaded, end) failed, as :669-671.  Empty: never stop.
  // With `pipeline` it is also called from the helper thread preparing the
  // next wave, so it must be thread-safe (ShouldContinue takes a lock).
  std::function<bool()> should_continue;
};

namespace detail {

template <class Pool>
struct Wave {
  size_t first = 0;  // index of its first part
  bool cancelled = false;  // should_continue() was false before it took a buffer
  std::vector<typename Pool::buffer_type> bufs;
  std::vector<uint8_t> dig;
  int backend = 0;
  double gather_s = 0, hash_s = 0;
};

// Handles already handed over are null (Pool::data() == nullptr) and are
// skipped: a real pool must never be given a null buffer back.
template <class Pool>
void release_all(Pool& pool, std::vector<typename Pool::buffer_type>& bufs, size_t from = 0) {
  for (size_t k = from; k < bufs.size(); ++k)
    if (Pool::data(bufs[k])) pool.release(bufs[k]);
  bufs.resize(std::min(from, bufs.size()));
}

// Take the buffers of the wave starting at part `first` (block for one while
// holding none, then only what is free), gather its parts, hash them.  On any
// failure every buffer it took is back in the pool before it throws.
// keep_half: the first wave of a pipelined upload keeps half of the buffers
// it could get and gives the rest back at once, so that the next wave (on the
// helper thread) has buffers to fill while this one uploads: the pool's
// buffers then alternate between the wave in upload and the wave in hashing.
template <class Pool, class Read>
Wave<Pool> prepare_wave(const std::vector<qsmd5_part>& parts, size_t first, Pool& pool, Read& read,
                        size_t max_wave, bool keep_half, const std::function<bool()>& should_continue) {
  using clock = std::chrono::steady_clock;
  Wave<Pool> w;
  w.first = first;
  if (should_continue && !should_continue()) {
    w.cancelled = true;
    return w;
  }
  const size_t want = std::min(max_wave ? max_wave : parts.size(), parts.size() - first);
  typename Pool::buffer_type b = pool.acquire();
  if (!Pool::data(b)) throw std::runtime_error("transfer buffer pool is shut down: upload stopped");
  try {
    w.bufs.push_back(b);
    while (w.bufs.size() < want && pool.try_acquire(&b)) w.bufs.push_back(b);
    if (keep_half && w.bufs.size() < parts.size() - first) release_all(pool, w.bufs, (w.bufs.size() + 1) / 2);
    const size_t n = w.bufs.size();
    const auto t0 = clock::now();
    std::vector<qsmd5_chunk> chunks(n);
    for (size_t k = 0; k < n; ++k) {
      const qsmd5_part& p = parts[first + k];
      if (Pool::size(w.bufs[k]) < p.size) throw std::invalid_argument("pool buffer smaller than a part");
      const size_t got = read(p, Pool::data(w.bufs[k]));
      if (got != p.size)
        throw std::runtime_error("short read of part " + std::to_string(p.part_number) + ": " +
                                 std::to_string(got) + " of " + std::to_string(p.size) + " bytes");
      chunks[k] = qsmd5_chunk{Pool::data(w.bufs[k]), p.size};
    }
    const auto t1 = clock::now();
    w.dig.resize(16 * n);
    check(qsmd5_hash_batch_ex(chunks.data(), n, reinterpret_cast<uint8_t(*)[16]>(w.dig.data()),
                              QSMD5_FLAG_HOST),
          "qsmd5_hash_batch_ex");
    w.backend = qsmd5_last_backend();  // this thread's call
    w.gather_s = std::chrono::duration<double>(t1 - t0).count();
    w.hash_s = std::chrono::duration<double>(clock::now() - t1).count();
  } catch (...) {
    release_all(pool, w.bufs);
    throw;
  }
  return w;
}

}  // namespace detail

// parts:    the file's parts as PrepareUpload slices them (qsmd5_plan_parts).
// pool:     the transfer buffer pool (see BlockingPool for the members used),
//           each buffer at least the largest part; shared with other uploads.
// read:     read(part, char* buf) -> bytes gathered (File::ReadNoLoad).  With
//           `pipeline` it runs on a helper thread, one wave at a time.
// upload:   upload(part, const buffer_type& buf, const std::string& hex) hands
//           the part on (UploadMultipart with SetContentMD5(hex)), on the
//           calling thread, in part order.  If it throws, the buffer goes back
//           to the pool and the upload stops there.  If it returns: with
//           opt.upload_releases the buffer is now upload()'s, whose completion
//           handler releases it; otherwise it goes back to the pool at once.
template <class Pool, class Read, class Upload>
WaveStats upload_parts_prehashed(const std::vector<qsmd5_part>& parts, Pool& pool, Read&& read,
                                 Upload&& upload, const PrehashOptions& opt = PrehashOptions()) {
  using clock = std::chrono::steady_clock;
  typedef detail::Wave<Pool> W;
  WaveStats st;
  const auto t_start = clock::now();
  if (parts.empty()) return st;
  auto secs = [](clock::time_point a, clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
  };
  auto prep = [&](size_t first) {
    return detail::prepare_wave(parts, first, pool, read, opt.max_wave, opt.pipeline && first == 0,
                                opt.should_continue);
  };
  std::future<W> ahead;  // the next wave, being prepared on the helper thread
  // On the way out after a failure: the wave in preparation finishes (its
  // thread may be waiting for a buffer this thread just released), and its
  // buffers go back to the pool.
  auto drain_ahead = [&]() noexcept {
    if (!ahead.valid()) return;
    try {
      W w = ahead.get();
      detail::release_all(pool, w.bufs);
    } catch (...) {
    }
  };
  auto stop_requested = [&] { return opt.should_continue && !opt.should_continue(); };
  W cur = prep(0);
  for (;;) {
    if (cur.cancelled) {  // stopped before this wave took a buffer; nothing is ahead of it
      st.stopped = true;
      break;
    }
    const size_t n = cur.bufs.size(), next = cur.first + n;
    ++st.waves;
    st.parts += n;
    st.widest_wave = std::max(st.widest_wave, n);
    st.gather_s += cur.gather_s;
    st.hash_s += cur.hash_s;
    switch (cur.backend) {
      case QSMD5_BACKEND_GPU: ++st.gpu_waves; break;
      case QSMD5_BACKEND_SPLIT: ++st.split_waves; break;  // longest parts on the CPU, the rest on the GPU
      default: ++st.cpu_waves; break;
    }
    if (opt.pipeline && next < parts.size()) {
      try {
        ahead = std::async(std::launch::async, prep, next);
      } catch (...) {
        // no thread to spare (std::system_error) or no memory for the shared
        // state (std::bad_alloc): this wave uploads, then the next is prepared
        // here; the wave's buffers are still cur's, released as it uploads
      }
    }
    const auto t0 = clock::now();
    size_t k = 0;
    try {
      for (; k < n; ++k) {
        if (stop_requested()) break;
        const qsmd5_part& p = parts[cur.first + k];
        const std::string hex = detail::hex(&cur.dig[16 * k]);
        // A buffer is upload()'s once upload() returns (upload_releases: its
        // completion handler releases it); if upload() throws, it was not
        // taken and goes back to the pool here.
        try {
          upload(p, cur.bufs[k], hex);
        } catch (...) {
          pool.release(cur.bufs[k]);
          cur.bufs[k] = typename Pool::buffer_type();
          throw;
        }
        if (!opt.upload_releases) pool.release(cur.bufs[k]);  // ReceivedHandlerMultipleUpload
        cur.bufs[k] = typename Pool::buffer_type();
        ++st.uploaded;
      }
    } catch (...) {
      // parts of this wave never handed over: from k on (a throwing upload()'s
      // own buffer is already back and null; a throwing should_continue() or
      // hex formatting left bufs[k] still held)
      detail::release_all(pool, cur.bufs, k);
      drain_ahead();
      throw;
    }
    const auto t1 = clock::now();
    st.upload_s += secs(t0, t1);
    if (k < n) {  // stopped inside the wave: the rest of it and the wave ahead go back
      detail::release_all(pool, cur.bufs, k);
      drain_ahead();
      st.stopped = true;
      break;
    }
    if (next >= parts.size()) break;
    if (ahead.valid()) {
      cur = ahead.get();  // rethrows the helper's failure (its buffers are already back)
      st.wait_s += secs(t1, clock::now());
    } else {
      cur = prep(next);
      st.wait_s += secs(t1, clock::now());
    }
  }
  st.wall_s = secs(t_start, clock::now());
  return st;
}

// ---- the whole file pre-hashed, then the reference's own upload loop ----------
// waves over pool buffers are at most -n parts wide (5 at
// qsfs's default), which keeps every wave below the GPU's break-even.  Here
// the pre-hash does not use the pool at all: qsmd5_hash_read pulls each part's
// bytes from the caller's File::ReadNoLoad (File.cpp:308-375) in column
// windows through the library's own bounded pinned staging, so one call hashes
// every queued part of the file as one GPU batch.  Each digest then rides on
// its part into the reference's loop: one pool buffer per part (Acquire
// blocks only while this thread holds none), ReadNoLoad into it,
// UploadMultipart with the stored digest (QSTransferManager.cpp:602-673) --
// plus, round 6, the next part read into a second buffer behind the upload
// when one is free at that instant (StagedOptions::read_ahead).

struct StagedOptions {
  uint64_t staging_bytes = 0;  // qsmd5_hash_read's budget (0: QSMD5_READ_STAGING_BYTES, 256 MiB)
  size_t wave_parts = 0;       // parts per pre-hash call (0: every part of the file at once)
  // Ramp (with pipeline and wave_parts): the first wave has this many parts
  // and each next one twice the last, up to wave_parts (0: every wave
  // wave_parts).  The first upload then waits only for a small wave (the
  // CPU's, ~ms) instead of a GPU wave's chain time (~85 ms per 10 MiB part),
  // and each larger wave is pre-hashed while the smaller one before it uploads.
  size_t first_wave_parts = 0;
  // With pipeline: the waves after the first are pre-hashed while the one
  // before them uploads.  Where that hides their latency they go out with
  // QSMD5_FLAG_BACKGROUND (the GPU whenever one is usable, leaving the host's
  // cores to the daemon's own threads): when the wave uploading meanwhile,
  // at the upload loop's own measured pace per part so far, lasts at least
  // 1.25 x the next wave's GPU time (its longest part's chain at the
  // library's GPU chain rate, qsmd5_get_rates, plus its bytes read at 12
  // GiB/s).  Otherwise -- the first wave, which the first upload waits for,
  // a wave behind one too short to hide it, and every wave when uploads
  // return at once -- the wave is routed for speed.  Round 5 sent every wave
  // after the first to the GPU: behind the ramp's 4-part first wave the
  // 8-part second one (one ~85 ms chain) outlasted 40 ms of uploads and the
  // uploader waited.  false: every wave for speed.
  bool background_waves = true;
  bool pipeline = true;        // pre-hash the next wave on a helper thread while this one uploads
                               // (read_range then runs there too: PrehashOptions::pipeline)
  bool upload_releases = false;  // as PrehashOptions::upload_releases
  int flags = 0;               // qsmd5_hash_read flags (QSMD5_FLAG_GPU_ONLY / _CPU_ONLY; with
                               // QSMD5_FLAG_READ_PARALLEL read_range runs on several library
                               // threads at once and must be thread-safe, as pread is)
  std::function<bool()> should_continue;  // as PrehashOptions::should_continue (thread-safe)
  // With pipeline: while a part uploads, the next part of the wave is read
  // into a buffer the pool has free at that moment (try_acquire, never a
  // blocking acquire while this thread holds a buffer) on a helper thread,
  // wherever the last upload() took longer than the last read, so the loop's
  // own ReadNoLoad runs behind the upload instead of between uploads (512 reads of ~0.8 ms each, serial with the
  // uploads, were the staged flow's 0.42 s over pure upload time).  The file
  // then has two parts in flight for one flush, as the reference's async
  // path has up to -n (QSTransferManager.cpp:654-659).  Needs a pool with
  // try_acquire (without one the loop reads as the reference's does).  false:
  // one buffer at a time, exactly the reference's loop.
  bool read_ahead = true;
  // The pre-hash reads the file before the upload loop reads each part again
  // into its buffer: a write in between would send a Content-MD5 that does not
  // match the part (the reference hashes the very buffer it sends,
  // QSClient.cpp:369-371).  source_changed() is asked after each part lands
  // in its buffer; true (the file was written since the pre-hash began: the
  // binding compares File's write version) re-hashes that part from the
  // buffer (qsmd5_hash_one), so the digest always matches the bytes sent.
  // Empty: the file does not change during the upload.
  std::function<bool()> source_changed;
};

namespace detail {

// read_range(file_offset, len, char* dst) -> bytes copied (File::ReadNoLoad(...).first).
// With QSMD5_FLAG_READ_PARALLEL in the flags, thunk runs on several library
// threads at once: the first exception is kept (under a mutex)
// and every later read returns 0 at once.
template <class ReadRange>
struct RangeReader {
  const std::vector<qsmd5_part>* parts;
  size_t first;
  ReadRange* read;
  std::atomic<bool> failed{false};
  std::mutex mu;
  std::exception_ptr err;
  RangeReader(const std::vector<qsmd5_part>* p, size_t f, ReadRange* r) : parts(p), first(f), read(r) {}
  static uint64_t thunk(void* user, size_t chunk, uint64_t offset, uint64_t len, void* dst) {
    RangeReader* r = static_cast<RangeReader*>(user);
    if (r->failed.load(std::memory_order_acquire)) return 0;
    try {
      const qsmd5_part& p = (*r->parts)[r->first + chunk];
      return (uint64_t)(*r->read)(p.offset + offset, (size_t)len, static_cast<char*>(dst));
    } catch (...) {  // never through the C library: carried out below
      std::lock_guard<std::mutex> lk(r->mu);
      if (!r->err) r->err = std::current_exception();
      r->failed.store(true, std::memory_order_release);
      return 0;
    }
  }
  // After the call returned (every library thread is done with thunk).
  void rethrow_if_failed() {
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> lk(mu);
      e = err;
    }
    if (e) std::rethrow_exception(e);
  }
};

// Whether Pool has the non-blocking try_acquire the read-ahead needs (a pool
// with acquire/release only -- the reference's ResourceManager as it stands --
// runs the reference's one-buffer loop without read-ahead).
template <class Pool, class = void>
struct has_try_acquire : std::false_type {};
template <class Pool>
struct has_try_acquire<Pool, decltype((void)std::declval<Pool&>().try_acquire(
                                 static_cast<typename Pool::buffer_type*>(nullptr)))> : std::true_type {};

template <class Pool>
bool try_acquire_if_any(Pool& pool, typename Pool::buffer_type* out, std::true_type) {
  return pool.try_acquire(out);
}
template <class Pool>
bool try_acquire_if_any(Pool&, typename Pool::buffer_type*, std::false_type) {
  return false;
}

// One helper thread for the upload loop's read-ahead: at most one read in
// flight; get() waits for it and rethrows what it threw.
class ReadAhead {
 public:
  ReadAhead() = default;
  ReadAhead(const ReadAhead&) = delete;
  ReadAhead& operator=(const ReadAhead&) = delete;
  ~ReadAhead() {
    if (!th_.joinable()) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  // Starts job on the helper (made on first use); false if no thread could be
  // made (the caller then reads on its own thread).
  bool start(std::function<size_t()> job) {
    if (!th_.joinable()) {
      try {
        th_ = std::thread([this] { loop(); });
      } catch (...) {
        return false;
      }
    }
    std::lock_guard<std::mutex> lk(mu_);
    job_ = std::move(job);
    has_job_ = true;
    done_ = false;
    err_ = nullptr;
    cv_.notify_all();
    return true;
  }
  size_t get() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return done_; });
    if (err_) std::rethrow_exception(err_);
    return got_;
  }
  double last_s() {  // how long the last job ran (after get())
    std::lock_guard<std::mutex> lk(mu_);
    return last_s_;
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || has_job_; });
      if (stop_ && !has_job_) return;
      std::function<size_t()> job = std::move(job_);
      has_job_ = false;
      lk.unlock();
      size_t got = 0;
      std::exception_ptr err;
      const auto t0 = std::chrono::steady_clock::now();
      try {
        got = job();
      } catch (...) {
        err = std::current_exception();
      }
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      lk.lock();
      last_s_ = s;
      got_ = got;
      err_ = err;
      done_ = true;
      cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
  std::function<size_t()> job_;
  bool has_job_ = false, done_ = true, stop_ = false;
  size_t got_ = 0;
  double last_s_ = 0;
  std::exception_ptr err_;
};

struct StagedWave {
  size_t first = 0, count = 0;
  bool cancelled = false;
  std::vector<uint8_t> dig;
  int backend = 0;
  double hash_s = 0;
};

template <class ReadRange>
StagedWave prehash_wave(const std::vector<qsmd5_part>& parts, size_t first, size_t count,
                        ReadRange& read_range, const StagedOptions& opt, int extra_flags = 0) {
  StagedWave w;
  w.first = first;
  if (opt.should_continue && !opt.should_continue()) {
    w.cancelled = true;
    return w;
  }
  w.count = count;
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<uint64_t> lens(count);
  for (size_t k = 0; k < count; ++k) lens[k] = parts[first + k].size;
  w.dig.resize(16 * count);
  RangeReader<ReadRange> rr(&parts, first, &read_range);
  const int rc = qsmd5_hash_read(lens.data(), count, &RangeReader<ReadRange>::thunk, &rr, opt.staging_bytes,
                                 reinterpret_cast<uint8_t(*)[16]>(w.dig.data()), opt.flags | extra_flags);
  rr.rethrow_if_failed();
  check(rc, "qsmd5_hash_read");
  w.backend = qsmd5_last_backend();  // this thread's call
  w.hash_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return w;
}

}  // namespace detail

// Digests of every part, pulled through read_range in bounded staging (no pool
// buffer used): hex text in part order.
template <class ReadRange>
std::vector<std::string> md5_parts_read(const std::vector<qsmd5_part>& parts, ReadRange&& read_range,
                                        uint64_t staging_bytes = 0, int flags = 0) {
  StagedOptions opt;
  opt.staging_bytes = staging_bytes;
  opt.flags = flags;
  const detail::StagedWave w = detail::prehash_wave(parts, 0, parts.size(), read_range, opt);
  std::vector<std::string> out(parts.size());
  for (size_t k = 0; k < parts.size(); ++k) out[k] = detail::hex(&w.dig[16 * k]);
  return out;
}

// parts, pool, upload: as upload_parts_prehashed.  read_range(file_offset,
// len, char* dst) -> bytes copied: File::ReadNoLoad(off, len, dst).first; with
// `pipeline` it is also called from the helper thread pre-hashing the next
// wave, so it must be thread-safe (ReadNoLoad locks the file) and must not
// wait for a lock this thread holds (PrehashOptions::pipeline).  Stats: waves =
// pre-hash calls, gpu_waves / cpu_waves by their backend, hash_s = time in
// them (reads included), upload_s = the upload loop (its own reads included),
// wait_s = upload time spent waiting for a pre-hash (hashing not hidden),
// and the loop's own split (acquire_s, loop_read_s, upload_call_s, read_ahead).
// A short read or a hashing failure throws before any part of that wave is
// uploaded; the pool is never held by the pre-hash.  The pool needs acquire,
// release, data and size; try_acquire (optional) enables the read-ahead.
template <class Pool, class ReadRange, class Upload>
WaveStats upload_parts_staged(const std::vector<qsmd5_part>& parts, Pool& pool, ReadRange&& read_range,
                              Upload&& upload, const StagedOptions& opt = StagedOptions()) {
  using clock = std::chrono::steady_clock;
  auto secs = [](clock::time_point a, clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
  };
  WaveStats st;
  const auto t_start = clock::now();
  if (parts.empty()) return st;
  const size_t per = opt.wave_parts ? opt.wave_parts : parts.size();
  // the size of the wave after one of `prev` parts (0: the first wave)
  auto wave_size = [&](size_t prev) {
    if (!opt.first_wave_parts || !opt.wave_parts || !opt.pipeline) return per;
    return prev ? std::min(per, 2 * prev) : std::min(per, opt.first_wave_parts);
  };
  auto prep = [&](size_t first, size_t count, bool background) {
    return detail::prehash_wave(parts, first, std::min(count, parts.size() - first), read_range, opt,
                                background ? QSMD5_FLAG_BACKGROUND : 0);
  };
  // Whether the wave [first, first + count) is hidden behind `uploading`
  // parts' uploads (StagedOptions::background_waves).
  double loop_s = 0;  // the upload loop's time so far, and the parts it uploaded
  size_t loop_parts = 0;
  auto hidden = [&](size_t first, size_t count, size_t uploading) {
    if (!(opt.pipeline && opt.background_waves) || first == 0 || loop_parts == 0) return false;
    qsmd5_rates r;
    if (qsmd5_get_rates(&r) != 0 || r.gpu_chain_gibs <= 0) return false;
    uint64_t longest = 0, total = 0;
    for (size_t i = first; i < std::min(parts.size(), first + count); ++i) {
      longest = std::max<uint64_t>(longest, parts[i].size);
      total += parts[i].size;
    }
    const double gib = 1073741824.0;
    const double gpu_s = (double)longest / (r.gpu_chain_gibs * gib) + (double)total / (12.0 * gib);
    return (double)uploading * (loop_s / (double)loop_parts) >= 1.25 * gpu_s;
  };
  std::future<detail::StagedWave> ahead;
  auto drain_ahead = [&]() noexcept {
    if (!ahead.valid()) return;
    try {
      (void)ahead.get();
    } catch (...) {
    }
  };
  auto stop_requested = [&] { return opt.should_continue && !opt.should_continue(); };
  const bool read_ahead = opt.pipeline && opt.read_ahead;
  detail::ReadAhead reader;  // joined on return, after every read it ran was waited for
  double last_upload_s = 0, last_read_s = 0;  // the last part's upload() and read
  const auto tw = clock::now();
  detail::StagedWave cur = prep(0, wave_size(0), false);
  st.wait_s += secs(tw, clock::now());
  for (;;) {
    if (cur.cancelled) {
      st.stopped = true;
      break;
    }
    const size_t n = cur.count, next = cur.first + n;
    ++st.waves;
    st.parts += n;
    st.widest_wave = std::max(st.widest_wave, n);
    st.hash_s += cur.hash_s;
    switch (cur.backend) {
      case QSMD5_BACKEND_GPU: ++st.gpu_waves; break;
      case QSMD5_BACKEND_SPLIT: ++st.split_waves; break;
      default: ++st.cpu_waves; break;
    }
    if (opt.pipeline && next < parts.size()) {
      try {
        ahead = std::async(std::launch::async, prep, next, wave_size(n), hidden(next, wave_size(n), n));
      } catch (...) {
        // no thread or no memory for one: the next wave is pre-hashed here, after this one
      }
    }
    const auto t0 = clock::now();
    const size_t uploaded0 = st.uploaded;
    size_t k = 0;
    // the read-ahead in flight: part cur.first + ra_k into ra_buf
    bool ra_valid = false;
    size_t ra_k = 0;
    typename Pool::buffer_type ra_buf = typename Pool::buffer_type();
    auto drop_read_ahead = [&]() noexcept {
      if (!ra_valid) return;
      try {
        (void)reader.get();
      } catch (...) {
      }
      pool.release(ra_buf);
      ra_valid = false;
    };
    try {
      for (; k < n; ++k) {
        if (stop_requested()) break;
        const qsmd5_part& p = parts[cur.first + k];
        // The reference's loop body (QSTransferManager.cpp:609-665): one
        // buffer, acquired while this thread holds none -- or the buffer the
        // read-ahead already filled with this part.
        typename Pool::buffer_type b;
        size_t got = 0;
        const auto r0 = clock::now();
        if (ra_valid && ra_k == k) {
          ra_valid = false;
          b = ra_buf;
          try {
            got = reader.get();
          } catch (...) {
            pool.release(b);
            throw;
          }
          st.loop_read_s += secs(r0, clock::now());
          last_read_s = reader.last_s();
        } else {
          b = pool.acquire();
          st.acquire_s += secs(r0, clock::now());
          if (!Pool::data(b)) throw std::runtime_error("transfer buffer pool is shut down: upload stopped");
          if (Pool::size(b) < p.size) {
            pool.release(b);
            throw std::invalid_argument("pool buffer smaller than a part");
          }
          const auto r1 = clock::now();
          try {
            got = read_range(p.offset, (size_t)p.size, Pool::data(b));
          } catch (...) {
            pool.release(b);
            throw;
          }
          last_read_s = secs(r1, clock::now());
          st.loop_read_s += last_read_s;
        }
        try {
          if (got != p.size)
            throw std::runtime_error("short read of part " + std::to_string(p.part_number) + ": " +
                                     std::to_string(got) + " of " + std::to_string(p.size) + " bytes");
          if (stop_requested()) {  // asked again after the read, as the reference (:645)
            pool.release(b);
            break;
          }
          if (opt.source_changed && opt.source_changed()) {
            uint8_t d[16];
            detail::check(qsmd5_hash_one(Pool::data(b), p.size, d), "qsmd5_hash_one");
            std::memcpy(&cur.dig[16 * k], d, 16);
            ++st.rehashed;
          }
          // The next part's read, behind this part's upload, into a buffer
          // that is free right now (never a blocking acquire while holding b)
          // -- where the uploads take longer than the reads (the last part's
          // of each, measured): uploads that return at once hide nothing, and
          // the read would only contend with the next wave's pre-hash.
          if (read_ahead && k + 1 < n && last_upload_s > last_read_s) {
            typename Pool::buffer_type b2;
            const qsmd5_part& q = parts[cur.first + k + 1];
            if (detail::try_acquire_if_any(pool, &b2, detail::has_try_acquire<Pool>())) {
              if (Pool::size(b2) >= q.size &&
                  reader.start([&read_range, q, b2] {
                    return (size_t)read_range(q.offset, (size_t)q.size, Pool::data(b2));
                  })) {
                ra_valid = true;
                ra_k = k + 1;
                ra_buf = b2;
                ++st.read_ahead;
              } else {
                pool.release(b2);
              }
            }
          }
          const auto u0 = clock::now();
          upload(p, b, detail::hex(&cur.dig[16 * k]));
          last_upload_s = secs(u0, clock::now());
          st.upload_call_s += last_upload_s;
        } catch (...) {
          pool.release(b);  // not handed over
          throw;
        }
        if (!opt.upload_releases) pool.release(b);  // ReceivedHandlerMultipleUpload
        ++st.uploaded;
      }
    } catch (...) {
      drop_read_ahead();
      drain_ahead();
      throw;
    }
    drop_read_ahead();  // stopped inside the wave: the part read ahead is not uploaded
    st.upload_s += secs(t0, clock::now());
    loop_s += secs(t0, clock::now());
    loop_parts += st.uploaded - uploaded0;
    if (k < n) {
      drain_ahead();
      st.stopped = true;
      break;
    }
    if (next >= parts.size()) break;
    const auto t1 = clock::now();
    cur = ahead.valid() ? ahead.get() : prep(next, wave_size(n), false);
    st.wait_s += secs(t1, clock::now());
  }
  st.wall_s = secs(t_start, clock::now());
  return st;
}

// The vector-of-buffers form: `pool` is this upload's own set of buffers
// (a BlockingPool over them), and upload(part, const char* buf, hex) returns
// when the part is sent.
template <class Read, class Upload>
WaveStats upload_parts_prehashed(const std::vector<qsmd5_part>& parts,
                                 const std::vector<PoolBuffer>& buffers, Read&& read, Upload&& upload,
                                 const PrehashOptions& opt = PrehashOptions()) {
  if (buffers.empty() && !parts.empty()) throw std::invalid_argument("empty buffer pool");
  BlockingPool pool(buffers);
  PrehashOptions o = opt;
  o.upload_releases = false;
  return upload_parts_prehashed(
      parts, pool, read,
      [&](const qsmd5_part& p, const PoolBuffer& b, const std::string& hex) { upload(p, b.data, hex); }, o);
}

}  // namespace qsmd5

#endif  // QSFS_AMD_QSFS_MULTIPART_HPP_
