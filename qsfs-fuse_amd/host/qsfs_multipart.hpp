// qsfs-fuse_amd/host/qsfs_multipart.hpp -- the batch pre-hash inside qsfs's
// multipart upload loop.
//
// The reference uploads a file's parts in QSTransferManager::DoMultiPartUpload
// (src/client/QSTransferManager.cpp:602-673): for each queued part it acquires
// a pooled transfer buffer (ResourceManager::Acquire, ResourceManager.cpp:54-70),
// gathers the part's bytes from the file's pages into it (File::ReadNoLoad,
// src/data/File.cpp:308-375), wraps it in an IOStream of the part's size, and
// hands it to UploadMultipart, which computes md5(stream) for the
// Content-MD5 (QSClient.cpp:369-371): one buffer, one serial hash, at a time.
//
// upload_parts_prehashed() keeps that loop and its buffer discipline but
// hashes in waves: it gathers as many parts as the pool has buffers, hashes the
// whole wave with ONE qsmd5_hash_batch_ex(QSMD5_FLAG_HOST) call (pool buffers
// are host memory), then hands each part, its buffer and its hex digest to the
// uploader.  The library routes the wave by size (QSMD5_BACKEND=auto): a
// default qsfs pool (50 MiB of 10 MiB buffers = 5, configure/Default.cpp:157,
// TransferManager.cpp:78-84) is below the GPU break-even and hashes on the CPU;
// a larger pool (-Z) or a whole flushed file goes to the gfx950 kernels.
//
// Header-only over the C-ABI (include/qsmd5.h).  Throws qsmd5::Error on a
// hashing failure and std::runtime_error on a short read, as the reference
// stops the upload there (QSTransferManager.cpp:622-643).
#ifndef QSFS_AMD_QSFS_MULTIPART_HPP_
#define QSFS_AMD_QSFS_MULTIPART_HPP_

#include <algorithm>
#include <chrono>
#include <stdexcept>
#include <string>
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

// What one wave did: parts hashed, and which backend the library picked.
struct WaveStats {
  size_t waves = 0, parts = 0;
  size_t gpu_waves = 0, cpu_waves = 0, split_waves = 0;  // by qsmd5_last_backend of each wave
  double gather_s = 0, hash_s = 0, upload_s = 0;  // wall time in each phase
};

// parts:    the file's parts as PrepareUpload slices them (qsmd5_plan_parts).
// pool:     the transfer buffers, each at least the largest part.
// read:     read(part, char* buf) -> bytes gathered (File::ReadNoLoad).
// upload:   upload(part, const char* buf, const std::string& hex) hands the part
//           on (UploadMultipart with SetContentMD5(hex)); the buffer may be
//           reused once it returns.
template <class Read, class Upload>
WaveStats upload_parts_prehashed(const std::vector<qsmd5_part>& parts,
                                 const std::vector<PoolBuffer>& pool, Read&& read,
                                 Upload&& upload) {
  if (pool.empty() && !parts.empty()) throw std::invalid_argument("empty buffer pool");
  WaveStats st;
  std::vector<qsmd5_chunk> chunks;
  std::vector<uint8_t> dig;
  for (size_t first = 0; first < parts.size(); first += pool.size()) {
    using clock = std::chrono::steady_clock;
    auto secs = [](clock::time_point a, clock::time_point b) {
      return std::chrono::duration<double>(b - a).count();
    };
    const auto t0 = clock::now();
    const size_t n = std::min(pool.size(), parts.size() - first);
    chunks.resize(n);
    for (size_t k = 0; k < n; ++k) {
      const qsmd5_part& p = parts[first + k];
      if (pool[k].size < p.size) throw std::invalid_argument("pool buffer smaller than a part");
      const size_t got = read(p, pool[k].data);
      if (got != p.size)
        throw std::runtime_error("short read of part " + std::to_string(p.part_number) + ": " +
                                 std::to_string(got) + " of " + std::to_string(p.size) + " bytes");
      chunks[k] = qsmd5_chunk{pool[k].data, p.size};
    }
    const auto t1 = clock::now();
    dig.resize(16 * n);
    detail::check(qsmd5_hash_batch_ex(chunks.data(), n, reinterpret_cast<uint8_t(*)[16]>(dig.data()),
                                      QSMD5_FLAG_HOST),
                  "qsmd5_hash_batch_ex");
    ++st.waves;
    st.parts += n;
    switch (qsmd5_last_backend()) {
      case QSMD5_BACKEND_GPU: ++st.gpu_waves; break;
      case QSMD5_BACKEND_SPLIT: ++st.split_waves; break;  // longest parts on the CPU, the rest on the GPU
      default: ++st.cpu_waves; break;
    }
    const auto t2 = clock::now();
    for (size_t k = 0; k < n; ++k) upload(parts[first + k], pool[k].data, detail::hex(&dig[16 * k]));
    const auto t3 = clock::now();
    st.gather_s += secs(t0, t1);
    st.hash_s += secs(t1, t2);
    st.upload_s += secs(t2, t3);
  }
  return st;
}

}  // namespace qsmd5

#endif  // QSFS_AMD_QSFS_MULTIPART_HPP_
