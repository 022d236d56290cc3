// tests/cpp/multipart_harness.cpp -- QSTransferManager::DoMultiPartUpload with
// the batch pre-hash, end to end.
//
// Builds a file the way qsfs holds one after File::Flush loaded it: its bytes
// live in many separately allocated pages of assorted sizes (Page,
// src/data/Page.h; qsfs pages follow the FUSE write sizes), keyed by offset.
// Then it runs the reference's upload loop through the drop-in helper
// qsmd5::upload_parts_prehashed (qsfs-fuse_amd/host/qsfs_multipart.hpp):
//   - parts sliced as PrepareUpload does (qsmd5_plan_parts, QSTransferManager.cpp:475-550);
//   - a pool of transfer buffers (ResourceManager; default 5 x 10 MiB);
//   - each part gathered from the pages into a pool buffer by a ReadNoLoad
//     restatement (File.cpp:308-375: the pages intersecting [off, off + len),
//     copied piece by piece; bytes no page holds are a short read);
//   - one qsmd5_hash_batch_ex(QSMD5_FLAG_HOST) per wave of pool-size parts;
//   - each part's hex digest handed to the "uploader" (UploadMultipart's
//     SetContentMD5, QSClient.cpp:369-371), which records it.
// File content: part-aligned mode (--aligned) makes part i = LCG(12345 + i),
// the parts of tests/golden/batch_10MiB.json; otherwise the file is one
// LCG(seed) stream.  Prints one JSON object with the digests in part order
// and where the time went (the last pass; hash_s_runs lists every pass's hash
// time); tests/test_gpu_multipart.py and
// tests/test_multipart_cpu.py check the digests.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../../qsfs-fuse_amd/host/qsfs_multipart.hpp"

namespace {

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

}  // namespace

int main(int argc, char** argv) {
  uint64_t size = 64ull * 10 * 1024 * 1024;
  size_t pool_n = 5;
  bool aligned = false, pinned = false, slab = false, reg = false;
  uint32_t seed = 12345;
  uint64_t buf = 10ull << 20;
  int repeat = 1;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* key) { return a.rfind(key, 0) == 0 ? a.c_str() + strlen(key) : nullptr; };
    if (const char* v = val("--size=")) size = strtoull(v, nullptr, 0);
    else if (const char* v = val("--pool=")) pool_n = strtoull(v, nullptr, 0);
    else if (const char* v = val("--seed=")) seed = (uint32_t)strtoul(v, nullptr, 0);
    else if (const char* v = val("--buf=")) buf = strtoull(v, nullptr, 0);
    else if (const char* v = val("--repeat=")) repeat = std::max(1, atoi(v));
    else if (a == "--aligned") aligned = true;
    else if (a == "--pinned") pinned = true;
    else if (a == "--slab") slab = true;
    else if (a == "--register") reg = true;
    else {
      fprintf(stderr, "unknown argument %s\n", argv[i]);
      return 2;
    }
  }
  // The file's bytes, cut into pages of 1 KiB .. 3 MiB.
  PagedFile file;
  file.size = size;
  {
    std::vector<uint8_t> all(size);
    if (aligned) {
      for (uint64_t p = 0; p * buf < size; ++p)
        lcg(12345u + (uint32_t)p, all.data() + p * buf, std::min(buf, size - p * buf));
    } else {
      lcg(seed, all.data(), size);
    }
    std::mt19937_64 rng(seed);
    for (uint64_t off = 0; off < size;) {
      const uint64_t len = std::min<uint64_t>(size - off, 1024 + rng() % (3u << 20));
      file.pages.emplace(off, std::vector<char>(all.begin() + off, all.begin() + off + len));
      off += len;
    }
  }
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
  std::vector<std::string> md5(n);
  (void)qsmd5_init(0);  // runtime start-up outside the timed uploads (-ENODEV without a GPU)
  // --register: lock the pageable pool's pages once, as a daemon would at start-up
  double register_s = 0;
  if (reg && !pinned) {
    const auto r0 = std::chrono::steady_clock::now();
    // one registration per allocation: the slab at once, else each buffer
    std::vector<qsmd5::PoolBuffer> regs =
        slab ? std::vector<qsmd5::PoolBuffer>{{slab_pool->data(), slab_pool->bytes()}} : pool;
    for (auto& b : regs)
      if (qsmd5_register_host(b.data, b.size)) {
        fprintf(stderr, "qsmd5_register_host: %s\n", qsmd5_last_error());
        return 1;
      }
    register_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - r0).count();
  }
  // --repeat: upload the file again through the same pool, as a daemon reuses
  // its buffers; the first pass pays HIP's first-touch locking of pageable pages.
  std::vector<double> hash_runs;
  qsmd5::WaveStats st;
  double total = 0;
  for (int rep = 0; rep < repeat; ++rep) {
    const auto t0 = std::chrono::steady_clock::now();
    try {
      st = qsmd5::upload_parts_prehashed(
          parts, pool,
          [&](const qsmd5_part& p, char* dst) { return file.read(p.offset, p.size, dst); },
          [&](const qsmd5_part& p, const char*, const std::string& hex) { md5[p.part_number - 1] = hex; });
    } catch (const std::exception& e) {
      fprintf(stderr, "upload failed: %s\n", e.what());
      return 1;
    }
    total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    hash_runs.push_back(st.hash_s);
  }
  if (pinned && !slab)
    for (auto& b : pool) qsmd5_free_pinned(b.data);
  if (reg && !pinned) {
    if (slab) qsmd5_unregister_host(slab_pool->data());
    else
      for (auto& b : pool) qsmd5_unregister_host(b.data);
  }
  printf("{\"size\": %llu, \"parts\": %zu, \"pages\": %zu, \"pool\": %zu, \"pinned\": %s, "
         "\"slab\": %s, \"registered\": %s, \"register_s\": %.6f, \"waves\": %zu, \"gpu_waves\": %zu, \"cpu_waves\": %zu, \"split_waves\": %zu, \"seconds\": %.6f, "
         "\"gather_s\": %.6f, \"hash_s\": %.6f, \"upload_s\": %.6f, \"part_sizes\": [",
         (unsigned long long)size, n, file.pages.size(), pool_n, pinned ? "true" : "false",
         slab ? "true" : "false", reg && !pinned ? "true" : "false", register_s, st.waves,
         st.gpu_waves, st.cpu_waves, st.split_waves, total, st.gather_s, st.hash_s, st.upload_s);
  for (size_t i = 0; i < n; ++i) printf("%s%llu", i ? ", " : "", (unsigned long long)parts[i].size);
  printf("], \"hash_s_runs\": [");
  for (size_t i = 0; i < hash_runs.size(); ++i) printf("%s%.6f", i ? ", " : "", hash_runs[i]);
  printf("], \"md5\": [");
  for (size_t i = 0; i < n; ++i) printf("%s\"%s\"", i ? ", " : "", md5[i].c_str());
  printf("]}\n");
  return 0;
}
