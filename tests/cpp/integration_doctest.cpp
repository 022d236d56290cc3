// tests/cpp/integration_doctest.cpp -- compiles and runs the DoMultiPartUpload
// binding exactly as INTEGRATION.md §3 prints it.
//
// tests/test_integration_doc.py cuts the §3 code block in two -- the adapter
// (namespace scope, INTEGRATION_ADAPTER) and the loop that replaces
// QSTransferManager::DoMultiPartUpload's (:602-673; INTEGRATION_LOOP) -- and
// compiles this file with both.  Around them stand minimal mocks with the
// SHAPE the snippet relies on (our own test doubles of qsfs's interfaces,
// written here, not qsfs code): a blocking pool with the added TryAcquire, a
// paged file, a transfer handle with a cancel flag, and an upload handler that
// releases the part's buffer, as ReceivedHandlerMultipleUpload does
// (QSTransferManager.cpp:215-220).  The run checks the wiring: every part
// handed on carries the MD5 of its bytes, cancelled or unsent parts are marked
// failed, and every buffer is back in the pool.
//
// usage: integration_doctest <file_bytes> <part_bytes> <pool_buffers> <cancel_after|-1> [flush] [write_after]
//   flush: async (this program's default; qsfs's -M mode: File::Flush
//   submitted the upload and returned, no lock held), sync (qsfs's default
//   single-threaded mode: the flushing thread holds the file's lock through
//   the upload and sets the flag, as File::Flush's synchronous branch with
//   the binding's addition), sync_unflagged (the negative control: the lock held,
//   the flag not set -- a helper thread's read waits forever; the watchdog
//   exits 3).  write_after: once that many parts went out, the file is
//   written (the part after the next to go out changes) as by another descriptor.
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
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/qsmd5.h"

using std::make_shared;
using std::shared_ptr;

// ---- test doubles of the qsfs interfaces the snippet names --------------------
namespace QS {
namespace Data {
typedef shared_ptr<std::vector<char>> Buffer;
}
}  // namespace QS
typedef QS::Data::Buffer Resource;

class ResourceManager {  // blocking Acquire (ResourceManager.cpp:53-67) + the added TryAcquire
 public:
  ResourceManager(size_t n, size_t size) {
    for (size_t i = 0; i < n; ++i) free_.push_back(make_shared<std::vector<char>>(size));
    total_ = n;
  }
  Resource Acquire() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !free_.empty(); });
    Resource r = free_.back();
    free_.pop_back();
    return r;
  }
  Resource TryAcquire() {
    std::lock_guard<std::mutex> lk(mu_);
    if (free_.empty()) return Resource();
    Resource r = free_.back();
    free_.pop_back();
    return r;
  }
  void Release(const Resource& r) {
    if (!r) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      free_.push_back(r);
    }
    cv_.notify_one();
  }
  size_t Free() {
    std::lock_guard<std::mutex> lk(mu_);
    return free_.size();
  }
  size_t total_ = 0;

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Resource> free_;
};

struct Part {
  uint16_t id;
  uint64_t begin, size;
  std::string md5;
  void SetContentMD5(const std::string& hex) { md5 = hex; }
  const std::string& GetContentMD5() const { return md5; }
};

namespace TransferStatus {
enum Value { InProgress, Failed };
}

struct TransferHandle {  // locked like the real one (TransferHandle.h:159-162): asked from two threads
  int cancel_after = -1;  // Cancel() once this many parts went out
  std::vector<uint16_t> pending, failed;
  TransferStatus::Value status = TransferStatus::InProgress;
  mutable std::mutex mu;
  bool ShouldContinue() const {
    std::lock_guard<std::mutex> lk(mu);
    return cancel_after < 0 || (int)pending.size() < cancel_after;
  }
  void AddPendingPart(const shared_ptr<Part>& p) {
    std::lock_guard<std::mutex> lk(mu);
    pending.push_back(p->id);
  }
  void ChangePartToFailed(const shared_ptr<Part>& p) {
    std::lock_guard<std::mutex> lk(mu);
    failed.push_back(p->id);
  }
  void UpdateStatus(TransferStatus::Value v) {
    std::lock_guard<std::mutex> lk(mu);
    status = v;
  }
};

struct PagedFile {  // File::ReadNoLoad: bytes [off, off + len) into dst, under the file's lock
  std::vector<char> bytes;
  mutable std::recursive_mutex m_mutex;  // File's (File.h); ReadNoLoad locks it (File.cpp:310)
  bool m_flushingUnderLock = false;      // the binding's added flag
  bool IsFlushingUnderLock() const { return m_flushingUnderLock; }
  std::atomic<uint64_t> m_writeVersion{0};  // the binding's added write counter
  uint64_t GetWriteVersion() const { return m_writeVersion.load(); }
  void Write(uint64_t off, const char* src, size_t len) {  // File::Write, under the lock
    std::lock_guard<std::recursive_mutex> lock(m_mutex);
    memcpy(bytes.data() + off, src, len);
    ++m_writeVersion;
  }
  std::pair<size_t, int> ReadNoLoad(uint64_t off, uint64_t len, char* dst) const {
    std::lock_guard<std::recursive_mutex> lock(m_mutex);
    memcpy(dst, bytes.data() + off, len);
    return std::make_pair((size_t)len, 0);
  }
};

struct IOStream {  // a view of the pooled buffer's first `len` bytes (StreamBuf.cpp:32-48)
  IOStream(const Resource& b, uint64_t n) : buf(b), len(n) {}
  Resource buf;
  uint64_t len;
};

struct Client {
  std::map<uint16_t, std::string> sent;   // part id -> Content-MD5 the SDK got
  std::map<uint16_t, std::string> truth;  // part id -> MD5 of the bytes the SDK got
};
typedef int UploadResult;

struct ReceivedHandlerMultipleUpload {  // releases the part's buffer (QSTransferManager.cpp:215-220)
  ReceivedHandlerMultipleUpload(shared_ptr<TransferHandle>, shared_ptr<Part>, shared_ptr<IOStream> s,
                                shared_ptr<ResourceManager> m, shared_ptr<Client>)
      : stream(std::move(s)), mgr(std::move(m)) {}
  void operator()(UploadResult) {
    mgr->Release(stream->buf);
    stream->buf.reset();
  }
  shared_ptr<IOStream> stream;
  shared_ptr<ResourceManager> mgr;
};

static void DebugError(const std::string& m) { fprintf(stderr, "DebugError: %s\n", m.c_str()); }

// ---- the adapter, as INTEGRATION.md §3 prints it -------------------------------
#include INTEGRATION_ADAPTER

struct Uploader {
  shared_ptr<ResourceManager> rm;
  shared_ptr<Client> client = make_shared<Client>();
  PagedFile* writer = nullptr;  // another descriptor writing the file mid-upload
  int write_after = -1;         // ... once this many parts went out
  uint64_t write_off = 0;
  shared_ptr<ResourceManager> GetBufferManager() { return rm; }
  shared_ptr<Client> GetClient() { return client; }
  // QSTransferManager::MultipleUploadWrapper (:721-727) with the digest argument
  UploadResult MultipleUploadWrapper(const shared_ptr<TransferHandle>&, const shared_ptr<Part>& part,
                                     const shared_ptr<IOStream>& stream) {
    if (!stream->buf || stream->len != part->size) return -1;
    client->sent[part->id] = part->GetContentMD5();
    uint8_t d[16];
    char hex[33];
    if (qsmd5_hash_one(stream->buf->data(), stream->len, d)) return -1;
    qsmd5_hex(d, hex);
    client->truth[part->id] = hex;
    if (writer && (int)client->sent.size() == write_after) {
      const char junk[] = "written by another descriptor during the upload";
      writer->Write(write_off, junk, sizeof(junk));
    }
    return 0;
  }

  void DoMultiPartUpload(const shared_ptr<TransferHandle>& handle, const PagedFile* file,
                         std::map<uint16_t, shared_ptr<Part>>& queuedParts, std::vector<qsmd5_part> queued) {
    // ---- the loop, as INTEGRATION.md §3 prints it; its first line's `parts`
    // ("from handle->GetQueuedParts(), in part order") is initialised from
    // `queued` (the one substitution tests/test_integration_doc.py makes)
#include INTEGRATION_LOOP
  }
};

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: integration_doctest <file_bytes> <part_bytes> <pool_buffers> <cancel_after|-1>\n");
    return 2;
  }
  const uint64_t fsz = strtoull(argv[1], nullptr, 0), psz = strtoull(argv[2], nullptr, 0);
  const size_t pool_n = strtoull(argv[3], nullptr, 0);
  const int cancel_after = atoi(argv[4]);
  PagedFile file;
  file.bytes.resize(fsz);
  uint32_t x = 777;
  for (auto& c : file.bytes) c = (char)((x = x * 1103515245u + 12345u) >> 16);
  size_t n = 0;
  if (qsmd5_plan_parts(fsz, psz, 4ull << 20, 0, 0, nullptr, 0, &n)) return 1;
  std::vector<qsmd5_part> plan(n);
  if (qsmd5_plan_parts(fsz, psz, 4ull << 20, 0, 0, plan.data(), n, &n)) return 1;
  std::map<uint16_t, shared_ptr<Part>> queued;
  for (const auto& p : plan) queued[(uint16_t)p.part_number] = make_shared<Part>(Part{(uint16_t)p.part_number, p.offset, p.size, ""});
  uint64_t largest = 0;
  for (const auto& p : plan) largest = std::max<uint64_t>(largest, p.size);

  const std::string flush = argc > 5 ? argv[5] : "async";
  Uploader up;
  up.write_after = argc > 6 ? atoi(argv[6]) : -1;
  if (up.write_after >= 0) {
    up.writer = &file;
    // the part after the next one to go out: already pre-hashed (its wave is
    // the one uploading) and not yet read into a buffer (the next one may be:
    // the loop's read-ahead reads it while this part uploads)
    const qsmd5_part& next = plan[std::min<size_t>(up.write_after + 1, plan.size() - 1)];
    up.write_off = next.offset + next.size / 2;
  }
  up.rm = make_shared<ResourceManager>(pool_n, largest);
  auto handle = make_shared<TransferHandle>();
  handle->cancel_after = cancel_after;
  std::atomic<bool> done{false};
  std::thread watchdog([&] {
    for (int i = 0; i < 300 && !done.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(50));
    if (!done.load()) {
      printf("{\"deadlock\": true, \"flush\": \"%s\"}\n", flush.c_str());
      fflush(stdout);
      _exit(3);
    }
  });
  {
    std::unique_lock<std::recursive_mutex> held(file.m_mutex, std::defer_lock);
    if (flush != "async") held.lock();  // File::Flush's lock_guard (File.cpp:619)
    file.m_flushingUnderLock = flush == "sync";
    up.DoMultiPartUpload(handle, &file, queued, plan);
    file.m_flushingUnderLock = false;
  }
  done.store(true);
  watchdog.join();

  int bad = 0;
  auto expect = [&](bool ok, const char* what) {
    if (!ok) {
      fprintf(stderr, "FAIL: %s\n", what);
      ++bad;
    }
  };
  const size_t want_sent = cancel_after < 0 ? n : std::min<size_t>(n, (size_t)cancel_after);
  expect(up.client->sent.size() == want_sent, "parts handed to the SDK");
  for (const auto& kv : up.client->sent) {
    expect(kv.second == up.client->truth[kv.first], "a part's Content-MD5 is the MD5 of the bytes sent");
    if (up.write_after >= 0) continue;
    const Part& p = *queued[kv.first];
    uint8_t d[16];
    char hex[33];
    if (qsmd5_hash_one(file.bytes.data() + p.begin, p.size, d)) return 1;
    qsmd5_hex(d, hex);
    expect(kv.second == hex, "a part's Content-MD5 is the MD5 of the file's bytes");
  }
  std::set<uint16_t> failed(handle->failed.begin(), handle->failed.end());
  expect(failed.size() == n - want_sent, "every part not sent is marked failed");
  for (uint16_t id : failed) expect(!up.client->sent.count(id), "a failed part was not sent");
  expect(up.rm->Free() == pool_n, "every buffer is back in the pool");
  printf("{\"parts\": %zu, \"sent\": %zu, \"failed\": %zu, \"pool_free\": %zu, \"bad\": %d, \"deadlock\": false}\n", n,
         up.client->sent.size(), failed.size(), up.rm->Free(), bad);
  return bad ? 1 : 0;
}
