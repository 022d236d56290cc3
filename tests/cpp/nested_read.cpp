// tests/cpp/nested_read.cpp -- read callbacks of qsmd5_hash_read that call
// back into the library (include/qsmd5.h: "It may call other qsmd5 entry
// points (not qsmd5_shutdown)"), ADVICE r05.
//
// Mode "shutdown" (ADVICE r05, medium): QSMD5_FLAG_READ_PARALLEL, so the
// window's rows are read on the library's reader threads too.  The first read
// that runs on a reader thread starts a thread calling qsmd5_shutdown, waits
// until that shutdown is pending (it waits for this call, which holds the
// runtime's call lock), then calls qsmd5_hash_one from the reader thread.
// That nested call must not wait at the shutdown gate: the outer call would
// never finish, and shutdown would wait for it forever.  Every read callback
// also hashes its window with qsmd5_hash_one (nested calls from every thread).
//
// Mode "nested-read" (ADVICE r05, low): each read callback of the outer batch
// calls qsmd5_hash_read itself (the window as one chunk).  Under auto routing
// the nested batch takes the CPU path (it needs no read slot); under
// QSMD5_FLAG_GPU_ONLY it gets a slot only if one is free (-EDEADLK otherwise):
// with QSMD5_READ_SLOTS=1 and the outer batch on the GPU, never a deadlock.
//
// argv: mode [outer flags: "gpu" = QSMD5_FLAG_GPU_ONLY, "cpu", "auto"] [inner: same]
// A watchdog prints {"deadlock": true} and exits 3 after 30 s.  Prints one JSON
// line; exit 0 = digests right and no deadlock.
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/qsmd5.h"

namespace {

constexpr size_t kChunks = 64;
constexpr uint64_t kLen = (1u << 20) + 77;

struct Ctx {
  std::vector<std::vector<uint8_t>> data;
  std::thread::id caller;
  std::atomic<bool> shutdown_started{false};
  std::atomic<int> shutdown_rc{1};
  std::atomic<bool> shutdown_done{false};
  std::thread shutter;
  std::mutex mu;
  std::atomic<uint64_t> nested_calls{0}, nested_errors{0}, reader_thread_reads{0};
  std::atomic<uint64_t> nested_edeadlk{0}, nested_ok{0};
  int inner_flags = 0;
  bool nested_read = false;
};

int flags_of(const char* s) {
  if (!strcmp(s, "gpu")) return QSMD5_FLAG_GPU_ONLY;
  if (!strcmp(s, "cpu")) return QSMD5_FLAG_CPU_ONLY;
  return 0;
}

struct One {
  const uint8_t* p;
  static uint64_t read(void* user, size_t, uint64_t offset, uint64_t len, void* dst) {
    memcpy(dst, static_cast<One*>(user)->p + offset, len);
    return len;
  }
};

uint64_t read_cb(void* user, size_t chunk, uint64_t offset, uint64_t len, void* dst) {
  Ctx& c = *static_cast<Ctx*>(user);
  const uint8_t* src = c.data[chunk].data() + offset;
  memcpy(dst, src, len);
  const bool reader_thread = std::this_thread::get_id() != c.caller;
  if (reader_thread) c.reader_thread_reads.fetch_add(1);
  if (!c.nested_read && reader_thread && !c.shutdown_started.exchange(true)) {
    // a shutdown from another thread, pending while this call is in flight
    c.shutter = std::thread([&c] {
      c.shutdown_rc.store(qsmd5_shutdown());
      c.shutdown_done.store(true);
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(100));  // it is pending by now
  }
  uint8_t d[16], want[16];
  c.nested_calls.fetch_add(1);
  if (c.nested_read) {
    One one{src};
    const int rc = qsmd5_hash_read(&len, 1, &One::read, &one, 0, reinterpret_cast<uint8_t(*)[16]>(d),
                                   c.inner_flags);
    if (rc == -EDEADLK) {
      c.nested_edeadlk.fetch_add(1);
      return len;
    }
    if (rc != 0) {
      c.nested_errors.fetch_add(1);
      return len;
    }
    c.nested_ok.fetch_add(1);
  } else if (qsmd5_hash_one(src, len, d) != 0) {
    c.nested_errors.fetch_add(1);
    return len;
  }
  qsmd5_chunk ch = {src, len};
  if (qsmd5_hash_batch_ex(&ch, 1, reinterpret_cast<uint8_t(*)[16]>(want), QSMD5_FLAG_CPU_ONLY) != 0 ||
      memcmp(d, want, 16) != 0)
    c.nested_errors.fetch_add(1);
  return len;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "shutdown";
  const int outer = argc > 2 ? flags_of(argv[2]) : 0;
  Ctx c;
  c.nested_read = mode == "nested-read";
  c.inner_flags = argc > 3 ? flags_of(argv[3]) : 0;
  c.caller = std::this_thread::get_id();
  c.data.resize(kChunks);
  uint32_t x = 4242;
  for (auto& v : c.data) {
    v.resize(kLen);
    for (auto& b : v) {
      x = x * 1103515245u + 12345u;
      b = (uint8_t)(x >> 16);
    }
  }
  std::vector<uint64_t> lens(kChunks, kLen);
  std::vector<uint8_t> want(16 * kChunks), got(16 * kChunks);
  std::vector<qsmd5_chunk> ch(kChunks);
  for (size_t i = 0; i < kChunks; ++i) ch[i] = qsmd5_chunk{c.data[i].data(), kLen};
  if (qsmd5_hash_batch_ex(ch.data(), kChunks, reinterpret_cast<uint8_t(*)[16]>(want.data()),
                          QSMD5_FLAG_CPU_ONLY) != 0)
    return 1;
  std::atomic<bool> finished{false};
  std::thread watchdog([&] {
    for (int i = 0; i < 300 && !finished.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
    if (!finished.load()) {
      printf("{\"deadlock\": true, \"mode\": \"%s\"}\n", mode.c_str());
      fflush(stdout);
      _exit(3);
    }
  });
  const int flags = outer | (c.nested_read ? 0 : QSMD5_FLAG_READ_PARALLEL);
  const auto t0 = std::chrono::steady_clock::now();
  // a 4 MiB budget: many windows, each window's rows over 4 reader threads
  const int rc = qsmd5_hash_read(lens.data(), kChunks, read_cb, &c, 4u << 20,
                                 reinterpret_cast<uint8_t(*)[16]>(got.data()), flags);
  const int backend = qsmd5_last_backend();
  if (c.shutter.joinable()) c.shutter.join();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  finished.store(true);
  watchdog.join();
  const bool ok_digests = rc == 0 && got == want;
  printf("{\"deadlock\": false, \"mode\": \"%s\", \"rc\": %d, \"backend\": %d, \"digests_ok\": %s, "
         "\"seconds\": %.3f, \"nested_calls\": %llu, \"nested_errors\": %llu, \"nested_ok\": %llu, "
         "\"nested_edeadlk\": %llu, \"reader_thread_reads\": %llu, \"shutdown_started\": %s, "
         "\"shutdown_rc\": %d}\n",
         mode.c_str(), rc, backend, ok_digests ? "true" : "false", s,
         (unsigned long long)c.nested_calls.load(), (unsigned long long)c.nested_errors.load(),
         (unsigned long long)c.nested_ok.load(), (unsigned long long)c.nested_edeadlk.load(),
         (unsigned long long)c.reader_thread_reads.load(), c.shutdown_started.load() ? "true" : "false",
         c.shutdown_rc.load());
  const bool shut_ok = c.nested_read || (c.shutdown_started.load() && c.shutdown_rc.load() == 0);
  return ok_digests && shut_ok && c.nested_errors.load() == 0 ? 0 : 1;
}
