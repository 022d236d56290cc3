// tests/cpp/shutdown_starvation.cpp -- qsmd5_shutdown while calls keep
// overlapping.
//
// qsfs's executor and FUSE threads call into the library at any time; a
// daemon's exit path calls qsmd5_shutdown while some of them may still be
// hashing.  The header promises that shutdown waits for the calls in flight
// and that calls starting meanwhile wait for it.  Every call holds the
// runtime's call lock shared, shutdown takes it exclusively, and glibc's
// rwlock prefers readers: with calls that always overlap, a writer could wait
// forever.  Here T threads hash back to back on the CPU backend (no GPU
// needed) so that at every instant some call holds the lock; the main thread
// calls qsmd5_shutdown after 100 ms.  It must return within 5 s, and the
// hashing threads must go on working after it (their next calls re-initialise).
// A watchdog stops the hashers after 20 s so that a starved run still ends.
// Prints one JSON line; exit 0 = not starved.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/qsmd5.h"

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 6;
  std::vector<uint8_t> buf(256 << 10, 0x5a);
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> calls{0}, after{0};
  std::atomic<bool> shut{false};
  std::atomic<int> errors{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&] {
      qsmd5_chunk c = {buf.data(), buf.size()};
      uint8_t d[16];
      while (!stop.load()) {
        if (qsmd5_hash_batch_ex(&c, 1, reinterpret_cast<uint8_t(*)[16]>(d), QSMD5_FLAG_CPU_ONLY) != 0)
          errors.fetch_add(1);
        calls.fetch_add(1);
        if (shut.load()) after.fetch_add(1);
      }
    });
  std::thread watchdog([&] {
    for (int i = 0; i < 200 && !shut.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
    stop.store(true);  // a starved shutdown gets the lock once the hashers stop
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  const uint64_t before = calls.load();
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = qsmd5_shutdown();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const bool starved = stop.load();  // the watchdog had to stop the hashers first
  shut.store(true);
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  stop.store(true);
  for (auto& x : th) x.join();
  watchdog.join();
  printf("{\"threads\": %d, \"shutdown_rc\": %d, \"shutdown_s\": %.4f, \"starved\": %s, "
         "\"calls_before\": %llu, \"calls_after\": %llu, \"errors\": %d}\n",
         T, rc, s, starved ? "true" : "false", (unsigned long long)before,
         (unsigned long long)after.load(), errors.load());
  return (rc == 0 && !starved && s < 5.0 && after.load() > 0 && errors.load() == 0) ? 0 : 1;
}
