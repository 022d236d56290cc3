// tests/cpp/coalesce_bench.cpp -- native callers of the group commit
// (qsmd5_rt_route.cpp): T threads each hash one P-byte part R times in a tight
// loop, as qsfs's numtransfer executor threads call md5() part after part
// (TransferManager.cpp:55-60, QSClient.cpp:370).  Prints one JSON line with
// the wall time and whether every digest matched the first round's.
// usage: coalesce_bench [threads=5] [rounds=4] [part_bytes=10485760]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/qsmd5.h"

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 5;
  const int R = argc > 2 ? atoi(argv[2]) : 4;
  const size_t P = argc > 3 ? strtoull(argv[3], nullptr, 10) : (10u << 20);
  if (qsmd5_init(0) != 0) {
    fprintf(stderr, "no GPU: %s\n", qsmd5_last_error());
    return 2;
  }
  std::vector<std::vector<unsigned char>> buf(T, std::vector<unsigned char>(P));
  for (int t = 0; t < T; ++t) {
    uint32_t x = 777u + t;
    for (size_t i = 0; i < P; ++i) {
      x = x * 1103515245u + 12345u;
      buf[t][i] = (unsigned char)(x >> 16);
    }
  }
  std::vector<std::vector<uint8_t>> first(T, std::vector<uint8_t>(16));
  for (int t = 0; t < T; ++t)
    if (qsmd5_hash_one(buf[t].data(), P, first[t].data()) != 0) return 3;
  std::atomic<int> bad{0}, ready{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      ready.fetch_add(1);
      while (ready.load() < T) {
      }
      uint8_t d[16];
      for (int r = 0; r < R; ++r) {
        if (qsmd5_hash_one(buf[t].data(), P, d) != 0 || memcmp(d, first[t].data(), 16) != 0)
          bad.fetch_add(1);
      }
    });
  for (auto& x : th) x.join();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"threads\": %d, \"rounds\": %d, \"part_bytes\": %zu, \"wall_s\": %.4f, "
         "\"parts_per_s\": %.1f, \"ok\": %s}\n", T, R, P, s, T * R / s, bad.load() ? "false" : "true");
  return bad.load() ? 1 : 0;
}
