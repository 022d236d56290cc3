// ubench/thread_cpu_probe.hip -- which host threads a synchronous GPU wait
// keeps busy, and how the wait is done (round 4).
//
// The route sweep (profiles/r04_route_sweep.jsonl) found a GPU wave of 10 MiB
// parts costing ~2 host cores for its ~85 ms: the caller's wait, plus one
// thread the process keeps alive.  This probe separates the two on raw HIP
// (no qsmd5 code): a kernel that holds the GPU for `ms` milliseconds
// (s_memrealtime, 100 MHz), waited for by
//   stream     hipStreamSynchronize
//   event      hipEventSynchronize on a default event
//   blocking   hipEventSynchronize on a hipEventBlockingSync event
//   poll       hipEventQuery + sleep (the caller sleeps)
//   copy1d / copy2d / samestream   poll, after an 80 MiB pinned H2D copy on
//              a second stream (event-ordered) or on the kernel's stream
//   timing     poll, with timing-enabled events around the kernel
//   d2h_pinned / d2h_spin   a 4 KiB D2H copy into pinned memory after the
//              kernel, then poll / hipStreamSynchronize
// and, for each, the CPU time of every thread of the process over 10 waits
// (/proc/self/task/*/stat), so the caller's share and HIP's/HSA's own threads'
// shares show apart.  Usage: thread_cpu_probe [ms=80] [reps=10]
#include <dirent.h>
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <map>
#include <string>
#include <thread>
#include <vector>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void hold(uint64_t ticks, uint32_t* out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[blockIdx.x] = (uint32_t)(t - t0);
}

// tid -> (name, CPU seconds) of every live thread
std::map<int, std::pair<std::string, double>> threads_cpu() {
  std::map<int, std::pair<std::string, double>> m;
  const long hz = sysconf(_SC_CLK_TCK);
  DIR* dir = opendir("/proc/self/task");
  if (!dir) return m;
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
    unsigned long ut = 0, st = 0;
    if (sscanf(r + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %lu %lu", &ut, &st) != 2) continue;
    m[atoi(de->d_name)] = {std::string(l + 1, r), (double)(ut + st) / hz};
  }
  closedir(dir);
  return m;
}

int main(int argc, char** argv) {
  const double ms = argc > 1 ? atof(argv[1]) : 80.0;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  // argv[3] = path of libqsmd5.so: load it and run qsmd5_init first, so that
  // whatever the library's initialisation starts shows up in the same modes
  if (argc > 3) {
    void* so = dlopen(argv[3], RTLD_NOW);
    if (!so) {
      fprintf(stderr, "dlopen: %s\n", dlerror());
      return 1;
    }
    auto init = reinterpret_cast<int (*)(int)>(dlsym(so, "qsmd5_init"));
    printf("qsmd5_init -> %d\n", init ? init(0) : -999);
  }
  uint32_t* d = nullptr;
  CHECK(hipMalloc(&d, 4096));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev_default, ev_block;
  CHECK(hipEventCreateWithFlags(&ev_default, hipEventDisableTiming));
  CHECK(hipEventCreateWithFlags(&ev_block, hipEventBlockingSync | hipEventDisableTiming));
  const uint64_t ticks = (uint64_t)(ms * 1e5);  // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(hold, dim3(1), dim3(64), 0, s, (uint64_t)1000, d);  // load the code object
  CHECK(hipStreamSynchronize(s));
  const int me = (int)gettid();
  // modes 4-6: what the runtime's host batches add around the kernel -- an
  // H2D copy of 8 x 10 MiB from pinned memory (1-D or 2-D) on a second stream
  // ordered before the kernel by an event, or on the kernel's own stream
  const size_t row = 10u << 20, rows = 8;
  void* h = nullptr;
  uint8_t* dbuf = nullptr;
  CHECK(hipHostMalloc(&h, rows * row, hipHostMallocDefault));
  CHECK(hipMalloc(&dbuf, rows * (row + 4096)));
  memset(h, 1, rows * row);
  hipStream_t s2;
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev_t0, ev_t1;  // mode 7: timing-enabled events around the kernel, as run_batch keeps
  CHECK(hipEventCreateWithFlags(&ev_t0, hipEventDefault));
  CHECK(hipEventCreateWithFlags(&ev_t1, hipEventDefault));
  const char* modes[] = {"stream", "event", "blocking", "poll", "copy1d", "copy2d", "samestream",
                         "timing", "d2h_pinned", "d2h_spin", "pipe40", "pipe40_1s", "pipe40_noev",
                         "pipe40_host"};
  // modes 10-12: the runtime's column pipeline -- 40 slices, each a 2-D copy
  // of 8 rows x 256 KiB on a copy stream, an event, the compute stream
  // waiting on it, and a kernel of 1/40 of the wave -- then the poll wait;
  // pipe40_1s puts copies and kernels on one stream (no events);
  // pipe40_noev keeps two streams but orders them with one event at the end;
  // pipe40_host orders them on the host: kernel k is launched once the host
  // sees copy k's event complete (hipEventQuery, 50 us sleeps), no stream waits.
  std::vector<hipEvent_t> evs(40);
  for (auto& e : evs) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  uint8_t* hsmall = nullptr;  // modes 8-9: the digests' D2H copy into pinned memory after the kernel
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&hsmall), 1 << 16, hipHostMallocDefault));
  for (int m = 0; m < 14; ++m) {
    const auto before = threads_cpu();
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
      if (m == 4 || m == 5) {
        if (m == 4) CHECK(hipMemcpyAsync(dbuf, h, rows * row, hipMemcpyHostToDevice, s2));
        else CHECK(hipMemcpy2DAsync(dbuf, row + 4096, h, row, row, rows, hipMemcpyHostToDevice, s2));
        CHECK(hipEventRecord(ev_block, s2));
        CHECK(hipStreamWaitEvent(s, ev_block, 0));
      } else if (m == 6) {
        CHECK(hipMemcpyAsync(dbuf, h, rows * row, hipMemcpyHostToDevice, s));
      }
      if (m == 13) {
        for (int k = 0; k < 40; ++k) {
          CHECK(hipMemcpy2DAsync(dbuf + (size_t)k * (256 << 10), row + 4096, (uint8_t*)h + (size_t)k * (256 << 10),
                                 row, 256 << 10, rows, hipMemcpyHostToDevice, s2));
          CHECK(hipEventRecord(evs[k], s2));
        }
        for (int k = 0; k < 40; ++k) {
          while (hipEventQuery(evs[k]) == hipErrorNotReady)
            std::this_thread::sleep_for(std::chrono::microseconds(50));
          hipLaunchKernelGGL(hold, dim3(8), dim3(64), 0, s, ticks / 40, d);
        }
      } else if (m >= 10) {
        for (int k = 0; k < 40; ++k) {
          hipStream_t cs = m == 11 ? s : s2;
          CHECK(hipMemcpy2DAsync(dbuf + (size_t)k * (256 << 10), row + 4096, (uint8_t*)h + (size_t)k * (256 << 10),
                                 row, 256 << 10, rows, hipMemcpyHostToDevice, cs));
          if (m == 10) {
            CHECK(hipEventRecord(evs[k], s2));
            CHECK(hipStreamWaitEvent(s, evs[k], 0));
          }
          if (m != 12) hipLaunchKernelGGL(hold, dim3(8), dim3(64), 0, s, ticks / 40, d);
        }
        if (m == 12) {
          CHECK(hipEventRecord(evs[0], s2));
          CHECK(hipStreamWaitEvent(s, evs[0], 0));
          for (int k = 0; k < 40; ++k) hipLaunchKernelGGL(hold, dim3(8), dim3(64), 0, s, ticks / 40, d);
        }
      } else {
      if (m == 7) CHECK(hipEventRecord(ev_t0, s));
      hipLaunchKernelGGL(hold, dim3(8), dim3(64), 0, s, ticks, d);
      if (m == 7) CHECK(hipEventRecord(ev_t1, s));
      if (m >= 8) CHECK(hipMemcpyAsync(hsmall, d, 4096, hipMemcpyDeviceToHost, s));
      }
      if (m == 9) {
        CHECK(hipStreamSynchronize(s));
      } else if (m >= 4) {
        CHECK(hipEventRecord(ev_default, s));
        std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(ms * 900)));
        while (hipEventQuery(ev_default) == hipErrorNotReady)
          std::this_thread::sleep_for(std::chrono::microseconds(100));
        if (m == 7) {
          float t = 0;
          CHECK(hipEventElapsedTime(&t, ev_t0, ev_t1));
        }
      } else if (m == 0) {
        CHECK(hipStreamSynchronize(s));
      } else if (m == 1 || m == 2) {
        hipEvent_t ev = m == 1 ? ev_default : ev_block;
        CHECK(hipEventRecord(ev, s));
        CHECK(hipEventSynchronize(ev));
      } else {
        CHECK(hipEventRecord(ev_default, s));
        std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(ms * 900)));
        while (hipEventQuery(ev_default) == hipErrorNotReady)
          std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
    }
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const auto after = threads_cpu();
    printf("%-9s %d waits of %.0f ms: wall %.3f s;", modes[m], reps, ms, wall);
    double other = 0;
    for (const auto& kv : after) {
      const auto it = before.find(kv.first);
      const double used = kv.second.second - (it == before.end() ? 0.0 : it->second.second);
      if (kv.first == me) {
        printf(" caller %.3f s;", used);
      } else if (used > 0.005) {
        printf(" [%s:%d] %.3f s;", kv.second.first.c_str(), kv.first - me, used);
        other += used;
      }
    }
    printf(" other threads %.3f s (%.2f cores)\n", other, other / wall);
    fflush(stdout);
  }
  const char* envs[] = {"HSA_ENABLE_INTERRUPT", "ROC_ACTIVE_WAIT_TIMEOUT", "HIP_FORCE_DEV_KERNARG",
                        "AMD_SERIALIZE_KERNEL"};
  for (const char* e : envs) printf("env %s=%s\n", e, getenv(e) ? getenv(e) : "(unset)");
  CHECK(hipFree(d));
  CHECK(hipFree(dbuf));
  CHECK(hipHostFree(h));
  CHECK(hipHostFree(hsmall));
  return 0;
}
