// ubench/ubench_classify.cpp -- cost of classifying chunk pointers (host vs
// device) with hipPointerGetAttributes, per thread count, for pageable host,
// pinned host and device pointers; and hipMemGetAddressRange on device ones.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

static double classify_ms(const std::vector<const void*>& p, int T, int* ndev) {
  std::vector<int> cnt(T, 0);
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      for (size_t i = t; i < p.size(); i += T) {
        hipPointerAttribute_t a;
        memset(&a, 0, sizeof(a));
        if (hipPointerGetAttributes(&a, p[i]) != hipSuccess) {
          (void)hipGetLastError();
          continue;
        }
        cnt[t] += a.type == hipMemoryTypeDevice;
      }
    });
  for (auto& x : th) x.join();
  *ndev = 0;
  for (int c : cnt) *ndev += c;
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
  const size_t n = 1 << 20, L = 1024;
  hipSetDevice(0);
  hipFree(nullptr);
  char* pageable = (char*)malloc(n * L);
  memset(pageable, 1, n * L);
  char* pinned = nullptr;
  char* dev = nullptr;
  hipHostMalloc((void**)&pinned, n * L, hipHostMallocDefault);
  hipMalloc((void**)&dev, n * L);
  for (const char* what : {"pageable", "pinned", "device"}) {
    char* base = !strcmp(what, "pageable") ? pageable : !strcmp(what, "pinned") ? pinned : dev;
    std::vector<const void*> p(n);
    for (size_t i = 0; i < n; ++i) p[i] = base + i * L;
    for (int T : {1, 2, 4, 8, 16}) {
      int nd = 0;
      const double ms = classify_ms(p, T, &nd);
      printf("%-8s %2d threads: %8.2f ms for %zu pointers (%.0f ns each), %d device\n", what, T, ms,
             n, ms * 1e6 / n, nd);
    }
  }
  // device range query
  {
    auto t0 = std::chrono::steady_clock::now();
    size_t ok = 0;
    for (size_t i = 0; i < n; i += 1) {
      hipDeviceptr_t b;
      size_t sz = 0;
      if (hipMemGetAddressRange(&b, &sz, (hipDeviceptr_t)(dev + i * L)) == hipSuccess) ok += sz >= n * L;
    }
    const double ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("hipMemGetAddressRange on device ptrs: %.2f ms (%zu with the whole range)\n", ms, ok);
    hipDeviceptr_t b;
    size_t sz = 0;
    hipError_t e = hipMemGetAddressRange(&b, &sz, (hipDeviceptr_t)(pinned + 12345));
    printf("hipMemGetAddressRange on pinned host: %s base_off=%lld size=%zu\n", hipGetErrorString(e),
           e == hipSuccess ? (long long)((char*)b - pinned) : -1ll, sz);
    (void)hipGetLastError();
  }
  return 0;
}
