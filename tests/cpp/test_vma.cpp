// tests/cpp/test_vma.cpp -- CPU checks of qsfs-fuse_amd/csrc/qsmd5_vma.h, the
// rule for which /proc/self/maps VMAs the runtime's pointer classifier may
// remember as host memory (qsmd5_rt.h Classifier).
//   1. readable anonymous, [heap], [stack], [anon:...] and regular-file VMAs
//      qualify, with their exact [lo, hi);
//   2. unreadable reservations (---p: where VRAM is mapped), /dev files
//      (/dev/dri/renderD*, /dev/kfd, /dev/shm), anon_inode mappings
//      (dma-bufs), [vvar]/[vdso] and malformed lines do not;
//   3. live: this process's malloc'd heap, a large mmap and its stack each
//      lie in a qualifying VMA of its own /proc/self/maps.
// Prints "vma ok <cases>" and exits 0, or the first failures and exits 1.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <initializer_list>

#include "../../qsfs-fuse_amd/csrc/qsmd5_vma.h"

static int fails = 0, cases = 0;

static void expect(const char* line, bool want, uint64_t lo = 0, uint64_t hi = 0) {
  ++cases;
  uint64_t a = 0, b = 0;
  const bool got = qsmd5::host_vma_from_maps_line(line, &a, &b);
  if (got != want || (want && (a != lo || b != hi))) {
    if (fails++ < 10)
      fprintf(stderr, "FAIL: '%s' -> %d [%llx, %llx), want %d [%llx, %llx)\n", line, got,
              (unsigned long long)a, (unsigned long long)b, want, (unsigned long long)lo,
              (unsigned long long)hi);
  }
}

static bool live_host(const void* p) {
  FILE* f = fopen("/proc/self/maps", "r");
  if (!f) return false;
  char line[4096];
  bool found = false;
  const uint64_t x = (uint64_t)(uintptr_t)p;
  uint64_t lo = 0, hi = 0;
  while (fgets(line, sizeof(line), f))
    if (qsmd5::host_vma_from_maps_line(line, &lo, &hi) && x >= lo && x < hi) found = true;
  fclose(f);
  return found;
}

int main() {
  expect("7f0000000000-7f0000100000 rw-p 00000000 00:00 0 \n", true, 0x7f0000000000ull, 0x7f0000100000ull);
  expect("7f0000000000-7f0000100000 rw-p 00000000 00:00 0", true, 0x7f0000000000ull, 0x7f0000100000ull);
  expect("55d0c0000000-55d0c0200000 rw-p 00000000 00:00 0                          [heap]\n", true,
         0x55d0c0000000ull, 0x55d0c0200000ull);
  expect("7ffc00000000-7ffc00021000 rw-p 00000000 00:00 0                          [stack]\n", true,
         0x7ffc00000000ull, 0x7ffc00021000ull);
  expect("7f1000000000-7f1000001000 rw-p 00000000 00:00 0                          [anon:pool]\n", true,
         0x7f1000000000ull, 0x7f1000001000ull);
  expect("7f2000000000-7f2040000000 r--p 00000000 103:02 1234567                   /data/big.bin\n", true,
         0x7f2000000000ull, 0x7f2040000000ull);
  expect("7f2000000000-7f2040000000 r--s 00000000 103:02 1234567                   /memfd:buf (deleted)\n",
         true, 0x7f2000000000ull, 0x7f2040000000ull);
  // not host-cacheable
  expect("7f3000000000-7f3100000000 ---p 00000000 00:00 0 \n", false);
  expect("7f4000000000-7f4000200000 rw-s 100200000 00:06 500                       /dev/dri/renderD128\n", false);
  expect("7f4000000000-7f4000200000 rw-s 00000000 00:06 501                        /dev/kfd\n", false);
  expect("7f4000000000-7f4000200000 rw-s 00000000 00:19 777                        /dev/shm/seg\n", false);
  expect("7f5000000000-7f5000200000 rw-s 00000000 00:0e 99                         anon_inode:dmabuf\n", false);
  expect("7ffc00100000-7ffc00104000 r--p 00000000 00:00 0                          [vvar]\n", false);
  expect("7ffc00104000-7ffc00106000 r-xp 00000000 00:00 0                          [vdso]\n", false);
  expect("7f6000000000-7f6000001000 -w-p 00000000 00:00 0 \n", false);
  expect("7f6000001000-7f6000000000 rw-p 00000000 00:00 0 \n", false);  // hi <= lo
  expect("garbage\n", false);
  expect("", false);
  // live
  char* heap = (char*)malloc(1 << 20);
  memset(heap, 1, 1 << 20);
  void* big = mmap(nullptr, 64 << 20, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  char stack_byte = 1;
  for (const void* p : {(const void*)heap, (const void*)big, (const void*)&stack_byte}) {
    ++cases;
    if (!live_host(p) && fails++ < 10) fprintf(stderr, "FAIL: live pointer %p not in a host VMA\n", p);
  }
  munmap(big, 64 << 20);
  free(heap);
  printf("vma %s %d cases\n", fails ? "FAIL" : "ok", cases);
  return fails ? 1 : 0;
}
