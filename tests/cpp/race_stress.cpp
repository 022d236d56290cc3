// tests/cpp/race_stress.cpp -- concurrent callers of every C-ABI entry point
// qsfs reaches from several threads at once, for the host-sanitizer builds
// (scripts/build_sanitized.sh: the runtime's host code under ThreadSanitizer,
// and under AddressSanitizer + UBSan).
//
// The reference calls md5() from FUSE threads and from up to `numtransfer`
// executor workers at the same time (TransferManager.cpp:55-60,
// QSClient.cpp:370, 446) and has no race detection of its own.
// The C-ABI promises to be reentrant, so T threads here race:
//   - qsmd5_init (lazy, call_once) as their first call;
//   - qsmd5_hash_one over pageable buffers (group commit merges these);
//   - qsmd5_hash_batch / _ex over ragged, unaligned sub-ranges;
//   - qsmd5_hash_read pulling ragged sub-ranges through a read callback;
//   - the streaming context (MD5 class) fed in pieces;
//   - qsmd5_alloc_pinned / qsmd5_free_pinned around a hash;
//   - qsmd5_hex / qsmd5_base64;
// and, once every thread has returned, qsmd5_shutdown (twice, then a call
// that re-initialises, then shutdown again) before a normal process exit.
// Every digest is checked against the CPU oracle (oracle/md5_oracle.c, the
// checker, linked only into this test).
// usage: race_stress [threads=6] [rounds=12] [max_len=3145728] [racy]
// Without a GPU it runs only with QSMD5_BACKEND=cpu (the library's CPU
// backend: its worker threads and multi-buffer lanes, under the same
// sanitizers, in the container's `not gpu` suite); pinned buffers are then
// refused with -ENODEV and the case hashes a heap copy instead.
// `racy` adds a deliberate unsynchronised counter shared by the threads: the
// negative control showing that the TSan build, with its HIP suppressions,
// still reports a race in instrumented code.
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/qsmd5.h"

#if defined(__has_feature)
#if __has_feature(address_sanitizer)
#include <sanitizer/allocator_interface.h>  // __sanitizer_purge_allocator
#endif
#endif

extern "C" void oracle_md5(const uint8_t* p, uint64_t len, uint8_t out[16]);
extern "C" void oracle_lcg_fill(uint8_t* dst, uint64_t len, uint32_t seed);

namespace {

std::atomic<int> g_bad{0};
std::atomic<long> g_checked{0};
bool g_racy = false;
bool g_cpu_only = false;  // no GPU, QSMD5_BACKEND=cpu
long g_racy_counter = 0;  // written without a lock when g_racy (negative control)

void check(const uint8_t* p, uint64_t len, const uint8_t got[16], const char* what, int t, int r) {
  uint8_t want[16];
  oracle_md5(p, len, want);
  g_checked.fetch_add(1);
  if (memcmp(want, got, 16) != 0) {
    char a[33], b[33];
    qsmd5_hex(got, a);
    qsmd5_hex(want, b);
    fprintf(stderr, "MISMATCH %s thread %d round %d len %llu: %s != %s\n", what, t, r,
            (unsigned long long)len, a, b);
    g_bad.fetch_add(1);
  }
}

void fail(const char* what, int rc, int t, int r) {
  fprintf(stderr, "ERROR %s thread %d round %d: rc %d (%s) %s\n", what, t, r, rc, qsmd5_strerror(rc),
          qsmd5_last_error());
  g_bad.fetch_add(1);
}

// xorshift: per-thread, deterministic
uint32_t next(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}

// Every chunk a case builds must lie inside the worker's buffer.  Round 3's
// negative control (max_len 64 KiB) built 128-256 KiB chunks in case 4 from a
// 64 KiB buffer: `buf.size() - len + 1` wrapped, the chunk started up to 4 GiB
// past the buffer, and the runtime's H2D copy of that pageable "chunk" read
// unmapped TSan heap (GPUTEST_r03: SEGV, READ of 0x72c456febf4b).  Each range
// is checked here before it is handed to the library.
void in_buf(const std::vector<uint8_t>& buf, const void* p, size_t len, const char* what) {
  const uint8_t* b = buf.data();
  const uint8_t* q = static_cast<const uint8_t*>(p);
  if (q < b || q > b + buf.size() || len > (size_t)(b + buf.size() - q)) {
    fprintf(stderr, "race_stress bug: %s range [%p, +%zu) outside the %zu-byte buffer\n", what, p, len,
            buf.size());
    abort();
  }
}

void worker(int t, int rounds, size_t max_len, std::atomic<int>* ready, int nthreads) {
  std::vector<uint8_t> buf(max_len + 64);
  oracle_lcg_fill(buf.data(), buf.size(), 1000u + (uint32_t)t);
  uint32_t s = 0x9e3779b9u * (uint32_t)(t + 1);
  ready->fetch_add(1);
  while (ready->load() < nthreads) {
  }
  int rc = qsmd5_init(0);
  if (rc == -ENODEV && g_cpu_only) rc = 0;  // no GPU to bind: the calls hash on the CPU
  if (rc != 0) {
    fail("init", rc, t, -1);
    return;
  }
  for (int r = 0; r < rounds; ++r) {
    uint8_t d[16];
    switch ((t + r) % 6) {
      case 0: {  // one part, pageable, arbitrary offset and length
        const size_t off = next(s) % 61, len = next(s) % (max_len - 64) + 1;
        in_buf(buf, buf.data() + off, len, "hash_one");
        if ((rc = qsmd5_hash_one(buf.data() + off, len, d)) != 0) fail("hash_one", rc, t, r);
        else check(buf.data() + off, len, d, "hash_one", t, r);
        break;
      }
      case 1: {  // ragged batch of sub-ranges, including an empty chunk
        const int n = 1 + (int)(next(s) % 9);
        std::vector<qsmd5_chunk> ch(n);
        std::vector<uint8_t> dg(16 * n);
        for (int i = 0; i < n; ++i) {
          const size_t off = next(s) % std::min<size_t>(4099, buf.size());
          size_t len = i == 0 ? 0 : next(s) % (max_len / 4);
          if (off + len > buf.size()) len = buf.size() - off;
          ch[i].ptr = buf.data() + off;
          ch[i].len = len;
          in_buf(buf, ch[i].ptr, len, "hash_batch");
        }
        rc = (r & 4) ? qsmd5_hash_batch_ex(ch.data(), n, (uint8_t(*)[16])dg.data(), QSMD5_FLAG_HOST)
                     : qsmd5_hash_batch(ch.data(), n, (uint8_t(*)[16])dg.data());
        if (rc != 0) fail("hash_batch", rc, t, r);
        else
          for (int i = 0; i < n; ++i)
            check((const uint8_t*)ch[i].ptr, ch[i].len, dg.data() + 16 * i, "hash_batch", t, r);
        break;
      }
      case 2: {  // streaming context (MD5 class: update()* then finalize())
        qsmd5_ctx* c = nullptr;
        if ((rc = qsmd5_ctx_create(&c)) != 0) {
          fail("ctx_create", rc, t, r);
          break;
        }
        const size_t len = next(s) % (max_len / 2) + 1;
        const size_t fork_at = next(s) % len;  // a copy of the context taken here (MD5 is a value type)
        qsmd5_ctx* copy = nullptr;
        size_t at = 0;
        while (at < len && rc == 0) {
          size_t piece = next(s) % (len / 3 + 70) + 1;
          if (piece > len - at) piece = len - at;
          if (!copy && at + piece > fork_at) piece = fork_at - at;
          if (!copy && at == fork_at) {
            if ((rc = qsmd5_ctx_copy(c, &copy)) != 0) break;
            continue;
          }
          rc = qsmd5_ctx_update(c, buf.data() + at, piece);
          at += piece;
        }
        if (rc == 0) rc = qsmd5_ctx_final(c, d);
        qsmd5_ctx_destroy(c);
        if (rc != 0) fail("ctx", rc, t, r);
        else check(buf.data(), len, d, "ctx", t, r);
        if (copy && rc == 0) {  // the copy hashes the rest in one piece, by itself
          uint8_t dc[16];
          if ((rc = qsmd5_ctx_update(copy, buf.data() + fork_at, len - fork_at)) == 0) rc = qsmd5_ctx_final(copy, dc);
          if (rc != 0) fail("ctx copy", rc, t, r);
          else check(buf.data(), len, dc, "ctx copy", t, r);
        }
        qsmd5_ctx_destroy(copy);
        break;
      }
      case 3: {  // pinned buffer from the pool API
        const size_t len = next(s) % (max_len / 2) + 1;
        void* p = nullptr;
        if ((rc = qsmd5_alloc_pinned(len, &p)) != 0) {
          if (rc != -ENODEV || !g_cpu_only) {
            fail("alloc_pinned", rc, t, r);
            break;
          }
          std::vector<uint8_t> heap(buf.begin() + 7, buf.begin() + 7 + len);  // no GPU: a heap copy
          if ((rc = qsmd5_hash_one(heap.data(), len, d)) != 0) fail("hash_one(heap)", rc, t, r);
          else check(heap.data(), len, d, "hash_one(heap)", t, r);
          break;
        }
        // (the library makes the pinned allocator's hand-off between threads
        // visible to TSan: qsmd5_rt.h pinned_handed_out / pinned_handed_back)
        memcpy(p, buf.data() + 7, len);
        if ((rc = qsmd5_hash_one(p, len, d)) != 0) fail("hash_one(pinned)", rc, t, r);
        else check((const uint8_t*)p, len, d, "hash_one(pinned)", t, r);
        if ((rc = qsmd5_free_pinned(p)) != 0) fail("free_pinned", rc, t, r);
        break;
      }
      case 4: {  // ragged: two long chunks among many short ones (split under auto routing)
        const int n = 48;
        std::vector<qsmd5_chunk> ch(n);
        std::vector<uint8_t> dg(16 * n);
        for (int i = 0; i < n; ++i) {
          // the short ones are 128-256 KiB at the default 3 MiB max_len;
          // scaled down with smaller buffers, never longer than the buffer
          const size_t lo = std::min<size_t>(128u << 10, max_len / 24 + 1);
          size_t len = i < 2 ? max_len / 4 + next(s) % 4096 : lo + next(s) % lo;
          len = std::min(len, buf.size());
          const size_t off = next(s) % (buf.size() - len + 1);
          ch[(i * 7) % n].ptr = buf.data() + off;  // long ones land mid-batch
          ch[(i * 7) % n].len = len;
          in_buf(buf, ch[(i * 7) % n].ptr, len, "split batch");
        }
        if ((rc = qsmd5_hash_batch(ch.data(), n, (uint8_t(*)[16])dg.data())) != 0) fail("split batch", rc, t, r);
        else
          for (int i = 0; i < n; ++i)
            check((const uint8_t*)ch[i].ptr, ch[i].len, dg.data() + 16 * i, "split batch", t, r);
        break;
      }
      case 5: {  // pull-driven batch (qsmd5_hash_read): the library reads sub-ranges in windows
        struct Src {
          const uint8_t* base;
          std::vector<size_t> off;
          std::vector<uint64_t> len;
          static uint64_t read(void* user, size_t c, uint64_t o, uint64_t n, void* dst) {
            const Src* s = static_cast<const Src*>(user);
            if (o + n > s->len[c]) return 0;
            memcpy(dst, s->base + s->off[c] + o, n);
            return n;
          }
        } src;
        src.base = buf.data();
        const int n = 1 + (int)(next(s) % 24);
        for (int i = 0; i < n; ++i) {
          size_t len = next(s) % (max_len / 3 + 1);
          const size_t off = next(s) % (buf.size() - std::min(len, buf.size()) + 1);
          len = std::min(len, buf.size() - off);
          in_buf(buf, buf.data() + off, len, "hash_read");
          src.off.push_back(off);
          src.len.push_back(len);
        }
        const uint64_t staging = (uint64_t)(64u << 10) << (next(s) % 7);  // 64 KiB .. 4 MiB
        std::vector<uint8_t> dg(16 * n);
        const int rflags = (r & 2) ? QSMD5_FLAG_READ_PARALLEL : 0;  // Src::read is thread-safe
        if ((rc = qsmd5_hash_read(src.len.data(), n, &Src::read, &src, staging, (uint8_t(*)[16])dg.data(),
                                  rflags)) != 0)
          fail("hash_read", rc, t, r);
        else
          for (int i = 0; i < n; ++i) check(buf.data() + src.off[i], src.len[i], dg.data() + 16 * i, "hash_read", t, r);
        break;
      }
    }
    if (g_racy) g_racy_counter += 1;
    char hex[33], b64[25];
    qsmd5_hex(d, hex);
    qsmd5_base64(d, b64);
    if (strlen(hex) != 32 || strlen(b64) != 24) {
      fprintf(stderr, "bad hex/base64 length\n");
      g_bad.fetch_add(1);
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 6;
  const int R = argc > 2 ? atoi(argv[2]) : 12;
  const size_t L = argc > 3 ? strtoull(argv[3], nullptr, 10) : (3u << 20);
  if (T < 1 || R < 1 || L < 1024) {
    fprintf(stderr, "usage: race_stress [threads>=1] [rounds>=1] [max_len>=1024]\n");
    return 2;
  }
  g_racy = argc > 4 && strcmp(argv[4], "racy") == 0;
  if (qsmd5_device_count() < 1) {
    const char* be = getenv("QSMD5_BACKEND");
    if (!be || strcmp(be, "cpu") != 0) {
      fprintf(stderr, "no GPU\n");
      return 2;
    }
    g_cpu_only = true;
  }
  std::atomic<int> ready{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(worker, t, R, L, &ready, T);
  for (auto& x : th) x.join();
  // The exit path of a qsfs daemon: every thread has returned, so release the
  // runtime (streams, events, scratch, staging, pinned metadata, registered
  // ranges) before static destructors run.  Twice (idempotent), then a call
  // after it must initialise afresh and a second shutdown release that too.
  int rc = qsmd5_shutdown();
  if (rc != 0) fail("shutdown", rc, -1, -1);
  if ((rc = qsmd5_shutdown()) != 0) fail("shutdown (again)", rc, -1, -1);
  {
    uint8_t d[16];
    static const char kAbc[] = "abc";
    static const uint8_t kWant[16] = {0x90, 0x01, 0x50, 0x98, 0x3c, 0xd2, 0x4f, 0xb0,
                                      0xd6, 0x96, 0x3f, 0x7d, 0x28, 0xe1, 0x7f, 0x72};
    if ((rc = qsmd5_hash_one(kAbc, 3, d)) != 0) fail("hash after shutdown", rc, -1, -1);
    else if (memcmp(d, kWant, 16) != 0) {
      fprintf(stderr, "MISMATCH hash after shutdown\n");
      g_bad.fetch_add(1);
    }
    if ((rc = qsmd5_shutdown()) != 0) fail("shutdown (after re-init)", rc, -1, -1);
  }
#if defined(__has_feature)
#if __has_feature(address_sanitizer)
  // ROCm's ASan keeps freed HSA (device and pinned) allocations in its
  // quarantine.  HIP's own teardown (__cxa_finalize of libamdhip64) shuts HSA
  // down and then frees host objects; a quarantine recycle at that point
  // returns a device chunk after the device runtime is gone and ASan's CHECK
  // (sanitizer_allocator_device.h:125, dev_runtime_unloaded_) aborts the
  // process (profiles/r02_gpu_suite_asan_teardown.log).  Drain the
  // quarantine while HSA is still up: the chunks our shutdown just freed are
  // returned now, not during HIP's teardown.
  __sanitizer_purge_allocator();
#endif
#endif
  printf("race_stress %s: %d threads x %d rounds, %ld digests checked, %d failures\n",
         g_bad.load() ? "FAILED" : "ok", T, R, g_checked.load(), g_bad.load());
  fflush(stdout);
  fflush(stderr);
  return g_bad.load() ? 1 : 0;
}
