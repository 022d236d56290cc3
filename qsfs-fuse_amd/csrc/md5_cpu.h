// qsfs-fuse_amd/csrc/md5_cpu.h -- the library's own CPU MD5 (product code).
//
// SURVEY.md §8b asks the C-ABI to pick the backend by size (CPU below a
// break-even, GPU above) and to fall back to the CPU when the GPU fails,
// returning the same digest.  This is that CPU backend: RFC 1321 MD5 written
// for a host core, not the test oracle (oracle/ is test infrastructure and is
// never linked into libqsmd5.so) and nothing built from /root/reference.
// It is pinned against every committed golden fixture by tests/test_cpu_backend.py.
//
// One chunk is a serial chain of 64-byte compressions, so a lone chunk runs
// on one core; the rate is set by the chain's dependent-instruction latency.
// The step functions use the forms that take the fewest operations on that
// chain: F = d ^ (b & (c ^ d)) (c ^ d is ready before b), G = (c & ~d) + (b & d)
// (the two terms share no bits, and c & ~d does not wait for b), I = c ^ (b | ~d).
// The message word and round constant join `a` before b is known.
#pragma once

#include <stdint.h>
#include <string.h>

namespace qsmd5 {
namespace cpu {

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "MD5 words are little-endian loads");

// Folds nblocks consecutive 64-byte blocks at p into h[4] (md5_cpu.cpp: its
// own translation unit, built by g++; hipcc's clang made the same 64 steps
// 25-60% slower).
void compress(uint32_t h[4], const uint8_t* p, uint64_t nblocks);

constexpr uint32_t kIV[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};

// Multi-buffer form (md5_cpu_mb.cpp): 16 independent messages per host thread
// in the lanes of AVX-512 registers, each lane refilled from `pull` when its
// message ends.  pull(ctx, &i) hands out message i (ptrs[i], lens[i] -> out[i])
// or returns false when none is left.  Call only if mb16_available().
typedef bool (*MbPull)(void* ctx, uint32_t* i);
bool mb16_available();
void md5_mb16(const uint8_t* const* ptrs, const uint64_t* lens, uint8_t (*out)[16], MbPull pull,
              void* ctx);
// The same with 32 lanes: two 16-lane groups whose chains interleave, for
// cores with the vector pipes to run both (the runtime times both once and
// keeps the faster, qsmd5_rt_route.cpp measure_cpu_rates).
void md5_mb32(const uint8_t* const* ptrs, const uint64_t* lens, uint8_t (*out)[16], MbPull pull,
              void* ctx);

// Resumable multi-buffer form (pull-driven batches, qsmd5_rt_read.cpp): job i
// continues state[i] over nblocks[i] whole 64-B blocks at ptrs[i], 16 jobs at
// a time in the lanes; each state is written back when its job ends, with no
// padding (the running Ctx finishes the message).  Call only if
// mb16_available().
void md5_mb16_blocks(uint32_t (*state)[4], const uint8_t* const* ptrs, const uint64_t* nblocks, size_t count);

// Streaming state: the MD5 class (update()* then final()), any piece sizes.
struct Ctx {
  uint32_t h[4] = {kIV[0], kIV[1], kIV[2], kIV[3]};
  uint64_t total = 0;  // message bytes so far (the length field is 8 * total mod 2^64)
  uint8_t tail[64];
  uint32_t tail_len = 0;

  void update(const void* data, uint64_t len) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    total += len;
    if (tail_len) {
      const uint32_t take = (uint32_t)(len < 64 - tail_len ? len : 64 - tail_len);
      memcpy(tail + tail_len, p, take);
      tail_len += take;
      p += take;
      len -= take;
      if (tail_len < 64) return;
      compress(h, tail, 1);
      tail_len = 0;
    }
    compress(h, p, len / 64);
    p += len & ~63ull;
    tail_len = (uint32_t)(len & 63);
    if (tail_len) memcpy(tail, p, tail_len);
  }

  // 0x80, zeros to 56 mod 64, the bit length little-endian; the state as bytes.
  void final(uint8_t out[16]) {
    uint8_t pad[128] = {0};
    memcpy(pad, tail, tail_len);
    pad[tail_len] = 0x80;
    const uint32_t nb = tail_len < 56 ? 1 : 2;
    const uint64_t bits = total << 3;
    memcpy(pad + 64 * nb - 8, &bits, 8);
    compress(h, pad, nb);
    memcpy(out, h, 16);
  }
};

// MD5 of [p, p + len) with the full 64-bit length.
inline void md5(const void* p, uint64_t len, uint8_t out[16]) {
  Ctx c;
  c.update(p, len);
  c.final(out);
}

}  // namespace cpu
}  // namespace qsmd5
