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

// floor(2^32 * |sin(i + 1)|), RFC 1321 §3.4.
constexpr uint32_t kT[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

// Per-round left-rotation amounts, RFC 1321 §3.4 (S11..S44).
constexpr int kRot[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};

// Message word of step i: i, 5i+1, 3i+5, 7i (mod 16) in rounds 1..4.
constexpr int word_of(int i) {
  return i < 16 ? i : i < 32 ? (5 * i + 1) & 15 : i < 48 ? (3 * i + 5) & 15 : (7 * i) & 15;
}

inline uint32_t rotl(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

// Folds nblocks consecutive 64-byte blocks at p into h[4].
inline void compress(uint32_t h[4], const uint8_t* p, uint64_t nblocks) {
  for (; nblocks; --nblocks, p += 64) {
    uint32_t x[16];
    memcpy(x, p, 64);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#pragma GCC unroll 64
    for (int i = 0; i < 64; ++i) {
      uint32_t t = a + x[word_of(i)] + kT[i];
      if (i < 16) {
        t += d ^ (b & (c ^ d));
      } else if (i < 32) {
        t += (c & ~d) + (b & d);
      } else if (i < 48) {
        t += b ^ c ^ d;
      } else {
        t += c ^ (b | ~d);
      }
      const uint32_t nb = b + rotl(t, kRot[i >> 4][i & 3]);
      a = d;
      d = c;
      c = b;
      b = nb;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
  }
}

constexpr uint32_t kIV[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};

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
