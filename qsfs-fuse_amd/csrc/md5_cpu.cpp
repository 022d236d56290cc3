// qsfs-fuse_amd/csrc/md5_cpu.cpp -- the 64-step compression of the library's
// CPU MD5 (md5_cpu.h), in its own translation unit so the Makefile builds it
// with g++ -O3: for this serial chain hipcc's clang scheduled the same source
// 25-60% slower (10 MiB: 17 ms with g++, 22-28 ms with clang, this container).
#include "md5_cpu.h"

namespace qsmd5 {
namespace cpu {
namespace {

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

// The round function of step I, in the forms of md5_cpu.h's header comment.
template <int I>
inline uint32_t round_fn(uint32_t b, uint32_t c, uint32_t d) {
  if constexpr (I < 16) return d ^ (b & (c ^ d));
  else if constexpr (I < 32) return (c & ~d) + (b & d);
  else if constexpr (I < 48) return b ^ c ^ d;
  else return c ^ (b | ~d);
}

// Steps I..63, unrolled at compile time.  Step I updates `a`; the roles then
// rotate: the next step's (a, b, c, d) is this step's (d, a, b, c).
template <int I>
inline void steps(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, const uint32_t* x) {
  if constexpr (I < 64) {
    const uint32_t t = a + x[word_of(I)] + kT[I] + round_fn<I>(b, c, d);
    a = b + rotl(t, kRot[I >> 4][I & 3]);
    steps<I + 1>(d, a, b, c, x);
  }
}

}  // namespace

void compress(uint32_t h[4], const uint8_t* p, uint64_t nblocks) {
  for (; nblocks; --nblocks, p += 64) {
    uint32_t x[16];
    memcpy(x, p, 64);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    steps<0>(a, b, c, d, x);
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
  }
}

}  // namespace cpu
}  // namespace qsmd5
