// qsfs-fuse_amd/csrc/md5_cpu_mb.cpp -- multi-buffer MD5 for the CPU backend:
// 16 independent messages per host thread, one per 32-bit lane of AVX-512
// registers (md5_cpu.h md5_mb16).
//
// A message is a serial chain of 64-byte compressions, so one chain keeps a
// core's integer pipes mostly idle waiting on its own dependencies (~4 cycles
// per step).  Sixteen chains in the lanes of one zmm register take the same
// ~4 cycles per step: vpternlogd is the round function in one instruction
// (the truth tables md5_kernels.hip feeds v_bitop3_b32), vprold the rotate.
// A lane whose message runs out is refilled from the caller's queue, so lanes
// of a ragged batch never wait for the longest one.
//
// Built by g++ with the default ISA; only the functions marked QS_AVX512 use
// AVX-512, and the caller reaches them only after mb16_available() said the
// host has AVX-512F.  No standard-library template is instantiated here (an
// AVX-512 copy of a shared inline function could be the one the linker keeps).
// RFC 1321 semantics as md5_cpu.cpp (reference src/base/MD5.cpp:151-312).
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include "md5_cpu.h"

#define QS_AVX512 __attribute__((target("avx512f")))

namespace qsmd5 {
namespace cpu {
namespace {

constexpr uint32_t kT[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

constexpr int kRot[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};

constexpr int word_of(int i) {
  return i < 16 ? i : i < 32 ? (5 * i + 1) & 15 : i < 48 ? (3 * i + 5) & 15 : (7 * i) & 15;
}

// vpternlogd immediates: the round function evaluated on b=0xF0, c=0xCC, d=0xAA.
constexpr int kTern[4] = {0xCA /* F */, 0xE4 /* G */, 0x96 /* H */, 0x39 /* I */};

alignas(64) const uint8_t kZeroBlock[64] = {0};

// Steps I..63 over 16 lanes; roles rotate as in md5_cpu.cpp.
template <int I>
QS_AVX512 inline void steps16(__m512i& a, __m512i& b, __m512i& c, __m512i& d, const __m512i* x) {
  if constexpr (I < 64) {
    // a + x + K does not wait for b: only ternlog, add, rotate, add are serial
    const __m512i amk = _mm512_add_epi32(_mm512_add_epi32(a, x[word_of(I)]),
                                         _mm512_set1_epi32((int)kT[I]));
    const __m512i f = _mm512_ternarylogic_epi32(b, c, d, kTern[I >> 4]);
    a = _mm512_add_epi32(b, _mm512_rol_epi32(_mm512_add_epi32(amk, f), kRot[I >> 4][I & 3]));
    steps16<I + 1>(d, a, b, c, x);
  }
}

// x[w] lane l = little-endian word w of the 64 bytes at p[l]: 16 row loads and
// a 16 x 16 dword transpose (unpack 32, unpack 64, then 128-bit blocks).
QS_AVX512 inline void load_transpose(__m512i (&x)[16], const uint8_t* const (&p)[16]) {
  __m512i r[16], t[16];
  for (int l = 0; l < 16; ++l) r[l] = _mm512_loadu_si512((const void*)p[l]);
  for (int i = 0; i < 8; ++i) {
    t[2 * i] = _mm512_unpacklo_epi32(r[2 * i], r[2 * i + 1]);
    t[2 * i + 1] = _mm512_unpackhi_epi32(r[2 * i], r[2 * i + 1]);
  }
  // r[4i + c], 128-bit block k: rows 4i..4i+3 of column 4k + c
  for (int i = 0; i < 4; ++i) {
    r[4 * i + 0] = _mm512_unpacklo_epi64(t[4 * i], t[4 * i + 2]);
    r[4 * i + 1] = _mm512_unpackhi_epi64(t[4 * i], t[4 * i + 2]);
    r[4 * i + 2] = _mm512_unpacklo_epi64(t[4 * i + 1], t[4 * i + 3]);
    r[4 * i + 3] = _mm512_unpackhi_epi64(t[4 * i + 1], t[4 * i + 3]);
  }
  for (int c = 0; c < 4; ++c) {
    const __m512i v0 = _mm512_shuffle_i32x4(r[c], r[4 + c], 0x44);
    const __m512i v1 = _mm512_shuffle_i32x4(r[c], r[4 + c], 0xEE);
    const __m512i v2 = _mm512_shuffle_i32x4(r[8 + c], r[12 + c], 0x44);
    const __m512i v3 = _mm512_shuffle_i32x4(r[8 + c], r[12 + c], 0xEE);
    x[c] = _mm512_shuffle_i32x4(v0, v2, 0x88);
    x[4 + c] = _mm512_shuffle_i32x4(v0, v2, 0xDD);
    x[8 + c] = _mm512_shuffle_i32x4(v1, v3, 0x88);
    x[12 + c] = _mm512_shuffle_i32x4(v1, v3, 0xDD);
  }
}

// The tail bytes, 0x80, zeros and the 64-bit bit length (MD5.cpp:282-312), on
// the scalar compression; then the state as the digest.
void finish_scalar(uint32_t h[4], const uint8_t* tail, uint32_t rem, uint64_t len,
                   uint8_t out[16]) {
  uint8_t pad[128];
  memset(pad, 0, sizeof(pad));
  if (rem) memcpy(pad, tail, rem);
  pad[rem] = 0x80;
  const uint32_t nb = rem < 56 ? 1 : 2;
  const uint64_t bits = len << 3;
  memcpy(pad + 64 * nb - 8, &bits, 8);
  compress(h, pad, nb);
  memcpy(out, h, 16);
}

QS_AVX512 void run16(const uint8_t* const* ptrs, const uint64_t* lens, uint8_t (*out)[16],
                     MbPull pull, void* ctx) {
  const uint8_t* p[16];
  uint64_t left[16];  // whole blocks still to run
  uint32_t idx[16];
  bool busy[16];
  alignas(64) uint32_t s[4][16];
  for (int l = 0; l < 16; ++l) {
    p[l] = kZeroBlock;
    left[l] = 0;
    busy[l] = false;
  }
  __m512i A = _mm512_setzero_si512(), B = A, C = A, D = A;
  bool more = true;  // the queue may still hold messages
  for (;;) {
    // refill idle lanes; messages shorter than one block finish right here
    __mmask16 fresh = 0;
    for (int l = 0; l < 16 && more; ++l) {
      while (!busy[l] && more) {
        uint32_t i;
        if (!pull(ctx, &i)) {
          more = false;
          break;
        }
        const uint64_t nb = lens[i] >> 6;
        if (nb == 0) {
          uint32_t h[4] = {kIV[0], kIV[1], kIV[2], kIV[3]};
          finish_scalar(h, ptrs[i], (uint32_t)lens[i], lens[i], out[i]);
          continue;
        }
        busy[l] = true;
        idx[l] = i;
        p[l] = ptrs[i];
        left[l] = nb;
        fresh |= (__mmask16)(1u << l);
      }
    }
    A = _mm512_mask_mov_epi32(A, fresh, _mm512_set1_epi32((int)kIV[0]));
    B = _mm512_mask_mov_epi32(B, fresh, _mm512_set1_epi32((int)kIV[1]));
    C = _mm512_mask_mov_epi32(C, fresh, _mm512_set1_epi32((int)kIV[2]));
    D = _mm512_mask_mov_epi32(D, fresh, _mm512_set1_epi32((int)kIV[3]));
    __mmask16 live = 0;
    uint64_t run = ~0ull;
    for (int l = 0; l < 16; ++l)
      if (busy[l]) {
        live |= (__mmask16)(1u << l);
        run = left[l] < run ? left[l] : run;
      }
    if (!live) return;
    // every live lane has `run` whole blocks: run them in lockstep (idle
    // lanes read a zero block and keep their registers)
    for (uint64_t j = 0; j < run; ++j) {
      __m512i x[16];
      load_transpose(x, p);
      __m512i a = A, b = B, c = C, d = D;
      steps16<0>(a, b, c, d, x);
      A = _mm512_mask_add_epi32(A, live, A, a);
      B = _mm512_mask_add_epi32(B, live, B, b);
      C = _mm512_mask_add_epi32(C, live, C, c);
      D = _mm512_mask_add_epi32(D, live, D, d);
      for (int l = 0; l < 16; ++l)
        if (busy[l]) p[l] += 64;
    }
    _mm512_store_si512((void*)s[0], A);
    _mm512_store_si512((void*)s[1], B);
    _mm512_store_si512((void*)s[2], C);
    _mm512_store_si512((void*)s[3], D);
    for (int l = 0; l < 16; ++l) {
      if (!busy[l]) continue;
      left[l] -= run;
      if (left[l]) continue;
      const uint32_t i = idx[l];
      uint32_t h[4] = {s[0][l], s[1][l], s[2][l], s[3][l]};
      finish_scalar(h, p[l], (uint32_t)(lens[i] & 63), lens[i], out[i]);
      busy[l] = false;
      p[l] = kZeroBlock;
    }
  }
}

}  // namespace

bool mb16_available() { return __builtin_cpu_supports("avx512f"); }

void md5_mb16(const uint8_t* const* ptrs, const uint64_t* lens, uint8_t (*out)[16], MbPull pull,
              void* ctx) {
  run16(ptrs, lens, out, pull, ctx);
}

}  // namespace cpu
}  // namespace qsmd5
