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

// Steps I..63 over G groups of 16 lanes.  Register roles rotate every step,
// as in md5_core.h: at step i the reference's "a" is v[(4 - i) & 3].  With
// G = 2 the two groups' independent chains interleave, so that one group's
// dependent ternlog/add/rotate/add fills the other's latency.
template <int G, int I>
QS_AVX512 inline void stepsG(__m512i (&v)[4][G], const __m512i (&x)[G][16]) {
  if constexpr (I < 64) {
    constexpr int ia = (4 - (I & 3)) & 3, ib = (ia + 1) & 3, ic = (ia + 2) & 3, id = (ia + 3) & 3;
    for (int g = 0; g < G; ++g) {
      // a + x + K does not wait for b: only ternlog, add, rotate, add are serial
      const __m512i amk = _mm512_add_epi32(_mm512_add_epi32(v[ia][g], x[g][word_of(I)]),
                                           _mm512_set1_epi32((int)kT[I]));
      const __m512i f = _mm512_ternarylogic_epi32(v[ib][g], v[ic][g], v[id][g], kTern[I >> 4]);
      v[ia][g] = _mm512_add_epi32(v[ib][g], _mm512_rol_epi32(_mm512_add_epi32(amk, f), kRot[I >> 4][I & 3]));
    }
    stepsG<G, I + 1>(v, x);
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

// 16 x G lanes, each holding one message, refilled from `pull` when its
// message ends; every live lane runs the same number of whole blocks in
// lockstep, then the lanes whose messages ended finish on the scalar path.
template <int G>
QS_AVX512 void runG(const uint8_t* const* ptrs, const uint64_t* lens, uint8_t (*out)[16], MbPull pull,
                    void* ctx) {
  constexpr int L = 16 * G;
  const uint8_t* p[L];
  uint64_t left[L];  // whole blocks still to run
  uint32_t idx[L];
  bool busy[L];
  alignas(64) uint32_t s[4][L];
  for (int l = 0; l < L; ++l) {
    p[l] = kZeroBlock;
    left[l] = 0;
    busy[l] = false;
  }
  __m512i S[4][G];
  for (int k = 0; k < 4; ++k)
    for (int g = 0; g < G; ++g) S[k][g] = _mm512_setzero_si512();
  bool more = true;  // the queue may still hold messages
  for (;;) {
    // refill idle lanes; messages shorter than one block finish right here
    __mmask16 fresh[G] = {};
    for (int l = 0; l < L && more; ++l) {
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
        fresh[l / 16] |= (__mmask16)(1u << (l % 16));
      }
    }
    for (int k = 0; k < 4; ++k)
      for (int g = 0; g < G; ++g) S[k][g] = _mm512_mask_mov_epi32(S[k][g], fresh[g], _mm512_set1_epi32((int)kIV[k]));
    __mmask16 live[G] = {};
    bool any = false;
    uint64_t run = ~0ull;
    for (int l = 0; l < L; ++l)
      if (busy[l]) {
        live[l / 16] |= (__mmask16)(1u << (l % 16));
        any = true;
        run = left[l] < run ? left[l] : run;
      }
    if (!any) return;
    // every live lane has `run` whole blocks: run them in lockstep (idle
    // lanes read a zero block and keep their registers)
    for (uint64_t j = 0; j < run; ++j) {
      __m512i x[G][16];
      for (int g = 0; g < G; ++g) {
        const uint8_t* const(&pg)[16] = *reinterpret_cast<const uint8_t* const(*)[16]>(p + 16 * g);
        load_transpose(x[g], pg);
      }
      __m512i v[4][G];
      for (int k = 0; k < 4; ++k)
        for (int g = 0; g < G; ++g) v[k][g] = S[k][g];
      stepsG<G, 0>(v, x);
      for (int k = 0; k < 4; ++k)
        for (int g = 0; g < G; ++g) S[k][g] = _mm512_mask_add_epi32(S[k][g], live[g], S[k][g], v[k][g]);
      for (int l = 0; l < L; ++l)
        if (busy[l]) p[l] += 64;
    }
    for (int k = 0; k < 4; ++k)
      for (int g = 0; g < G; ++g) _mm512_store_si512((void*)(s[k] + 16 * g), S[k][g]);
    for (int l = 0; l < L; ++l) {
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

// The resumable form (md5_mb16_blocks): job i continues state[i] over
// nblocks[i] whole blocks at ptrs[i]; 16 lanes run in lockstep, a lane whose
// job is done takes the next one, and each state is written back as its job
// ends (no padding: the caller's running context finishes the message).
QS_AVX512 void run_blocks(uint32_t (*state)[4], const uint8_t* const* ptrs, const uint64_t* nblocks,
                          size_t count) {
  constexpr int L = 16;
  const uint8_t* p[L];
  uint64_t left[L];
  size_t idx[L];
  bool busy[L];
  alignas(64) uint32_t s[4][L];
  for (int l = 0; l < L; ++l) {
    p[l] = kZeroBlock;
    left[l] = 0;
    busy[l] = false;
  }
  __m512i S[4];
  for (int k = 0; k < 4; ++k) S[k] = _mm512_setzero_si512();
  size_t next = 0;
  for (;;) {
    // refill idle lanes with the next job's state
    for (int k = 0; k < 4; ++k) _mm512_store_si512((void*)s[k], S[k]);
    for (int l = 0; l < L; ++l)
      while (!busy[l] && next < count) {
        const size_t i = next++;
        if (nblocks[i] == 0) continue;  // nothing to run: the state stands
        busy[l] = true;
        idx[l] = i;
        p[l] = ptrs[i];
        left[l] = nblocks[i];
        for (int k = 0; k < 4; ++k) s[k][l] = state[i][k];
      }
    for (int k = 0; k < 4; ++k) S[k] = _mm512_load_si512((const void*)s[k]);
    __mmask16 live = 0;
    uint64_t run = ~0ull;
    for (int l = 0; l < L; ++l)
      if (busy[l]) {
        live |= (__mmask16)(1u << l);
        run = left[l] < run ? left[l] : run;
      }
    if (!live) return;
    for (uint64_t j = 0; j < run; ++j) {
      __m512i x[1][16];
      const uint8_t* const(&pg)[16] = *reinterpret_cast<const uint8_t* const(*)[16]>(p);
      load_transpose(x[0], pg);
      __m512i v[4][1];
      for (int k = 0; k < 4; ++k) v[k][0] = S[k];
      stepsG<1, 0>(v, x);
      for (int k = 0; k < 4; ++k) S[k] = _mm512_mask_add_epi32(S[k], live, S[k], v[k][0]);
      for (int l = 0; l < L; ++l)
        if (busy[l]) p[l] += 64;
    }
    for (int k = 0; k < 4; ++k) _mm512_store_si512((void*)s[k], S[k]);
    for (int l = 0; l < L; ++l) {
      if (!busy[l]) continue;
      left[l] -= run;
      if (left[l]) continue;
      for (int k = 0; k < 4; ++k) state[idx[l]][k] = s[k][l];
      busy[l] = false;
      p[l] = kZeroBlock;
    }
  }
}

}  // namespace

bool mb16_available() { return __builtin_cpu_supports("avx512f"); }

void md5_mb16_blocks(uint32_t (*state)[4], const uint8_t* const* ptrs, const uint64_t* nblocks, size_t count) {
  run_blocks(state, ptrs, nblocks, count);
}

void md5_mb16(const uint8_t* const* ptrs, const uint64_t* lens, uint8_t (*out)[16], MbPull pull,
              void* ctx) {
  runG<1>(ptrs, lens, out, pull, ctx);
}

void md5_mb32(const uint8_t* const* ptrs, const uint64_t* lens, uint8_t (*out)[16], MbPull pull,
              void* ctx) {
  runG<2>(ptrs, lens, out, pull, ctx);
}

}  // namespace cpu
}  // namespace qsmd5
