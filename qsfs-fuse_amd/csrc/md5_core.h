// qsfs-fuse_amd/csrc/md5_core.h -- RFC 1321 MD5 compression for gfx950 lanes.
//
// Device-side building blocks shared by every MD5 kernel in md5_kernels.hip.
// One lane owns one message chain (a qsfs upload part); the 64 steps of a
// block are fully unrolled with compile-time constants so that each step
// lowers to v_bitop3_b32 (round function) + v_add3_u32 + v_alignbit_b32
// (rotate) + v_add_u32, the constants landing in SGPRs/literals.
//
// Semantics follow the reference MD5 class (qsfs-fuse v1.0.11):
//   init constants       src/base/MD5.cpp:112-123
//   LE word decode       src/base/MD5.cpp:129-133
//   F/G/H/I, rotate      src/base/MD5.cpp:61-72
//   step a=b+rotl(a+f+x+k,s)  src/base/MD5.cpp:76-94
//   transform + feed-fwd src/base/MD5.cpp:151-234
//   finalize padding     src/base/MD5.cpp:282-312
// The formulation (template-indexed steps, no message copy) is our own.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qsmd5 {

struct Md5Tables {
  // floor(2^32 * |sin(i+1)|)
  static constexpr uint32_t K[64] = {
      0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au,
      0xa8304613u, 0xfd469501u, 0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu,
      0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u, 0xf61e2562u, 0xc040b340u,
      0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
      0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u,
      0x676f02d9u, 0x8d2a4c8au, 0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu,
      0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u, 0x289b7ec6u, 0xeaa127fau,
      0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
      0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u,
      0xffeff47du, 0x85845dd1u, 0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u,
      0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};
};

constexpr uint32_t kInit0 = 0x67452301u;
constexpr uint32_t kInit1 = 0xefcdab89u;
constexpr uint32_t kInit2 = 0x98badcfeu;
constexpr uint32_t kInit3 = 0x10325476u;

// Left-rotation amount of step i.
__host__ __device__ constexpr int md5_shift(int i) {
  return (i < 16)   ? ((i & 3) == 0 ? 7 : (i & 3) == 1 ? 12 : (i & 3) == 2 ? 17 : 22)
         : (i < 32) ? ((i & 3) == 0 ? 5 : (i & 3) == 1 ? 9 : (i & 3) == 2 ? 14 : 20)
         : (i < 48) ? ((i & 3) == 0 ? 4 : (i & 3) == 1 ? 11 : (i & 3) == 2 ? 16 : 23)
                    : ((i & 3) == 0 ? 6 : (i & 3) == 1 ? 10 : (i & 3) == 2 ? 15 : 21);
}

// Message word consumed by step i.
__host__ __device__ constexpr int md5_word(int i) {
  return (i < 16) ? i
         : (i < 32) ? ((5 * (i - 16) + 1) & 15)
         : (i < 48) ? ((3 * (i - 32) + 5) & 15)
                    : ((7 * (i - 48)) & 15);
}

// Round function truth tables as v_bitop3_b32 immediates.  The ISA indexes the
// 8-entry table by (S0<<2 | S1<<1 | S2), so evaluating the boolean function on
// S0=0xF0, S1=0xCC, S2=0xAA yields the immediate directly.
__host__ __device__ constexpr uint32_t md5_fn_host(int round, uint32_t x, uint32_t y, uint32_t z) {
  return round == 0   ? ((x & y) | (~x & z))   // F  (MD5.cpp:61)
         : round == 1 ? ((x & z) | (y & ~z))   // G  (MD5.cpp:63)
         : round == 2 ? (x ^ y ^ z)            // H  (MD5.cpp:65)
                      : (y ^ (x | ~z));        // I  (MD5.cpp:67)
}
__host__ __device__ constexpr uint32_t md5_bitop3_imm(int round) {
  return md5_fn_host(round, 0xF0u, 0xCCu, 0xAAu) & 0xFFu;
}

// The builtin keeps the round function one instruction: written as C the
// compiler rewrites F/G as a disjoint sum and spends an extra VALU per step.
template <int I>
__device__ __forceinline__ uint32_t md5_round_fn(uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_amdgcn_bitop3_b32(b, c, d, md5_bitop3_imm(I >> 4));
}

// Register roles rotate every step: at step i the reference's "a" is v[(4-i)&3].
template <int I>
__device__ __forceinline__ void md5_steps(uint32_t (&v)[4], const uint32_t (&w)[16]) {
  if constexpr (I < 64) {
    constexpr int ia = (4 - (I & 3)) & 3;
    constexpr int ib = (ia + 1) & 3;
    constexpr int ic = (ia + 2) & 3;
    constexpr int id = (ia + 3) & 3;
    // a + x + k does not depend on the freshest register: off the critical path.
    const uint32_t amk = v[ia] + w[md5_word(I)] + Md5Tables::K[I];
    const uint32_t t = amk + md5_round_fn<I>(v[ib], v[ic], v[id]);
    v[ia] = v[ib] + __builtin_rotateleft32(t, md5_shift(I));
    md5_steps<I + 1>(v, w);
  }
}

// Steps with the message-and-constant term mk[i] = x[word(i)] + K[i] supplied
// precomputed (by the producer wave of qsmd5_batch_pc_kernel): each step is then
// exactly v_bitop3 + v_add3 + v_alignbit + v_add.
template <int I, int kEnd = 64>
__device__ __forceinline__ void md5_steps_mk(uint32_t (&v)[4], const uint32_t (&mk)[64]) {
  if constexpr (I < kEnd) {
    constexpr int ia = (4 - (I & 3)) & 3;
    constexpr int ib = (ia + 1) & 3;
    constexpr int ic = (ia + 2) & 3;
    constexpr int id = (ia + 3) & 3;
    const uint32_t t = v[ia] + md5_round_fn<I>(v[ib], v[ic], v[id]) + mk[I];
    v[ia] = v[ib] + __builtin_rotateleft32(t, md5_shift(I));
    md5_steps_mk<I + 1, kEnd>(v, mk);
  }
}

__device__ __forceinline__ void md5_compress_mk(uint32_t (&st)[4], const uint32_t (&mk)[64]) {
  uint32_t v[4] = {st[0], st[1], st[2], st[3]};
  md5_steps_mk<0>(v, mk);
  st[0] += v[0];
  st[1] += v[1];
  st[2] += v[2];
  st[3] += v[3];
}

// One 64-byte compression with feed-forward: st <- st + F(st, w).
__device__ __forceinline__ void md5_compress(uint32_t (&st)[4], const uint32_t (&w)[16]) {
  uint32_t v[4] = {st[0], st[1], st[2], st[3]};
  md5_steps<0>(v, w);
  st[0] += v[0];
  st[1] += v[1];
  st[2] += v[2];
  st[3] += v[3];
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
#define QS_GLOBAL __attribute__((address_space(1)))

// 16-byte load from a 4-byte-aligned global address (global_load_dwordx4;
// the generic-pointer form would lower to flat_load and force vmcnt(0)+lgkmcnt(0)).
// kNT: the non-temporal cache policy (nt), for message bytes read exactly once.
template <bool kNT = false>
__device__ __forceinline__ u32x4 load16_a4(const uint32_t* p) {
  if constexpr (kNT)
    return __builtin_nontemporal_load((const QS_GLOBAL u32x4_a4*)(reinterpret_cast<uintptr_t>(p)));
  else
    return *(const QS_GLOBAL u32x4_a4*)(reinterpret_cast<uintptr_t>(p));
}
__device__ __forceinline__ uint32_t load4(const uint32_t* p) {
  return *(const QS_GLOBAL uint32_t*)(reinterpret_cast<uintptr_t>(p));
}

__device__ __forceinline__ void unpack4(uint32_t (&w)[16], int k, u32x4 q) {
  w[4 * k + 0] = q.x;
  w[4 * k + 1] = q.y;
  w[4 * k + 2] = q.z;
  w[4 * k + 3] = q.w;
}

}  // namespace qsmd5
