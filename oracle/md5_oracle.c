/*
 * oracle/md5_oracle.c -- CPU restatement of the qsfs reference MD5 path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the
 * MI355X HIP path in qsfs-fuse_amd/csrc.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker or the
 * timed CPU baseline -- never as the thing shipped.  The product library
 * (libqsmd5.so) does not link, load or call anything under oracle/.
 *
 * Pinning: the digests this file produces are checked against
 *   - the RFC 1321 appendix A.5 test suite (tests/golden/rfc1321.json),
 *   - the LCG golden table produced by the REFERENCE's own MD5.cpp compiled
 *     in this container (oracle/build_ref.sh -> oracle/_ref/,
 *     tests/golden/make_golden.py -> tests/golden/lcg_*.json),
 *   - Python hashlib on random inputs (tests/test_oracle.py).
 *
 * What it restates (file:line into the reference, qsfs-fuse v1.0.11):
 *   MD5::init                src/base/MD5.cpp:112-123
 *   MD5::decode (LE words)   src/base/MD5.cpp:129-133
 *   F/G/H/I, rotate_left     src/base/MD5.cpp:61-72
 *   FF/GG/HH/II step         src/base/MD5.cpp:76-94
 *   MD5::transform           src/base/MD5.cpp:151-234 (64 steps, feed-forward)
 *   MD5::update              src/base/MD5.cpp:240-269 (32-bit size_type,
 *                            bit counter with carry into count[1])
 *   MD5::finalize            src/base/MD5.cpp:282-312 (0x80 pad to 56 mod 64,
 *                            8-byte LE bit count)
 *   MD5::hexdigest           src/base/MD5.cpp:317-325 (lowercase %02x)
 *   md5(std::string)         src/base/MD5.cpp:335-339 -- note MD5(text)
 *                            passes text.length() into a 32-bit size_type
 *                            (MD5.h:53, MD5.cpp:106): the reference hashes
 *                            only the first (len mod 2^32) bytes.
 *                            oracle_md5_reference_string() reproduces that.
 *
 * The step schedule is written table-driven (message index, shift and
 * constant per step) rather than as the reference's 64 hand-unrolled macro
 * calls; the arithmetic is RFC 1321's and is identical bit for bit.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_EXPORT __attribute__((visibility("default")))

/* RFC 1321 sine table: K[i] = floor(2^32 * |sin(i + 1)|). */
static const uint32_t kK[64] = {
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

/* Per-round left-rotation amounts (RFC 1321 S11..S44, MD5.cpp:41-56). */
static const int kS[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};

static inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* Message-word index used by step i (round r = i/16, position j = i%16). */
static inline int msg_index(int i) {
  int j = i & 15;
  switch (i >> 4) {
    case 0: return j;
    case 1: return (5 * j + 1) & 15;
    case 2: return (3 * j + 5) & 15;
    default: return (7 * j) & 15;
  }
}

static inline uint32_t round_fn(int r, uint32_t x, uint32_t y, uint32_t z) {
  switch (r) {
    case 0: return (x & y) | (~x & z);
    case 1: return (x & z) | (y & ~z);
    case 2: return x ^ y ^ z;
    default: return y ^ (x | ~z);
  }
}

/* One compression over a 64-byte block (MD5.cpp:151-234). */
static void oracle_compress(uint32_t st[4], const uint8_t* blk) {
  uint32_t w[16];
  for (int k = 0; k < 16; ++k)
    w[k] = (uint32_t)blk[4 * k] | ((uint32_t)blk[4 * k + 1] << 8) |
           ((uint32_t)blk[4 * k + 2] << 16) | ((uint32_t)blk[4 * k + 3] << 24);
  uint32_t v[4] = {st[0], st[1], st[2], st[3]};
  /* v[(4 - i) & 3] is the register the reference calls "a" at step i. */
#pragma GCC unroll 64
  for (int i = 0; i < 64; ++i) {
    uint32_t* a = &v[(4 - (i & 3)) & 3];
    uint32_t b = v[(5 - (i & 3)) & 3];
    uint32_t c = v[(6 - (i & 3)) & 3];
    uint32_t d = v[(7 - (i & 3)) & 3];
    *a = b + rotl32(*a + round_fn(i >> 4, b, c, d) + w[msg_index(i)] + kK[i],
                    kS[i >> 4][i & 3]);
  }
  st[0] += v[0];
  st[1] += v[1];
  st[2] += v[2];
  st[3] += v[3];
}

typedef struct {
  uint32_t state[4];
  uint32_t count[2]; /* bit count, lo/hi (MD5.h:80) */
  uint8_t buffer[64];
  int finalized;
  uint8_t digest[16];
} oracle_md5_ctx;

ORACLE_EXPORT void oracle_md5_init(oracle_md5_ctx* c) {
  memset(c, 0, sizeof(*c));
  c->state[0] = 0x67452301u;
  c->state[1] = 0xefcdab89u;
  c->state[2] = 0x98badcfeu;
  c->state[3] = 0x10325476u;
}

/* MD5::update (MD5.cpp:240-269): length is a 32-bit size_type. */
ORACLE_EXPORT void oracle_md5_update(oracle_md5_ctx* c, const uint8_t* in, uint32_t len) {
  uint32_t idx = (c->count[0] >> 3) & 63u;
  uint32_t bits_lo = len << 3;
  c->count[0] += bits_lo;
  if (c->count[0] < bits_lo) c->count[1]++;
  c->count[1] += len >> 29;
  uint32_t room = 64u - idx;
  uint32_t i = 0;
  if (len >= room) {
    memcpy(c->buffer + idx, in, room);
    oracle_compress(c->state, c->buffer);
    for (i = room; i + 64u <= len; i += 64u) oracle_compress(c->state, in + i);
    idx = 0;
  }
  memcpy(c->buffer + idx, in + i, len - i);
}

/* MD5::finalize (MD5.cpp:282-312). */
ORACLE_EXPORT void oracle_md5_final(oracle_md5_ctx* c, uint8_t out[16]) {
  if (!c->finalized) {
    uint8_t lenle[8];
    for (int k = 0; k < 4; ++k) {
      lenle[k] = (uint8_t)(c->count[0] >> (8 * k));
      lenle[4 + k] = (uint8_t)(c->count[1] >> (8 * k));
    }
    static const uint8_t pad[64] = {0x80};
    uint32_t idx = (c->count[0] >> 3) & 63u;
    uint32_t padlen = idx < 56u ? 56u - idx : 120u - idx;
    oracle_md5_update(c, pad, padlen);
    oracle_md5_update(c, lenle, 8);
    for (int k = 0; k < 4; ++k)
      for (int b = 0; b < 4; ++b) c->digest[4 * k + b] = (uint8_t)(c->state[k] >> (8 * b));
    memset(c->buffer, 0, sizeof c->buffer);
    c->count[0] = c->count[1] = 0;
    c->finalized = 1;
  }
  memcpy(out, c->digest, 16);
}

/* MD5::hexdigest (MD5.cpp:317-325): 32 lowercase hex chars + NUL. */
ORACLE_EXPORT void oracle_md5_hex(const uint8_t d[16], char out[33]) {
  static const char hx[] = "0123456789abcdef";
  for (int k = 0; k < 16; ++k) {
    out[2 * k] = hx[d[k] >> 4];
    out[2 * k + 1] = hx[d[k] & 15];
  }
  out[32] = 0;
}

/* Full 64-bit-length MD5 (RFC 1321) -- what the HIP path computes. */
ORACLE_EXPORT void oracle_md5(const uint8_t* p, uint64_t len, uint8_t out[16]) {
  oracle_md5_ctx c;
  oracle_md5_init(&c);
  /* feed in < 4 GiB slices; count[] carries correctly across calls */
  const uint64_t kSlice = 1ull << 30;
  while (len > 0) {
    uint64_t n = len < kSlice ? len : kSlice;
    oracle_md5_update(&c, p, (uint32_t)n);
    p += n;
    len -= n;
  }
  oracle_md5_final(&c, out);
}

/* md5(const std::string) exactly as the reference behaves, including the
 * 32-bit truncation of the length at MD5.cpp:106 (MD5.h:53). */
ORACLE_EXPORT void oracle_md5_reference_string(const uint8_t* p, uint64_t len, uint8_t out[16]) {
  oracle_md5_ctx c;
  oracle_md5_init(&c);
  oracle_md5_update(&c, p, (uint32_t)len);
  oracle_md5_final(&c, out);
}

/* ------------------------------------------------------------------------ */
/* Batch helper: hash n independent chunks on nthreads host threads.         */

typedef struct {
  const uint8_t* const* ptrs;
  const uint64_t* lens;
  uint8_t (*out)[16];
  size_t n;
  size_t next; /* guarded by mu */
  pthread_mutex_t mu;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->n) break;
    oracle_md5(j->ptrs[i], j->lens[i], j->out[i]);
  }
  return NULL;
}

ORACLE_EXPORT int oracle_md5_batch(const uint8_t* const* ptrs, const uint64_t* lens, size_t n,
                                   uint8_t (*out)[16], int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  batch_job j;
  j.ptrs = ptrs;
  j.lens = lens;
  j.out = out;
  j.n = n;
  j.next = 0;
  pthread_mutex_init(&j.mu, NULL);
  pthread_t th[256];
  int started = 0;
  for (int t = 1; t < nthreads; ++t)
    if (pthread_create(&th[started], NULL, batch_worker, &j) == 0) ++started;
  batch_worker(&j);
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&j.mu);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Deterministic test-data generator:                        */
/*   x <- x * 1103515245 + 12345 (mod 2^32), applied BEFORE each byte;       */
/*   byte = (x >> 16) & 0xff; x0 = seed.                                     */

ORACLE_EXPORT void oracle_lcg_fill(uint8_t* dst, uint64_t len, uint32_t seed) {
  uint32_t x = seed;
  for (uint64_t i = 0; i < len; ++i) {
    x = x * 1103515245u + 12345u;
    dst[i] = (uint8_t)(x >> 16);
  }
}
