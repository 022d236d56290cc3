// qsfs-fuse_amd/csrc/md5_kernels.hip -- gfx950 kernels for the qsfs MD5 path.
//
// Batch kernels (one lane per chunk = one qsfs upload part; each hashes the
// whole message incl. RFC 1321 padding and writes the 16-byte digest, i.e.
// md5(shared_ptr<iostream>), reference src/base/MD5.cpp:341-349, for a batch):
//   qsmd5_batch_pc_kernel    latency kernel, <= 256 x 64 chunks (every
//                            BASELINE config): producer wave streams blocks and
//                            precomputes x[g]+K into LDS, chain wave runs only
//                            the serial 4-VALU steps.  qsmd5_batch_pc64/32_kernel
//                            are the same with 64 / 32 chains per workgroup
//                            fixed at compile time (what the runtime launches).
//   qsmd5_batch_pc2_kernel   the same with a 64 KiB ring (two workgroups per
//                            CU): <= 2 x 256 x 64 chunks.
//   qsmd5_batch_coal_kernel  throughput kernel, more chunks, 16-B aligned:
//                            coalesced LDS-DMA staging of 128 B per chain.
//   qsmd5_batch_kernel       throughput kernel, more chunks, any alignment:
//                            per-lane loads, 5 VALU per step.
//   qsmd5_column_pc[2]_kernel  the latency kernels over one column of a
//                            host-staged batch: chains resume from and park in
//                            HBM state (qsmd5_rt_staging.cpp run_batch).
// Streaming (the MD5 class, MD5.cpp:240-312): update() runs its blocks as a
// one-lane qsmd5_column_pc_kernel batch; then
//   qsmd5_final_kernel       tail + padding + length (finalize()).
// Test/bench support:
//   qsmd5_lcg_fill_kernel    SURVEY.md §8c LCG data, jump-ahead parallel.
//
// Why lane-per-chunk: MD5 is Merkle-Damgard, so a chunk is a strictly serial
// chain of 64-byte compressions; parallelism exists only across chunks.  On
// gfx950 one wave issues a dependent VALU op every ~4.4 cycles whether 1 or 64
// lanes are active (ubench/ubench_md5.hip "issue"), so the per-chain rate is
// set by the dependent instructions per block (4 per step, 256 per block at
// best), not by lanes per wave: 64 chains share one wave at no cost per chain
// and leave the other SIMDs free.  Batch workgroups each own 64 chunks, so the
// dispatcher spreads them over all 8 XCDs / 256 CUs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "md5_core.h"

namespace qsmd5 {

struct ChunkDesc {  // layout-identical to qsmd5_chunk in include/qsmd5.h
  const uint8_t* ptr;
  uint64_t len;
};

// Whole blocks from a 4-byte-aligned pointer.  Four blocks (64 VGPRs) are
// kept in flight so the ~1-2 us HBM latency hides behind ~3 blocks of compute.
// Prefetch addresses are clamped to the last block (always in bounds).
__device__ __forceinline__ void blocks_aligned4(uint32_t (&st)[4], const uint32_t* p,
                                                uint32_t nblk) {
  if (nblk == 0) return;
  const uint32_t last = nblk - 1;
  u32x4 a0, a1, a2, a3, b0, b1, b2, b3, c0, c1, c2, c3, d0, d1, d2, d3;
#define QS_LOAD(X, blk)                                   \
  do {                                                    \
    const uint32_t* q_ = p + (uint64_t)(blk) * 16u;       \
    X##0 = load16_a4(q_);                                 \
    X##1 = load16_a4(q_ + 4);                             \
    X##2 = load16_a4(q_ + 8);                             \
    X##3 = load16_a4(q_ + 12);                            \
  } while (0)
#define QS_COMPRESS(X)            \
  do {                            \
    uint32_t w_[16];              \
    unpack4(w_, 0, X##0);         \
    unpack4(w_, 1, X##1);         \
    unpack4(w_, 2, X##2);         \
    unpack4(w_, 3, X##3);         \
    md5_compress(st, w_);         \
  } while (0)
  QS_LOAD(a, 0);
  QS_LOAD(b, min(1u, last));
  QS_LOAD(c, min(2u, last));
  QS_LOAD(d, min(3u, last));
  uint32_t j = 0;
  for (; j + 4 <= nblk; j += 4) {
    QS_COMPRESS(a);
    QS_LOAD(a, min(j + 4, last));
    QS_COMPRESS(b);
    QS_LOAD(b, min(j + 5, last));
    QS_COMPRESS(c);
    QS_LOAD(c, min(j + 6, last));
    QS_COMPRESS(d);
    QS_LOAD(d, min(j + 7, last));
  }
  if (j < nblk) QS_COMPRESS(a);
  if (j + 1 < nblk) QS_COMPRESS(b);
  if (j + 2 < nblk) QS_COMPRESS(c);
#undef QS_COMPRESS
#undef QS_LOAD
}

// Whole blocks from an arbitrary byte address: aligned dword window of 17
// words per block, realigned with v_alignbyte_b32.  Every dword read holds at
// least one byte of the message, so nothing past the buffer's last aligned
// dword is touched.
__device__ __forceinline__ void blocks_unaligned(uint32_t (&st)[4], const uint8_t* bp,
                                                 uint32_t nblk) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(bp);
  const uint32_t* base = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t off = static_cast<uint32_t>(a & 3u);
  for (uint32_t j = 0; j < nblk; ++j) {
    const uint32_t* q = base + (uint64_t)j * 16u;
    u32x4 x0 = load16_a4(q), x1 = load16_a4(q + 4), x2 = load16_a4(q + 8),
          x3 = load16_a4(q + 12);
    uint32_t e = load4(q + 16);
    uint32_t d[17] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w, x2.x,
                      x2.y, x2.z, x2.w, x3.x, x3.y, x3.z, x3.w, e};
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], off);
    md5_compress(st, w);
  }
}

// Final 1 or 2 blocks: the rem (< 64) trailing bytes, 0x80, zero fill, and the
// 64-bit little-endian bit count (MD5.cpp:282-312).  Only dwords holding at
// least one of the rem bytes are read (none when rem == 0), so an empty or
// short tail never touches memory outside the message.
__device__ __forceinline__ void finish(uint32_t (&st)[4], const uint8_t* tp, uint32_t rem,
                                       uint64_t total_len) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(tp);
  const uint32_t* base = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t off = static_cast<uint32_t>(a & 3u);
  uint32_t d[17];
#pragma unroll
  for (int k = 0; k < 17; ++k)
    d[k] = (rem != 0u && (uint32_t)(4 * k) < off + rem) ? load4(base + k) : 0u;
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint32_t x = __builtin_amdgcn_alignbyte(d[k + 1], d[k], off);
    const uint32_t lo = 4u * k;
    uint32_t m = rem >= lo + 4u ? 0xffffffffu : rem <= lo ? 0u : ((1u << (8u * (rem - lo))) - 1u);
    x &= m;
    if ((rem >> 2) == (uint32_t)k) x |= 0x80u << (8u * (rem & 3u));
    w[k] = x;
  }
  const uint64_t bits = total_len << 3;
  if (rem < 56u) {
    w[14] = (uint32_t)bits;
    w[15] = (uint32_t)(bits >> 32);
    md5_compress(st, w);
  } else {
    md5_compress(st, w);
#pragma unroll
    for (int k = 0; k < 14; ++k) w[k] = 0u;
    w[14] = (uint32_t)bits;
    w[15] = (uint32_t)(bits >> 32);
    md5_compress(st, w);
  }
}

__device__ __forceinline__ void hash_message(uint32_t (&st)[4], const uint8_t* p, uint64_t len) {
  const uint32_t nblk = (uint32_t)(len >> 6);
  if ((reinterpret_cast<uintptr_t>(p) & 3u) == 0)
    blocks_aligned4(st, reinterpret_cast<const uint32_t*>(p), nblk);
  else
    blocks_unaligned(st, p, nblk);
  finish(st, p + ((uint64_t)nblk << 6), (uint32_t)(len & 63u), len);
}


__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// Wave-uniform copy of a 32-bit value as UNSIGNED: the builtin returns int, and
// widening that int to 64 bits would sign-extend (fatal for pointer halves).
__device__ __forceinline__ uint32_t rfl_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// LDS-only workgroup barrier: wait for this wave's LDS traffic, then s_barrier.
// Deliberately not __syncthreads(): its fence would also drain vmcnt and kill
// the producer's global-load prefetch that spans the barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- producer/consumer batch kernel -------------------------------------------
// Workgroup = 2 waves over the same 64 chunks.  Wave 1 (producer) streams the
// message blocks from HBM, realigns them, and writes mk[i] = x[word(i)] + K[i]
// for all 64 steps of each block into an LDS ring; wave 0 (chain) runs only the
// serial part: 4 VALU per step plus one ds_read_b128 per 4 steps.  The two waves
// sit on different SIMDs, so the chain wave's issue slots are not shared.
constexpr int kPcHalf = 4;  // blocks per ring half (one phase): 8 x 16 KiB = 128 KiB of LDS
// Steps of each phase's first block that run on its first kPcLead / 4 operand
// reads (chain_phase kLead): 1188-1192 against 1199-1202 cycles per block at
// 512 x 10 MiB, 1195 against 1208 at 8192 x 1 MiB (profiles/r02_lead_ab.log).
constexpr int kPcLead = 8;
// s_waitcnt immediate (gfx9 encoding) for lgkmcnt(0) alone: vmcnt 63, expcnt 7.
constexpr int kLgkmcnt0 = 0xC07F;

struct PcBlockRegs {
  u32x4 q[4];
  uint32_t e;
};

template <bool kNT>
__device__ __forceinline__ void pc_load_block(PcBlockRegs& r, const uint32_t* base, uint32_t off,
                                              uint32_t blk) {
  const uint32_t* q = base + (uint64_t)blk * 16u;
  r.q[0] = load16_a4<kNT>(q);
  r.q[1] = load16_a4<kNT>(q + 4);
  r.q[2] = load16_a4<kNT>(q + 8);
  r.q[3] = load16_a4<kNT>(q + 12);
  r.e = off ? load4(q + 16) : 0u;  // 17th dword holds message bytes only if off != 0
}

__device__ __forceinline__ void pc_write_mk(u32x4 (*slot)[64], uint32_t lane, const PcBlockRegs& r,
                                            uint32_t off) {
  uint32_t d[17] = {r.q[0].x, r.q[0].y, r.q[0].z, r.q[0].w, r.q[1].x, r.q[1].y,
                    r.q[1].z, r.q[1].w, r.q[2].x, r.q[2].y, r.q[2].z, r.q[2].w,
                    r.q[3].x, r.q[3].y, r.q[3].z, r.q[3].w, r.e};
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], off);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    u32x4 m;
    m.x = w[md5_word(4 * g + 0)] + Md5Tables::K[4 * g + 0];
    m.y = w[md5_word(4 * g + 1)] + Md5Tables::K[4 * g + 1];
    m.z = w[md5_word(4 * g + 2)] + Md5Tables::K[4 * g + 2];
    m.w = w[md5_word(4 * g + 3)] + Md5Tables::K[4 * g + 3];
    slot[g][lane] = m;
  }
}


// One phase of the chain wave: kPcHalf blocks from ring slots s0.., the
// operands of block h+1 read from LDS while block h compresses.  kAllLive
// drops the per-block lane predicate (every lane has blocks blk0..blk0+H-1).
//
// kLead > 0: the first block of the phase, whose 16 reads go out right after
// the phase barrier, waits only for its first kLead/4 reads (LDS returns in
// order), runs steps [0, kLead), then waits for the rest and sends block 1's
// reads.  The full-block wait exposes all 16 reads' latency once per phase.
template <bool kAllLive, int kHalf = kPcHalf, int kLead = 0, int kLead2 = 0>
__device__ __forceinline__ void chain_phase(uint32_t (&st)[4], const u32x4 (*ring)[16][64],
                                            uint32_t s0, uint32_t lane, uint32_t blk0,
                                            uint32_t nblk) {
  u32x4 a[16], b[16];
  auto read_slot = [&](u32x4 (&dst)[16], uint32_t slot) {
#pragma unroll
    for (int g = 0; g < 16; ++g) dst[g] = ring[slot][g][lane];
  };
  auto unpack_slot = [&](uint32_t (&mk)[64], const u32x4 (&src)[16]) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      mk[4 * g + 0] = src[g].x;
      mk[4 * g + 1] = src[g].y;
      mk[4 * g + 2] = src[g].z;
      mk[4 * g + 3] = src[g].w;
    }
  };
  auto compress_slot = [&](const u32x4 (&src)[16]) {
    uint32_t mk[64];
    unpack_slot(mk, src);
    md5_compress_mk(st, mk);
  };
  read_slot(a, s0);
  if constexpr (kLead > 0) {
    static_assert(kLead % 4 == 0 && kLead < 64, "kLead: whole ds_read_b128 groups");
    // block 0 with a graded wait; blocks 1.. below as usual
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt((kLgkmcnt0 & ~(0xF << 8)) | ((16 - kLead / 4) << 8));
    __builtin_amdgcn_sched_barrier(0);
    const bool run0 = kAllLive || blk0 < nblk;
    uint32_t mk[64];
    unpack_slot(mk, a);
    uint32_t v[4] = {st[0], st[1], st[2], st[3]};
    if (run0) md5_steps_mk<0, kLead>(v, mk);
    constexpr int kRest = kLead2 > kLead ? kLead2 : kLead;
    if constexpr (kLead2 > kLead) {
      static_assert(kLead2 % 4 == 0 && kLead2 < 64, "kLead2: whole ds_read_b128 groups");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt((kLgkmcnt0 & ~(0xF << 8)) | ((16 - kLead2 / 4) << 8));
      __builtin_amdgcn_sched_barrier(0);
      if (run0) md5_steps_mk<kLead, kLead2>(v, mk);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
    if (1 < kHalf) read_slot(b, s0 + 1);
    __builtin_amdgcn_sched_barrier(0);
    if (run0) {
      md5_steps_mk<kRest, 64>(v, mk);
      st[0] += v[0];
      st[1] += v[1];
      st[2] += v[2];
      st[3] += v[3];
    }
  }
#pragma unroll
  for (int h = (kLead > 0 ? 1 : 0); h < kHalf; ++h) {
    // One wait per block: the operands of block h (read a whole block ago)
    // are complete, then the 16 reads of block h+1 go out and the 256 VALU of
    // block h need no wait at all.  Left to itself the compiler hoists two
    // blocks of reads (32 > the 15 lgkmcnt can count) and then waits before
    // every ds_read_b128's first use: 8 waits (issue slots) per block.
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
    if (h + 1 < kHalf) read_slot((h & 1) ? a : b, s0 + h + 1);
    __builtin_amdgcn_sched_barrier(0);
    if (kAllLive || blk0 + (uint32_t)h < nblk) compress_slot((h & 1) ? b : a);  // blk0 may wrap (skew)
  }
}


}  // namespace qsmd5

using namespace qsmd5;

// digests: n x 16 bytes (4 LE words each), indexed by chunk index.
// order: optional lane -> chunk permutation (length-bucketed by the host).
extern "C" __global__ __launch_bounds__(64) void qsmd5_batch_kernel(
    const ChunkDesc* __restrict__ chunks, const uint32_t* __restrict__ order, uint32_t n,
    uint32_t* __restrict__ digests) {
  const uint32_t t = blockIdx.x * 64u + threadIdx.x;
  if (t >= n) return;
  const uint32_t idx = order ? order[t] : t;
  const ChunkDesc cd = chunks[idx];
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
  hash_message(st, cd.ptr, cd.len);
  u32x4 o = {st[0], st[1], st[2], st[3]};
  *reinterpret_cast<u32x4*>(digests + 4u * (uint64_t)idx) = o;
}

// Streaming finalize: tail bytes (< 64, host-provided in device memory) + pad.
extern "C" __global__ __launch_bounds__(64) void qsmd5_final_kernel(uint32_t* __restrict__ state,
                                                                    const uint8_t* tail,
                                                                    uint32_t rem,
                                                                    uint64_t total_len) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t st[4] = {state[0], state[1], state[2], state[3]};
  finish(st, tail, rem, total_len);
  state[0] = st[0];
  state[1] = st[1];
  state[2] = st[2];
  state[3] = st[3];
}

// ---------------------------------------------------------------------------
// Synthetic data: chunk i of `nchunks` at base + i*stride holds `len` bytes of
// LCG(seed0 + i): x <- x*1103515245 + 12345 before each byte, byte = x>>16.
// Each thread writes one 1 KiB segment after jumping the LCG ahead.
namespace {
constexpr uint32_t kLcgA = 1103515245u;
constexpr uint32_t kLcgC = 12345u;
constexpr uint32_t kSeg = 1024u;

__device__ __forceinline__ uint32_t lcg_jump(uint32_t x, uint64_t n) {
  uint32_t am = kLcgA, cm = kLcgC;  // T^(2^k)
  uint32_t ar = 1u, cr = 0u;        // accumulated map
  while (n) {
    if (n & 1u) {
      ar = ar * am;
      cr = cr * am + cm;
    }
    cm = cm * am + cm;
    am = am * am;
    n >>= 1;
  }
  return ar * x + cr;
}
}  // namespace

extern "C" __global__ __launch_bounds__(256) void qsmd5_lcg_fill_kernel(
    uint8_t* __restrict__ base, uint64_t stride, uint64_t len, uint32_t seed0,
    uint32_t nchunks, uint64_t segs_per_chunk) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t chunk = g / segs_per_chunk;
  if (chunk >= nchunks) return;
  const uint64_t seg = g - chunk * segs_per_chunk;
  const uint64_t start = seg * kSeg;
  if (start >= len) return;
  const uint64_t end = start + kSeg < len ? start + kSeg : len;
  uint32_t x = lcg_jump(seed0 + (uint32_t)chunk, start);
  uint8_t* out = base + chunk * stride;
  uint64_t i = start;
  if (((reinterpret_cast<uintptr_t>(out) + start) & 3u) == 0) {
    for (; i + 4 <= end; i += 4) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        x = x * kLcgA + kLcgC;
        v |= ((x >> 16) & 0xffu) << (8 * b);
      }
      *reinterpret_cast<uint32_t*>(out + i) = v;
    }
  }
  for (; i < end; ++i) {
    x = x * kLcgA + kLcgC;
    out[i] = (uint8_t)(x >> 16);
  }
}

// Latency-regime batch kernel body (B up to one resident round, 256 x 64
// chunks): see the producer/consumer notes at kPcHalf.
//
// kColumn = false: chunks[order[t]] is a whole chunk; digest -> digests[idx].
// kColumn = true (column-pipelined host batches, qsmd5_rt_staging.cpp): the batch
// is cut into columns [col_off, col_off + col_w) of every chunk.  chunks[t] is
// lane t's staged SEGMENT {ptr = segment start, len = the chunk's TOTAL
// length L} and idx = order[t] names the chunk.  A lane resumes from
// states[idx] (or the MD5 IV when col_off == 0), runs the segment's blocks,
// and then either parks the state (L - col_off > col_w) or finishes with the
// tail and the full length L (MD5.cpp:279-312 over the whole message).
// col_off and col_w are multiples of 64, so block boundaries line up.
//
// skew (whole-chunk batches only; a multiple of kPcHalf): in a wave whose
// longest chunk has >= kSkewMinBlocks blocks (32 MiB), lane l starts its chain
// perm(l) x skew blocks late, so the 64 lanes read addresses spread over up to
// 63 x skew x 64 B instead of the same offset of every chunk at once.  Long
// parts at a power-of-two stride (a contiguous device file cut into 32 or
// 64 MiB parts, qsfs -b 32/64) otherwise send every lane's request to the same
// HBM channels: measured 512 x 64 MiB 42.1 -> 54.5 GiB/s, 512 x 32 MiB
// 48.6 -> 54.7 (profiles/r01_ubench_skew.log).  Cost: 63 x skew blocks per
// wave (0.05% of a 32 MiB chain); shorter chunks never pay it.  0 = off.
constexpr uint32_t kSkewMinBlocks = 1u << 19;
//
// kNT: the producer's loads carry the non-temporal cache policy (chosen per
// launch by the host, qsmd5_rt_staging.cpp load_nt_for).
// kTrace (ubench only): the chain wave's lane 0 stamps s_memtime and
// s_memrealtime every 4096 phases into trace[workgroup][2 * (p / 4096) + {0,1}],
// and at the end the cycles each wave spent: trace[workgroup][1019] producer
// total, [1020] chain waiting at the phase barriers, [1021] chain total,
// [1022] producer waiting at the barriers, [1023] producer writing the ring
// (including its wait for the loads).
// kProbe (ubench attribution only; 0 in every shipped kernel): bit 0 = the
// producer skips its ring writes, bit 1 = it skips its global loads.  The
// digests are then wrong; the chain's cycles say what the producer's LDS
// writes and HBM loads cost it (profiles/r03_attrib.log).
template <bool kColumn, int kDepth = 1, int kHalf = kPcHalf, bool kNT = false, bool kTrace = false,
          int kPace = 0, int kGap = 0, int kLead = kPcLead, int kLead2 = 0, int kProbe = 0>
__device__ __forceinline__ void pc_body(const ChunkDesc* __restrict__ chunks,
                                        const uint32_t* __restrict__ order, uint32_t n,
                                        uint32_t* __restrict__ digests, uint64_t col_off,
                                        uint64_t col_w, uint32_t* __restrict__ states,
                                        uint32_t skew, uint64_t* __restrict__ trace = nullptr,
                                        uint32_t lanes = 64) {
  __shared__ u32x4 ring[2 * kHalf][16][64];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  // `lanes` chains per workgroup (64, or fewer to spread long chains over more
  // CUs); lanes past it, or past the batch, idle.
  const uint32_t t = blockIdx.x * lanes + lane;
  const bool live = lane < lanes && t < n;
  uint32_t idx = 0;
  ChunkDesc cd = {nullptr, 0};
  uint64_t seg = 0;     // message bytes of this lane's segment
  bool final = true;    // this segment ends the chunk
  if (live) {
    if (kColumn) {
      idx = order[t];
      cd = chunks[t];
      const uint64_t rest = cd.len - col_off;
      final = rest <= col_w;
      seg = final ? rest : col_w;
    } else {
      idx = order ? order[t] : t;
      cd = chunks[idx];
      seg = cd.len;
    }
  }
  const uint32_t nblk = (uint32_t)(seg >> 6);
  // start delay in blocks; lanes take the delays in a scrambled order (37 is odd,
  // so l -> 37 l mod 64 is a permutation) so that no affine chunk stride can
  // cancel the spread
  const bool skewed = !kColumn && skew != 0 && wave_max_u32(nblk) >= kSkewMinBlocks;
  const uint32_t delta = (skewed && nblk) ? skew * ((lane * 37u) & 63u) : 0u;
  const uint32_t phases = (wave_max_u32(nblk + delta) + kHalf - 1) / kHalf;
  const uintptr_t pa = reinterpret_cast<uintptr_t>(cd.ptr);
  const uint32_t off = (uint32_t)(pa & 3u);

  if (wave == 1) {
    // ---------------- producer ----------------
    const uint32_t* base = reinterpret_cast<const uint32_t*>(pa & ~uintptr_t(3));
    const uint32_t last = nblk ? nblk - 1 : 0;
    // kDepth register sets of one phase each: the loads of phase q go into set
    // q % kDepth and are written to the ring kDepth phases after they were
    // issued, so a load has kDepth phases (~2 us each) to land.
    PcBlockRegs r[kDepth][kHalf];
    if constexpr ((kProbe & 2) != 0) {
#pragma unroll
      for (int k = 0; k < kDepth; ++k)
#pragma unroll
        for (int h = 0; h < kHalf; ++h) r[k][h] = PcBlockRegs{{lane, lane, lane, lane}, lane};
    }
    auto load_phase = [&](PcBlockRegs (&rs)[kHalf], uint32_t p) {
      if constexpr ((kProbe & 2) != 0) return;
      if (nblk) {
#pragma unroll
        for (int h = 0; h < kHalf; ++h) {
          const uint32_t j = p * kHalf + h;  // virtual block; the lane's block is j - delta
          pc_load_block<kNT>(rs[h], base, off, j < delta ? 0u : min(j - delta, last));
        }
      }
    };
    auto write_phase = [&](const PcBlockRegs (&rs)[kHalf], uint32_t p) {
      if (nblk) {
#pragma unroll
        for (int h = 0; h < kHalf; ++h) {
          if constexpr (kGap > 0) {
            if (h) __builtin_amdgcn_s_sleep(kGap);
          }
          if constexpr ((kProbe & 1) == 0) pc_write_mk(ring[(p & 1u) * kHalf + h], lane, rs[h], off);
        }
      }
    };
    uint64_t t_start = 0, t_wait = 0, t_write = 0;
    if constexpr (kTrace) t_start = __builtin_amdgcn_s_memtime();
    if (phases > 0) {
#pragma unroll
      for (int k = 0; k < kDepth; ++k) load_phase(r[k], (uint32_t)k);
      write_phase(r[0], 0);
      load_phase(r[0], kDepth);
    }
    lds_barrier();
    // iteration p writes phase p + 1 from set (p + 1) % kDepth and refills that
    // set with phase p + 1 + kDepth; unrolled by kDepth so every set is static
    for (uint32_t p0 = 0; p0 < phases; p0 += kDepth) {
#pragma unroll
      for (int u = 0; u < kDepth; ++u) {
        const uint32_t p = p0 + (uint32_t)u;
        if (p < phases) {
          if (p + 1 < phases) {
            uint64_t tw = 0;
            if constexpr (kTrace) tw = __builtin_amdgcn_s_memtime();
            if constexpr (kPace > 0) __builtin_amdgcn_s_sleep(kPace);
            write_phase(r[(u + 1) % kDepth], p + 1);
            if constexpr (kTrace) t_write += __builtin_amdgcn_s_memtime() - tw;
            load_phase(r[(u + 1) % kDepth], p + 1 + kDepth);
          }
          uint64_t tb = 0;
          if constexpr (kTrace) tb = __builtin_amdgcn_s_memtime();
          lds_barrier();
          if constexpr (kTrace) t_wait += __builtin_amdgcn_s_memtime() - tb;
        }
      }
    }
    if constexpr (kTrace) {
      if (lane == 0) {
        uint64_t* tr = trace + (uint64_t)blockIdx.x * 1024u;
        tr[1019] = __builtin_amdgcn_s_memtime() - t_start;
        tr[1022] = t_wait;
        tr[1023] = t_write;
      }
    }
    return;
  }

  // ---------------- chain ----------------
  // Phases in which every live lane still has all kHalf blocks run without a
  // per-block lane predicate (wave-uniform branch on an SGPR).
  const uint32_t live_lo = rfl_u32((wave_max_u32(delta) + kHalf - 1) / kHalf);
  const uint32_t live_hi = rfl_u32(wave_min_u32(live ? nblk + delta : 0xffffffffu) / kHalf);
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
  if (kColumn && col_off != 0 && live) {
    const u32x4 s4 = *reinterpret_cast<const u32x4*>(states + 4u * (uint64_t)idx);
    st[0] = s4.x;
    st[1] = s4.y;
    st[2] = s4.z;
    st[3] = s4.w;
  }
  uint64_t c_start = 0, c_wait = 0;
  if constexpr (kTrace) c_start = __builtin_amdgcn_s_memtime();
  lds_barrier();
  for (uint32_t p = 0; p < phases; ++p) {
    if constexpr (kTrace) {
      if (lane == 0 && (p & 4095u) == 0u) {
        uint64_t* tr = trace + (uint64_t)blockIdx.x * 1024u + 2u * (p >> 12);
        tr[0] = __builtin_amdgcn_s_memtime();
        tr[1] = __builtin_amdgcn_s_memrealtime();
      }
    }
    const uint32_t s0 = (p & 1u) * kHalf;
    if (p >= live_lo && p < live_hi)
      chain_phase<true, kHalf, kLead, kLead2>(st, ring, s0, lane, p * kHalf - delta, nblk);
    else
      chain_phase<false, kHalf, kLead, kLead2>(st, ring, s0, lane, p * kHalf - delta, nblk);
    uint64_t tb = 0;
    if constexpr (kTrace) tb = __builtin_amdgcn_s_memtime();
    lds_barrier();
    if constexpr (kTrace) c_wait += __builtin_amdgcn_s_memtime() - tb;
  }
  if constexpr (kTrace) {
    if (lane == 0) {
      uint64_t* tr = trace + (uint64_t)blockIdx.x * 1024u;
      tr[1020] = c_wait;
      tr[1021] = __builtin_amdgcn_s_memtime() - c_start;
    }
  }
  if (!live) return;
  if (kColumn && !final) {
    u32x4 o = {st[0], st[1], st[2], st[3]};
    *reinterpret_cast<u32x4*>(states + 4u * (uint64_t)idx) = o;
    return;
  }
  finish(st, cd.ptr + ((uint64_t)nblk << 6), (uint32_t)(seg & 63u), cd.len);
  u32x4 o = {st[0], st[1], st[2], st[3]};
  *reinterpret_cast<u32x4*>(digests + 4u * (uint64_t)idx) = o;
}

// Whole-chunk batches: producer loads two phases ahead (kDepth 2) and, after
// each phase barrier, a ~512-cycle pause before it writes the next phase, so
// its 64 ring writes do not queue ahead of the chain's first operand reads of
// the phase: 1200 against 1210-1219 cycles per block at 512 x 10 MiB
// (profiles/r02_pace_ab.log).  Longer pauses make the producer late.
constexpr int kPcDepth = 2;
constexpr int kPcPace = 8;  // s_sleep units of 64 cycles

extern "C" __global__ __launch_bounds__(128) void qsmd5_batch_pc_kernel(
    const ChunkDesc* __restrict__ chunks, const uint32_t* __restrict__ order, uint32_t n,
    uint32_t* __restrict__ digests, uint32_t skew, uint32_t lanes) {
  pc_body<false, kPcDepth, kPcHalf, false, false, kPcPace>(chunks, order, n, digests, 0, ~0ull,
                                                           nullptr, skew, nullptr, lanes);
}

// The same kernel with the lanes per workgroup fixed at compile time (the
// runtime's two choices, 64 and 32): the lane bounds fold away, worth ~1% of
// the chain's cycles at 512 x 10 MiB (profiles/r02_pace_ab.log).
#define QSMD5_PC_FIXED(NAME, LANES, NT)                                                        \
  extern "C" __global__ __launch_bounds__(128) void NAME(                                     \
      const ChunkDesc* __restrict__ chunks, const uint32_t* __restrict__ order, uint32_t n,   \
      uint32_t* __restrict__ digests, uint32_t skew) {                                        \
    pc_body<false, kPcDepth, kPcHalf, NT, false, kPcPace>(chunks, order, n, digests, 0, ~0ull, \
                                                          nullptr, skew, nullptr, LANES);      \
  }
QSMD5_PC_FIXED(qsmd5_batch_pc64_kernel, 64u, false)
QSMD5_PC_FIXED(qsmd5_batch_pc64_nt_kernel, 64u, true)
QSMD5_PC_FIXED(qsmd5_batch_pc32_kernel, 32u, false)
QSMD5_PC_FIXED(qsmd5_batch_pc32_nt_kernel, 32u, true)
#undef QSMD5_PC_FIXED

// 2-block phases: a 64 KiB ring, so two workgroups (four waves) share a CU and
// one launch keeps 2 x 256 x 64 chunks resident (kKernelLatency2).
extern "C" __global__ __launch_bounds__(128) void qsmd5_batch_pc2_kernel(
    const ChunkDesc* __restrict__ chunks, const uint32_t* __restrict__ order, uint32_t n,
    uint32_t* __restrict__ digests, uint32_t skew, uint32_t lanes) {
  pc_body<false, 1, 2>(chunks, order, n, digests, 0, ~0ull, nullptr, skew, nullptr, lanes);
}

// The same two kernels with non-temporal producer loads.
extern "C" __global__ __launch_bounds__(128) void qsmd5_batch_pc_nt_kernel(
    const ChunkDesc* __restrict__ chunks, const uint32_t* __restrict__ order, uint32_t n,
    uint32_t* __restrict__ digests, uint32_t skew, uint32_t lanes) {
  pc_body<false, kPcDepth, kPcHalf, true, false, kPcPace>(chunks, order, n, digests, 0, ~0ull,
                                                          nullptr, skew, nullptr, lanes);
}

extern "C" __global__ __launch_bounds__(128) void qsmd5_batch_pc2_nt_kernel(
    const ChunkDesc* __restrict__ chunks, const uint32_t* __restrict__ order, uint32_t n,
    uint32_t* __restrict__ digests, uint32_t skew, uint32_t lanes) {
  pc_body<false, 1, 2, true>(chunks, order, n, digests, 0, ~0ull, nullptr, skew, nullptr, lanes);
}

extern "C" __global__ __launch_bounds__(128) void qsmd5_column_pc_kernel(
    const ChunkDesc* __restrict__ segs, const uint32_t* __restrict__ order, uint32_t n,
    uint32_t* __restrict__ digests, uint64_t col_off, uint64_t col_w,
    uint32_t* __restrict__ states) {
  pc_body<true>(segs, order, n, digests, col_off, col_w, states, 0u);
}

extern "C" __global__ __launch_bounds__(128) void qsmd5_column_pc2_kernel(
    const ChunkDesc* __restrict__ segs, const uint32_t* __restrict__ order, uint32_t n,
    uint32_t* __restrict__ digests, uint64_t col_off, uint64_t col_w,
    uint32_t* __restrict__ states) {
  pc_body<true, 1, 2>(segs, order, n, digests, col_off, col_w, states, 0u);
}

// ---------------------------------------------------------------------------
// Throughput kernel with coalesced LDS-DMA staging (batches of >> 16 K chunks).
//
// Each lane walking its own chunk makes every load instruction touch 64
// different lines; that pattern alone tops out at ~4.0-4.6 TB/s on MI355X
// (ubench lane_stream) against 7.1 TB/s for coalesced reads.  Here the wave
// instead stages 2 blocks (128 B) of each of its 64 chains per tile with 8
// global_load_lds_dwordx4: instruction i fetches chains 8i..8i+7, 8 lanes x 16 B
// contiguous per chain, straight into LDS rows [chain][8 x 16 B].  Each lane
// then reads its own row back (8 ds_read_b128).  The 16-B slots of row c are
// XOR-swizzled by (c >> 1) & 7 on the SOURCE address (the LDS-DMA destination
// is lane-linear), which makes the row reads bank-conflict-free.  Tiles are
// double-buffered: tile t+1 is in flight (vmcnt 8) while tile t compresses.
// Requires 16-byte-aligned chunks (the host routes others to qsmd5_batch_kernel).
#define QS_GP(p) ((const __attribute__((address_space(1))) void*)(uintptr_t)(p))
#define QS_LP(p) ((__attribute__((address_space(3))) void*)(uintptr_t)(uint32_t)(uintptr_t)(p))

// One fast-region tile U of a group (see batch_coal_body): prefetch the next
// tile into buffer (U + 1) & 1, then compress tile U from buffer U & 1 with no
// lane predicate.  kImm = false: each DMA source pointer is bumped per tile
// (1 VALU each).  kImm = true: the pointers stay at the group's first prefetch
// tile and tile U is reached with the instruction's immediate offset U x 128.
// The hardware adds that offset to the LDS destination as well as to the
// global address, so the LDS base passed in (M0) is lowered by the same amount
// (the caller pads the LDS buffer in front to keep it non-negative).
// Cache policy (aux) of the coalesced kernel's LDS-DMA loads: 2 = nt (non-temporal).
// Every byte is read once; nt ran the saturation lines 1-2 points of HBM peak
// higher than the default policy, A/B/A/B on one box.
#ifndef QS_COAL_AUX
#define QS_COAL_AUX 2
#endif
template <int U, int kU, int kTB, int kS, int kCPI, bool kImm>
__device__ __forceinline__ void coal_fast_group(uint32_t (&st)[4], const uint8_t* (&gp)[kS],
                                                u32x4 (*tile_buf)[64][kS], uint32_t lane,
                                                uint32_t rswz) {
  if constexpr (U < kU) {
#pragma unroll
    for (int i = 0; i < kS; ++i) {
      if constexpr (kImm) {
        constexpr int kOff = U * kTB * 64;
        __builtin_amdgcn_global_load_lds(
            QS_GP(gp[i]),
            QS_LP(reinterpret_cast<uintptr_t>(&tile_buf[(U + 1) & 1][i * kCPI][0]) - kOff), 16,
            kOff, QS_COAL_AUX);
      } else {
        __builtin_amdgcn_global_load_lds(QS_GP(gp[i]), QS_LP(&tile_buf[(U + 1) & 1][i * kCPI][0]),
                                         16, 0, QS_COAL_AUX);
        gp[i] += kTB * 64;
      }
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kS) : "memory");
#pragma unroll
    for (int h = 0; h < kTB; ++h) {
      uint32_t w[16];
      unpack4(w, 0, tile_buf[U & 1][lane][(4 * h + 0) ^ rswz]);
      unpack4(w, 1, tile_buf[U & 1][lane][(4 * h + 1) ^ rswz]);
      unpack4(w, 2, tile_buf[U & 1][lane][(4 * h + 2) ^ rswz]);
      unpack4(w, 3, tile_buf[U & 1][lane][(4 * h + 3) ^ rswz]);
      md5_compress(st, w);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    coal_fast_group<U + 1, kU, kTB, kS, kCPI, kImm>(st, gp, tile_buf, lane, rswz);
  }
}

// kPrioEpoch (ubench only; 0 in every product kernel): every 2^kPrioEpoch
// tiles of the fast region, a wave sets its issue priority to
// (epoch ^ WAVE_ID) & 1, so the two waves of a SIMD take turns at the
// higher priority instead of the older one finishing first (round 5 stamps).
template <int kTB, int kBufs, bool kImm = false, int kPrioEpoch = 0>
__device__ __forceinline__ void batch_coal_body(const ChunkDesc* __restrict__ chunks,
                                                const uint32_t* __restrict__ order, uint32_t n,
                                                uint32_t* __restrict__ digests) {
  // kTB blocks (kTB x 64 B) per chain per tile; kBufs tile buffers: kBufs - 1
  // tiles in flight while one compresses.  A row of kS 16-B slots per chain;
  // one LDS-DMA instruction covers 64 / kS chains, kS instructions per tile.
  constexpr int kS = 4 * kTB;
  constexpr int kCPI = 64 / kS;  // chains per instruction
  // kImm: pad in front of the tiles so that M0 = destination - offset >= 0
  constexpr int kUImm = 4;
  constexpr int kPad = kImm ? ((kUImm - 1) * kTB * 64 + 15) / 16 : 0;
  __shared__ u32x4 tile_raw[kPad + kBufs * 64 * kS];
  u32x4 (*tile_buf)[64][kS] = reinterpret_cast<u32x4 (*)[64][kS]>(tile_raw + kPad);
  const uint32_t lane = threadIdx.x;
  const uint32_t t = blockIdx.x * 64u + lane;
  uint32_t idx = 0;
  ChunkDesc cd = {nullptr, 0};
  if (t < n) {
    idx = order ? order[t] : t;
    cd = chunks[idx];
  }
  const uint32_t nblk = (uint32_t)(cd.len >> 6);
  const uint32_t ntiles = rfl_u32((wave_max_u32(nblk) + (kTB - 1)) / kTB);
  // Slot swizzle making the row reads (lane l reads row l) bank-conflict-free
  // for ds_read_b128's 16-lane groups: rows of 128 B alternate bank halves.
  auto swz = [](uint32_t c) -> uint32_t {
    return kTB == 2 ? ((c >> 1) & 7u) : (c & 15u);
  };

  // Loader role of this lane in instruction i: chain kCPI*i + lane / kS, slot lane % kS.
  const uint32_t slot = lane % kS;
  const uint64_t myptr = reinterpret_cast<uint64_t>(cd.ptr);
  const uint8_t* src[kS];
  uint32_t src_nblk[kS], piece[kS];
#pragma unroll
  for (int i = 0; i < kS; ++i) {
    const int c = i * kCPI + (int)(lane / kS);
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)myptr, c, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(myptr >> 32), c, 64);
    src[i] = reinterpret_cast<const uint8_t*>(((uint64_t)hi << 32) | lo);
    src_nblk[i] = (uint32_t)__shfl((int)nblk, c, 64);
    piece[i] = slot ^ swz((uint32_t)c);  // 16-B piece this lane fetches
  }
  // Exactly kS LDS-DMA instructions per tile, whatever the chain lengths: the
  // counted vmcnt waits below depend on it.  Lanes whose chain has no whole
  // block left (or no chain) fetch 16 harmless bytes from the descriptor array.
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(chunks);
  auto issue_tile = [&](uint32_t b, uint32_t tl) {
#pragma unroll
    for (int i = 0; i < kS; ++i) {
      const uint32_t blk = min(tl * (uint32_t)kTB + (piece[i] >> 2), src_nblk[i] - 1u);
      const uint8_t* g = src_nblk[i] ? src[i] + (uint64_t)blk * 64u + (piece[i] & 3u) * 16u
                                     : dummy;
      __builtin_amdgcn_global_load_lds(QS_GP(g), QS_LP(&tile_buf[b][i * kCPI][0]), 16, 0,
                                       QS_COAL_AUX);
    }
  };
  const uint32_t rswz = swz(lane);
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
#pragma unroll
  for (int k = 0; k < kBufs - 1; ++k)
    if ((uint32_t)k < ntiles) issue_tile((uint32_t)k, (uint32_t)k);
  uint32_t tl = 0;
  if constexpr (kBufs == 2) {
    // Fast region: a full wave whose every chain still has whole tiles.  No
    // clamp, no dummy source, no per-block lane predicate: each DMA source is
    // one 64-bit pointer bumped per tile (1 VALU), and the row reads are
    // loop-invariant per-lane addresses.  This removes ~24 VALU per block
    // (352 -> 328, ~7%) in a regime bound by VALU x clock
    // (profiles/r01_ubench_probe.log).
    constexpr int kU = kImm ? kUImm : 2;  // tiles per loop trip (even: static buffer index)
    const bool full_wave = (blockIdx.x + 1u) * 64u <= n;
    const uint32_t fast_tiles = full_wave ? rfl_u32(wave_min_u32(nblk)) / (uint32_t)kTB : 0u;
    const uint8_t* gp[kS];  // source of tile tl + 1 for DMA instruction i
#pragma unroll
    for (int i = 0; i < kS; ++i)
      gp[i] = src[i] + kTB * 64u + (piece[i] >> 2) * 64u + (piece[i] & 3u) * 16u;
    for (; tl + (uint32_t)kU < fast_tiles; tl += (uint32_t)kU) {
      if constexpr (kPrioEpoch > 0) {
        const uint32_t wave_id = __builtin_amdgcn_s_getreg((3 << 11) | 4) & 0xfu;  // HW_ID[3:0]
        if (((tl >> kPrioEpoch) ^ wave_id) & 1u) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      coal_fast_group<0, kU, kTB, kS, kCPI, kImm>(st, gp, tile_buf, lane, rswz);
      if constexpr (kImm) {
#pragma unroll
        for (int i = 0; i < kS; ++i) gp[i] += kU * kTB * 64;
      }
    }
  }
  for (; tl < ntiles; ++tl) {
    const uint32_t b = tl % kBufs;
    if (tl + (kBufs - 1) < ntiles) {
      issue_tile((tl + (kBufs - 1)) % kBufs, tl + (kBufs - 1));
      // the kBufs - 1 younger tiles (kS LDS-DMA each) may stay in flight
      if constexpr (kS * (kBufs - 1) == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if constexpr (kS * (kBufs - 1) == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      // last kBufs - 1 tiles: fewer follow, drain
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int h = 0; h < kTB; ++h) {
      u32x4 q0 = tile_buf[b][lane][(4 * h + 0) ^ rswz];
      u32x4 q1 = tile_buf[b][lane][(4 * h + 1) ^ rswz];
      u32x4 q2 = tile_buf[b][lane][(4 * h + 2) ^ rswz];
      u32x4 q3 = tile_buf[b][lane][(4 * h + 3) ^ rswz];
      if (tl * (uint32_t)kTB + h < nblk) {
        uint32_t w[16];
        unpack4(w, 0, q0);
        unpack4(w, 1, q1);
        unpack4(w, 2, q2);
        unpack4(w, 3, q3);
        md5_compress(st, w);
      }
    }
    // the next issue_tile may overwrite a buffer: make sure the row reads are done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (t >= n) return;
  finish(st, cd.ptr + ((uint64_t)nblk << 6), (uint32_t)(cd.len & 63u), cd.len);
  u32x4 o = {st[0], st[1], st[2], st[3]};
  *reinterpret_cast<u32x4*>(digests + 4u * (uint64_t)idx) = o;
}

// 2-block tiles, two tile buffers (16 KiB LDS per wave, up to 10 waves per
// CU).  Measured alternatives (profiles/r01_ubench_coal_variants.log): a third
// buffer, or 4-block tiles (32 KiB per wave), both lose 25-35% at
// 131072 x 64 KiB -- fewer resident waves, the batch no longer fits one round.
extern "C" __global__ __launch_bounds__(64) void qsmd5_batch_coal_kernel(
    const ChunkDesc* __restrict__ chunks, const uint32_t* __restrict__ order, uint32_t n,
    uint32_t* __restrict__ digests) {
  batch_coal_body<2, 2>(chunks, order, n, digests);
}

#undef QS_GP
#undef QS_LP

// ---------------------------------------------------------------------------
// Gather of host rows into the staging ring (qsmd5_rt_staging.cpp run_batch).
// Rows that cannot share a 2-D DMA copy -- pinned buffers in separate
// allocations, each one HIP allocation on its own -- would otherwise cost one
// hipMemcpyAsync each (~8-10 us of overhead per 256 KiB column row).  Pinned
// and registered host memory is mapped for the GPU, so one launch per slice
// reads every row over PCIe instead.  The host only hands over rows that lie
// inside one HIP-known host allocation, 16-B aligned at both ends of the
// dwordx4 body; the last len % 16 bytes go byte by byte, so nothing past a
// row is read.  A few persistent workgroups walk the rows: 8 of them, with 4
// loads of 16 B in flight per thread (128 KiB in flight), keep the link full,
// as 4 already do.  More hurt: the chains of earlier columns run beside the
// gathers of later ones, and with one workgroup per row their 2 ms columns
// took up to 94 ms, with 64 workgroups 5-6 ms -- the chains' HBM loads queue
// behind the gathers' PCIe reads.  8 workgroups leave them at 2.05-2.1 ms
// (profiles/r02_gather_groups.log).  Each also reserves 80 KiB of LDS it never
// uses, so a CU holding one cannot take a latency-kernel workgroup (128 KiB).
struct GatherRow {
  const uint8_t* src;  // device-visible address of the host bytes
  uint8_t* dst;        // staging segment (256-B aligned)
  uint64_t len;
};

__device__ __forceinline__ void gather_row(const GatherRow g) {
  const uint64_t nvec = g.len >> 4;
  const u32x4* __restrict__ src = reinterpret_cast<const u32x4*>(g.src);
  u32x4* __restrict__ dst = reinterpret_cast<u32x4*>(g.dst);
  constexpr uint32_t kU = 4;
  uint64_t i = threadIdx.x;
  for (; i + (kU - 1) * 256u < nvec; i += kU * 256u) {
    u32x4 v[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) v[u] = __builtin_nontemporal_load(src + i + u * 256u);
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) dst[i + u * 256u] = v[u];
  }
  for (; i < nvec; i += 256u) dst[i] = __builtin_nontemporal_load(src + i);
  const uint64_t tail = g.len & 15u;
  if (threadIdx.x < tail) g.dst[(nvec << 4) + threadIdx.x] = g.src[(nvec << 4) + threadIdx.x];
}

extern "C" __global__ __launch_bounds__(256) void qsmd5_gather_kernel(const GatherRow* __restrict__ rows,
                                                                     uint32_t nrows) {
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) gather_row(rows[r]);
}

// ---------------------------------------------------------------------------
// Host launchers (md5_launch.h).
#include "md5_launch.h"

namespace qsmd5 {

// Each launcher returns hipGetLastError() after its launch, and that reports
// the last failure of ANY HIP call on the thread: a stale one -- the runtime's
// own out-of-memory hipMalloc before a CPU fallback, or the caller's -- would
// fail a good launch (and every later one until read).  So each launcher
// clears it first (clear_stale_error), and the launch's own status is what
// comes back.
static inline void clear_stale_error() { (void)hipGetLastError(); }

hipError_t launch_batch(const void* chunks, const uint32_t* order, uint32_t n, uint32_t* digests,
                        int kind, hipStream_t s, uint32_t skew_blocks, bool load_nt, uint32_t lanes) {
  if (n == 0) return hipSuccess;
  clear_stale_error();
  const uint32_t groups = (n + 63u) / 64u;
  if (lanes < 1 || lanes > 64) return hipErrorInvalidValue;
  const uint32_t pc_groups = (n + lanes - 1) / lanes;
  if (kind == kKernelLatency) {
    const ChunkDesc* c = static_cast<const ChunkDesc*>(chunks);
    const uint32_t skew = skew_blocks / kPcHalf * kPcHalf;
    if (lanes == 64)
      hipLaunchKernelGGL(load_nt ? qsmd5_batch_pc64_nt_kernel : qsmd5_batch_pc64_kernel,
                         dim3(pc_groups), dim3(128), 0, s, c, order, n, digests, skew);
    else if (lanes == 32)
      hipLaunchKernelGGL(load_nt ? qsmd5_batch_pc32_nt_kernel : qsmd5_batch_pc32_kernel,
                         dim3(pc_groups), dim3(128), 0, s, c, order, n, digests, skew);
    else
      hipLaunchKernelGGL(load_nt ? qsmd5_batch_pc_nt_kernel : qsmd5_batch_pc_kernel, dim3(pc_groups),
                         dim3(128), 0, s, c, order, n, digests, skew, lanes);
  } else if (kind == kKernelLatency2) {
    hipLaunchKernelGGL(load_nt ? qsmd5_batch_pc2_nt_kernel : qsmd5_batch_pc2_kernel, dim3(pc_groups),
                       dim3(128), 0, s, static_cast<const ChunkDesc*>(chunks), order, n, digests,
                       skew_blocks / kPcHalf * kPcHalf, lanes);
  } else if (kind == kKernelCoalesced) {
    hipLaunchKernelGGL(qsmd5_batch_coal_kernel, dim3(groups), dim3(64), 0, s,
                       static_cast<const ChunkDesc*>(chunks), order, n, digests);
  } else {
    hipLaunchKernelGGL(qsmd5_batch_kernel, dim3(groups), dim3(64), 0, s,
                       static_cast<const ChunkDesc*>(chunks), order, n, digests);
  }
  return hipGetLastError();
}

hipError_t launch_column(const void* segs, const uint32_t* order, uint32_t n, uint32_t* digests,
                         uint64_t col_off, uint64_t col_w, uint32_t* states, hipStream_t s) {
  if (n == 0) return hipSuccess;
  clear_stale_error();
  if (n > kLatencyKernelResident)  // beyond one resident round: two workgroups per CU
    hipLaunchKernelGGL(qsmd5_column_pc2_kernel, dim3((n + 63u) / 64u), dim3(128), 0, s,
                       static_cast<const ChunkDesc*>(segs), order, n, digests, col_off, col_w,
                       states);
  else
    hipLaunchKernelGGL(qsmd5_column_pc_kernel, dim3((n + 63u) / 64u), dim3(128), 0, s,
                       static_cast<const ChunkDesc*>(segs), order, n, digests, col_off, col_w,
                       states);
  return hipGetLastError();
}


hipError_t launch_gather(const void* rows, uint32_t nrows, hipStream_t s, uint32_t groups) {
  if (nrows == 0) return hipSuccess;
  constexpr size_t kGatherLds = 80u << 10;  // keeps latency-kernel workgroups off these CUs
  if (groups == 0) groups = 1;
  clear_stale_error();
  hipLaunchKernelGGL(qsmd5_gather_kernel, dim3(nrows < groups ? nrows : groups),
                     dim3(256), kGatherLds, s, static_cast<const GatherRow*>(rows), nrows);
  return hipGetLastError();
}

hipError_t launch_final(uint32_t* state, const uint8_t* tail, uint32_t rem, uint64_t total_len,
                        hipStream_t s) {
  clear_stale_error();
  hipLaunchKernelGGL(qsmd5_final_kernel, dim3(1), dim3(64), 0, s, state, tail, rem, total_len);
  return hipGetLastError();
}

// One empty launch: loads the library's code object (all kernels) at init
// instead of on the first hash (first 10 MiB call 107 -> ~85 ms), and fails
// init early if the device cannot run gfx950 code.
hipError_t warm_up(hipStream_t s) {
  clear_stale_error();
  hipLaunchKernelGGL(qsmd5_lcg_fill_kernel, dim3(1), dim3(64), 0, s, nullptr, 0, 0, 0u, 0u, 1);
  return hipGetLastError();
}

hipError_t launch_lcg_fill(uint8_t* base, uint64_t stride, uint64_t len, uint32_t seed0,
                           uint32_t nchunks, hipStream_t s) {
  if (nchunks == 0 || len == 0) return hipSuccess;
  const uint64_t segs = (len + kSeg - 1) / kSeg;
  const uint64_t threads = segs * nchunks;
  const uint64_t blocks = (threads + 255) / 256;
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  clear_stale_error();
  hipLaunchKernelGGL(qsmd5_lcg_fill_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, base, stride,
                     len, seed0, nchunks, segs);
  return hipGetLastError();
}

}  // namespace qsmd5
