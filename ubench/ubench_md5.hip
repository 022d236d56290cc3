// ubench/ubench_md5.hip -- gfx950 micro-measurements behind the MD5 kernel design.
//
// 1. VALU issue/latency for one wave alone on its SIMD (inline-asm loops timed
//    with s_memtime): dependent vs independent v_add_u32, v_alignbit_b32,
//    v_bitop3_b32, v_add3_u32.  These set the per-chain MD5 rate.
// 2. qsmd5_batch_kernel on B chunks x L bytes of device-resident LCG data:
//    wall time per launch (hipEvents) -> per-chain rate r1 and B*r1, with every
//    digest checked against the CPU oracle.
// Test infrastructure, not product code.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <chrono>
#include <vector>

#include "../qsfs-fuse_amd/csrc/md5_kernels.hip"
extern "C" {
#include "../oracle/md5_oracle.c"
}

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
              __LINE__);                                                           \
      exit(2);                                                                     \
    }                                                                              \
  } while (0)

// Latency kernel with a deeper producer prefetch (kDepth phases of loads in flight).
template <int D>
__global__ __launch_bounds__(128) void k_pc_depth(const ChunkDesc* __restrict__ c,
                                                  const uint32_t* __restrict__ o, uint32_t n,
                                                  uint32_t* __restrict__ d, uint32_t skew) {
  pc_body<false, D>(c, o, n, d, 0, ~0ull, nullptr, skew);
}

// Latency kernel with 2-block phases: a 64 KiB LDS ring, two workgroups per CU.
__global__ __launch_bounds__(128) void k_pc_half2(const ChunkDesc* __restrict__ c,
                                                  const uint32_t* __restrict__ o, uint32_t n,
                                                  uint32_t* __restrict__ d, uint32_t skew) {
  pc_body<false, 1, 2>(c, o, n, d, 0, ~0ull, nullptr, skew);
}

// Latency kernel with the chain wave stamping its clocks every 4096 phases.
__global__ __launch_bounds__(128) void k_pc_trace(const ChunkDesc* __restrict__ c,
                                                  const uint32_t* __restrict__ o, uint32_t n,
                                                  uint32_t* __restrict__ d, uint32_t skew,
                                                  uint64_t* __restrict__ tr, uint32_t lanes) {
  pc_body<false, kPcDepth, kPcHalf, false, true, kPcPace>(c, o, n, d, 0, ~0ull, nullptr, skew, tr,
                                                          lanes);
}

// The shipped 64-lane latency kernel with parts of its producer switched off
// (pc_body kProbe): what the producer's ring writes and HBM loads cost the chain.
template <int kProbe>
__global__ __launch_bounds__(128) void k_pc_probe(const ChunkDesc* __restrict__ c,
                                                  const uint32_t* __restrict__ o, uint32_t n,
                                                  uint32_t* __restrict__ d, uint32_t skew) {
  pc_body<false, kPcDepth, kPcHalf, false, false, kPcPace, 0, kPcLead, 0, kProbe>(
      c, o, n, d, 0, ~0ull, nullptr, skew, nullptr, 64u);
}

// chain_phase with the 16 LDS reads of block h+1 spread through block h's 256
// VALU (one read per kR VALU, placed with sched_group_barrier) instead of
// issued together at the block's start.
template <int kR, int kHalf = kPcHalf>
__device__ __forceinline__ void chain_phase_spread(uint32_t (&st)[4], const u32x4 (*ring)[16][64],
                                                   uint32_t s0, uint32_t lane) {
  u32x4 a[16], b[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) a[g] = ring[s0][g][lane];
#pragma unroll
  for (int h = 0; h < kHalf; ++h) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
    __builtin_amdgcn_sched_barrier(0);
    u32x4 (&cur)[16] = (h & 1) ? b : a;
    u32x4 (&nxt)[16] = (h & 1) ? a : b;
    if (h + 1 < kHalf) {
#pragma unroll
      for (int g = 0; g < 16; ++g) nxt[g] = ring[s0 + h + 1][g][lane];
    }
    uint32_t mk[64];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      mk[4 * g + 0] = cur[g].x;
      mk[4 * g + 1] = cur[g].y;
      mk[4 * g + 2] = cur[g].z;
      mk[4 * g + 3] = cur[g].w;
    }
    md5_compress_mk(st, mk);
    if (h + 1 < kHalf) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);   // one DS read
        __builtin_amdgcn_sched_group_barrier(0x0002, kR, 0);  // kR VALU
      }
    }
  }
}

template <int kR>
__global__ __launch_bounds__(128) void k_chain_spread(uint64_t* out, uint32_t* sink, int phases) {
  __shared__ u32x4 ring[2 * kPcHalf][16][64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (int k = threadIdx.x; k < 2 * kPcHalf * 16 * 64; k += blockDim.x)
    (&ring[0][0][0])[k] = u32x4{(uint32_t)k * 2654435761u, (uint32_t)k, 7u, 9u};
  __syncthreads();
  if (wave == 1) return;
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int p = 0; p < phases; ++p) chain_phase_spread<kR>(st, ring, (uint32_t)(p & 1) * kPcHalf, lane);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = t1 - t0;
  sink[lane] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

// Decomposition of the latency kernel's chain-wave cost per 64-B block:
//   kMode 0: chain_phase<true> over a pre-filled LDS ring, no producer, no barrier
//   kMode 1: mode 0 + lds_barrier() after every phase, with a second wave that
//            only meets the barriers (the producer's role without its loads)
//   kMode 2: md5_compress_mk from registers (no LDS reads at all)
// out[0] = s_memtime cycles of the chain wave over `phases` phases of 4 blocks.
template <int kMode, uint32_t kLanes = 64, int kL = 0>
__global__ __launch_bounds__(128) void k_chain_cost(uint64_t* out, uint32_t* sink, int phases) {
  __shared__ u32x4 ring[2 * kPcHalf][16][64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (int k = threadIdx.x; k < 2 * kPcHalf * 16 * 64; k += blockDim.x)
    (&ring[0][0][0])[k] = u32x4{(uint32_t)k * 2654435761u, (uint32_t)k, 7u, 9u};
  __syncthreads();
  if (wave == 1) {
    if (kMode == 1)
      for (int p = 0; p < phases; ++p) lds_barrier();
    return;
  }
  if (lane >= kLanes) return;  // fewer active chains: a narrower EXEC mask
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
  uint32_t mk[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) mk[i] = (&ring[0][0][0])[i * 64 + lane].x;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int p = 0; p < phases; ++p) {
    if constexpr (kMode == 2) {
#pragma unroll
      for (int h = 0; h < kPcHalf; ++h) md5_compress_mk(st, mk);
      asm volatile("" : "+v"(st[0]), "+v"(st[1]));
    } else {
      chain_phase<true, kPcHalf, kL>(st, ring, (uint32_t)(p & 1) * kPcHalf, lane, 0, 1u << 30);
      if (kMode == 1) lds_barrier();
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = t1 - t0;
  sink[lane] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

// Round 3 (session 2): where could the chain's operands come from, if not the
// LDS ring the producer shares with it?  The chain wave alone, continuous (no
// phases, no barrier): block h+1's 16 operand groups are requested while block
// h compresses, one wait per block.
//   kSrc 0: LDS ring of 8 blocks (ds_read_b128)
//   kSrc 1..3: a global ring of kRing blocks, buffer_load_dwordx4 with the
//     cache policy aux = 0 (default), 1 (sc0: L2, the policy a ring written by
//     another CU needs), 2 (nt)
// out[0] = s_memtime cycles over `blocks` blocks.
template <int kSrc, int kRing = 8>
__global__ __launch_bounds__(128) void k_chain_ring(uint64_t* out, uint32_t* sink, int blocks,
                                                    const u32x4* __restrict__ gring) {
  __shared__ u32x4 ring[8][16][64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  if (kSrc == 0) {
    for (int k = threadIdx.x; k < 8 * 16 * 64; k += blockDim.x)
      (&ring[0][0][0])[k] = u32x4{(uint32_t)k * 2654435761u, (uint32_t)k, 7u, 9u};
    __syncthreads();
  }
  if (wave == 1) return;
  constexpr int kAux = kSrc == 1 ? 0 : kSrc == 2 ? 1 : 2;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)gring, 0, kRing * 16384, 0x00020000);
  u32x4 a[16], b[16];
  auto read_blk = [&](u32x4 (&dst)[16], uint32_t blk) {
    const uint32_t slot = blk & (kRing - 1);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      if constexpr (kSrc == 0)
        dst[g] = ring[blk & 7u][g][lane];
      else
        dst[g] = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lane * 16u + g * 1024u),
                                                         (int)(slot * 16384u), kAux));
    }
  };
  auto compress = [&](uint32_t (&st)[4], const u32x4 (&src)[16]) {
    uint32_t mk[64];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      mk[4 * g + 0] = src[g].x;
      mk[4 * g + 1] = src[g].y;
      mk[4 * g + 2] = src[g].z;
      mk[4 * g + 3] = src[g].w;
    }
    md5_compress_mk(st, mk);
  };
  constexpr int kWait = kSrc == 0 ? kLgkmcnt0 : 0x0F70;  // lgkmcnt(0) / vmcnt(0)
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
  read_blk(a, 0);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int h = 0; h < blocks; h += 2) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(kWait);
    read_blk(b, h + 1);
    __builtin_amdgcn_sched_barrier(0);
    compress(st, a);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(kWait);
    read_blk(a, h + 2);
    __builtin_amdgcn_sched_barrier(0);
    compress(st, b);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = t1 - t0;
  sink[lane] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

// The continuous LDS chain with block h+1's 16 operand reads issued after
// step kS of block h instead of at its start (the graded phase-start wait puts
// block 1's reads after step 8 of block 0; is that placement better for every
// block?).  kS = 0 is k_chain_ring<0>.
template <int kS>
__global__ __launch_bounds__(128) void k_chain_at(uint64_t* out, uint32_t* sink, int blocks,
                                                  const u32x4* __restrict__ gring) {
  (void)gring;
  __shared__ u32x4 ring[8][16][64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (int k = threadIdx.x; k < 8 * 16 * 64; k += blockDim.x)
    (&ring[0][0][0])[k] = u32x4{(uint32_t)k * 2654435761u, (uint32_t)k, 7u, 9u};
  __syncthreads();
  if (wave == 1) return;
  u32x4 a[16], b[16];
  auto read_blk = [&](u32x4 (&dst)[16], uint32_t blk) {
#pragma unroll
    for (int g = 0; g < 16; ++g) dst[g] = ring[blk & 7u][g][lane];
  };
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
  auto block = [&](const u32x4 (&cur)[16], u32x4 (&nxt)[16], uint32_t next_blk) {
    uint32_t mk[64];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      mk[4 * g + 0] = cur[g].x;
      mk[4 * g + 1] = cur[g].y;
      mk[4 * g + 2] = cur[g].z;
      mk[4 * g + 3] = cur[g].w;
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t v[4] = {st[0], st[1], st[2], st[3]};
    if constexpr (kS > 0) md5_steps_mk<0, kS>(v, mk);
    __builtin_amdgcn_sched_barrier(0);
    read_blk(nxt, next_blk);
    __builtin_amdgcn_sched_barrier(0);
    md5_steps_mk<kS, 64>(v, mk);
    st[0] += v[0];
    st[1] += v[1];
    st[2] += v[2];
    st[3] += v[3];
  };
  read_blk(a, 0);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int h = 0; h < blocks; h += 2) {
    block(a, b, h + 1);
    block(b, a, h + 2);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = t1 - t0;
  sink[lane] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

// The same continuous chain over an L1-sized global ring of kSlots blocks with
// kLanes live chains: slot = [16 groups][kLanes lanes] x 16 B, contiguous (the
// L1 footprint; kCompact = false spreads the groups 1 KiB apart).  Dead
// lanes keep EXEC full (a partial EXEC mask slows memory instructions) and
// read past the buffer's range (num_records): zeros, no memory access.
// kBar: an s_barrier after every block that a second wave meets (the
// per-block hand-off a producer would need).
template <int kSlots, int kLanes, bool kBar, bool kCompact = true>
__global__ __launch_bounds__(128) void k_chain_l1(uint64_t* out, uint32_t* sink, int blocks,
                                                  const u32x4* __restrict__ gring) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  if (wave == 1) {
    if (kBar)
      for (int p = 0; p < blocks + 1; ++p) __builtin_amdgcn_s_barrier();
    return;
  }
  constexpr uint32_t kRow = kCompact ? kLanes * 16u : 1024u;  // bytes per group row
  constexpr uint32_t kSlotB = 16u * kRow;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)gring, 0, kSlots * kSlotB, 0x00020000);
  const uint32_t vbase = lane < (uint32_t)kLanes ? lane * 16u : 0x40000000u;
  u32x4 a[16], b[16];
  auto read_blk = [&](u32x4 (&dst)[16], uint32_t slot) {
#pragma unroll
    for (int g = 0; g < 16; ++g)
      dst[g] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(vbase + g * kRow),
                                                       (int)(slot * kSlotB), 0));
  };
  auto compress = [&](uint32_t (&st)[4], const u32x4 (&src)[16]) {
    uint32_t mk[64];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      mk[4 * g + 0] = src[g].x;
      mk[4 * g + 1] = src[g].y;
      mk[4 * g + 2] = src[g].z;
      mk[4 * g + 3] = src[g].w;
    }
    md5_compress_mk(st, mk);
  };
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
  uint32_t slot = 0;
  auto next = [&]() { slot = slot + 1 == (uint32_t)kSlots ? 0u : slot + 1; return slot; };
  read_blk(a, 0);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int h = 0; h < blocks; h += 2) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    read_blk(b, next());
    __builtin_amdgcn_sched_barrier(0);
    compress(st, a);
    if (kBar) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    read_blk(a, next());
    __builtin_amdgcn_sched_barrier(0);
    compress(st, b);
    if (kBar) __builtin_amdgcn_s_barrier();
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (kBar) __builtin_amdgcn_s_barrier();
  if (lane == 0) out[0] = t1 - t0;
  sink[lane] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

// The hand-off the L1 ring would need: wave 1 stores block h+2 into slot
// h % 2 while the chain compresses block h, drains its stores (vmcnt(0)) and
// meets the chain at a per-block barrier; the chain waits for block h+1's
// operands before that barrier, then requests block h+2's.  Does the chain
// still hit L1 after another wave's stores, and does it see them?  Each group
// g of block j holds {j, lane, g, 0x5a}; out[1] counts the chain's mismatches.
// kStoreAux: the producer's store cache policy.
template <int kStoreAux>
__global__ __launch_bounds__(128) void k_l1_handoff(uint64_t* out, uint32_t* sink, int blocks,
                                                    u32x4* __restrict__ gring) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)gring, 0, 2 * 16384, 0x00020000);
  if (wave == 1) {
    auto put = [&](uint32_t blk) {
#pragma unroll
      for (int g = 0; g < 16; ++g)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) int,
                               u32x4{blk, lane, (uint32_t)g, 0x5au}),
            rs, (int)(lane * 16u + g * 1024u), (int)((blk & 1u) * 16384u), kStoreAux);
    };
    put(0);
    put(1);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_barrier();
    for (int h = 0; h < blocks; ++h) {
      put((uint32_t)h + 2u);
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __builtin_amdgcn_s_barrier();
    }
    return;
  }
  u32x4 a[16], b[16];
  auto read_blk = [&](u32x4 (&dst)[16], uint32_t blk) {
#pragma unroll
    for (int g = 0; g < 16; ++g)
      dst[g] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lane * 16u + g * 1024u),
                                                       (int)((blk & 1u) * 16384u), 0));
  };
  uint32_t bad = 0;
  auto compress = [&](uint32_t (&st)[4], const u32x4 (&src)[16], uint32_t blk) {
    uint32_t mk[64];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      bad += (src[g].x != blk) | (src[g].y != lane) | (src[g].z != (uint32_t)g);
      mk[4 * g + 0] = src[g].x;
      mk[4 * g + 1] = src[g].y;
      mk[4 * g + 2] = src[g].z;
      mk[4 * g + 3] = src[g].w;
    }
    md5_compress_mk(st, mk);
  };
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
  __builtin_amdgcn_s_barrier();
  read_blk(a, 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int h = 0; h < blocks; h += 2) {
    __builtin_amdgcn_sched_barrier(0);
    read_blk(b, (uint32_t)h + 1u);
    __builtin_amdgcn_sched_barrier(0);
    compress(st, a, (uint32_t)h);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    read_blk(a, (uint32_t)h + 2u);
    __builtin_amdgcn_sched_barrier(0);
    compress(st, b, (uint32_t)h + 1u);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_barrier();
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = t1 - t0;
  bad = __builtin_amdgcn_readfirstlane(bad) + 0u;  // lane 0's count is enough for a probe
  if (lane == 0) out[1] = bad;
  sink[lane] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

// Latency kernel with 5-block phases: a 160 KiB ring (all of a gfx950 CU's
// LDS), one barrier per 5 blocks instead of per 4.
// producer sleeps kP x ~64 cycles after each phase barrier before writing the
// ring, so the chain's first operand reads of the phase are not queued behind
// the producer's 64 ds_write_b128
template <int kP, int kG = 0, int kD = 1>
__global__ __launch_bounds__(128) void k_pc_pace(const ChunkDesc* __restrict__ c,
                                                 const uint32_t* __restrict__ o, uint32_t n,
                                                 uint32_t* __restrict__ d, uint32_t skew) {
  pc_body<false, kD, kPcHalf, false, false, kP, kG>(c, o, n, d, 0, ~0ull, nullptr, skew);
}

// Graded wait at each phase's first block (chain_phase kLead): the shipped
// producer (depth 2, pause 8) and 64 lanes fixed, as qsmd5_batch_pc64_kernel.
template <int kL, int kL2 = 0, int kP = 8, int kD = 2>
__global__ __launch_bounds__(128) void k_pc_lead(const ChunkDesc* __restrict__ c,
                                                 const uint32_t* __restrict__ o, uint32_t n,
                                                 uint32_t* __restrict__ d, uint32_t skew) {
  pc_body<false, kD, kPcHalf, false, false, kP, 0, kL, kL2>(c, o, n, d, 0, ~0ull, nullptr, skew, nullptr,
                                                      64u);
}

// 64 KiB-ring latency kernel (2-block phases) with the whole-chunk producer
// options of the 128 KiB kernel: pause kP after each barrier, depth kD
template <int kP, int kD>
__global__ __launch_bounds__(128) void k_pc2_pace(const ChunkDesc* __restrict__ c,
                                                  const uint32_t* __restrict__ o, uint32_t n,
                                                  uint32_t* __restrict__ d, uint32_t skew) {
  pc_body<false, kD, 2, false, false, kP>(c, o, n, d, 0, ~0ull, nullptr, skew, nullptr, 64u);
}

__global__ __launch_bounds__(128) void k_pc_half5(const ChunkDesc* __restrict__ c,
                                                  const uint32_t* __restrict__ o, uint32_t n,
                                                  uint32_t* __restrict__ d, uint32_t skew) {
  pc_body<false, 1, 5>(c, o, n, d, 0, ~0ull, nullptr, skew);
}

// Coalesced kernel with immediate-offset DMA in the fast region.
__global__ __launch_bounds__(64) void k_coal_imm(const ChunkDesc* __restrict__ c,
                                                 const uint32_t* __restrict__ o, uint32_t n,
                                                 uint32_t* __restrict__ d) {
  batch_coal_body<2, 2, true>(c, o, n, d);
}

// ---- 1. issue / latency ----------------------------------------------------
#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void k_dep_add(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t v0 = threadIdx.x, v1 = 3;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP64("v_add_u32 %0, %0, %1\n") : "+v"(v0) : "v"(v1));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = v0;
}

__global__ void k_ind_add(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3, one = 1;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP8(REP8("v_add_u32 %0, %0, %4\nv_add_u32 %1, %1, %4\nv_add_u32 %2, %2, %4\nv_add_u32 %3, %3, %4\n"))
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
                 : "v"(one));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = a + b + c + d;
}

__global__ void k_dep_alignbit(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t v0 = threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP64("v_alignbit_b32 %0, %0, %0, 7\n") : "+v"(v0));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = v0;
}

__global__ void k_dep_bitop3(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t v0 = threadIdx.x, v1 = 5, v2 = 9;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP64("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca\n") : "+v"(v0) : "v"(v1), "v"(v2));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = v0;
}

__global__ void k_dep_add3(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t v0 = threadIdx.x, v1 = 5, v2 = 9;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP64("v_add3_u32 %0, %0, %1, %2\n") : "+v"(v0) : "v"(v1), "v"(v2));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = v0;
}

// MD5-shaped dependent step: bitop3 -> add3 -> alignbit -> add (4-deep chain)
// plus one off-path add: 5 instructions / step.
__global__ void k_md5_step(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = 1, c = 2, d = 3, m = 7, t = 0, s;
  asm volatile("s_mov_b32 %0, 0x12345" : "=s"(s));
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP8(REP8(
        "v_add3_u32 %4, %0, %5, %6\n"
        "v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca\n"
        "v_add_u32 %0, %0, %4\n"
        "v_alignbit_b32 %0, %0, %0, 25\n"
        "v_add_u32 %0, %0, %1\n"))
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(t)
                 : "v"(m), "s"(s));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = a + b + c + d;
}

// MD5-shaped step with the a+x+k term precomputed elsewhere (4 instr/step).
__global__ void k_md5_step4(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = 1, c = 2, d = 3, mk = 7;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP8(REP8(
        "v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca\n"
        "v_add3_u32 %0, %0, %4, %1\n"
        "v_alignbit_b32 %0, %0, %0, 25\n"
        "v_add_u32 %0, %0, %1\n"))
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
                 : "v"(mk));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = a + b + c + d;
}

// VALU + ds_read_b128 interleaved (1 LDS read per 4 VALU, as the chain wave).
__global__ void k_mix_lds(uint64_t* out, uint32_t* sink, int iters) {
  __shared__ u32x4 lds[64];
  lds[threadIdx.x] = u32x4{threadIdx.x, 1, 2, 3};
  __syncthreads();
  uint32_t v0 = threadIdx.x, v1 = 3;
  u32x4 r;
  uint32_t addr = threadIdx.x * 16;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP64("ds_read_b128 %2, %3\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n")
                 : "+v"(v0), "+v"(v1), "=&v"(r) : "v"(addr));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  sink[threadIdx.x] = v0 + r.x;
}

typedef void (*ukern)(uint64_t*, uint32_t*, int);

static double run_issue(ukern k, int instr_per_iter, int iters, int threads) {
  uint64_t* d_out;
  uint32_t* d_sink;
  CK(hipMalloc(&d_out, 8));
  CK(hipMalloc(&d_sink, 4 * 1024));
  hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, d_out, d_sink, 10);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, d_out, d_sink, iters);
  CK(hipDeviceSynchronize());
  uint64_t cyc;
  CK(hipMemcpy(&cyc, d_out, 8, hipMemcpyDeviceToHost));
  CK(hipFree(d_out));
  CK(hipFree(d_sink));
  return (double)cyc / ((double)iters * instr_per_iter);
}

// ---- 1b. Stamped coalesced kernel (round 5) ---------------
// Diagnostic build of qsmd5_batch_coal_kernel: each wave stamps its start and
// end in shader cycles (s_memtime) and in the 100 MHz constant clock
// (s_memrealtime), plus where it ran (HW_ID: SIMD, CU, SE; XCC_ID), into a
// buffer of its own that no other code reads; no output is computed from
// them.  Splits a dispatch's time into the clock the waves ran at and the
// spread of wave start / end times, by waves per SIMD.  `extra_lds` bytes of
// dynamic LDS per workgroup cap the workgroups a CU can hold (160 KiB / LDS
// per workgroup), which decides how the dispatcher spreads them.
template <int kPrioEpoch>
__global__ __launch_bounds__(64) void k_coal_stamped(const ChunkDesc* __restrict__ chunks, uint32_t n,
                                                     uint32_t* __restrict__ digests, uint64_t* stamps) {
  extern __shared__ uint32_t pad_lds[];
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  batch_coal_body<2, 2, false, kPrioEpoch>(chunks, nullptr, n, digests);
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  // s_getreg_b32 HW_REG_HW_ID (4) and HW_REG_XCC_ID (20), all 32 bits
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  if (threadIdx.x == 0) {
    uint64_t* q = stamps + 6ull * blockIdx.x;
    q[0] = c0;
    q[1] = r0;
    q[2] = c1;
    q[3] = r1;
    q[4] = hw;
    q[5] = xcc | ((uint64_t)pad_lds[0] << 63 >> 63 << 32);  // keeps the dynamic LDS referenced
  }
}

static double pctl(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[(size_t)std::min<double>(v.size() - 1, q * (v.size() - 1) + 0.5)];
}

// One line per launch of n x L (stride L + pad): event ms, the waves' clock,
// start and end spread, the share of (first start .. last end) an average wave
// is alive, and the waves per SIMD / per CU with each class's mean lifetime.
static void run_stamps(uint32_t n, uint64_t L, int reps, uint64_t pad, uint32_t extra_lds, int prio = 0) {
  const uint64_t stride = L + pad;
  uint8_t* d_data;
  CK(hipMalloc(&d_data, stride * (uint64_t)n));
  const uint64_t segs = (L + 1023) / 1024, thr = segs * (uint64_t)n;
  hipLaunchKernelGGL(qsmd5_lcg_fill_kernel, dim3((thr + 255) / 256), dim3(256), 0, 0, d_data, stride, L,
                     12345u, n, segs);
  std::vector<ChunkDesc> h(n);
  for (uint32_t i = 0; i < n; ++i) h[i] = {d_data + stride * (uint64_t)i, L};
  ChunkDesc* d_desc;
  uint32_t* d_dig;
  uint64_t* d_st;
  const uint32_t waves = (n + 63) / 64;
  CK(hipMalloc(&d_desc, sizeof(ChunkDesc) * n));
  CK(hipMalloc(&d_dig, 16ull * n));
  CK(hipMalloc(&d_st, 48ull * waves));
  CK(hipMemcpy(d_desc, h.data(), sizeof(ChunkDesc) * n, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<uint64_t> st(6ull * waves);
  for (int rep = 0; rep <= reps; ++rep) {  // rep 0: warm-up, not reported
    CK(hipEventRecord(e0, 0));
    if (prio == 0)
      hipLaunchKernelGGL(k_coal_stamped<0>, dim3(waves), dim3(64), extra_lds, 0, d_desc, n, d_dig, d_st);
    else if (prio == 2)
      hipLaunchKernelGGL(k_coal_stamped<2>, dim3(waves), dim3(64), extra_lds, 0, d_desc, n, d_dig, d_st);
    else
      hipLaunchKernelGGL(k_coal_stamped<4>, dim3(waves), dim3(64), extra_lds, 0, d_desc, n, d_dig, d_st);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
    if (rep == 0) continue;
    uint64_t r_min = ~0ull, r_max = 0;
    for (uint32_t w = 0; w < waves; ++w) {
      r_min = std::min(r_min, st[6 * w + 1]);
      r_max = std::max(r_max, st[6 * w + 3]);
    }
    // where each wave ran: (xcc, se, cu) -> CU key; SIMD key adds simd
    auto cu_key = [&](uint32_t w) {
      const uint64_t hw = st[6 * w + 4], xcc = st[6 * w + 5] & 0xf;
      return (xcc << 16) | ((hw >> 8) & 0xff);  // CU_ID [11:8], SH_ID [12], SE_ID [15:13]
    };
    auto simd_key = [&](uint32_t w) { return (cu_key(w) << 2) | ((st[6 * w + 4] >> 4) & 3); };
    std::map<uint64_t, int> per_cu, per_simd;
    for (uint32_t w = 0; w < waves; ++w) {
      ++per_cu[cu_key(w)];
      ++per_simd[simd_key(w)];
    }
    std::vector<double> clk(waves), start_us(waves), end_us(waves);
    double alive = 0;
    std::map<int, std::pair<double, int>> life_by_simd_load;  // waves on the SIMD -> (sum life, count)
    for (uint32_t w = 0; w < waves; ++w) {
      const double dr = (double)(st[6 * w + 3] - st[6 * w + 1]);  // 10 ns ticks
      clk[w] = dr > 0 ? (double)(st[6 * w + 2] - st[6 * w + 0]) / (dr * 10.0) : 0.0;  // GHz
      start_us[w] = (st[6 * w + 1] - r_min) * 0.01;
      end_us[w] = (st[6 * w + 3] - r_min) * 0.01;
      alive += dr * 0.01;
      auto& e = life_by_simd_load[per_simd[simd_key(w)]];
      e.first += dr * 0.01;
      e.second += 1;
    }
    std::map<int, int> cu_hist, simd_hist;
    for (auto& kv : per_cu) ++cu_hist[kv.second];
    for (auto& kv : per_simd) ++simd_hist[kv.second];
    const double span_us = (r_max - r_min) * 0.01;
    printf("{\"mode\": \"stamps\", \"prio_epoch\": %d, \"chains\": %u, \"chunk_KiB\": %llu, \"extra_lds\": %u, \"rep\": %d, "
           "\"event_ms\": %.4f, \"GBps\": %.1f, \"span_us\": %.1f, \"clock_GHz_p10_p50_p90\": [%.3f, %.3f, %.3f], "
           "\"start_us_p50_max\": [%.1f, %.1f], \"end_us_min_p50_max\": [%.1f, %.1f, %.1f], "
           "\"alive_share\": %.4f, \"cus\": %zu, \"simds\": %zu",
           prio, n, (unsigned long long)(L >> 10), extra_lds, rep, ms, (double)n * L / (ms * 1e-3) / 1e9, span_us,
           pctl(clk, 0.1), pctl(clk, 0.5), pctl(clk, 0.9), pctl(start_us, 0.5), pctl(start_us, 1.0),
           pctl(end_us, 0.0), pctl(end_us, 0.5), pctl(end_us, 1.0), alive / (waves * span_us), per_cu.size(),
           per_simd.size());
    printf(", \"waves_per_cu_hist\": {");
    bool first = true;
    for (auto& kv : cu_hist) printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second), first = false;
    printf("}, \"waves_per_simd_hist\": {");
    first = true;
    for (auto& kv : simd_hist) printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second), first = false;
    printf("}, \"mean_life_us_by_waves_on_simd\": {");
    first = true;
    for (auto& kv : life_by_simd_load)
      printf("%s\"%d\": %.1f", first ? "" : ", ", kv.first, kv.second.first / kv.second.second), first = false;
    printf("}}\n");
    fflush(stdout);
  }
  // the last launch's digests of 64 chains spread over the batch, against the oracle
  int bad = 0;
  std::vector<uint8_t> buf(L);
  uint8_t got[16], want[16];
  for (uint32_t k = 0; k < 64; ++k) {
    const uint32_t i = (uint32_t)(((uint64_t)k * 2039u) % n);
    CK(hipMemcpy(buf.data(), d_data + stride * (uint64_t)i, L, hipMemcpyDeviceToHost));
    CK(hipMemcpy(got, d_dig + 4ull * i, 16, hipMemcpyDeviceToHost));
    oracle_md5(buf.data(), L, want);
    bad += memcmp(got, want, 16) != 0;
  }
  printf("{\"mode\": \"stamps_parity\", \"prio_epoch\": %d, \"chunk_KiB\": %llu, \"checked\": 64, \"bad\": %d}\n",
         prio, (unsigned long long)(L >> 10), bad);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  CK(hipFree(d_st));
  CK(hipFree(d_dig));
  CK(hipFree(d_desc));
  CK(hipFree(d_data));
}

// ---- 2. MD5 batch kernel -----------------------------------------------------
static bool g_host_pinned = false;  // "zc" mode: chunks in pinned host memory (zero-copy)
static uint32_t g_skew = kPcSkewBlocks;  // latency kernel start skew (blocks per lane)

// lane order: 0 chunk i; 1 lane l of wave w gets chunk l * (B/64) + w; 2 random
// permutation inside each group of 64; 3 random permutation of all chunks
static int g_interleave = 0;
static void run_md5(int B, uint64_t L, int reps, bool check, int which = 0, uint64_t pad = 0) {
  uint64_t stride = ((L + 255) & ~uint64_t(255)) + pad;
  uint8_t* d_data;
  if (g_host_pinned)
    CK(hipHostMalloc(&d_data, stride * (uint64_t)B, hipHostMallocDefault));
  else
    CK(hipMalloc(&d_data, stride * (uint64_t)B));
  const uint64_t segs = (L + 1023) / 1024;
  const uint64_t thr = segs * (uint64_t)B;
  hipLaunchKernelGGL(qsmd5_lcg_fill_kernel, dim3((thr + 255) / 256), dim3(256), 0, 0, d_data,
                     stride, L, 12345u, (uint32_t)B, segs);
  std::vector<ChunkDesc> h(B);
  for (int i = 0; i < B; ++i) {
    h[i].ptr = d_data + stride * (uint64_t)i;
    h[i].len = L;
  }
  if (g_interleave) {
    std::vector<ChunkDesc> p(h);
    uint64_t x = 88172645463325252ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    if (g_interleave == 1 && B % 64 == 0)
      for (int i = 0; i < B; ++i) p[i] = h[(uint64_t)(i % 64) * (B / 64) + i / 64];
    const int grp = g_interleave == 2 ? 64 : B;
    if (g_interleave >= 2)
      for (int g0 = 0; g0 < B; g0 += grp)
        for (int i = std::min(B, g0 + grp) - 1; i > g0; --i) std::swap(p[i], p[g0 + rnd() % (i - g0 + 1)]);
    h = p;
  }
  ChunkDesc* d_desc;
  uint32_t* d_dig;
  CK(hipMalloc(&d_desc, sizeof(ChunkDesc) * B));
  CK(hipMalloc(&d_dig, 16 * (size_t)B));
  CK(hipMemcpy(d_desc, h.data(), sizeof(ChunkDesc) * B, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = (B + 63) / 64;
  auto launch = [&]() {
    if (which == 0)
      hipLaunchKernelGGL(qsmd5_batch_kernel, dim3(grid), dim3(64), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig);
    else if (which == 1)  // what the runtime launches at 64 chains per workgroup
      hipLaunchKernelGGL(qsmd5_batch_pc64_kernel, dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 19)  // the same kernel with the lanes per workgroup a runtime argument
      hipLaunchKernelGGL(qsmd5_batch_pc_kernel, dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew, 64u);
    else if (which == 2)
      hipLaunchKernelGGL(qsmd5_batch_coal_kernel, dim3(grid), dim3(64), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig);
    else if (which == 3)
      hipLaunchKernelGGL(k_pc_depth<2>, dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 5)
      hipLaunchKernelGGL(k_pc_half2, dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 6)
      hipLaunchKernelGGL(k_coal_imm, dim3(grid), dim3(64), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig);
    else if (which == 7)
      hipLaunchKernelGGL(k_pc_half5, dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, 0u);
    else if (which == 20)
      hipLaunchKernelGGL((k_pc_pace<0,0,1>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 21)
      hipLaunchKernelGGL((k_pc_pace<8,0,1>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 22)
      hipLaunchKernelGGL((k_pc_pace<10,0,1>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 23)
      hipLaunchKernelGGL((k_pc_pace<8,0,2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 24)
      hipLaunchKernelGGL((k_pc_pace<16,0,2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 25)
      hipLaunchKernelGGL((k_pc_pace<24,0,2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 26)
      hipLaunchKernelGGL((k_pc_pace<32,0,2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 30)
      hipLaunchKernelGGL(k_pc_lead<8>, dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 31)
      hipLaunchKernelGGL((k_pc_lead<8, 24>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 32)
      hipLaunchKernelGGL((k_pc_lead<4, 16>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 35)
      hipLaunchKernelGGL((k_pc_lead<8, 0, 4, 2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 36)
      hipLaunchKernelGGL((k_pc_lead<8, 0, 12, 2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 37)
      hipLaunchKernelGGL((k_pc_lead<8, 0, 8, 3>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 38)
      hipLaunchKernelGGL((k_pc_lead<8, 0, 16, 3>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 39)
      hipLaunchKernelGGL((k_pc_lead<8, 0, 0, 2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 40)
      hipLaunchKernelGGL((k_pc2_pace<0, 1>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 41)
      hipLaunchKernelGGL((k_pc2_pace<0, 2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 42)
      hipLaunchKernelGGL((k_pc2_pace<4, 2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 43)
      hipLaunchKernelGGL((k_pc2_pace<8, 2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 44)
      hipLaunchKernelGGL((k_pc2_pace<2, 2>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr,
                         (uint32_t)B, d_dig, g_skew);
    else if (which == 34)
      hipLaunchKernelGGL((k_pc_lead<0>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 33)
      hipLaunchKernelGGL((k_pc_lead<8, 32>), dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 50)
      hipLaunchKernelGGL(k_pc_probe<1>, dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 51)
      hipLaunchKernelGGL(k_pc_probe<2>, dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else if (which == 52)
      hipLaunchKernelGGL(k_pc_probe<3>, dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
    else
      hipLaunchKernelGGL(k_pc_depth<3>, dim3(grid), dim3(128), 0, 0, d_desc, nullptr, (uint32_t)B,
                         d_dig, g_skew);
  };
  launch();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<float> ms(reps);
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[r], e0, e1));
  }
  float best = ms[0], med;
  for (float m : ms) best = m < best ? m : best;
  std::vector<float> s = ms;
  std::sort(s.begin(), s.end());
  med = s[s.size() / 2];
  double gib = (double)L * B / (1u << 30);
  if (pad) printf("(stride pad %llu) ", (unsigned long long)pad);
  if ((which == 1 || which == 3 || which == 4 || which == 5) && g_skew)
    printf("(skew %u) ", g_skew);
  if (g_host_pinned) printf("[pinned host, zero-copy] ");
  printf("md5[%s] B=%d L=%llu: median %.3f ms best %.3f ms -> %.2f GiB/s total, r1=%.4f GiB/s/chain, "
         "%.1f cycles/block @2.4GHz\n",
         which == 0 ? "v1" : which == 1 ? "pc" : which == 2 ? "coal" : which == 3 ? "pc-d2" : which == 5 ? "pc-h2" : which == 6 ? "coal-imm" : which == 19 ? "pc (runtime lanes)" : which == 20 ? "pc-r1 (depth 1, no pause)" : which == 21 ? "pace8" : which == 22 ? "pace10" : which == 23 ? "d2-pace8" : which == 24 ? "d2-pace16" : which == 25 ? "d2-pace24" : which == 26 ? "d2-pace32" : which == 30 ? "lead8" : which == 31 ? "lead8+24" : which == 32 ? "lead4+16" : which == 33 ? "lead8+32" : which == 34 ? "lead0 (no graded wait)" : which == 40 ? "pc2 d1 (64u fixed)" : which == 41 ? "pc2 d2" : which == 42 ? "pc2 d2 pace4" : which == 43 ? "pc2 d2 pace8" : which == 44 ? "pc2 d2 pace2" : which == 35 ? "lead8 pace4" : which == 36 ? "lead8 pace12" : which == 37 ? "lead8 pace8 depth3" : which == 38 ? "lead8 pace16 depth3" : which == 39 ? "lead8 no pause" : which == 50 ? "probe: producer writes no ring" : which == 51 ? "probe: producer loads nothing" : which == 52 ? "probe: producer neither loads nor writes" : "pc-d3", B, (unsigned long long)L, med, best, gib / (med / 1e3), (double)L / (1u << 30) / (med / 1e3),
         (med / 1e3) * 2.4e9 / (double)(L / 64));
  if (check) {
    std::vector<uint32_t> dig(4 * (size_t)B);
    CK(hipMemcpy(dig.data(), d_dig, 16 * (size_t)B, hipMemcpyDeviceToHost));
    std::vector<uint8_t> host(L);
    int bad = 0;
    int ncheck = B < 16 ? B : 16;
    for (int i = 0; i < ncheck; ++i) {
      int ci = (i * 7919) % B;
      CK(hipMemcpy(host.data(), d_data + stride * (uint64_t)ci, L, hipMemcpyDeviceToHost));
      std::vector<uint8_t> ref(L);
      oracle_lcg_fill(ref.data(), L, 12345u + ci);
      if (memcmp(ref.data(), host.data(), L) != 0) {
        printf("  generator mismatch chunk %d\n", ci);
        ++bad;
      }
      uint8_t od[16];
      oracle_md5(host.data(), L, od);
      if (memcmp(od, &dig[4 * (size_t)ci], 16) != 0) {
        char hx[33], hg[33];
        oracle_md5_hex(od, hx);
        oracle_md5_hex((const uint8_t*)&dig[4 * (size_t)ci], hg);
        printf("  DIGEST MISMATCH chunk %d: oracle %s gpu %s\n", ci, hx, hg);
        ++bad;
      }
    }
    printf("  check %d chunks: %s\n", ncheck, bad ? "FAIL" : "ok");
  }
  if (g_host_pinned) CK(hipHostFree(d_data)); else CK(hipFree(d_data));
  CK(hipFree(d_desc));
  CK(hipFree(d_dig));
}

// Edge lengths on unaligned offsets, 1 launch each, all checked.
static int run_edges(int which) {
  const uint64_t lens[] = {0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 1000, 4096, 8191, 100003};
  const int nl = sizeof(lens) / sizeof(lens[0]);
  int bad = 0;
  uint8_t* d;
  CK(hipMalloc(&d, 1 << 20));
  std::vector<uint8_t> h(1 << 20);
  oracle_lcg_fill(h.data(), h.size(), 777u);
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  std::vector<ChunkDesc> desc;
  std::vector<std::pair<uint64_t, uint64_t>> ref;
  for (int off = 0; off < 8; ++off)
    for (int i = 0; i < nl; ++i) {
      uint64_t o = which >= 2 ? off * 4096 + 16 * off : off * 4099 + off;
      desc.push_back({d + o, lens[i]});
      ref.push_back({o, lens[i]});
    }
  int n = desc.size();
  ChunkDesc* dd;
  uint32_t* dg;
  CK(hipMalloc(&dd, sizeof(ChunkDesc) * n));
  CK(hipMalloc(&dg, 16 * n));
  CK(hipMemcpy(dd, desc.data(), sizeof(ChunkDesc) * n, hipMemcpyHostToDevice));
  CK(hipMemset(dg, 0, 16 * n));
  if (which == 0)
    hipLaunchKernelGGL(qsmd5_batch_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, dd, nullptr,
                       (uint32_t)n, dg);
  else if (which == 1)
    hipLaunchKernelGGL(qsmd5_batch_pc64_kernel, dim3((n + 63) / 64), dim3(128), 0, 0, dd, nullptr,
                       (uint32_t)n, dg, g_skew);
  else if (which == 19)
    hipLaunchKernelGGL(qsmd5_batch_pc_kernel, dim3((n + 63) / 64), dim3(128), 0, 0, dd, nullptr,
                       (uint32_t)n, dg, g_skew, 64u);
  else if (which == 2)
    hipLaunchKernelGGL(qsmd5_batch_coal_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, dd, nullptr,
                       (uint32_t)n, dg);
  else if (which == 3)
    hipLaunchKernelGGL(k_pc_depth<2>, dim3((n + 63) / 64), dim3(128), 0, 0, dd, nullptr,
                       (uint32_t)n, dg, g_skew);
  else if (which == 5)
    hipLaunchKernelGGL(k_pc_half2, dim3((n + 63) / 64), dim3(128), 0, 0, dd, nullptr,
                       (uint32_t)n, dg, g_skew);
  else if (which == 6)
    hipLaunchKernelGGL(k_coal_imm, dim3((n + 63) / 64), dim3(64), 0, 0, dd, nullptr, (uint32_t)n,
                       dg);
  else if (which == 7)
    hipLaunchKernelGGL(k_pc_half5, dim3((n + 63) / 64), dim3(128), 0, 0, dd, nullptr, (uint32_t)n,
                       dg, 0u);
  else if (which == 21)
    hipLaunchKernelGGL((k_pc_pace<8, 0, 1>), dim3((n + 63) / 64), dim3(128), 0, 0, dd, nullptr,
                       (uint32_t)n, dg, g_skew);
  else if (which == 24)
    hipLaunchKernelGGL((k_pc_pace<16, 0, 2>), dim3((n + 63) / 64), dim3(128), 0, 0, dd, nullptr,
                       (uint32_t)n, dg, g_skew);
  else if (which >= 30 && which <= 33) {
    auto k = which == 30 ? k_pc_lead<8> : which == 31 ? k_pc_lead<8, 24>
           : which == 32 ? k_pc_lead<4, 16> : k_pc_lead<8, 32>;
    hipLaunchKernelGGL(k, dim3((n + 63) / 64), dim3(128), 0, 0, dd, nullptr, (uint32_t)n, dg, g_skew);
  } else
    hipLaunchKernelGGL(k_pc_depth<3>, dim3((n + 63) / 64), dim3(128), 0, 0, dd, nullptr,
                       (uint32_t)n, dg, g_skew);
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> got(16 * n);
  CK(hipMemcpy(got.data(), dg, 16 * n, hipMemcpyDeviceToHost));
  for (int i = 0; i < n; ++i) {
    uint8_t od[16];
    oracle_md5(h.data() + ref[i].first, ref[i].second, od);
    if (memcmp(od, &got[16 * i], 16)) {
      printf("  edge mismatch off=%llu len=%llu\n", (unsigned long long)ref[i].first,
             (unsigned long long)ref[i].second);
      ++bad;
    }
  }
  printf("edges[%d]: %d cases, %d bad\n", which, n, bad);
  CK(hipFree(d));
  CK(hipFree(dd));
  CK(hipFree(dg));
  return bad;
}

// Coalesced streaming read (16 B/lane, grid-stride): the FETCH_SIZE calibration
// reference of MI355X_MICROARCH.md §HBM and the achievable HBM read rate here.
__global__ __launch_bounds__(256) void k_stream_read(const u32x4* __restrict__ p, uint64_t n16,
                                                     uint32_t* sink) {
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16;
       i += (uint64_t)gridDim.x * 256) {
    u32x4 v = __builtin_nontemporal_load(p + i);
    acc ^= v;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

// Per-lane sequential streams (the MD5 access pattern with no compute): lane l
// reads chunk l's bytes 64 B at a time, 8 blocks per iteration in flight.
template <bool kNT>
__global__ __launch_bounds__(64) void k_lane_stream(const uint8_t* __restrict__ base,
                                                    uint64_t stride, uint32_t nblk,
                                                    uint32_t* sink) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  const u32x4* p = reinterpret_cast<const u32x4*>(base + stride * t);
  u32x4 acc = {0, 0, 0, 0};
  for (uint32_t j = 0; j < nblk; j += 8) {
    u32x4 v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = kNT ? __builtin_nontemporal_load(p + 4 * j + k) : p[4 * j + k];
#pragma unroll
    for (int k = 0; k < 32; ++k) acc ^= v[k];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = t;
}

static void run_lane_stream(uint32_t B, uint64_t L, uint64_t pad, bool nt) {
  uint64_t stride = L + pad;
  uint8_t* d;
  uint32_t* sink;
  CK(hipMalloc(&d, stride * B));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(d, 3, stride * B));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 4; ++r) {
    CK(hipEventRecord(e0, 0));
    if (nt)
      hipLaunchKernelGGL(k_lane_stream<true>, dim3(B / 64), dim3(64), 0, 0, d, stride,
                         (uint32_t)(L / 64), sink);
    else
      hipLaunchKernelGGL(k_lane_stream<false>, dim3(B / 64), dim3(64), 0, 0, d, stride,
                         (uint32_t)(L / 64), sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r) best = ms < best ? ms : best;
  }
  printf("lane_stream%s B=%u L=%llu pad=%llu: %.3f ms -> %.1f GB/s\n", nt ? "[nt]" : "", B,
         (unsigned long long)L, (unsigned long long)pad, best, (double)L * B / (best * 1e-3) / 1e9);
  CK(hipFree(d));
  CK(hipFree(sink));
}

static void run_stream_read(uint64_t bytes, int reps) {
  u32x4* d;
  uint32_t* sink;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(d, 1, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_stream_read, dim3(256 * 8), dim3(256), 0, 0, d, bytes / 16, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  printf("stream_read %llu bytes: best %.3f ms -> %.1f GB/s\n", (unsigned long long)bytes, best,
         bytes / (best * 1e-3) / 1e9);
  CK(hipFree(d));
  CK(hipFree(sink));
}

// Raw H2D bandwidth from pinned host memory: the ceiling for host-resident
// batches (BASELINE config 3).  `total` bytes in `piece`-sized copies
// alternating over `nstreams` streams.
static void run_h2d(size_t total, size_t piece, int nstreams) {
  void* h = nullptr;
  void* d = nullptr;
  CK(hipHostMalloc(&h, total, hipHostMallocDefault));
  CK(hipMalloc(&d, total));
  memset(h, 1, total);
  hipStream_t st[4];
  for (int i = 0; i < nstreams; ++i) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
  double best = 1e30;
  for (int r = 0; r < 3; ++r) {
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    int k = 0;
    for (size_t o = 0; o < total; o += piece, ++k)
      CK(hipMemcpyAsync((char*)d + o, (char*)h + o, std::min(piece, total - o),
                        hipMemcpyHostToDevice, st[k % nstreams]));
    CK(hipDeviceSynchronize());
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, s);
  }
  printf("h2d total=%.1f GiB piece=%.0f MiB streams=%d: %.3f s -> %.2f GiB/s (%.1f GB/s)\n",
         total / 1073741824.0, piece / 1048576.0, nstreams, best, total / 1073741824.0 / best,
         total / 1e9 / best);
  for (int i = 0; i < nstreams; ++i) CK(hipStreamDestroy(st[i]));
  CK(hipFree(d));
  CK(hipHostFree(h));
}

// Column copies: `rows` chunks of `len` bytes at host stride `len`, copied as
// columns of `width` bytes per chunk with one hipMemcpy2DAsync per column
// (device pitch = len + skew) -- the H2D pattern of a column-pipelined batch.
static void run_h2d_2d(int rows, size_t len, size_t width, int nstreams) {
  const size_t skew = 4352;
  const size_t total = (size_t)rows * len;
  void* h = nullptr;
  void* d = nullptr;
  CK(hipHostMalloc(&h, total, hipHostMallocDefault));
  CK(hipMalloc(&d, (size_t)rows * (len + skew)));
  memset(h, 1, total);
  hipStream_t st[4];
  for (int i = 0; i < nstreams; ++i) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
  double best = 1e30;
  for (int r = 0; r < 3; ++r) {
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    int k = 0;
    for (size_t o = 0; o < len; o += width, ++k)
      CK(hipMemcpy2DAsync((char*)d + o, len + skew, (char*)h + o, len, std::min(width, len - o),
                          rows, hipMemcpyHostToDevice, st[k % nstreams]));
    CK(hipDeviceSynchronize());
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, s);
  }
  // spot-check placement
  std::vector<uint8_t> probe(16);
  CK(hipMemcpy(probe.data(), (char*)d + (size_t)(rows - 1) * (len + skew) + len - 16, 16,
               hipMemcpyDeviceToHost));
  printf("h2d-2d rows=%d len=%.1f MiB width=%.2f MiB streams=%d: %.3f s -> %.2f GiB/s (%.1f GB/s)%s\n",
         rows, len / 1048576.0, width / 1048576.0, nstreams, best, total / 1073741824.0 / best,
         total / 1e9 / best, probe[15] == 1 ? "" : "  PLACEMENT WRONG");
  for (int i = 0; i < nstreams; ++i) CK(hipStreamDestroy(st[i]));
  CK(hipFree(d));
  CK(hipHostFree(h));
}


#define QS_GP(p) ((const __attribute__((address_space(1))) void*)(uintptr_t)(p))
#define QS_LP(p) ((__attribute__((address_space(3))) void*)(uintptr_t)(uint32_t)(uintptr_t)(p))
// ---- 3. throughput-kernel probes ---------------------------------------------
// Copy of batch_coal_body<2,2> with a probe mode: 0 = as shipped, 1 = memory
// only (compress replaced by an XOR fold), 2 = compute only (no LDS-DMA, the
// tile buffers hold garbage).  Lane 0 stamps s_memtime / s_memrealtime at entry
// and exit: clock = d(memtime) / d(realtime) x 100 MHz.
template <int kMode>
__global__ __launch_bounds__(64) void k_coal_probe(const ChunkDesc* __restrict__ chunks, uint32_t n,
                                                   uint32_t* __restrict__ digests,
                                                   uint64_t* __restrict__ stamps) {
  constexpr int kTB = 2, kBufs = 2, kS = 8, kCPI = 8;
  __shared__ u32x4 tile_buf[kBufs][64][kS];
  const uint64_t m0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t lane = threadIdx.x;
  const uint32_t t = blockIdx.x * 64u + lane;
  ChunkDesc cd = {nullptr, 0};
  if (t < n) cd = chunks[t];
  const uint32_t nblk = (uint32_t)(cd.len >> 6);
  const uint32_t ntiles = rfl_u32((wave_max_u32(nblk) + (kTB - 1)) / kTB);
  auto swz = [](uint32_t c) -> uint32_t { return (c >> 1) & 7u; };
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
    piece[i] = slot ^ swz((uint32_t)c);
  }
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(chunks);
  auto issue_tile = [&](uint32_t b, uint32_t tl) {
    if (kMode == 2) return;
#pragma unroll
    for (int i = 0; i < kS; ++i) {
      const uint32_t blk = min(tl * (uint32_t)kTB + (piece[i] >> 2), src_nblk[i] - 1u);
      const uint8_t* g = src_nblk[i] ? src[i] + (uint64_t)blk * 64u + (piece[i] & 3u) * 16u : dummy;
      __builtin_amdgcn_global_load_lds(QS_GP(g), QS_LP(&tile_buf[b][i * kCPI][0]), 16, 0, 0);
    }
  };
  const uint32_t rswz = swz(lane);
  uint32_t st[4] = {kInit0, kInit1, kInit2, kInit3};
  issue_tile(0, 0);
  for (uint32_t tl = 0; tl < ntiles; ++tl) {
    const uint32_t b = tl % kBufs;
    if (tl + 1 < ntiles) {
      issue_tile((tl + 1) % kBufs, tl + 1);
      if (kMode != 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      if (kMode != 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int h = 0; h < kTB; ++h) {
      u32x4 q0 = tile_buf[b][lane][(4 * h + 0) ^ rswz];
      u32x4 q1 = tile_buf[b][lane][(4 * h + 1) ^ rswz];
      u32x4 q2 = tile_buf[b][lane][(4 * h + 2) ^ rswz];
      u32x4 q3 = tile_buf[b][lane][(4 * h + 3) ^ rswz];
      if (tl * (uint32_t)kTB + h < nblk) {
        if (kMode == 1) {
          st[0] ^= q0.x ^ q1.y ^ q2.z ^ q3.w;
          st[1] += q0.y ^ q1.z ^ q2.w ^ q3.x;
          st[2] ^= q0.z + q1.w + q2.x + q3.y;
          st[3] += q0.w + q1.x + q2.y + q3.z;
        } else {
          uint32_t w[16];
          unpack4(w, 0, q0);
          unpack4(w, 1, q1);
          unpack4(w, 2, q2);
          unpack4(w, 3, q3);
          md5_compress(st, w);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (t < n) {
    u32x4 o = {st[0], st[1], st[2], st[3]};
    *reinterpret_cast<u32x4*>(digests + 4u * (uint64_t)t) = o;
  }
  const uint64_t m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    stamps[4 * blockIdx.x + 0] = m0;
    stamps[4 * blockIdx.x + 1] = r0;
    stamps[4 * blockIdx.x + 2] = m1;
    stamps[4 * blockIdx.x + 3] = r1;
  }
}

template <int kMode>
static void run_coal_probe(int B, uint64_t L, uint64_t pad, int reps) {
  uint64_t stride = ((L + 255) & ~uint64_t(255)) + pad;
  uint8_t* d_data;
  CK(hipMalloc(&d_data, stride * (uint64_t)B));
  const uint64_t segs = (L + 1023) / 1024;
  const uint64_t thr = segs * (uint64_t)B;
  hipLaunchKernelGGL(qsmd5_lcg_fill_kernel, dim3((thr + 255) / 256), dim3(256), 0, 0, d_data,
                     stride, L, 12345u, (uint32_t)B, segs);
  std::vector<ChunkDesc> h(B);
  for (int i = 0; i < B; ++i) h[i] = {d_data + stride * (uint64_t)i, L};
  ChunkDesc* d_desc;
  uint32_t* d_dig;
  uint64_t* d_st;
  const int grid = (B + 63) / 64;
  CK(hipMalloc(&d_desc, sizeof(ChunkDesc) * B));
  CK(hipMalloc(&d_dig, 16 * (size_t)B));
  CK(hipMalloc(&d_st, 32 * (size_t)grid));
  CK(hipMemcpy(d_desc, h.data(), sizeof(ChunkDesc) * B, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms(reps);
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_coal_probe<kMode>, dim3(grid), dim3(64), 0, 0, d_desc, (uint32_t)B, d_dig, d_st);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[r], e0, e1));
  }
  std::vector<uint64_t> st(4 * (size_t)grid);
  CK(hipMemcpy(st.data(), d_st, 32 * (size_t)grid, hipMemcpyDeviceToHost));
  std::vector<double> clk, dur;
  for (int g = 0; g < grid; ++g) {
    double dm = (double)(st[4 * g + 2] - st[4 * g]), dr = (double)(st[4 * g + 3] - st[4 * g + 1]);
    if (dr > 0) clk.push_back(dm / dr * 100.0), dur.push_back(dr / 100.0);
  }
  std::sort(clk.begin(), clk.end());
  std::sort(dur.begin(), dur.end());
  std::vector<float> s = ms;
  std::sort(s.begin(), s.end());
  const double med = s[s.size() / 2];
  printf("probe[%s] B=%d L=%llu pad=%llu: median %.3f ms best %.3f ms -> %.1f GB/s; wave clock median %.0f MHz "
         "(p10 %.0f p90 %.0f); wave time median %.1f us max %.1f us\n",
         kMode == 0 ? "full" : kMode == 1 ? "mem-only" : "compute-only", B, (unsigned long long)L,
         (unsigned long long)pad, med, s[0], (double)L * B / (med * 1e-3) / 1e9, clk[clk.size() / 2],
         clk[clk.size() / 10], clk[clk.size() * 9 / 10], dur[dur.size() / 2], dur.back());
  CK(hipFree(d_data));
  CK(hipFree(d_desc));
  CK(hipFree(d_dig));
  CK(hipFree(d_st));
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "all";
  if (!strcmp(mode, "calib")) {
    // one launch each, for rocprofv3 --pmc FETCH_SIZE
    run_stream_read(4ull << 30, 2);
    run_md5(512, 10485760, 1, false, 1);
    run_md5(131072, 65536, 1, false, 0);
    return 0;
  }
  if (!strcmp(mode, "h2d")) {
    const size_t G = 1ull << 30;
    for (int ns : {1, 2, 4})
      for (size_t piece : {G / 16, 1 * G, 4 * G}) run_h2d(16 * G, piece, ns);
    run_h2d(40 * G, 4 * G, 2);
    for (size_t w : {256ull << 10, 1ull << 20, 10ull << 19})
      for (int ns : {1, 2}) run_h2d_2d(4096, 10 << 20, w, ns);
    // per-chunk 10 MiB copies, as the row-sliced pipeline issues them
    for (int ns : {1, 2}) run_h2d(40 * G, 10ull << 20, ns);
    for (int ns : {1, 2}) run_h2d(4 * G, 1ull << 20, ns);
    return 0;
  }
  if (!strcmp(mode, "zc")) {
    g_host_pinned = true;
    run_md5(64, 10485760, 2, true, 1);
    run_md5(512, 10485760, 2, true, 1);
    run_md5(512, 10485760, 2, true, 0);
    run_md5(2048, 10485760, 2, true, 1);
    run_md5(4096, 10485760, 2, true, 1);
    run_md5(4096, 10485760, 2, true, 0);
    return 0;
  }
  if (!strcmp(mode, "coal")) {
    int bad = run_edges(2);
    for (int w : {0, 2}) {
      run_md5(131072, 65536, 5, true, w, 0);
      run_md5(131072, 65536, 5, true, w, 4352);
      run_md5(262144, 32768, 5, true, w, 4352);
      run_md5(65536, 262144, 3, true, w, 4352);
      run_md5(32768, 1 << 20, 3, true, w, 4352);
    }
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "mem")) {
    run_stream_read(8ull << 30, 5);
    for (int nt = 0; nt < 2; ++nt) {
      run_lane_stream(131072, 65536, 0, nt);
      run_lane_stream(131072, 65536, 4352, nt);
      run_lane_stream(32768, 262144, 4352, nt);
      run_lane_stream(8192, 1 << 20, 4352, nt);
      run_lane_stream(512, 10485760, 0, nt);
    }
    return 0;
  }
  if (!strcmp(mode, "ab")) {
    int bad = run_edges(0) + run_edges(1);
    for (int r = 0; r < 3; ++r) {
      run_md5(512, 10485760, 3, r == 0, 0);
      run_md5(512, 10485760, 3, r == 0, 1);
    }
    run_md5(600, 1 << 20, 3, true, 1);
    run_md5(4096, 1 << 20, 3, true, 1);
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "issue")) {
    const int iters = 20000;
    printf("  dep v_add_u32      %.2f\n", run_issue(k_dep_add, 64, iters, 64));
    printf("  dep v_add_u32 32 lanes  %.2f\n", run_issue(k_dep_add, 64, iters, 32));
    printf("  dep v_add_u32 16 lanes  %.2f\n", run_issue(k_dep_add, 64, iters, 16));
    printf("  dep v_add_u32 1 lane    %.2f\n", run_issue(k_dep_add, 64, iters, 1));
    printf("  ind v_add_u32 x4 32 lanes %.2f\n", run_issue(k_ind_add, 256, iters, 32));
    printf("  md5 step4 64 lanes %.2f per instr\n", run_issue(k_md5_step4, 256, iters, 64));
    printf("  md5 step4 32 lanes %.2f per instr\n", run_issue(k_md5_step4, 256, iters, 32));
    printf("  md5 step4 1 lane   %.2f per instr\n", run_issue(k_md5_step4, 256, iters, 1));
    printf("  4 v_add + ds_read  %.2f per group\n", run_issue(k_mix_lds, 64, iters, 64));
    return 0;
  }
  if (!strcmp(mode, "stride")) {
    for (uint64_t mib : {10ull, 16ull, 32ull, 64ull}) {
      run_md5(512, mib << 20, 2, false, 1, 0);
      run_md5(512, mib << 20, 2, false, 1, 4096);
      run_md5(512, mib << 20, 2, false, 1, 65536 + 256);
    }
    run_md5(512, 32ull << 20, 2, false, 0, 0);
    run_md5(512, 32ull << 20, 2, false, 0, 4096);
    return 0;
  }
  if (!strcmp(mode, "span")) {
    // same footprint, different lane->chunk maps: per-wave address span vs stride
    static const char* names[] = {"in order", "interleaved", "shuffled in 64s", "shuffled all"};
    for (uint64_t pad : {(uint64_t)0, (uint64_t)4352})
      for (int m = 0; m < 4; ++m) {
        g_interleave = m;
        printf("(%s, pad %llu) ", names[m], (unsigned long long)pad);
        run_md5(512, 10ull << 20, 2, false, 1, pad);
      }
    for (uint64_t L : {32ull << 20, 64ull << 20})
      for (uint64_t pad : {(uint64_t)0, (uint64_t)4352})
        for (int m : {0, 2, 3}) {
          g_interleave = m;
          printf("(%s, pad %llu) ", names[m], (unsigned long long)pad);
          run_md5(512, L, 1, false, 1, pad);
        }
    g_interleave = 0;
    return 0;
  }
  if (!strcmp(mode, "fp_pmc")) {
    // one launch each under rocprofv3 --pmc: dense 10 MiB, strided 10 MiB, strided 64 MiB
    run_md5(512, 10ull << 20, 1, false, 1, 0);
    run_md5(512, 10ull << 20, 1, false, 1, (54ull << 20) + 4096);
    run_md5(512, 64ull << 20, 1, false, 1, 4096);
    return 0;
  }
  if (!strcmp(mode, "footprint")) {
    // 10 MiB chunks dense vs spread at a 32/64 MiB + 4 KiB stride; 10 000 dense
    // chunks (98 GiB footprint).  A two-producer-wave variant of the latency
    // kernel was measured here and dropped (profiles/r01_ubench_footprint_producers.log).
    for (int rep = 0; rep < 2; ++rep) {
      run_md5(512, 10ull << 20, 2, rep == 0, 1, 0);
      run_md5(512, 10ull << 20, 2, rep == 0, 1, (54ull << 20) + 4096);
      run_md5(512, 10ull << 20, 2, false, 1, (22ull << 20) + 4096);
      run_md5(512, 64ull << 20, 2, false, 1, 4096);
    }
    run_md5(10000, 10ull << 20, 2, true, 1, 0);
    return 0;
  }
  if (!strcmp(mode, "imm")) {
    // coalesced kernel: per-tile pointer bumps (shipped) vs immediate-offset DMA
    int bad = run_edges(2) + run_edges(6);
    for (int rep = 0; rep < 2; ++rep)
      for (int w : {2, 6}) {
        run_md5(131072, 65536, 10, rep == 0, w, 4352);
        run_md5(131072, 262144, 6, rep == 0, w, 4352);
      }
    run_md5(100000, 65536 + 17 * 64, 3, true, 6, 4352);
    run_md5(131072, 65536 + 64 * 3, 3, true, 6, 4352);
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "tlb")) {
    // 2 MiB-page aliasing test: pads that move each chunk to another 2 MiB page index
    for (uint64_t mib : {32ull, 64ull})
      for (uint64_t pad : {0ull, 4096ull, 1ull << 20, 2ull << 20, (2ull << 20) + 4096, 6ull << 20})
        run_md5(512, mib << 20, 2, false, 1, pad);
    run_md5(512, 10ull << 20, 2, false, 1, 0);
    return 0;
  }
  if (!strcmp(mode, "skew")) {
    // latency kernel on long strided chunks: start skew x producer prefetch depth
    int bad = 0;
    for (int w : {1, 3, 4}) {
      bad += run_edges(w);
      for (uint64_t mib : {10ull, 32ull, 64ull}) run_md5(512, mib << 20, 2, mib == 64, w, 0);
      for (uint64_t mib : {32ull, 64ull}) run_md5(512, mib << 20, 2, false, w, 4096);
      run_md5(512, 64ull << 20, 2, false, w, 65536 + 256);
      run_md5(100, (32ull << 20) + 64 * 7 + 13, 2, true, w, 0);  // ragged tail, partial wave
    }
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "ptrace")) {
    // ptrace B MiB pad: cycles per 64-B block and the SCLK of the latency
    // kernel's chain waves, per 16384 blocks (1 MiB) of progress: does a long
    // chain slow down with its block index, with time, or from the start?
    const int B = argc > 2 ? atoi(argv[2]) : 512;
    const uint64_t L = (argc > 3 ? strtoull(argv[3], nullptr, 10) : 64) << 20;
    const uint64_t pad = argc > 4 ? strtoull(argv[4], nullptr, 10) : 4352;
    const uint32_t lanes = argc > 5 ? (uint32_t)atoi(argv[5]) : 64u;
    const uint64_t stride = L + pad;
    uint8_t* d_data;
    CK(hipMalloc(&d_data, stride * (uint64_t)B));
    const uint64_t segs = (L + 1023) / 1024;
    hipLaunchKernelGGL(qsmd5_lcg_fill_kernel, dim3((segs * B + 255) / 256), dim3(256), 0, 0, d_data,
                       stride, L, 12345u, (uint32_t)B, segs);
    std::vector<ChunkDesc> h(B);
    for (int i = 0; i < B; ++i) h[i] = {d_data + (uint64_t)i * stride, L};
    ChunkDesc* d_c;
    uint32_t* d_dig;
    uint64_t* d_tr;
    const int groups = (B + (int)lanes - 1) / (int)lanes;
    CK(hipMalloc(&d_c, sizeof(ChunkDesc) * B));
    CK(hipMalloc(&d_dig, 16 * B));
    CK(hipMalloc(&d_tr, 8 * 1024 * groups));
    CK(hipMemset(d_tr, 0, 8 * 1024 * groups));
    CK(hipMemcpy(d_c, h.data(), sizeof(ChunkDesc) * B, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_pc_trace, dim3(groups), dim3(128), 0, 0, d_c, nullptr, (uint32_t)B, d_dig,
                       g_skew, d_tr, lanes);
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<uint64_t> tr(1024 * groups);
    CK(hipMemcpy(tr.data(), d_tr, 8 * tr.size(), hipMemcpyDeviceToHost));
    const uint64_t nblk = L / 64;
    printf("ptrace B=%d L=%llu MiB pad=%llu skew=%u lanes=%u: %.2f ms, %.1f cycles/block overall at 2.4 GHz\n",
           B, (unsigned long long)(L >> 20), (unsigned long long)pad, g_skew, lanes, ms,
           ms * 1e-3 * 2.4e9 / (double)nblk);
    {
      // where the waves' cycles go, per phase (4 blocks), averaged over workgroups
      double cw = 0, ct = 0, pw = 0, pwr = 0, pt = 0;
      for (int g = 0; g < groups; ++g) {
        const uint64_t* t = &tr[(uint64_t)g * 1024];
        pt += t[1019]; cw += t[1020]; ct += t[1021]; pw += t[1022]; pwr += t[1023];
      }
      const double ph = (double)groups * (double)(nblk / 4);
      printf("  per phase: chain %.0f cycles (%.0f waiting at the barrier); producer %.0f "
             "(%.0f writing the ring incl. load waits, %.0f at the barrier)\n",
             ct / ph, cw / ph, pt / ph, pwr / ph, pw / ph);
    }
    const int pts = (int)std::min<uint64_t>(510, (nblk / 4 + 4095) / 4096);
    for (int g = 0; g < groups; g += std::max(1, groups / 4)) {
      printf("  wg %d: MiB-index:cycles/block@GHz", g);
      for (int k = 1; k < pts; ++k) {
        const uint64_t* a = &tr[(uint64_t)g * 1024 + 2 * (k - 1)];
        const uint64_t* b = &tr[(uint64_t)g * 1024 + 2 * k];
        if (!b[0] || !a[0]) break;
        const double cyc = (double)(b[0] - a[0]), real = (double)(b[1] - a[1]);
        if (k % std::max(1, pts / 16) == 0 || k == pts - 1)
          printf(" %d:%.0f@%.2f", k, cyc / 16384.0, cyc / real * 0.1);
      }
      printf("\n");
    }
    CK(hipFree(d_data));
    CK(hipFree(d_c));
    CK(hipFree(d_dig));
    CK(hipFree(d_tr));
    return 0;
  }
  if (!strcmp(mode, "half5")) {
    // A/B/A/B: 4-block phases (128 KiB ring) vs 5-block phases (160 KiB ring)
    int bad = 0;
    bad += run_edges(7);
    for (int rep = 0; rep < 2; ++rep) {
      run_md5(512, 10ull << 20, 5, rep == 0, 1);
      run_md5(512, 10ull << 20, 5, rep == 0, 7);
    }
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "pace")) {
    // A/B: the shipped producer (pc: depth 2, ~512-cycle pause before it writes
    // the ring) vs round 1's (depth 1, no pause) and other pauses
    int bad = run_edges(1) + run_edges(19);
    for (int rep = 0; rep < 3; ++rep)
      for (int w : {1, 19, 20, 23}) run_md5(512, 10ull << 20, 7, rep == 0, w);
    for (int w : {1, 19, 20}) run_md5(8192, 1ull << 20, 5, true, w);
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "lead")) {
    // A/B: chain_phase's graded wait at each phase's first block (kLead steps
    // on the first kLead/4 reads) against the shipped qsmd5_batch_pc64_kernel
    // (the shipped kernel, which 1, runs lead 8 since this A/B; which 34 is
    // the kernel before it)
    int bad = 0;
    for (int w : {30, 31, 32, 33}) bad += run_edges(w);
    for (int rep = 0; rep < 3; ++rep)
      for (int w : {1, 34}) run_md5(512, 10ull << 20, 7, rep == 0, w);
    for (int rep = 0; rep < 4; ++rep)
      for (int w : {1, 30, 31, 32, 33}) run_md5(512, 10ull << 20, 7, rep == 0, w);
    for (int w : {1, 30, 31, 32, 33}) run_md5(8192, 1ull << 20, 5, true, w);
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "pc2_pace")) {
    // the 64 KiB-ring kernel (16 385..32 768 chunks): producer depth and pause
    for (int rep = 0; rep < 2; ++rep)
      for (int B : {20480, 32768})
        for (int w : {5, 40, 41, 42, 43, 44}) run_md5(B, 1ull << 20, 5, rep == 0, w, 4352);
    return 0;
  }
  if (!strcmp(mode, "lead_pace")) {
    // with the graded wait shipped: producer pause and depth again
    for (int rep = 0; rep < 3; ++rep)
      for (int w : {1, 35, 36, 37, 38, 39}) run_md5(512, 10ull << 20, 7, rep == 0, w);
    for (int w : {1, 37, 38}) run_md5(8192, 1ull << 20, 5, true, w);
    return 0;
  }
  if (!strcmp(mode, "attrib")) {
    // where the chain's last ~55 cycles per block go.  The
    // shipped kernel (1) against itself with the producer's ring writes (50),
    // its HBM loads (51) or both (52) switched off; 50-52 hash garbage, so only
    // the shipped kernel is checked.  (Round 3 also tried an unconditional
    // producer loop with exact vmcnt waits and an unconditional 17th-dword
    // load: both slower, profiles/r03_attrib2.log, r03_attrib3.log.)
    int bad = run_edges(1);
    for (int rep = 0; rep < 3; ++rep)
      for (int w : {1, 50, 51, 52}) run_md5(512, 10ull << 20, 5, rep == 0 && w == 1, w);
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "chaincost")) {
    // cycles per 64-B block of the chain wave, by what it does besides the steps
    uint64_t* d_out;
    uint32_t* d_sink;
    CK(hipMalloc(&d_out, 8));
    CK(hipMalloc(&d_sink, 4 * 128));
    const int phases = 4096;
    auto one = [&](auto kern, const char* what) {
      hipLaunchKernelGGL(kern, dim3(1), dim3(128), 0, 0, d_out, d_sink, 16);
      hipLaunchKernelGGL(kern, dim3(1), dim3(128), 0, 0, d_out, d_sink, phases);
      CK(hipDeviceSynchronize());
      uint64_t cyc;
      CK(hipMemcpy(&cyc, d_out, 8, hipMemcpyDeviceToHost));
      printf("  %-58s %.1f cycles/block\n", what, (double)cyc / (phases * kPcHalf));
    };
    one(k_chain_cost<2>, "steps from registers (no LDS, no barrier)");
    one(k_chain_cost<0>, "chain_phase: 16 ds_read_b128 + 1 wait per block");
    one(k_chain_cost<1>, "chain_phase + lds_barrier per 4 blocks (2nd wave barriers only)");
    one(k_chain_cost<0, 32>, "chain_phase, 32 active lanes");
    one(k_chain_cost<0, 16>, "chain_phase, 16 active lanes");
    one(k_chain_cost<0, 1>, "chain_phase, 1 active lane");
    one(k_chain_cost<2, 32>, "steps from registers, 32 active lanes");
    one(k_chain_spread<16>, "reads spread: 1 DS read per 16 VALU");
    one(k_chain_cost<0, 64, 4>, "chain_phase, graded wait on block 0 (lead 4 steps)");
    one(k_chain_cost<0, 64, 8>, "chain_phase, graded wait on block 0 (lead 8 steps)");
    one(k_chain_cost<0, 64, 16>, "chain_phase, graded wait on block 0 (lead 16 steps)");
    one(k_chain_cost<0, 64, 32>, "chain_phase, graded wait on block 0 (lead 32 steps)");
    one(k_chain_cost<1, 64, 16>, "+ lds_barrier per 4 blocks, lead 16");
    // operands from a continuous ring, no phases (k_chain_ring)
    u32x4* d_ring;
    CK(hipMalloc(&d_ring, 64 * 16384));
    {
      std::vector<uint32_t> h(64 * 4096);
      for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)i * 2654435761u;
      CK(hipMemcpy(d_ring, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    const int nb = phases * kPcHalf;
    auto ring_one = [&](auto kern, const char* what) {
      hipLaunchKernelGGL(kern, dim3(1), dim3(128), 0, 0, d_out, d_sink, 64, d_ring);
      hipLaunchKernelGGL(kern, dim3(1), dim3(128), 0, 0, d_out, d_sink, nb, d_ring);
      CK(hipDeviceSynchronize());
      uint64_t cyc;
      CK(hipMemcpy(&cyc, d_out, 8, hipMemcpyDeviceToHost));
      printf("  %-58s %.1f cycles/block\n", what, (double)cyc / nb);
    };
    ring_one(k_chain_ring<0>, "continuous LDS ring (no phases, no barrier)");
    ring_one(k_chain_at<0>, "continuous LDS, next reads after step 0");
    ring_one(k_chain_at<4>, "continuous LDS, next reads after step 4");
    ring_one(k_chain_at<8>, "continuous LDS, next reads after step 8");
    ring_one(k_chain_at<16>, "continuous LDS, next reads after step 16");
    ring_one(k_chain_at<32>, "continuous LDS, next reads after step 32");
    ring_one(k_chain_ring<1, 2>, "global ring 2 blocks, default policy");
    ring_one(k_chain_ring<1, 8>, "global ring 8 blocks, default policy");
    ring_one(k_chain_ring<2, 8>, "global ring 8 blocks, sc0 (L2)");
    ring_one(k_chain_ring<2, 64>, "global ring 64 blocks, sc0 (L2)");
    ring_one(k_chain_ring<3, 64>, "global ring 64 blocks, nt");
    ring_one(k_chain_l1<2, 64, false>, "L1 ring 2 slots x 64 lanes (32 KiB)");
    ring_one(k_chain_l1<2, 64, true>, "L1 ring 2 slots x 64 lanes, barrier per block");
    ring_one(k_chain_l1<3, 32, false, false>, "L1 ring 3 slots x 32 live lanes, 1 KiB rows");
    ring_one(k_chain_l1<3, 32, false>, "L1 ring 3 slots x 32 live lanes (24 KiB)");
    ring_one(k_chain_l1<3, 32, true>, "L1 ring 3 slots x 32 live lanes, barrier per block");
    ring_one(k_chain_l1<4, 32, true>, "L1 ring 4 slots x 32 live lanes (32 KiB), barrier");
    ring_one(k_chain_l1<2, 32, true>, "L1 ring 2 slots x 32 live lanes (16 KiB), barrier");
    ring_one(k_chain_l1<5, 16, true>, "L1 ring 5 slots x 16 live lanes (20 KiB), barrier");
    ring_one(k_chain_l1<8, 16, true>, "L1 ring 8 slots x 16 live lanes (32 KiB), barrier");
    ring_one(k_chain_l1<4, 16, true>, "L1 ring 4 slots x 16 live lanes (16 KiB), barrier");
    ring_one(k_chain_l1<2, 16, true>, "L1 ring 2 slots x 16 live lanes (8 KiB), barrier");
    ring_one(k_chain_l1<1, 64, false>, "L1 ring 1 slot x 64 lanes (16 KiB)");
    {
      uint64_t* d_o2;
      CK(hipMalloc(&d_o2, 16));
      auto hand = [&](auto kern, const char* what) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(128), 0, 0, d_o2, d_sink, 64, d_ring);
        hipLaunchKernelGGL(kern, dim3(1), dim3(128), 0, 0, d_o2, d_sink, nb, d_ring);
        CK(hipDeviceSynchronize());
        uint64_t r[2];
        CK(hipMemcpy(r, d_o2, 16, hipMemcpyDeviceToHost));
        printf("  %-58s %.1f cycles/block, %llu stale operand groups\n", what, (double)r[0] / nb,
               (unsigned long long)r[1]);
      };
      hand(k_l1_handoff<0>, "hand-off: 2 slots, producer stores, default policy");
      hand(k_l1_handoff<1>, "hand-off: 2 slots, producer stores sc0");
      hand(k_l1_handoff<2>, "hand-off: 2 slots, producer stores nt");
      CK(hipFree(d_o2));
    }
    CK(hipFree(d_ring));
    CK(hipFree(d_out));
    CK(hipFree(d_sink));
    return 0;
  }
  if (!strcmp(mode, "cross")) {
    // latency (pc) vs coalesced kernel around the selection threshold (16384 chunks)
    int bad = run_edges(5);
    for (int B : {512, 8192, 16384, 20480, 24576, 32768, 49152})
      for (int w : {1, 5, 2}) run_md5(B, 1 << 20, 3, w == 5, w, 4352);
    run_md5(512, 10 << 20, 3, true, 5, 0);
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "coalfast")) {
    // A/B: the previous coal body (probe copy, mode 0) vs the shipped kernel with the fast region
    int bad = run_edges(2);
    for (int rep = 0; rep < 2; ++rep) {
      run_coal_probe<0>(131072, 65536, 4352, 5);
      run_md5(131072, 65536, 5, rep == 0, 2, 4352);
    }
    run_coal_probe<0>(65536, 262144, 4352, 3);
    run_md5(65536, 262144, 3, true, 2, 4352);
    run_coal_probe<0>(32768, 1 << 20, 4352, 3);
    run_md5(32768, 1 << 20, 3, true, 2, 4352);
    run_md5(131072, 65536 + 64 * 3, 3, true, 2, 4352);
    run_md5(100000, 65536 + 17 * 64, 3, true, 2, 4352);
    return bad ? 1 : 0;
  }
  if (!strcmp(mode, "probe")) {
    for (int rep = 0; rep < 2; ++rep) {
      run_coal_probe<0>(131072, 65536, 4352, 5);
      run_coal_probe<1>(131072, 65536, 4352, 5);
      run_coal_probe<2>(131072, 65536, 4352, 5);
    }
    run_coal_probe<0>(65536, 262144, 4352, 3);
    run_coal_probe<1>(65536, 262144, 4352, 3);
    run_coal_probe<2>(65536, 262144, 4352, 3);
    run_coal_probe<0>(262144, 65536, 4352, 3);
    run_coal_probe<1>(262144, 65536, 4352, 3);
    run_coal_probe<2>(262144, 65536, 4352, 3);
    run_coal_probe<0>(8192, 1 << 20, 4352, 3);
    return 0;
  }
  if (!strcmp(mode, "prio")) {  // round 5: alternating issue priority, A/B/A/B after a warm-up
    run_stamps(131072, 64 << 10, 20, 4352, 0, 0);  // warm-up series (its lines are reported too)
    for (int round = 0; round < 2; ++round)
      for (int prio : {0, 2, 4})
        for (uint64_t kib : {64, 256}) run_stamps(131072, kib << 10, 5, 4352, 0, prio);
    return 0;
  }
  if (!strcmp(mode, "stamps")) {  // round 5: clock vs ramp/tail of the coalesced kernel
    // extra LDS per workgroup: 0 (16 KiB static: up to 10 per CU), 4 KiB (20 KiB: 8 per CU,
    // 2048 workgroups = exactly 8 on each of 256 CUs)
    for (uint32_t extra : {0u, 4096u})
      for (uint64_t kib : {64, 256}) run_stamps(131072, kib << 10, 6, 4352, extra);
    return 0;
  }
  if (!strcmp(mode, "sat")) {
    run_stream_read(8ull << 30, 5);
    run_md5(131072, 65536, 5, true, 0, 0);
    run_md5(131072, 65536, 5, true, 0, 4352);
    run_md5(262144, 32768, 5, true, 0, 4352);
    run_md5(524288, 16384, 5, true, 0, 4352);
    run_md5(65536, 262144, 3, true, 0, 4352);
    run_md5(16384, 1 << 20, 3, true, 1, 4352);
    run_md5(512, 10485760, 3, true, 0, 0);
    return 0;
  }
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  printf("device %s %s CUs=%d clock=%d kHz\n", prop.name, prop.gcnArchName,
         prop.multiProcessorCount, prop.clockRate);
  const int iters = 20000;
  printf("issue (cycles/instr, s_memtime ticks, 1 wave):\n");
  printf("  dep v_add_u32      %.2f\n", run_issue(k_dep_add, 64, iters, 64));
  printf("  ind v_add_u32 x4   %.2f\n", run_issue(k_ind_add, 256, iters, 64));
  printf("  dep v_alignbit     %.2f\n", run_issue(k_dep_alignbit, 64, iters, 64));
  printf("  dep v_bitop3       %.2f\n", run_issue(k_dep_bitop3, 64, iters, 64));
  printf("  dep v_add3_u32     %.2f\n", run_issue(k_dep_add3, 64, iters, 64));
  printf("  md5 step (5 ins)   %.2f per instr\n", run_issue(k_md5_step, 320, iters, 64));
  printf("  md5 step4 (4 ins)  %.2f per instr\n", run_issue(k_md5_step4, 256, iters, 64));
  printf("  4 v_add + ds_read  %.2f per group\n", run_issue(k_mix_lds, 64, iters, 64));
  printf("  dep v_add_u32 2 waves/WG   %.2f\n", run_issue(k_dep_add, 64, iters, 128));
  printf("  dep v_add_u32 8 waves/WG   %.2f\n", run_issue(k_dep_add, 64, iters, 512));
  printf("  dep v_add_u32 16 waves/WG  %.2f\n", run_issue(k_dep_add, 64, iters, 1024));
  int bad = run_edges(0) + run_edges(1);
  const uint64_t L = 10485760;
  for (int w = 0; w < 2; ++w) {
    run_md5(1, L, 3, true, w);
    run_md5(512, L, 5, true, w);
    run_md5(4096, L, 3, true, w);
    run_md5(65536, 65536, 5, true, w);
  }
  run_md5(512, 1 << 20, 5, true, 1);
  run_md5(4096, 1 << 20, 5, true, 1);
  run_md5(262144, 16384, 5, true, 0);
  return bad ? 1 : 0;
}
