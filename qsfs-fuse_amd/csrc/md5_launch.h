// qsfs-fuse_amd/csrc/md5_launch.h -- host-side launchers for md5_kernels.hip
// (private to libqsmd5; the public surface is include/qsmd5.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qsmd5 {

enum KernelKind : int {
  kKernelThroughput = 0,  // qsmd5_batch_kernel: 1 wave / 64 chunks, all work in-wave
  kKernelLatency = 1,     // qsmd5_batch_pc_kernel: producer + chain wave / 64 chunks
  kKernelCoalesced = 2,   // qsmd5_batch_coal_kernel: LDS-DMA coalesced staging, 16-B-aligned
  kKernelLatency2 = 3,    // qsmd5_batch_pc2_kernel: the latency kernel with a 64 KiB ring
};

// Chunks one launch of the latency kernel keeps resident at once: one
// 128 KiB-LDS workgroup per CU, 64 chunks each.  The 64 KiB-ring variant fits
// two workgroups per CU (2-block phases: ~3% slower per chain, measured).
constexpr uint32_t kLatencyKernelResident = 256u * 64u;
constexpr uint32_t kLatency2KernelResident = 2u * 256u * 64u;

// chunks: device array of {ptr,len}; order: optional device lane->chunk map;
// digests: device, 16 B per chunk indexed by chunk index.
// Start skew of the latency kernel for waves whose longest chunk is >= 32 MiB
// (see pc_body): lane l starts perm(l) x skew blocks late.
constexpr uint32_t kPcSkewBlocks = 4;

// skew_blocks: latency kernel only (rounded down to a multiple of 4; 0 = off).
// load_nt: latency kernels only: the producer's loads use the non-temporal
// cache policy.
// lanes: latency kernels only: chains per workgroup (1..64; fewer spread long
// chains over more CUs).
hipError_t launch_batch(const void* chunks, const uint32_t* order, uint32_t n, uint32_t* digests,
                        int kind, hipStream_t s, uint32_t skew_blocks = kPcSkewBlocks,
                        bool load_nt = false, uint32_t lanes = 64);
// Column-pipelined latency kernel: lane t hashes segment segs[t] = {staged
// start of bytes [col_off, col_off + col_w) of chunk order[t], that chunk's
// total length}; state parks in states[4 * order[t]] between columns and the
// digest lands in digests[4 * order[t]] after the chunk's last column.
hipError_t launch_column(const void* segs, const uint32_t* order, uint32_t n, uint32_t* digests,
                         uint64_t col_off, uint64_t col_w, uint32_t* states, hipStream_t s);
hipError_t launch_final(uint32_t* state, const uint8_t* tail, uint32_t rem, uint64_t total_len,
                        hipStream_t s);
// Gather rows {src (device-visible host address), dst (staging), len} into the
// staging ring, one workgroup per row; rows: device array of 24-B records.
constexpr size_t kGatherRowBytes = 24;
hipError_t launch_gather(const void* rows, uint32_t nrows, hipStream_t s, uint32_t groups);
hipError_t warm_up(hipStream_t s);
hipError_t launch_lcg_fill(uint8_t* base, uint64_t stride, uint64_t len, uint32_t seed0,
                           uint32_t nchunks, hipStream_t s);

}  // namespace qsmd5
