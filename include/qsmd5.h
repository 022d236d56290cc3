/*
 * include/qsmd5.h -- C-ABI of the MI355X MD5 chunk-hashing path for qsfs.
 *
 * Drop-in boundary for the reference's per-part Content-MD5 computation
 * (qingstor-incubating/qsfs-fuse v1.0.11):
 *
 *   std::string md5(const boost::shared_ptr<std::iostream>&)  src/base/MD5.h:96,
 *                                                              src/base/MD5.cpp:341-349
 *   std::string md5(const std::string)                         src/base/MD5.h:95,
 *                                                              src/base/MD5.cpp:335-339
 *   class MD5 { update(); finalize(); hexdigest(); }           src/base/MD5.h:51-93
 *
 * called from QSClient::UploadMultipart (src/client/QSClient.cpp:369-371) and
 * QSClient::UploadFile (src/client/QSClient.cpp:445-447).  The batch entry
 * points add what the reference lacks: one call that hashes every part of a
 * file (QSTransferManager::PrepareUpload / DoMultiPartUpload,
 * src/client/QSTransferManager.cpp:475-550, 602-673).
 *
 * Contract (all entry points):
 *   - extern "C", never throw, thread-safe, reentrant from any thread;
 *   - return 0 on success or a negative errno (-EINVAL, -ENODEV, -ENOMEM,
 *     -EIO); qsmd5_strerror() / qsmd5_last_error() describe failures;
 *   - digests are the 16 raw MD5 bytes (RFC 1321 byte order), identical to
 *     the reference's MD5::digest; qsmd5_hex() gives its hexdigest() text;
 *   - the backend is chosen per call: QSMD5_BACKEND=auto
 *     (default) hashes on the CPU when its estimated time is below the GPU's
 *     (a lone part, a few parts, tiny objects one call at a time) and on the
 *     GPU above that break-even; "gpu" forces the gfx950 kernels (no
 *     fallback: without a usable device every hashing call fails with
 *     -ENODEV); "cpu" forces the library's CPU MD5.  QSMD5_FLAG_GPU_ONLY /
 *     QSMD5_FLAG_CPU_ONLY override the environment per call.
 *   - in auto mode a GPU failure falls back to the CPU and returns the same
 *     digest (never an empty Content-MD5).  A sticky HIP error
 *     (a lost GPU context) is logged once to stderr and every later call of
 *     the process hashes on the CPU; qsmd5_get_stats reports it.
 *     qsmd5_set_log_callback sends each call's backend, reason and size to
 *     the host's logger (QSMD5_LOG=1: to stderr).
 *   - lengths up to 2^38 bytes per chunk; the full 64-bit MD5 length is used.
 *     The reference truncates lengths >= 4 GiB (MD5.h:53 32-bit size_type,
 *     MD5.cpp:106); set QSMD5_FLAG_REF_TRUNCATE32 to reproduce that.
 *
 * Lazily initialised: the first call (or qsmd5_init) picks the current HIP
 * device, so it is safe to call after fuse_main() has forked (reference
 * Operations.cpp:1520-1549 initialises threads after the fork for the same
 * reason).  A child forked AFTER the library first initialised (even if
 * qsmd5_shutdown ran since: HIP itself stays up in the parent) cannot use the
 * parent's HIP state: its GPU calls fail with -ENODEV, and auto routing
 * hashes on the CPU.
 *
 * Multi-GPU (one process, e.g. the qsfs daemon): QSMD5_DEVICES="all" or a
 * comma list of ordinals binds several GPUs at init.  qsmd5_hash_batch[_ex]
 * then splits a batch: device chunks run on the GPU that holds them, and host
 * chunks go in contiguous byte-balanced ranges to up to
 * ceil(host bytes / QSMD5_SHARD_BYTES) GPUs (default 4 GiB per GPU), one
 * thread per GPU.  A chunk in device memory of a GPU that is not bound is
 * rejected with -EINVAL (a kernel cannot read it safely).  Streaming contexts,
 * device-async batches and the fill helper use the first bound GPU.
 */
#ifndef QSMD5_H_
#define QSMD5_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define QSMD5_API __attribute__((visibility("default")))
#else
#define QSMD5_API
#endif

#define QSMD5_ABI_VERSION 1

/* One message to hash: `len` bytes at `ptr`.  `ptr` may point to device
 * memory (hipMalloc), pinned host memory (qsmd5_alloc_pinned / hipHostMalloc)
 * or ordinary pageable host memory, at any byte alignment; NULL only if
 * len == 0.  Layout-compatible with the kernel's descriptor. */
typedef struct qsmd5_chunk {
  const void* ptr;
  uint64_t len;
} qsmd5_chunk;

/* One multipart-upload part, as QSTransferManager::PrepareUpload slices a
 * file (QSTransferManager.cpp:475-550; Part, TransferHandle.h:45-101). */
typedef struct qsmd5_part {
  uint32_t part_number; /* 1-based, as the reference's part id */
  uint32_t reserved;
  uint64_t offset;      /* byte offset of the part in the file */
  uint64_t size;        /* bytes in the part */
} qsmd5_part;

/* Flags for qsmd5_init / qsmd5_hash_batch_ex. */
#define QSMD5_FLAG_NONE 0
#define QSMD5_FLAG_REF_TRUNCATE32 1 /* hash only len mod 2^32 bytes, like MD5(std::string) */
#define QSMD5_FLAG_ALIGNED16 2      /* device_async_ex: caller promises 16-B-aligned chunk ptrs */
#define QSMD5_FLAG_GPU_ONLY 8       /* hash_batch_ex: gfx950 kernels only, no CPU routing/fallback */
#define QSMD5_FLAG_CPU_ONLY 16      /* hash_batch_ex: the library's CPU MD5 only */
#define QSMD5_FLAG_BACKGROUND 32    /* hash_batch_ex / hash_read / route: the caller hides this
                                     * batch's latency behind other work (a pre-hash running ahead
                                     * of the uploads): under QSMD5_BACKEND=auto it goes to the GPU
                                     * whenever one is usable, leaving the host's cores to the
                                     * daemon (a GPU failure still falls back to the CPU); without
                                     * a usable GPU, routed as usual. */
#define QSMD5_FLAG_READ_PARALLEL 64 /* hash_read: `read` may run on several library threads at
                                     * once, for different chunks of a window (pread on a file,
                                     * say): QSMD5_READ_THREADS of them (default 4, at most 16).
                                     * Without it, read runs on the calling thread only. */
#define QSMD5_FLAG_HOST 4           /* hash_batch_ex: caller promises every chunk is host memory
                                     * (pageable, pinned or registered), as qsfs's part buffers
                                     * are; skips pointer classification (otherwise one query per
                                     * new allocation or VMA, cached by range).  A device pointer
                                     * in such a batch is a caller bug (it is staged as host). */

/* Initialise the runtime on the current HIP device, or on the QSMD5_DEVICES
 * list (idempotent).  Returns 0, -ENODEV when no GPU is usable or the list
 * names a missing GPU, or -EINVAL when the list is malformed. */
QSMD5_API int qsmd5_init(int flags);

/* Release everything the runtime holds -- each bound GPU's streams, events,
 * descriptor/digest scratch, staging ring and pinned metadata, and every host
 * range still registered through qsmd5_register_host -- before static
 * destructors run (a qsfs daemon's exit path; the reference has no such step:
 * MD5 holds no global state, MD5.cpp:283).  Waits until every call in flight
 * on any thread has returned; calls that start meanwhile wait for it and then
 * initialise afresh.  Streaming contexts must be destroyed first.  Called from
 * inside a qsmd5 call on the same thread it returns -EINVAL.  Idempotent: 0
 * when there is nothing to release.  In a child forked after initialisation it
 * drops the parent's handles without a HIP call and without a lock.  Returns
 * 0, or -EIO if a HIP release call failed (the resources are dropped either
 * way). */
QSMD5_API int qsmd5_shutdown(void);

QSMD5_API int qsmd5_abi_version(void);

/* Log sink for the library's messages (the digest backend and
 * batch size at qsfs's DebugInfo).  Levels are qsfs's LogLevel::Value
 * (src/base/LogLevel.h:27).  Once a sink is set, every message goes to it and
 * nothing to stderr:
 *   QSMD5_LOG_INFO   each hashing call's backend, reason, chunk count and
 *                    bytes ("qsmd5: backend=gpu reason=size chunks=64
 *                    bytes=671088640"), and the GPUs bound at initialisation;
 *   QSMD5_LOG_WARN   a GPU batch that failed and was re-hashed on the CPU, a
 *                    GPU runtime that could not initialise;
 *   QSMD5_LOG_ERROR  a lost GPU context (all later calls hash on the CPU).
 * `msg` has no trailing newline and is valid only during the call.  The sink
 * runs on the thread that made the qsmd5 call, possibly several at once; it
 * must not call back into this library.  NULL restores the default: warnings
 * and errors to stderr, Info lines only under QSMD5_LOG=1.  A qsfs binding:
 *   static void qsfs_md5_log(int lvl, const char* m, void*) {
 *     if (lvl == QSMD5_LOG_INFO) DebugInfo(m); else if (lvl == QSMD5_LOG_WARN)
 *     DebugWarning(m); else DebugError(m); }
 *   qsmd5_set_log_callback(qsfs_md5_log, NULL);   // in qsfs_init */
#define QSMD5_LOG_INFO 0
#define QSMD5_LOG_WARN 1
#define QSMD5_LOG_ERROR 2
typedef void (*qsmd5_log_fn)(int level, const char* msg, void* user);
QSMD5_API int qsmd5_set_log_callback(qsmd5_log_fn fn, void* user);

/* Number of HIP devices visible to this process (0 without a GPU); does not
 * initialise the runtime. */
QSMD5_API int qsmd5_device_count(void);

/* HIP's per-thread error state: the library reads and clears the calling
 * thread's last HIP error (hipGetLastError) before its own launches, so that a
 * stale failure of an earlier HIP call -- the caller's or its own -- cannot
 * fail a good batch.  A caller that wants its own last error must read it
 * before calling into this library. */

/* Static text for an error code returned by this library. */
QSMD5_API const char* qsmd5_strerror(int err);

/* Detail of the last failure on the calling thread ("" if none). */
QSMD5_API const char* qsmd5_last_error(void);

/* md5(std::string) / md5(iostream) for one buffer (MD5.cpp:335-349).
 * Synchronous. */
QSMD5_API int qsmd5_hash_one(const void* ptr, uint64_t len, uint8_t digest[16]);

/* Hash n independent chunks (qsfs upload parts) in one GPU batch.
 * digests[i] receives the MD5 of chunks[i].  Synchronous: returns when every
 * digest is in `digests` (host memory).  Host-resident chunks are copied to
 * the GPU in slices that overlap with hashing.  Device-resident chunks are
 * read on the library's own streams, which are not ordered after work the
 * caller enqueued on any stream (the legacy default stream included):
 * synchronise the stream that wrote them first, or hash them on that stream
 * with qsmd5_hash_batch_device_async. */
QSMD5_API int qsmd5_hash_batch(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16]);

/* As qsmd5_hash_batch with QSMD5_FLAG_* flags. */
QSMD5_API int qsmd5_hash_batch_ex(const qsmd5_chunk* chunks, size_t n, uint8_t (*digests)[16], int flags);

/* Device-resident fast path, asynchronous on `hip_stream` (a hipStream_t, or
 * NULL for the legacy default stream): d_chunks, d_order and d_digests are
 * device memory, every chunk ptr is device memory.  d_order (optional, may be
 * NULL) lists chunk indices in the order lanes take them.  For speed, sort by
 * length, descending, so that the lanes of a wavefront finish together; break
 * ties by address, so that neighbouring buffers share a wavefront and spread
 * over the HBM channels.  qsmd5_hash_batch does both itself.
 * Only enqueues work; the caller synchronises the stream. */
QSMD5_API int qsmd5_hash_batch_device_async(const qsmd5_chunk* d_chunks, const uint32_t* d_order, size_t n,
                                  uint8_t (*d_digests)[16], void* hip_stream);

/* As qsmd5_hash_batch_device_async; flags may carry QSMD5_FLAG_ALIGNED16,
 * which lets batches beyond the latency kernels' range (> 32 768 chunks) use
 * the coalesced LDS-DMA throughput kernel. */
QSMD5_API int qsmd5_hash_batch_device_async_ex(const qsmd5_chunk* d_chunks, const uint32_t* d_order,
                                     size_t n, uint8_t (*d_digests)[16], void* hip_stream,
                                     int flags);

/* Which kernel a device batch of n chunks gets: 1 = producer/consumer latency
 * kernel, 128 KiB LDS ring, one workgroup per CU (n <= 16 384); 3 = the same
 * with a 64 KiB ring, two workgroups per CU (n <= 32 768); 2 = coalesced
 * throughput kernel (larger, 16-B-aligned chunks); 0 = one-wave throughput
 * kernel (larger, any alignment).  QSMD5_KERNEL env ("pc"/"pc2"/"coal"/"v1")
 * overrides. */
QSMD5_API int qsmd5_kernel_choice(size_t n);
QSMD5_API int qsmd5_kernel_choice_ex(size_t n, int flags);

/* Lowercase hex, exactly MD5::hexdigest()'s "%02x" x 16 (MD5.cpp:317-325);
 * out must hold 33 bytes (NUL-terminated).  Host-only, needs no GPU. */
QSMD5_API void qsmd5_hex(const uint8_t digest[16], char out[33]);

/* RFC 1864 Content-MD5 header value: standard base64 (RFC 4648 §4, '='
 * padded) of the 16 raw digest bytes, 24 chars; out must hold 25 bytes.
 * The reference hands the SDK the hex text (QSClient.cpp:370, 446) and how
 * qingstor-sdk-cpp (unpinned, GIT_TAG master) puts it on the wire is not
 * covered by any reference test: this is the form S3-style
 * servers verify, offered for callers that set the header themselves.
 * Host-only, needs no GPU. */
QSMD5_API void qsmd5_base64(const uint8_t digest[16], char out[25]);

/* Streaming context: the reference MD5 class (update()* then finalize()). */
typedef struct qsmd5_ctx qsmd5_ctx;
QSMD5_API int qsmd5_ctx_create(qsmd5_ctx** out);
QSMD5_API int qsmd5_ctx_update(qsmd5_ctx* ctx, const void* ptr, uint64_t len);
QSMD5_API int qsmd5_ctx_final(qsmd5_ctx* ctx, uint8_t digest[16]);
QSMD5_API void qsmd5_ctx_destroy(qsmd5_ctx* ctx);
/* A copy of a context with its running state (the reference MD5 is a value
 * type: MD5.h:51-93 has the implicit copy members and operator<< takes it by
 * value, MD5.h:61).  The copy and the original then update and finalise
 * independently; a finalised or failed context copies as such.  Destroy the
 * copy with qsmd5_ctx_destroy. */
QSMD5_API int qsmd5_ctx_copy(const qsmd5_ctx* src, qsmd5_ctx** out);

/* Pinned (page-locked) host buffers for the transfer-buffer pool
 * (ResourceManager, src/data/ResourceManager.cpp:53-77): the page gather
 * (File::ReadNoLoad) can fill them and the GPU reads them by DMA. */
QSMD5_API int qsmd5_alloc_pinned(size_t bytes, void** out);
QSMD5_API int qsmd5_free_pinned(void* ptr);

/* Register existing host buffers with the GPU (hipHostRegister), e.g. qsfs's
 * transfer-buffer pool once at start-up (TransferManager::InitializeResources,
 * TransferManager.cpp:103-108): their pages are then locked once instead of on
 * each batch's first touch, and rows in separate registered buffers are
 * gathered by one kernel per column.  The range is widened to
 * whole pages.  Unregister (with the same ptr) before freeing the memory.
 * -EINVAL for a NULL/empty range, a ptr registered twice, a range starting
 * in the first page of one already registered, a range sharing a page with
 * one already registered that HIP refuses, or unregistering a ptr this
 * library did not register.  Ranges that share a boundary page (adjacent heap
 * buffers) are otherwise fine: each is registered in full. */
QSMD5_API int qsmd5_register_host(void* ptr, size_t bytes);
QSMD5_API int qsmd5_unregister_host(void* ptr);

/* Part slicing identical to QSTransferManager::PrepareUpload
 * (QSTransferManager.cpp:492-546): a single part below `threshold`, else
 * parts of `buf_size` with the last two averaged when the remainder is below
 * `min_part`.  Offsets start at `range_begin`.  Writes up to `cap` parts and
 * sets *nparts to the number needed (call with cap = 0 to size).
 * Host-only, needs no GPU.  Reference defaults: buf 10 MiB, min 4 MiB,
 * threshold 20 MiB (configure/Default.cpp:159-177).
 * More than 65 535 parts: -EINVAL, with the count in *nparts and nothing
 * written.  The reference's part ids are uint16_t (TransferHandle.h:50), so
 * its part 65 536 gets id 0 and part 65 537 collides with part 1 and is
 * dropped (TransferHandle.cpp:252-256); part numbers here are the
 * reference's for every plan it can carry out. */
QSMD5_API int qsmd5_plan_parts(uint64_t file_size, uint64_t buf_size, uint64_t min_part,
                     uint64_t threshold, uint64_t range_begin, qsmd5_part* parts, size_t cap,
                     size_t* nparts);

/* Batch pre-hash of a whole file's parts in one call: digests[i] = MD5 of
 * file[parts[i].offset - parts[0].offset ... + parts[i].size).  `file` points
 * at the byte for parts[0].offset (host or device memory). */
QSMD5_API int qsmd5_hash_parts(const void* file, const qsmd5_part* parts, size_t n, uint8_t (*digests)[16]);

/* Pull-driven batch: hash n chunks that are NOT whole buffers in memory -- a
 * qsfs file's parts, held in its page cache and gathered by File::ReadNoLoad
 * (src/data/File.cpp:308-375), the read QSTransferManager::DoMultiPartUpload
 * makes for every part before it hashes it (QSTransferManager.cpp:621-623,
 * MD5 at QSClient.cpp:369-371).  The library asks for the bytes through
 * `read` in COLUMN WINDOWS into its own pinned staging: every chunk of a group
 * (up to 32 768) is one GPU chain that parks its state between windows, so the
 * batch is as wide as the file has parts while the staging never exceeds
 * `staging_bytes` (0: QSMD5_READ_STAGING_BYTES, default 256 MiB), whatever the
 * file's size.  The reader fills the next window while the GPU copies and
 * hashes the last one.
 *
 *   read(user, chunk, offset, len, dst): copy bytes [offset, offset + len) of
 *   chunk `chunk` (0-based index into lens) to dst and return the number of
 *   bytes copied, as ReadNoLoad's readSize.  Any other count than len fails the
 *   call with -EIO (the reference stops the upload on a short read,
 *   QSTransferManager.cpp:625-643); nothing is hashed from it.
 *
 * read runs on the calling thread only (QSMD5_FLAG_READ_PARALLEL: on several
 * threads at once, each chunk's windows still in order), one window at a
 * time, with each chunk's windows in increasing offset order and every byte
 * asked for once --
 * except that in QSMD5_BACKEND=auto a GPU failure re-runs the whole batch on
 * the CPU, asking for every byte again from offset 0.  It may call other qsmd5
 * entry points (not qsmd5_shutdown), on any of those threads.  A nested
 * qsmd5_hash_read (from inside read) never waits for a read slot, as the
 * outer call holds one through its reads: under auto routing it runs on the
 * CPU; under QSMD5_FLAG_GPU_ONLY it takes a free slot or returns -EDEADLK.
 * lens[i] < 2^38.  Routed like qsmd5_hash_batch_ex (flags:
 * QSMD5_FLAG_GPU_ONLY / _CPU_ONLY / _REF_TRUNCATE32), by the wall time of
 * the reads and the hashing on each backend.  Calls from different threads
 * (files flushed at once) run side by side, each with its own streams and
 * staging, up to QSMD5_READ_SLOTS per GPU at a time (default 4, at most 8;
 * each slot holds up to staging_bytes of pinned host memory and as much HBM,
 * split into QSMD5_READ_REGIONS regions (default 2); slot 0 of the primary
 * GPU is taken at initialisation unless QSMD5_READ_PREWARM=0, the others on
 * first use, all kept until qsmd5_shutdown); a further call waits for a
 * slot.  The CPU path's pageable staging (up to staging_bytes per call) is
 * likewise kept for the next call, up to QSMD5_READ_SLOTS buffers, until
 * qsmd5_shutdown.  One bound GPU
 * hashes a whole call: the one with the fewest such calls in flight (the
 * first on a tie), so with QSMD5_DEVICES binding several, files flushed at
 * once spread over the GPUs. */
typedef uint64_t (*qsmd5_read_fn)(void* user, size_t chunk, uint64_t offset, uint64_t len, void* dst);
QSMD5_API int qsmd5_hash_read(const uint64_t* lens, size_t n, qsmd5_read_fn read, void* user,
                              uint64_t staging_bytes, uint8_t (*digests)[16], int flags);

/* Download-side integrity (new: the reference never
 * hashes downloads).  QSClient::DownloadFile keeps the object's ETag
 * (QSClient.cpp:321-323) and ReceivedHandlerSingleDownload
 * (QSTransferManager.cpp:85-98) is where a check belongs.  For a single-part
 * object the ETag is the MD5 as 32 hex digits, optionally in double quotes.
 * qsmd5_etag_matches: 1 = digest matches, 0 = mismatch, -EINVAL = the ETag is
 * not a plain MD5 (multipart "<hex>-<n>", empty, malformed).  Host-only. */
QSMD5_API int qsmd5_etag_matches(const uint8_t digest[16], const char* etag);

/* Hash [ptr, ptr+len) (host or device memory) and compare with etag:
 * 1 / 0 as above, or a negative errno. */
QSMD5_API int qsmd5_verify_etag(const void* ptr, uint64_t len, const char* etag);

/* Backend of the calling thread's last hashing call (hash_batch[_ex],
 * hash_one, hash_parts, verify_etag): QSMD5_BACKEND_GPU, QSMD5_BACKEND_CPU,
 * QSMD5_BACKEND_SPLIT (both at once: see qsmd5_route), or 0 before the first
 * call. */
#define QSMD5_BACKEND_GPU 1
#define QSMD5_BACKEND_CPU 2
#define QSMD5_BACKEND_SPLIT 3
QSMD5_API int qsmd5_last_backend(void);

/* The backend QSMD5_BACKEND=auto picks for this batch while the GPU is
 * healthy: QSMD5_BACKEND_CPU when the CPU's estimated time is the lower
 * (QSMD5_CPU_THREADS threads, default 4, at this host's measured chain rate
 * each: qsmd5_get_rates); QSMD5_BACKEND_SPLIT when the batch is ragged enough that
 * handing its longest host chunks to the CPU threads while the GPU hashes the
 * rest cuts the estimate by >= 10% (a device chunk in the CPU share is read
 * back to the host first; QSMD5_SPLIT=0 turns splitting off); else
 * QSMD5_BACKEND_GPU.  A split call counts once in both gpu_batches and
 * cpu_batches of qsmd5_stats. */
QSMD5_API int qsmd5_route(const qsmd5_chunk* chunks, size_t n, int flags);

/* The rates QSMD5_BACKEND=auto prices a batch with (qsmd5_route), in GiB/s.
 * They are this host's: the CPU rates are timed once, at the first routing
 * decision (~1 ms); the GPU chain rate is averaged over single-launch GPU
 * batches of <= 16 384 chunks whose longest is >= 4 MiB, each bound GPU's
 * first such batch not counted (0.119 before any; reset by qsmd5_shutdown).
 * QSMD5_CPU_GIBS, QSMD5_GPU_CHAIN_GIBS and QSMD5_LINK_GIBS override;
 * QSMD5_CALIBRATE=0 keeps the built-in CPU defaults. */
#define QSMD5_RATE_CPU_MEASURED 1   /* cpu_chain_gibs / cpu_lane_thread_gibs timed on this host */
#define QSMD5_RATE_CPU_ENV 2        /* cpu_chain_gibs from QSMD5_CPU_GIBS */
#define QSMD5_RATE_GPU_MEASURED 4   /* gpu_chain_gibs from a timed batch */
#define QSMD5_RATE_GPU_ENV 8        /* gpu_chain_gibs from QSMD5_GPU_CHAIN_GIBS */
typedef struct qsmd5_rates {
  double cpu_chain_gibs;       /* one host thread's scalar MD5 chain */
  double cpu_lane_thread_gibs; /* one host thread's 16 AVX-512 lanes together (0: no AVX-512F) */
  double gpu_chain_gibs;       /* one chunk's chain on a GPU lane (latency kernel) */
  double link_gibs;            /* host -> GPU copy */
  double d2h_gibs;             /* device chunk read back by the CPU backend */
  double gpu_call_ms;          /* fixed cost of a GPU batch */
  int cpu_threads;             /* QSMD5_CPU_THREADS (default 4) */
  int source;                  /* QSMD5_RATE_* bits */
} qsmd5_rates;
QSMD5_API int qsmd5_get_rates(qsmd5_rates* out);

/* The share of its priced rate the CPU backend got in its recent batches
 * (1.0 = as priced on an idle host; 0.5 = its batches took twice the
 * estimate: the host's cores are busy with other work).  Every CPU batch
 * priced at >= 2 ms is timed; a new sample weighs 1/2, and the value relaxes
 * back to 1 with a 10 s time constant (QSMD5_CPU_EFF_DECAY_S) when no CPU
 * batch runs.  QSMD5_BACKEND=auto divides its CPU estimates by it, so a busy
 * host sends batches to the GPU earlier (QSMD5_CPU_LOAD_FEEDBACK=0: always
 * 1).  Host-only, needs no GPU. */
QSMD5_API int qsmd5_get_cpu_efficiency(double* out);

/* Process-wide backend counters since load. */
typedef struct qsmd5_stats {
  uint64_t gpu_batches;  /* calls hashed by the gfx950 kernels */
  uint64_t cpu_batches;  /* calls hashed by the CPU MD5 (routed, forced or fallback) */
  uint64_t fallbacks;    /* of those, calls whose GPU attempt failed */
  uint64_t gpu_chunks, cpu_chunks;
  int gpu_lost;          /* 1 once a sticky HIP error was seen: all later calls run on the CPU */
  int inits;             /* runtime initialisations (HIP device setup) this process ran: 1 after
                          * the first call, +1 per re-init after qsmd5_shutdown; a forked child
                          * never adds one (it makes no HIP call) */
} qsmd5_stats;
QSMD5_API int qsmd5_get_stats(qsmd5_stats* out);

/* Timing of the most recent synchronous batch on this process (ms): total
 * wall, and GPU kernel time between the first and last kernel event. */
QSMD5_API int qsmd5_last_timing(double* wall_ms, double* kernel_ms);

/* Test/bench support (synthetic data, not used by the hashing path): fill
 * nchunks device chunks at base + i*stride with `len` bytes of the LCG of
 * SURVEY.md §8c seeded with seed0 + i.  Asynchronous on hip_stream. */
QSMD5_API int qsmd5_synth_fill_lcg(void* d_base, uint64_t stride, uint64_t len, uint32_t seed0,
                         uint32_t nchunks, void* hip_stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* QSMD5_H_ */
