/*
 * eloqstore_pcs.h — C ABI of the MI355X page-checksum engine (libeloqstore_pcs.so).
 *
 * The drop-in boundary for EloqStore's per-page checksum path.  Every entry
 * point takes plain pointers and sizes; no C++ or torch types cross it.  The
 * reference has no batched or device API: these functions replace the bodies
 * of
 *     void eloqstore::SetChecksum(std::string_view)      src/storage/page.cpp:18-23
 *     bool eloqstore::ValidateChecksum(std::string_view)  src/storage/page.cpp:25-31
 * (declared include/storage/page.h:25-26) at the batch points of their callers:
 *     IouringMgr::ReadPages validate loop        src/async_io_manager.cpp:353-366 (<=128 pages)
 *     IouringMgr::ReadPage validate              src/async_io_manager.cpp:239-244
 *     WriteTask::WritePage SetChecksum x3         src/tasks/write_task.cpp:58-79  (batched at
 *                                                 FlushBatchPages :155-167, <=256 pages)
 *     page_checksum_tool                         tools/page_checksum_tool.cpp:104-105
 * and the hash primitive they call, XXH3_64bits (external/xxhash.h:6185) /
 * XXH64 (external/xxhash.h:3678).
 *
 * Page convention (include/storage/page.h:11, include/coding.h:64-77,126-139):
 * digest = XXH3_64bits(page + 8, page_size - 8) (seed 0, default secret),
 * stored little-endian in page bytes [0, 8).  algo = PCS_XXH64 uses
 * XXH64(page + 8, page_size - 8, 0) with the same layout (BASELINE config 3).
 *
 * Conventions
 *  - Return value: PCS_OK (0) or a negative pcs_status.  pcs_last_error()
 *    gives a thread-local message for the last failure on the calling thread.
 *  - *_dev functions take caller-owned DEVICE pointers on the current HIP
 *    device and enqueue work on `stream` (0 = legacy default stream); they do
 *    not synchronise.  Results are valid after the stream is synchronised.
 *  - Validation never fails on a mismatch: mismatches are reported through
 *    d_ok[i] = 0 and *d_first_bad = smallest failing index (UINT64_MAX when all
 *    pages match).  d_first_bad may be NULL.  The caller maps a mismatch to
 *    KvError::Corrupted exactly as async_io_manager.cpp:243/362 does.
 *  - Thread-safety: reentrant; use one stream per host thread per device.
 *    The only global state is the immutable secret in device constant memory
 *    and a per-device CU-count cache.
 *  - The library has no CPU fallback: without a usable GPU every compute entry
 *    point returns PCS_ERR_NO_DEVICE.
 */
#ifndef ELOQSTORE_PCS_H
#define ELOQSTORE_PCS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* hipStream_t, kept opaque so that callers need no HIP headers. */
typedef struct ihipStream_t *pcs_stream_t;

enum pcs_status {
    PCS_OK = 0,
    PCS_ERR_INVALID = -1,     /* bad argument (null pointer, page_size < 8, ...) */
    PCS_ERR_NO_DEVICE = -2,   /* no usable GPU / HIP runtime failure at init */
    PCS_ERR_HIP = -3,         /* a HIP call or kernel launch failed */
    PCS_ERR_NOMEM = -4,       /* device or pinned-host allocation failed */
};

enum pcs_algo {
    PCS_XXH3_64 = 0, /* XXH3_64bits, seed 0 — the reference's page checksum */
    PCS_XXH64 = 1,   /* XXH64, seed 0 */
};

/* Flags of the validating host entry points (pcs_pages_validate_host_ex,
 * pcs_batch_submit_ex in PCS_BATCH_VALIDATE mode).  The flag-less names keep
 * their original 6-argument prototypes (= PCS_FLAG_NONE, always verify), so a
 * caller built against an older header can never pass a stray flag word.
 *   PCS_FLAG_SKIP_VERIFY  KvOptions::skip_verify_checksum (include/kv_options.h:41):
 *                         the reference skips the validate loop entirely
 *                         (async_io_manager.cpp:239, 353); here nothing is
 *                         hashed or copied, every verdict is 1 and first_bad is
 *                         UINT64_MAX.  Arguments are still checked; no GPU is
 *                         needed for this path (it computes nothing). */
enum pcs_flags {
    PCS_FLAG_NONE = 0,
    PCS_FLAG_SKIP_VERIFY = 1u << 0,
};

/* ---- library / device ----------------------------------------------------
 * ABI version of this header.  Compare pcs_abi_version() with PCS_ABI_VERSION
 * once at start-up: a library built from another header revision then fails
 * loudly instead of reading arguments it was not given.
 *   3  round 3: pcs_pages_validate_host and pcs_batch_submit lost the trailing
 *      flags word they had in round 2 (the flags moved to the _ex forms); a
 *      caller built against the old prototypes links but its flags are
 *      ignored, which pcs_abi_version() detects
 *   4  round 4: PCS_TUNE_SERVICE_TEAR_TEST / FAIL_INJECT / SERVICE_MAX_CALLERS,
 *      PCS_COUNTER_SERVICE_TORN_REQUESTS; the C++ single-page SetChecksum /
 *      ValidateChecksum moved to libeloqstore_pcs_dropin.so
 *   5  round 5: PCS_TUNE_SERVICE_REPOST_TEST, PCS_TUNE_ZC_STAMP_POLL_PAGES,
 *      PCS_COUNTER_SERVICE_REPOSTS (additive: no prototype changed)
 *   6  round 6: pcs_last_path / pcs_batch_path and the PCS_PATH_* bits,
 *      PCS_TUNE_SERVICE_SLOW_EXIT_TEST, PCS_TUNE_ZC_BATCH_EVENT, PCS_TUNE_SYNC_SPIN_US,
 *      PCS_TUNE_SERVICE_DEPARTURE, pcs_thread_prepare (additive);
 *      pcs_stream_read_dev writes
 *      one word per 4 KiB (was per 64 KiB: size d_out for the new count) */
#define PCS_ABI_VERSION 6
int pcs_abi_version(void);
const char *pcs_version(void);
const char *pcs_last_error(void);
int pcs_device_count(int *count);
/* Select the HIP device for subsequent calls on this host thread. */
int pcs_set_device(int device);
int pcs_synchronize(pcs_stream_t stream);

/* ---- device-resident, fixed page size (pages contiguous, stride page_size) --
 * Fast paths: XXH3 runs a 16-lane group per page for every page size of its
 * long path (page_size >= 249) at any alignment; fastest at page_size % 256
 * == 0 on a 16-byte-aligned base (every power-of-two data_page_size and 64 KiB
 * chunks), 5-7 TB/s for other sizes.  XXH64 needs an
 * 8-byte-aligned base, page_size % 8 == 0 and page_size >= 40.  Any other
 * shape is still computed exactly (generic kernel), only slower. */

/* d_digests[i] = digest of page i over [8, page_size). */
int pcs_pages_digest_dev(const void *d_pages, uint64_t page_size, uint64_t n_pages, int algo,
                         uint64_t *d_digests, pcs_stream_t stream);
/* d_ok[i] = (stored LE u64 at page i [0,8)) == digest; batched ValidateChecksum. */
int pcs_pages_validate_dev(const void *d_pages, uint64_t page_size, uint64_t n_pages, int algo,
                           uint8_t *d_ok, uint64_t *d_first_bad, pcs_stream_t stream);
/* In place: page i bytes [0,8) = digest (LE); batched SetChecksum. */
int pcs_pages_stamp_dev(void *d_pages, uint64_t page_size, uint64_t n_pages, int algo,
                        pcs_stream_t stream);

/* ---- device-resident descriptor batches (mixed page sizes) ----------------
 * Page i occupies [d_base + d_off[i], d_base + d_off[i] + d_len[i]).  Pages
 * shorter than 8 bytes never validate (ok = 0) and digest to 0. */
int pcs_desc_digest_dev(const void *d_base, const uint64_t *d_off, const uint32_t *d_len,
                        uint64_t n, int algo, uint64_t *d_digests, pcs_stream_t stream);
int pcs_desc_validate_dev(const void *d_base, const uint64_t *d_off, const uint32_t *d_len,
                          uint64_t n, int algo, uint8_t *d_ok, uint64_t *d_first_bad,
                          pcs_stream_t stream);
int pcs_desc_stamp_dev(void *d_base, const uint64_t *d_off, const uint32_t *d_len, uint64_t n,
                       int algo, pcs_stream_t stream);

/* ---- raw ranges (no page header): the hash primitive itself ---------------
 * d_out[i] = XXH3_64bits(range i)  (external/xxhash.h:6185), any length, or
 * XXH64(range i, seed)             (external/xxhash.h:3678). */
int pcs_xxh3_64_ranges_dev(const void *d_base, const uint64_t *d_off, const uint32_t *d_len,
                           uint64_t n, uint64_t *d_out, pcs_stream_t stream);
int pcs_xxh64_ranges_dev(const void *d_base, const uint64_t *d_off, const uint32_t *d_len,
                         uint64_t n, uint64_t seed, uint64_t *d_out, pcs_stream_t stream);

/* ---- host-memory batches (scattered pool pages, synchronous) --------------
 * The shape of IouringMgr::ReadPages / FlushBatchPages: an array of page
 * pointers into the caller's page pool (page.cpp:95-120).  Pages are gathered
 * into pinned staging, hashed on the current device and results copied back;
 * the call returns when done.  When the pages form one contiguous run in
 * pinned memory (hipHostMalloc / hipHostRegister, e.g. a registered io_uring
 * buffer ring), they are DMA'd directly with no gather copy.  32 MiB chunks
 * flow through three slots (H2D || kernel || D2H).  Safe to call concurrently
 * from several host threads (each thread owns its staging and streams). */
int pcs_pages_validate_host(const void *const *pages, uint64_t page_size, uint64_t n_pages,
                            int algo, uint8_t *ok, uint64_t *first_bad);
/* The same plus a flags word: PCS_FLAG_SKIP_VERIFY = KvOptions::skip_verify_checksum. */
int pcs_pages_validate_host_ex(const void *const *pages, uint64_t page_size, uint64_t n_pages,
                               int algo, uint8_t *ok, uint64_t *first_bad, uint32_t flags);
int pcs_pages_stamp_host(void *const *pages, uint64_t page_size, uint64_t n_pages, int algo);
int pcs_pages_digest_host(const void *const *pages, uint64_t page_size, uint64_t n_pages,
                          int algo, uint64_t *digests);

/* Pinned (page-locked) host memory, e.g. for an io_uring buffer ring or file
 * staging: batches over one contiguous pinned run are DMA'd with no gather.
 * The allocation is also a registered region (below). */
int pcs_host_alloc_pinned(uint64_t bytes, void **out);
int pcs_host_free_pinned(void *p);

/* Registered page pools (zero-copy).  EloqStore allocates its page pool in
 * chunks of 1024 pages (PagesPool::Extend, src/storage/page.cpp:95-120) and
 * its io_uring buffer rings once at start-up.  Registering such a region once
 * (page-locks it and maps it for the GPU) lets a host batch read and write its
 * pages in place over PCIe.  A host batch (pcs_pages_*_host, pcs_batch_submit)
 * whose pages all lie in registered regions, are 16-byte aligned and have a
 * fast size (XXH3: page_size % 256 == 0; XXH64: page_size % 64 == 0 and
 * >= 128) runs as ONE kernel launch.  That launch reads the page list and the
 * pages from host memory and writes the verdicts, digests or stamped headers
 * straight back: no gather copy and no staging DMA
 * (PCS_TUNE_ZERO_COPY).  Regions must not overlap.  A region must stay
 * registered until every batch over it has completed. */
int pcs_host_register(void *ptr, uint64_t bytes);
/* Optional, once per host thread that will issue host batches (a shard
 * thread at start-up): creates the thread's stream and the pinned result and
 * zero-copy buffers a batch of up to 256 pages uses on the current device,
 * and runs one 1-page zero-copy batch through them (the process's first
 * launch also loads the kernels).  Without it the thread's first host batch
 * pays for this: 16-35 ms with eight threads starting at once (soak
 * attribution).  Idempotent. */
int pcs_thread_prepare(void);
int pcs_host_unregister(void *ptr);  /* ptr = the base passed to pcs_host_register */

/* ---- asynchronous host batches (shard-loop integration) --------------------
 * EloqStore's shard thread never blocks: its work loop is Submit() ->
 * PollComplete() -> ExecuteReadyTasks() (src/storage/shard.cpp:67-130), and
 * a ReadPages / FlushBatchPages coroutine yields while I/O is in flight.  A
 * pcs_batch is the checksum analogue: submit gathers the pages (or DMAs a
 * pinned contiguous run directly), enqueues H2D + kernel + D2H on the batch's
 * own stream and returns; poll answers "done?" without blocking.  A batch
 * whose pages are one contiguous pinned run is DMA'd in place (the caller
 * must then not modify the pages until completion).  One batch
 * object holds one batch in flight; create several for more concurrency.
 * Pages must stay valid until the batch completes (stamp writes the digests
 * into them when poll/wait observes completion). */
typedef struct pcs_batch pcs_batch;
enum pcs_batch_mode { PCS_BATCH_DIGEST = 0, PCS_BATCH_VALIDATE = 1, PCS_BATCH_STAMP = 2 };
int pcs_batch_create(pcs_batch **out);  /* on the calling thread's current device */
/* A submit that fails leaves the batch idle: poll/wait/result then refuse
 * until a later submit succeeds. */
int pcs_batch_submit(pcs_batch *b, int mode, const void *const *pages, uint64_t page_size,
                     uint64_t n_pages, int algo);
/* flags: PCS_FLAG_SKIP_VERIFY (validate mode only) completes the batch at
 * submit with every verdict 1, sizing and pinning no staging. */
int pcs_batch_submit_ex(pcs_batch *b, int mode, const void *const *pages, uint64_t page_size,
                        uint64_t n_pages, int algo, uint32_t flags);
/* 1 = done, 0 = in flight, < 0 = error.  Never waits: on the service path a
 * poll that finds the service's lock held (another thread starting, stopping
 * or launching it) returns 0 and looks again at the next poll, and a service
 * stop or restart never drains the stream under that lock. */
int pcs_batch_poll(pcs_batch *b);
int pcs_batch_wait(pcs_batch *b);   /* blocks until done; PCS_OK or error */
/* After completion: verdicts / digests (either may be NULL) and the first
 * failing index (UINT64_MAX if none, validate mode). */
int pcs_batch_result(pcs_batch *b, uint8_t *ok, uint64_t *digests, uint64_t *first_bad);
int pcs_batch_destroy(pcs_batch *b);

/* ---- which path served a host batch (diagnostics) ------------------------
 * PCS_PATH_* bits of the calling thread's last synchronous host validate or
 * stamp (pcs_pages_validate_host(_ex), pcs_pages_stamp_host), or of a batch's
 * last submission (pcs_batch_path, complete or not).  0 before any call. */
enum pcs_path {
    PCS_PATH_SERVED = 1,          /* answered by the resident service kernel */
    PCS_PATH_LAUNCHED = 2,        /* ran on the launch path (a kernel launch of its own) */
    PCS_PATH_FALLBACK = 4,        /* posted to the service, then re-run on the launch path */
    PCS_PATH_REPOSTED = 8,        /* re-posted to a newer service generation at least once */
    PCS_PATH_NEW_GENERATION = 16, /* queued a new service kernel: none was certainly waiting */
    PCS_PATH_LOCK_SKIPPED = 32,   /* a poll found the service's lock held and returned without it, or a
                                     submit gave up waiting for it (20 us) and took the launch path */
};
int pcs_last_path(void);
int pcs_batch_path(const pcs_batch *b);

/* ---- pre-armed validate service (small read batches, opt-in) --------------
 * A launch per host batch costs ~14 µs before its first page is read.  While
 * the service is on, pcs_pages_validate_host(_ex) and pcs_pages_stamp_host
 * (and so eloqstore::ValidateChecksums / SetChecksums) serve eligible batches
 * through a resident
 * kernel of `workgroups` workgroups that polls a request line in pinned host
 * memory between requests.  Eligible: XXH3, 1-256 pages, all in registered
 * regions, 16-byte aligned, page_size % 256 == 0, called on a device whose
 * service is on; everything else takes the launch path.  Each device has its
 * own service: pcs_service_start / stop / running act on the calling
 * thread's current device (pcs_set_device).  One request per request line is
 * in flight at a time (one line by default, up to 8 with
 * pcs_service_start_ex); a call that finds every line owned, or arrives while
 * more eligible calls are in progress on the device than
 * PCS_TUNE_SERVICE_MAX_CALLERS + lines - 1 (a decaying average), takes the
 * launch path.  The kernel leaves
 * after idle_us (0 = 1000; else 200 .. 1000000) without a request and, between
 * requests, after 2 * idle_us of life, and the next request starts a new one:
 * it holds its CUs, and delays any device-synchronising HIP call of the
 * process, by at most 2 * idle_us.  Results are identical to the launch
 * path's.  PCS_ERR_INVALID for workgroups outside [1, 256] or
 * an idle_us out of range, or when the device's service is already running.
 * Services still running at exit are stopped by an atexit handler. */
int pcs_service_start(int workgroups, uint32_t idle_us);
/* The same with `lines` request lines (1 .. 8), each served by its own
 * `workgroups_per_line` workgroups (lines x workgroups_per_line <= 256): up
 * to `lines` calls on the device are in flight through the service at once,
 * each on a line of its own.  pcs_service_start(wg, idle) = _ex(1, wg, idle). */
int pcs_service_start_ex(int lines, int workgroups_per_line, uint32_t idle_us);
/* Turns the device's service off at once (new calls take the launch path),
 * then waits, without holding anything another thread's call needs, up to 2 s
 * for its kernels to leave; PCS_ERR_HIP if they have not.  Requests still in
 * flight re-run on the launch path. */
int pcs_service_stop(void);
int pcs_service_running(void); /* 1 while the service is on, 0 otherwise */

/* ---- manifest record checksum (next row: SURVEY.md §8f-3) -----------------
 * ManifestBuilder::CalcChecksum (src/storage/root_meta.cpp:150-174): XXH3-64
 * of each <= 1 MiB chunk of the content, folded as agg = rotl(agg, 1) ^ h;
 * agg *= 0x9e3779b97f4a7c15; empty content -> 0.  Chunks >= 2 KiB at 8-byte
 * alignment run on the long-range kernel (a workgroup per chunk). */
int pcs_manifest_checksum_dev(const void *d_content, uint64_t len, uint64_t *d_out, pcs_stream_t stream);
int pcs_manifest_checksum_host(const void *content, uint64_t len, uint64_t *out);
/* ManifestBuilder::ValidateChecksum (root_meta.cpp:138-148): a record is
 * checksum(8) | root(4) | ttl_root(4) | len(4) | payload; records shorter than
 * the 20-byte header never validate. */
int pcs_manifest_validate_host(const void *record, uint64_t size, int *valid);

/* ---- sharding ------------------------------------------------------------
 * Contiguous page range [begin, end) of rank `rank` of `world` for n pages:
 * begin = floor(rank * n / world).  Pages are independent, so G GPUs hash G
 * disjoint ranges with no collective. */
int pcs_shard_range(uint64_t n, int world, int rank, uint64_t *begin, uint64_t *end);

/* ---- tuning -------------------------------------------------------------
 * Process-wide launch knobs, read at every launch (defaults in brackets):
 *   PCS_TUNE_XXH3_BLOCKS_PER_CU   [0] grid cap in 256-thread blocks per CU for
 *                                     the XXH3 page kernels (grid-stride loop
 *                                     beyond it); 0 = auto: one block per 16
 *                                     pages up to 16 KiB pages, 8 per CU above
 *   PCS_TUNE_XXH64_BLOCKS_PER_CU  [0] same for XXH64 (one block per 64 pages)
 *   PCS_TUNE_NT_LOADS             [1] XXH3 page loads non-temporal (1) or
 *                                     default cache policy (0)
 *   PCS_TUNE_XXH64_LAYOUT         [0] segments in flight per XXH64 LDS-kernel
 *                                     step: 0 or 1 = default (2), 2 -> 1,
 *                                     3 -> 2, 4 -> 4, 5 -> 3
 *   PCS_TUNE_ZERO_COPY            [1] host batches over registered pages:
 *                                     1 = zero-copy (one launch, pages read in
 *                                     place); 0 = stage through device memory
 *                                     (gather or direct DMA)
 *   PCS_TUNE_XXH3_RT_BATCH        [1] XXH3 pages whose size is not a compiled
 *                                     case (mixed-size descriptors, odd
 *                                     multiples of 256): 1 = load 4 blocks per
 *                                     step like the fixed kernels; 0 = one
 *                                     block per step
 *   PCS_TUNE_XXH3_SPLIT_PAGES  [8192] fixed-size XXH3 pages of at least this
 *                                     many bytes (power of two, 8-64 KiB) are
 *                                     split over P/4096 groups, one 4 KiB slice
 *                                     each, with the scramble chain run from
 *                                     block sums in LDS; 0 = never
 *   PCS_TUNE_INLINE_LIST          [1] zero-copy XXH3 batches of <= 256 pages
 *                                     pass the page list in the kernel
 *                                     arguments (0 = read it from host memory)
 *   PCS_TUNE_MANIFEST_WIDE        [1] manifests at 8-byte alignment: block
 *                                     sums over the whole GPU, then one chain
 *                                     per chunk (0 = one workgroup per chunk)
 *   PCS_TUNE_XXH64_WAVES          [4] waves per workgroup of the XXH64 LDS
 *                                     kernel (1, 2 or 4; 16 pages per wave)
 *   PCS_TUNE_ZC_POLL              [1] validate batches from host memory, sync
 *                                     and async, zero-copy AND staged (gather
 *                                     or direct DMA), plus zero-copy XXH3
 *                                     stamps of <= PCS_TUNE_ZC_STAMP_POLL_PAGES
 *                                     pages: complete once
 *                                     every verdict / done byte has landed in
 *                                     host memory (1) or on the launch's
 *                                     completion signal (0)
 *   PCS_TUNE_ZC_STAMP_POLL_PAGES [256] zero-copy XXH3 stamps of up to this
 *                                     many pages complete from per-page done
 *                                     bytes (with PCS_TUNE_ZC_POLL on), larger
 *                                     ones on the launch's completion signal
 *   PCS_TUNE_SERVICE_STREAM       [1] stream of the validate service, read at
 *                                     pcs_service_start: 1 highest priority
 *                                     (hardware queues of its own), 0 plain
 *   PCS_TUNE_SERVICE_MAX_CALLERS  [2] validate service contention gate: while
 *                                     the decaying average of concurrent
 *                                     eligible calls on the device exceeds
 *                                     this + lines - 1 + 0.5, the service
 *                                     declines and calls take the launch
 *                                     path; 0 = off (values above 2^20 act
 *                                     as 2^20: the gate never closes)
 *   PCS_TUNE_SERVICE_TEAR_TEST    [0] test only: microseconds the service's
 *                                     host side waits between posting seq and
 *                                     writing the request words (the kernel
 *                                     must ignore the torn line meanwhile)
 *   PCS_TUNE_FAIL_INJECT          [0] test only: the next k host-batch calls
 *                                     (pcs_pages_*_host, pcs_batch_submit*,
 *                                     pcs_batch_poll / wait,
 *                                     pcs_manifest_*_host) fail with
 *                                     PCS_ERR_HIP; decremented per failure
 *   PCS_TUNE_SERVICE_REPOST_TEST  [0] test only: the next k service requests
 *                                     are posted as if an earlier generation
 *                                     had answered part of them and left: seq
 *                                     names the previous generation (no
 *                                     waiting kernel serves it) and the
 *                                     verdict words of pages 16 and up hold a
 *                                     stale answer (validate 0, stamp 1); the
 *                                     host must re-arm and re-post the whole
 *                                     request (PCS_COUNTER_SERVICE_REPOSTS)
 *   PCS_TUNE_SERVICE_SLOW_EXIT_TEST [0] test only: service kernels queued while
 *                                     this is > 0 serve no request and stay
 *                                     this many microseconds after deciding to
 *                                     leave (a stop or restart must not make
 *                                     pollers wait for them)
 *   PCS_TUNE_ZC_BATCH_EVENT       [0] asynchronous zero-copy batches that
 *                                     complete from their landed verdicts /
 *                                     done bytes: 1 records an event behind
 *                                     the kernel (round 5), 0 queries the
 *                                     batch's stream instead (one runtime
 *                                     call less per batch)
 *   PCS_TUNE_SYNC_SPIN_US         [0] synchronous host calls (validate, stamp,
 *                                     pcs_batch_wait) spin on their results
 *                                     for this many microseconds, then sleep
 *                                     ~10 µs between checks; 0 = spin
 *                                     throughout (lowest latency; a loaded
 *                                     store's sync callers then burn their
 *                                     cores)
 *   PCS_TUNE_SERVICE_DEPARTURE    [1] a service kernel's workgroups store
 *                                     their generation into the mailbox as
 *                                     they leave; 1: a waiting request learns
 *                                     that its line's workgroups have gone
 *                                     from those words (re-posting at once)
 *                                     and asks the runtime about the kernel
 *                                     every 1 ms; 0: asks the runtime every
 *                                     50 µs (round 6 before this key)
 * Keys 4, 5, 10, 12, 14, 16-22, 25, 29 and 32 selected variants that measured slower or no
 * better (XXH64 quad nt loads, in-place stamp widths, descriptor tile sorts,
 * 4 KiB slices, wave-dealt pages and slice streams, pipelined split-page
 * tiles, plain result stores, 4 KiB-aligned descriptor steps, a 4-waves-
 * per-SIMD descriptor body; round 3: an XXH64 direct-to-LDS segment ring,
 * XXH64 tile-order chunks; round 4: XXH64 equal-byte runs per quad; round 5:
 * validate-service polls kept in flight);
 * they were retired: setting one fails and reading one
 * returns -1. */
enum pcs_tune_key {
    PCS_TUNE_XXH3_BLOCKS_PER_CU = 1,
    PCS_TUNE_XXH64_BLOCKS_PER_CU = 2,
    PCS_TUNE_NT_LOADS = 3,
    PCS_TUNE_XXH64_LAYOUT = 6,
    PCS_TUNE_ZERO_COPY = 7,
    PCS_TUNE_XXH3_RT_BATCH = 8,
    PCS_TUNE_XXH3_SPLIT_PAGES = 9,
    PCS_TUNE_INLINE_LIST = 11,
    PCS_TUNE_MANIFEST_WIDE = 13,
    PCS_TUNE_XXH64_WAVES = 15,
    PCS_TUNE_ZC_POLL = 23,
    PCS_TUNE_SERVICE_STREAM = 24,
    PCS_TUNE_SERVICE_TEAR_TEST = 26,
    PCS_TUNE_FAIL_INJECT = 27,
    PCS_TUNE_SERVICE_MAX_CALLERS = 28,
    PCS_TUNE_SERVICE_REPOST_TEST = 30,
    PCS_TUNE_ZC_STAMP_POLL_PAGES = 31,
    PCS_TUNE_SERVICE_SLOW_EXIT_TEST = 33,
    PCS_TUNE_ZC_BATCH_EVENT = 34,
    PCS_TUNE_SYNC_SPIN_US = 35,
    PCS_TUNE_SERVICE_DEPARTURE = 36,
};
int pcs_set_tuning(int key, int64_t value);
int64_t pcs_get_tuning(int key); /* -1 for an unknown key */

/* ---- path counters ----------------------------------------------------------
 * Process-wide counts of how host batches were served (monotonic). */
enum pcs_counter {
    PCS_COUNTER_ZERO_COPY_LAUNCHES = 0, /* registered pages hashed in place */
    PCS_COUNTER_DIRECT_DMA_CHUNKS = 1,  /* contiguous pinned runs DMA'd as is */
    PCS_COUNTER_GATHER_CHUNKS = 2,      /* pages gathered into pinned staging */
    PCS_COUNTER_SERVICE_BATCHES = 3,    /* validate / stamp batches served by the pre-armed service */
    PCS_COUNTER_SERVICE_TORN_REQUESTS = 4, /* served requests whose line the kernel first saw torn
                                              (new seq, words failing the check word) and ignored */
    PCS_COUNTER_SERVICE_REPOSTS = 5,       /* service requests re-posted to a newer generation after
                                              the kernel they were posted to left unanswered */
};
uint64_t pcs_counter(int which); /* 0 for an unknown counter */

/* ---- workload tooling (benchmarks, tests, scrub drills) -------------------
 * Synthetic pages: word w of page p = splitmix64((seed ^ p) + (w+1) *
 * 0x9E3779B97F4A7C15), p = first_page_index + i. */
int pcs_gen_pages_dev(void *d_pages, uint64_t page_size, uint64_t n_pages, uint64_t seed,
                      uint64_t first_page_index, pcs_stream_t stream);
int pcs_gen_desc_dev(void *d_base, const uint64_t *d_off, const uint32_t *d_len, uint64_t n,
                     uint64_t seed, uint64_t first_page_index, pcs_stream_t stream);
/* XOR 0xFF into byte `byte_offset` of every `every`-th page (pages 0, every, ...). */
int pcs_flip_byte_dev(void *d_pages, uint64_t page_size, uint64_t n_pages, uint64_t every,
                      uint64_t byte_offset, pcs_stream_t stream);
/* Streaming-read ceiling: a plain read of [d_buf, d_buf + bytes) (16-byte
 * aligned; a trailing partial 16 bytes is ignored) with the headline hash
 * kernel's exact structure and load pattern (256-thread workgroups of 16 four-
 * KiB "pages", XCD-contiguous tile order, nt dwordx4 loads, one 128-byte
 * result store per tile) and no hash: each 4 KiB page folded into one word,
 * d_out[0 .. ceil(bytes / 4096)).  The roofline's measured companion: the
 * hash kernels are compared with the rate at which the same bytes can merely
 * be read the same way.  (ABI 6: one word per 4 KiB; rounds 2-5 wrote one
 * per 64 KiB window.) */
int pcs_stream_read_dev(const void *d_buf, uint64_t bytes, uint64_t *d_out, pcs_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* ELOQSTORE_PCS_H */
