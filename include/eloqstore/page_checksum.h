// page_checksum.h — C++ drop-in for EloqStore's page checksum call surface,
// backed by the MI355X kernels behind include/eloqstore_pcs.h.
//
// Reference surface (namespace eloqstore, include/storage/page.h:25-26):
//     void SetChecksum(std::string_view blob);      // src/storage/page.cpp:18-23
//     bool ValidateChecksum(std::string_view blob);  // src/storage/page.cpp:25-31
// This header only re-declares those two functions (an identical
// redeclaration is legal next to page.h) and defines nothing page.h defines:
// the header constants (checksum_bytes = 8, page_type_offset, page.h:11-12)
// stay page.h's, so both headers can be included in one translation unit
// (tests/test_integration_compile.py compiles INTEGRATION.md's call-site
// snippets against the reference's own page.h).
// Same names, namespace and argument meaning: blob is one whole page,
// blob.size() >= 8 is assumed exactly as in the reference (a shorter blob
// never validates and SetChecksum leaves it untouched); SetChecksum writes the
// little-endian digest into blob[0, 8) through const_cast, as page.cpp does.
// The two single-page functions are defined ONLY in the opt-in
// libeloqstore_pcs_dropin.so (for a store that deletes page.cpp's bodies);
// the batch library libeloqstore_pcs.so does not export them, so a store that
// keeps page.cpp's CPU definitions (the recommended integration,
// INTEGRATION.md §2.4) resolves them to page.cpp in any link or DSO order.
// They terminate the process on a GPU failure (the reference's functions
// cannot fail, and a silent `false` would be reported by callers as
// KvError::Corrupted).
//
// Batched forms for the natural batch points of the callers
// (IouringMgr::ReadPages, async_io_manager.cpp:353-366; FlushBatchPages,
// write_task.cpp:155-167) — scattered pool pages of one page size — in two
// flavours: the Try* forms return a status (PCS_OK or a negative pcs_status,
// message in LastChecksumError()) so a call site can fall back to the
// reference's per-page loop on a GPU failure, and
// the plain forms terminate with the message instead.
#pragma once

#include <cstddef>
#include <cstdint>
#include <span>
#include <string_view>
#include <vector>

struct pcs_batch;  // include/eloqstore_pcs.h (global namespace, C ABI)

namespace eloqstore {

void SetChecksum(std::string_view blob);
bool ValidateChecksum(std::string_view blob);

// Hash variant for the batched forms (the reference path is always XXH3).
enum class PageHash : int { XXH3_64 = 0, XXH64 = 1 };

// Batch-size policy for the call sites.  A GPU batch pays
// a fixed launch + completion cost before any byte is hashed (~14 µs for one
// page) while the reference's CPU loop pays per page (~0.6 µs per cache-cold
// 4 KiB page), so small batches stay on the reference's own per-page
// ValidateChecksum / SetChecksum (page.cpp:18-31): the 6-page scan prefetch
// (types.h:31, scan_task.cpp:215), short overflow reads (task.cpp:136), the
// tail of a write batch.  Defaults are the measured latency crossovers of one
// call against one core running the reference loop over the same scattered
// 4 KiB pool pages (integration_snippets --crossover, every repetition timing
// the columns in a fresh random order, with a control column that must agree
// within 3 %; DESIGN.md §5, profiles/r05/crossover_r05e.txt):
//   registered pool (RegisterPagePool, zero-copy): GPU faster from 32 pages
//   to validate (32 pages = 128 KiB) and from 32-48 pages to stamp (three
//   boxes: 32, 48, 48; the write gate is 48 pages = 192 KiB);
//   unregistered pages (gathered into staging):    GPU faster from 192-256 pages.
inline constexpr size_t kGpuChecksumMinBatchBytes = size_t(128) << 10;
inline constexpr size_t kGpuStampMinBatchBytes = size_t(192) << 10;  // FlushBatchPages
inline constexpr size_t kGpuChecksumMinBatchBytesStaged = size_t(1) << 20;
inline bool GpuChecksumPays(size_t n_pages, size_t page_size, size_t min_bytes = kGpuChecksumMinBatchBytes) {
    return n_pages * page_size >= min_bytes;
}

// Manifest records (ManifestBuilder::CalcChecksum, root_meta.cpp:150-174):
// the host-memory ManifestChecksum copies the record over PCIe and runs three
// launches (~54 µs at 64 KiB), so only records from this size on (snapshots,
// large mapping logs) are faster on the GPU; smaller ones keep the reference
// loop.  Measured crossover, same harness: 6 MiB (259 vs 239 µs; 64 MiB:
// 2.8 ms on one core, 1.44 ms on the GPU).
inline constexpr size_t kGpuManifestMinBytes = size_t(6) << 20;

// Non-aborting forms.  Return PCS_OK (0) or a negative pcs_status
// (include/eloqstore_pcs.h) with the message in LastChecksumError(); on
// PCS_OK, *first_bad (if given) is the first corrupted index or pages.size().
// A failed call has written nothing a caller may trust: the read path falls
// back to page.cpp's ValidateChecksum loop, as the reference would run it
// (async_io_manager.cpp:353-366), and the write path to SetChecksum.
int TryValidateChecksums(std::span<const char* const> pages, size_t page_size, uint8_t* ok_out, size_t* first_bad,
                         PageHash hash = PageHash::XXH3_64, bool skip_verify = false);
int TrySetChecksums(std::span<char* const> pages, size_t page_size, PageHash hash = PageHash::XXH3_64);
const char* LastChecksumError();  // the calling thread's last failure (pcs_last_error)

// Validates every page; ok_out[i] = 1 if page i's stored digest matches.
// Returns the index of the first corrupted page, or pages.size() if all match
// (the reference loop stops at the first failure, async_io_manager.cpp:357-363;
// the batch checks all and reports the first).  skip_verify mirrors
// KvOptions::skip_verify_checksum (kv_options.h:41): nothing is hashed and every
// page is reported valid (PCS_FLAG_SKIP_VERIFY; needs no GPU).
size_t ValidateChecksums(std::span<const char* const> pages, size_t page_size, uint8_t* ok_out,
                         PageHash hash = PageHash::XXH3_64, bool skip_verify = false);

// Stamps every page in place (batched SetChecksum).
void SetChecksums(std::span<char* const> pages, size_t page_size, PageHash hash = PageHash::XXH3_64);

// Digests without touching the pages.
void PageDigests(std::span<const char* const> pages, size_t page_size, uint64_t* digests_out,
                 PageHash hash = PageHash::XXH3_64);

// Registers a page-pool chunk or io_uring buffer ring once (PagesPool::Extend,
// src/storage/page.cpp:95-120): batches whose pages all lie in registered
// memory are then hashed in place over PCIe in one launch, with no gather
// copy (pcs_host_register).  Unregister only when no batch over it is in flight.
void RegisterPagePool(void* base, size_t bytes);
void UnregisterPagePool(void* base);

// Pre-armed validate service (pcs_service_start, opt-in): while it is on,
// ValidateChecksums, SetChecksums and ChecksumBatch's validate and stamp
// batches of up to 256 registered pages are served through a resident kernel
// polling a request line, instead of a launch per batch, and the GPU pays
// from kGpuChecksumMinBatchBytesService on (4 KiB pool pages,
// integration_snippets --crossover, profiles/r05/crossover_r05e.txt: one page
// 7.8 µs to validate instead of 14.8 and 8.2 µs to stamp instead of 15.2;
// faster than the reference loop from 24 pages, both ways).  The kernel holds
// `workgroups` CUs (16 serves 128-256 pages 10-15 % faster than 4) and
// leaves after idle_us without a request or 2 * idle_us of life; the next
// request starts a new one.  `lines` request lines (1-8) let that many calls
// be served at once, each line by its own `workgroups` workgroups.  A call
// that finds every line owned, or that arrives while more than
// PCS_TUNE_SERVICE_MAX_CALLERS + lines - 1 eligible calls are in progress on
// the device (a decaying average; the knob is 2 by default), takes the launch
// path.  Start and stop act on the calling thread's current device; each
// device has its own service.
void StartChecksumService(int workgroups = 4, uint32_t idle_us = 1000, int lines = 1);
void StopChecksumService();
// Optional, once per shard thread at start-up (pcs_thread_prepare): creates
// the thread's stream and the pinned buffers a batch of up to 256 pages uses
// and runs one 1-page batch, so the thread's first ReadPages / FlushBatchPages
// batch does not pay for that (16-35 ms with eight threads starting at once).
void PrepareChecksumThread();
inline constexpr size_t kGpuChecksumMinBatchBytesService = size_t(96) << 10;

// Asynchronous batch for coroutine call sites: Submit, then Poll() from the
// shard work loop (shard.cpp:67-130) until it returns true.  Pages must stay
// valid until then; SubmitStamp writes the digests into them on completion.
// With the validate service on, an eligible batch is posted to it (no
// launch) and Poll() watches its verdict words.
class ChecksumBatch {
public:
    ChecksumBatch();  // never aborts: a failed creation is Status(), and every call reports it
    ~ChecksumBatch();
    ChecksumBatch(const ChecksumBatch&) = delete;
    ChecksumBatch& operator=(const ChecksumBatch&) = delete;

    // skip_verify mirrors KvOptions::skip_verify_checksum (kv_options.h:41):
    // the batch completes at submit with every page reported valid.
    void SubmitValidate(std::span<const char* const> pages, size_t page_size, PageHash hash = PageHash::XXH3_64,
                        bool skip_verify = false);
    void SubmitStamp(std::span<char* const> pages, size_t page_size, PageHash hash = PageHash::XXH3_64);
    bool Poll();  // true once complete; never blocks
    void Wait();
    // Non-aborting forms: PCS_OK / a negative pcs_status (TrySubmit*), and
    // 1 complete / 0 in flight / a negative pcs_status (TryPoll).
    int TrySubmitValidate(std::span<const char* const> pages, size_t page_size, PageHash hash = PageHash::XXH3_64,
                          bool skip_verify = false);
    int TrySubmitStamp(std::span<char* const> pages, size_t page_size, PageHash hash = PageHash::XXH3_64);
    int TryPoll();
    int Status() const { return status_; }  // PCS_OK, or why the batch could not be created
    // Validate mode, after completion: index of the first corrupted page, or
    // the batch size if every page matched.
    size_t FirstBad() const { return first_bad_; }
    const uint8_t* Verdicts() const { return ok_.data(); }
    // PCS_PATH_* bits of the last submission: which path served it (pcs_batch_path).
    int Path() const;

private:
    int Collect();
    ::pcs_batch* batch_ = nullptr;
    int status_ = 0;
    std::vector<uint8_t> ok_;
    size_t n_ = 0, first_bad_ = 0;
    bool validate_ = false, collected_ = false;
};

// ManifestBuilder::CalcChecksum / ValidateChecksum (src/storage/root_meta.cpp:138-174).
uint64_t ManifestChecksum(std::string_view content);
bool ValidateManifestRecord(std::string_view record);

}  // namespace eloqstore
