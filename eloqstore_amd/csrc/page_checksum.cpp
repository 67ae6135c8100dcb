// page_checksum.cpp — the batched C++ forms of eloqstore's page checksum over
// the C ABI (include/eloqstore/page_checksum.h).  The single-page
// SetChecksum / ValidateChecksum live in page_checksum_dropin.cpp, a library
// of their own, so linking this one never interposes on page.cpp's.
#include "eloqstore/page_checksum.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "eloqstore_pcs.h"

namespace eloqstore {
namespace {

[[noreturn]] void die(const char* where, int rc) {
    std::fprintf(stderr, "eloqstore page checksum: %s failed (%d): %s\n", where, rc, pcs_last_error());
    std::abort();
}

}  // namespace

int TryValidateChecksums(std::span<const char* const> pages, size_t page_size, uint8_t* ok_out, size_t* first_bad,
                         PageHash hash, bool skip_verify) {
    uint64_t fb = UINT64_MAX;
    static_assert(sizeof(const char*) == sizeof(const void*));
    const int rc = pcs_pages_validate_host_ex(reinterpret_cast<const void* const*>(pages.data()), page_size,
                                              pages.size(), static_cast<int>(hash), ok_out, &fb,
                                              skip_verify ? PCS_FLAG_SKIP_VERIFY : PCS_FLAG_NONE);
    if (rc == PCS_OK && first_bad) *first_bad = fb == UINT64_MAX ? pages.size() : static_cast<size_t>(fb);
    return rc;
}

int TrySetChecksums(std::span<char* const> pages, size_t page_size, PageHash hash) {
    return pcs_pages_stamp_host(reinterpret_cast<void* const*>(pages.data()), page_size, pages.size(),
                                static_cast<int>(hash));
}

const char* LastChecksumError() { return pcs_last_error(); }

size_t ValidateChecksums(std::span<const char* const> pages, size_t page_size, uint8_t* ok_out, PageHash hash,
                         bool skip_verify) {
    size_t first_bad = pages.size();
    if (int rc = TryValidateChecksums(pages, page_size, ok_out, &first_bad, hash, skip_verify))
        die("ValidateChecksums", rc);
    return first_bad;
}

void SetChecksums(std::span<char* const> pages, size_t page_size, PageHash hash) {
    if (int rc = TrySetChecksums(pages, page_size, hash)) die("SetChecksums", rc);
}

void PageDigests(std::span<const char* const> pages, size_t page_size, uint64_t* digests_out, PageHash hash) {
    if (int rc = pcs_pages_digest_host(reinterpret_cast<const void* const*>(pages.data()), page_size, pages.size(),
                                       static_cast<int>(hash), digests_out))
        die("PageDigests", rc);
}

void RegisterPagePool(void* base, size_t bytes) {
    if (int rc = pcs_host_register(base, bytes)) die("RegisterPagePool", rc);
}

void UnregisterPagePool(void* base) {
    if (int rc = pcs_host_unregister(base)) die("UnregisterPagePool", rc);
}

void StartChecksumService(int workgroups, uint32_t idle_us, int lines) {
    if (int rc = pcs_service_start_ex(lines, workgroups, idle_us)) die("StartChecksumService", rc);
}

void StopChecksumService() {
    if (int rc = pcs_service_stop()) die("StopChecksumService", rc);
}

void PrepareChecksumThread() {
    if (int rc = pcs_thread_prepare()) die("PrepareChecksumThread", rc);
}

ChecksumBatch::ChecksumBatch() { status_ = pcs_batch_create(&batch_); }

ChecksumBatch::~ChecksumBatch() { pcs_batch_destroy(batch_); }

int ChecksumBatch::TrySubmitValidate(std::span<const char* const> pages, size_t page_size, PageHash hash,
                                     bool skip_verify) {
    if (status_) return status_;
    n_ = pages.size();
    validate_ = true;
    collected_ = false;
    ok_.assign(n_, 0);
    return pcs_batch_submit_ex(batch_, PCS_BATCH_VALIDATE, reinterpret_cast<const void* const*>(pages.data()),
                               page_size, n_, static_cast<int>(hash),
                               skip_verify ? PCS_FLAG_SKIP_VERIFY : PCS_FLAG_NONE);
}

int ChecksumBatch::TrySubmitStamp(std::span<char* const> pages, size_t page_size, PageHash hash) {
    if (status_) return status_;
    n_ = pages.size();
    validate_ = false;
    collected_ = false;
    return pcs_batch_submit(batch_, PCS_BATCH_STAMP, reinterpret_cast<const void* const*>(pages.data()), page_size,
                            n_, static_cast<int>(hash));
}

void ChecksumBatch::SubmitValidate(std::span<const char* const> pages, size_t page_size, PageHash hash,
                                   bool skip_verify) {
    if (int rc = TrySubmitValidate(pages, page_size, hash, skip_verify)) die("ChecksumBatch::SubmitValidate", rc);
}

void ChecksumBatch::SubmitStamp(std::span<char* const> pages, size_t page_size, PageHash hash) {
    if (int rc = TrySubmitStamp(pages, page_size, hash)) die("ChecksumBatch::SubmitStamp", rc);
}

int ChecksumBatch::Collect() {
    if (collected_) return PCS_OK;
    uint64_t fb = UINT64_MAX;
    if (int rc = pcs_batch_result(batch_, validate_ ? ok_.data() : nullptr, nullptr, &fb)) return rc;
    first_bad_ = fb == UINT64_MAX ? n_ : static_cast<size_t>(fb);
    collected_ = true;
    return PCS_OK;
}

int ChecksumBatch::Path() const { return batch_ ? pcs_batch_path(batch_) : 0; }

int ChecksumBatch::TryPoll() {
    if (status_) return status_;
    const int rc = pcs_batch_poll(batch_);
    if (rc == 1) {
        if (int c = Collect()) return c;
    }
    return rc;
}

bool ChecksumBatch::Poll() {
    const int rc = TryPoll();
    if (rc < 0) die("ChecksumBatch::Poll", rc);
    return rc == 1;
}

void ChecksumBatch::Wait() {
    if (status_) die("ChecksumBatch::Wait", status_);
    if (int rc = pcs_batch_wait(batch_)) die("ChecksumBatch::Wait", rc);
    if (int rc = Collect()) die("ChecksumBatch::Wait", rc);
}

uint64_t ManifestChecksum(std::string_view content) {
    uint64_t h = 0;
    if (int rc = pcs_manifest_checksum_host(content.data(), content.size(), &h)) die("ManifestChecksum", rc);
    return h;
}

bool ValidateManifestRecord(std::string_view record) {
    int valid = 0;
    if (int rc = pcs_manifest_validate_host(record.data(), record.size(), &valid)) die("ValidateManifestRecord", rc);
    return valid != 0;
}

}  // namespace eloqstore
