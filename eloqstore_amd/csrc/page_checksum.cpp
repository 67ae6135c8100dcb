// page_checksum.cpp — eloqstore::SetChecksum / ValidateChecksum (+ batched
// forms) over the C ABI.  See include/eloqstore/page_checksum.h.
#include "eloqstore/page_checksum.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "eloqstore_pcs.h"

namespace eloqstore {
namespace {

// Digest header width: eloqstore::checksum_bytes (include/storage/page.h:11),
// which this library's public header deliberately does not define.
constexpr size_t kChecksumBytes = 8;

[[noreturn]] void die(const char* where, int rc) {
    std::fprintf(stderr, "eloqstore page checksum: %s failed (%d): %s\n", where, rc, pcs_last_error());
    std::abort();
}

}  // namespace

void SetChecksum(std::string_view blob) {
    if (blob.size() < kChecksumBytes) return;
    void* page = const_cast<char*>(blob.data());
    if (int rc = pcs_pages_stamp_host(&page, blob.size(), 1, PCS_XXH3_64)) die("SetChecksum", rc);
}

bool ValidateChecksum(std::string_view blob) {
    if (blob.size() < kChecksumBytes) return false;
    const void* page = blob.data();
    uint8_t ok = 0;
    if (int rc = pcs_pages_validate_host(&page, blob.size(), 1, PCS_XXH3_64, &ok, nullptr))
        die("ValidateChecksum", rc);
    return ok != 0;
}

size_t ValidateChecksums(std::span<const char* const> pages, size_t page_size, uint8_t* ok_out, PageHash hash,
                         bool skip_verify) {
    uint64_t first_bad = UINT64_MAX;
    static_assert(sizeof(const char*) == sizeof(const void*));
    if (int rc = pcs_pages_validate_host_ex(reinterpret_cast<const void* const*>(pages.data()), page_size,
                                            pages.size(), static_cast<int>(hash), ok_out, &first_bad,
                                            skip_verify ? PCS_FLAG_SKIP_VERIFY : PCS_FLAG_NONE))
        die("ValidateChecksums", rc);
    return first_bad == UINT64_MAX ? pages.size() : static_cast<size_t>(first_bad);
}

void SetChecksums(std::span<char* const> pages, size_t page_size, PageHash hash) {
    if (int rc = pcs_pages_stamp_host(reinterpret_cast<void* const*>(pages.data()), page_size, pages.size(),
                                      static_cast<int>(hash)))
        die("SetChecksums", rc);
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

void StartChecksumService(int workgroups, uint32_t idle_us) {
    if (int rc = pcs_service_start(workgroups, idle_us)) die("StartChecksumService", rc);
}

void StopChecksumService() {
    if (int rc = pcs_service_stop()) die("StopChecksumService", rc);
}

ChecksumBatch::ChecksumBatch() {
    if (int rc = pcs_batch_create(&batch_)) die("ChecksumBatch", rc);
}

ChecksumBatch::~ChecksumBatch() { pcs_batch_destroy(batch_); }

void ChecksumBatch::SubmitValidate(std::span<const char* const> pages, size_t page_size, PageHash hash,
                                   bool skip_verify) {
    n_ = pages.size();
    validate_ = true;
    collected_ = false;
    ok_.assign(n_, 0);
    if (int rc = pcs_batch_submit_ex(batch_, PCS_BATCH_VALIDATE, reinterpret_cast<const void* const*>(pages.data()),
                                     page_size, n_, static_cast<int>(hash),
                                     skip_verify ? PCS_FLAG_SKIP_VERIFY : PCS_FLAG_NONE))
        die("ChecksumBatch::SubmitValidate", rc);
}

void ChecksumBatch::SubmitStamp(std::span<char* const> pages, size_t page_size, PageHash hash) {
    n_ = pages.size();
    validate_ = false;
    collected_ = false;
    if (int rc = pcs_batch_submit(batch_, PCS_BATCH_STAMP, reinterpret_cast<const void* const*>(pages.data()),
                                  page_size, n_, static_cast<int>(hash)))
        die("ChecksumBatch::SubmitStamp", rc);
}

void ChecksumBatch::Collect() {
    if (collected_) return;
    uint64_t fb = UINT64_MAX;
    if (int rc = pcs_batch_result(batch_, validate_ ? ok_.data() : nullptr, nullptr, &fb))
        die("ChecksumBatch::Collect", rc);
    first_bad_ = fb == UINT64_MAX ? n_ : static_cast<size_t>(fb);
    collected_ = true;
}

bool ChecksumBatch::Poll() {
    const int rc = pcs_batch_poll(batch_);
    if (rc < 0) die("ChecksumBatch::Poll", rc);
    if (rc == 1) Collect();
    return rc == 1;
}

void ChecksumBatch::Wait() {
    if (int rc = pcs_batch_wait(batch_)) die("ChecksumBatch::Wait", rc);
    Collect();
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
