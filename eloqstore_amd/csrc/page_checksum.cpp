// page_checksum.cpp — eloqstore::SetChecksum / ValidateChecksum (+ batched
// forms) over the C ABI.  See include/eloqstore/page_checksum.h.
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

void SetChecksum(std::string_view blob) {
    if (blob.size() < checksum_bytes) return;
    void* page = const_cast<char*>(blob.data());
    if (int rc = pcs_pages_stamp_host(&page, blob.size(), 1, PCS_XXH3_64)) die("SetChecksum", rc);
}

bool ValidateChecksum(std::string_view blob) {
    if (blob.size() < checksum_bytes) return false;
    const void* page = blob.data();
    uint8_t ok = 0;
    if (int rc = pcs_pages_validate_host(&page, blob.size(), 1, PCS_XXH3_64, &ok, nullptr))
        die("ValidateChecksum", rc);
    return ok != 0;
}

size_t ValidateChecksums(std::span<const char* const> pages, size_t page_size, uint8_t* ok_out, PageHash hash,
                         bool skip_verify) {
    if (skip_verify) {
        std::memset(ok_out, 1, pages.size());
        return pages.size();
    }
    uint64_t first_bad = UINT64_MAX;
    static_assert(sizeof(const char*) == sizeof(const void*));
    if (int rc = pcs_pages_validate_host(reinterpret_cast<const void* const*>(pages.data()), page_size, pages.size(),
                                         static_cast<int>(hash), ok_out, &first_bad))
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

}  // namespace eloqstore
