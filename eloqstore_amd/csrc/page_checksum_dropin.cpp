// page_checksum_dropin.cpp — eloqstore::SetChecksum / ValidateChecksum
// (include/storage/page.h:25-26, src/storage/page.cpp:18-31) over the C ABI,
// built as libeloqstore_pcs_dropin.so.
//
// A library of its own, opt-in: only a store that deletes page.cpp's two
// bodies links it.  The batch library (libeloqstore_pcs.so) does not export
// these names, so a store that keeps page.cpp's CPU definitions, the
// recommended integration, resolves them to page.cpp
// whatever the link order or DSO search order: an EloqStore built as a
// shared object (eloqstore_module.cpp embedding) can never have its
// single-page calls silently become GPU round trips.
#include <cstdio>
#include <cstdlib>
#include <string_view>

#include "eloqstore/page_checksum.h"
#include "eloqstore_pcs.h"

namespace eloqstore {
namespace {

// Digest header width: eloqstore::checksum_bytes (include/storage/page.h:11),
// which this library's public header deliberately does not define.
constexpr size_t kChecksumBytes = 8;

// The reference's functions cannot fail, and a silent `false` would be
// reported by callers as KvError::Corrupted: a GPU failure terminates.
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

}  // namespace eloqstore
