// ref_page_stub.cpp — TEST INFRASTRUCTURE: stands in for the reference's
// src/storage/page.cpp:18-31 linked into a SHARED object, the way an
// EloqStore embedded through eloqstore_module.cpp would carry it.  It defines
// eloqstore::SetChecksum / ValidateChecksum with the reference's signatures
// (include/storage/page.h:25-26) over the CPU oracle (checker), and counts
// its calls so tests/cpp/linkorder_test.cpp can tell whose definition a call
// resolved to.
#include <atomic>
#include <cstdint>
#include <string_view>

#include "xxh_oracle.h"

namespace {
std::atomic<uint64_t> g_calls{0};
}

extern "C" uint64_t ref_page_calls() { return g_calls.load(); }

namespace eloqstore {

void SetChecksum(std::string_view blob) {
    ++g_calls;
    oracle_set_checksum(const_cast<char*>(blob.data()), blob.size());
}

bool ValidateChecksum(std::string_view blob) {
    ++g_calls;
    return oracle_validate_checksum(blob.data(), blob.size()) != 0;
}

}  // namespace eloqstore
