// capi_sanitize_test.cpp — the C ABI's host code (pcs_capi.cpp,
// page_checksum.cpp) built with ASAN + UBSan and driven on a host with no GPU
// (eloqstore_amd/Makefile `sanitize`, tests/test_sanitizers.py).  Every
// compute entry point must fail loudly with PCS_ERR_NO_DEVICE and every
// argument check must run clean under the sanitizers: null pointers, page
// sizes, flags, shard ranges at the uint64 edge, tuning keys, batch handles,
// the skip_verify path (kv_options.h:41) that completes without a device, the
// thread-local last-error string, and the ABI 4 additions (service lines,
// injected failures, the Try forms and a ChecksumBatch that could not be made).
#include "eloqstore_pcs.h"
#include "eloqstore/page_checksum.h"

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static int g_fail = 0;
#define CHECK(c)                                                                       \
    do {                                                                               \
        if (!(c)) {                                                                    \
            std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #c);  \
            ++g_fail;                                                                  \
        }                                                                              \
    } while (0)

static void shard_ranges() {
    const uint64_t ns[] = {0, 1, 7, 8, 1000003, 1ull << 40, UINT64_MAX - 1, UINT64_MAX};
    for (uint64_t n : ns)
        for (int world : {1, 2, 3, 7, 8, 64, 1 << 20}) {
            uint64_t prev_end = 0, total = 0;
            for (int rank = 0; rank < world; rank += (world > 64 ? 9973 : 1)) {
                uint64_t b = 1, e = 0;
                CHECK(pcs_shard_range(n, world, rank, &b, &e) == PCS_OK);
                CHECK(b <= e && e <= n);
                if (world <= 64) {
                    CHECK(b == prev_end);  // contiguous, in rank order
                    prev_end = e;
                    total += e - b;
                    // balanced: sizes differ by at most one page
                    CHECK(e - b == n / world || e - b == n / world + 1);
                }
            }
            if (world <= 64) CHECK(prev_end == n && total == n);
        }
    uint64_t b, e;
    CHECK(pcs_shard_range(10, 0, 0, &b, &e) == PCS_ERR_INVALID);
    CHECK(pcs_shard_range(10, 4, 4, &b, &e) == PCS_ERR_INVALID);
    CHECK(pcs_shard_range(10, 4, -1, &b, &e) == PCS_ERR_INVALID);
    CHECK(pcs_shard_range(10, 4, 0, nullptr, &e) == PCS_ERR_INVALID);
}

static void no_device() {
    int count = 7;
    CHECK(pcs_device_count(&count) == PCS_ERR_NO_DEVICE && count == 0);
    CHECK(pcs_device_count(nullptr) == PCS_ERR_INVALID);
    CHECK(pcs_set_device(0) == PCS_ERR_NO_DEVICE);
    CHECK(std::strstr(pcs_last_error(), "no usable HIP device") != nullptr);
    CHECK(pcs_synchronize(nullptr) == PCS_ERR_NO_DEVICE);
    uint64_t dummy[4] = {};
    uint32_t len[1] = {4096};
    uint8_t ok[4] = {};
    CHECK(pcs_pages_digest_dev(dummy, 4096, 1, PCS_XXH3_64, dummy, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_pages_validate_dev(dummy, 4096, 1, PCS_XXH64, ok, dummy, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_pages_stamp_dev(dummy, 4096, 1, PCS_XXH3_64, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_desc_digest_dev(dummy, dummy, len, 1, PCS_XXH3_64, dummy, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_desc_validate_dev(dummy, dummy, len, 1, PCS_XXH3_64, ok, nullptr, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_desc_stamp_dev(dummy, dummy, len, 1, PCS_XXH3_64, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_xxh3_64_ranges_dev(dummy, dummy, len, 1, dummy, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_xxh64_ranges_dev(dummy, dummy, len, 1, 0, dummy, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_manifest_checksum_dev(dummy, 8, dummy, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_gen_pages_dev(dummy, 4096, 1, 1, 0, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_gen_desc_dev(dummy, dummy, len, 1, 1, 0, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_flip_byte_dev(dummy, 4096, 1, 1, 10, nullptr) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_stream_read_dev(dummy, 32, dummy, nullptr) == PCS_ERR_NO_DEVICE);

    std::vector<uint8_t> page(4096, 0xAB);
    const void* pages[1] = {page.data()};
    void* wpages[1] = {page.data()};
    uint64_t dig = 0, fb = 0;
    CHECK(pcs_pages_digest_host(pages, 4096, 1, PCS_XXH3_64, &dig) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_pages_validate_host(pages, 4096, 1, PCS_XXH3_64, ok, &fb) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_pages_validate_host_ex(pages, 4096, 1, PCS_XXH3_64, ok, &fb, PCS_FLAG_NONE) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_pages_stamp_host(wpages, 4096, 1, PCS_XXH3_64) == PCS_ERR_NO_DEVICE);
    CHECK(page[0] == 0xAB);  // nothing written without a device
    CHECK(pcs_manifest_checksum_host(page.data(), 100, &dig) == PCS_ERR_NO_DEVICE);
    int valid = -1;
    CHECK(pcs_manifest_validate_host(page.data(), 100, &valid) == PCS_ERR_NO_DEVICE);

    void* pinned = reinterpret_cast<void*>(0x1);
    CHECK(pcs_host_alloc_pinned(4096, &pinned) == PCS_ERR_NO_DEVICE && pinned == nullptr);
    CHECK(pcs_host_register(page.data(), page.size()) == PCS_ERR_NO_DEVICE);
    pcs_batch* b = reinterpret_cast<pcs_batch*>(0x1);
    CHECK(pcs_batch_create(&b) == PCS_ERR_NO_DEVICE && b == nullptr);
    CHECK(pcs_service_start(4, 0) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_service_start(0, 0) == PCS_ERR_INVALID);
    CHECK(pcs_service_start(4, 2000000) == PCS_ERR_INVALID);
    CHECK(pcs_service_start(4, 100) == PCS_ERR_INVALID);
    CHECK(pcs_service_running() == 0 && pcs_service_stop() == PCS_OK);
}

static void arguments() {
    uint64_t dummy[4] = {};
    uint8_t ok[8] = {};
    std::vector<uint8_t> page(4096, 0x5A);
    const void* pages[2] = {page.data(), nullptr};
    // skip_verify (kv_options.h:41): argument checks only, every page passes, no device needed
    uint64_t fb = 0;
    std::memset(ok, 0, sizeof ok);
    CHECK(pcs_pages_validate_host_ex(pages, 4096, 1, PCS_XXH3_64, ok, &fb, PCS_FLAG_SKIP_VERIFY) == PCS_OK);
    CHECK(ok[0] == 1 && fb == UINT64_MAX);
    CHECK(pcs_pages_validate_host_ex(pages, 4096, 0, PCS_XXH3_64, nullptr, nullptr, PCS_FLAG_SKIP_VERIFY) == PCS_OK);
    CHECK(pcs_pages_validate_host_ex(pages, 4096, 2, PCS_XXH3_64, ok, &fb, PCS_FLAG_SKIP_VERIFY) == PCS_ERR_INVALID);
    CHECK(pcs_pages_validate_host_ex(pages, 4, 1, PCS_XXH3_64, ok, &fb, PCS_FLAG_SKIP_VERIFY) == PCS_ERR_INVALID);
    CHECK(pcs_pages_validate_host_ex(pages, 4096, 1, 9, ok, &fb, PCS_FLAG_SKIP_VERIFY) == PCS_ERR_INVALID);
    CHECK(pcs_pages_validate_host_ex(pages, 4096, 1, PCS_XXH3_64, nullptr, &fb, PCS_FLAG_SKIP_VERIFY) == PCS_ERR_INVALID);
    CHECK(pcs_pages_validate_host_ex(pages, 4096, 1, PCS_XXH3_64, ok, &fb, 0x80) == PCS_ERR_INVALID);
    CHECK(pcs_pages_validate_host_ex(nullptr, 4096, 1, PCS_XXH3_64, ok, &fb, PCS_FLAG_SKIP_VERIFY) == PCS_ERR_INVALID);
    // n * page_size past 2^64 is refused before any page pointer is read
    CHECK(pcs_pages_validate_host_ex(pages, 4096, 1ull << 53, PCS_XXH3_64, ok, &fb, PCS_FLAG_SKIP_VERIFY) == PCS_ERR_INVALID);
    CHECK(std::strstr(pcs_last_error(), "overflows") != nullptr);
    CHECK(pcs_pages_digest_host(pages, 4096, 1, PCS_XXH3_64, nullptr) == PCS_ERR_INVALID);
    // batches: null handles
    CHECK(pcs_batch_create(nullptr) == PCS_ERR_INVALID);
    CHECK(pcs_batch_submit(nullptr, 0, pages, 4096, 1, 0) == PCS_ERR_INVALID);
    CHECK(pcs_batch_submit_ex(nullptr, 0, pages, 4096, 1, 0, 0) == PCS_ERR_INVALID);
    CHECK(pcs_batch_poll(nullptr) == PCS_ERR_INVALID);
    CHECK(pcs_batch_wait(nullptr) == PCS_ERR_INVALID);
    CHECK(pcs_batch_result(nullptr, ok, dummy, &fb) == PCS_ERR_INVALID);
    CHECK(pcs_batch_destroy(nullptr) == PCS_OK);
    // host memory bookkeeping without a device
    CHECK(pcs_host_free_pinned(nullptr) == PCS_OK);
    CHECK(pcs_host_free_pinned(page.data()) == PCS_ERR_INVALID);  // never allocated here
    CHECK(pcs_host_alloc_pinned(16, nullptr) == PCS_ERR_INVALID);
    CHECK(pcs_host_register(nullptr, 4096) == PCS_ERR_INVALID);
    CHECK(pcs_host_register(page.data(), 0) == PCS_ERR_INVALID);
    CHECK(pcs_host_unregister(nullptr) == PCS_ERR_INVALID);
    CHECK(pcs_host_unregister(page.data()) == PCS_ERR_INVALID);
    // manifest record shorter than its header: invalid without touching the GPU
    int valid = -1;
    CHECK(pcs_manifest_validate_host(page.data(), 19, &valid) == PCS_OK && valid == 0);
    CHECK(pcs_manifest_validate_host(nullptr, 100, &valid) == PCS_ERR_INVALID);
    CHECK(pcs_manifest_validate_host(page.data(), 100, nullptr) == PCS_ERR_INVALID);
    // tuning and counters
    const int64_t nt = pcs_get_tuning(PCS_TUNE_NT_LOADS);
    CHECK(nt >= 0);
    CHECK(pcs_set_tuning(PCS_TUNE_NT_LOADS, 0) == PCS_OK && pcs_get_tuning(PCS_TUNE_NT_LOADS) == 0);
    CHECK(pcs_set_tuning(PCS_TUNE_NT_LOADS, nt) == PCS_OK);
    CHECK(pcs_set_tuning(PCS_TUNE_NT_LOADS, -1) == PCS_ERR_INVALID);
    CHECK(pcs_set_tuning(12345, 1) == PCS_ERR_INVALID && pcs_get_tuning(12345) == -1);
    CHECK(pcs_set_tuning(-7, 1) == PCS_ERR_INVALID && pcs_get_tuning(-7) == -1);
    CHECK(pcs_counter(-1) == 0 && pcs_counter(3) == 0);
    CHECK(std::strstr(pcs_version(), "gfx950") != nullptr);
}

// pcs_last_error is per thread: one thread's failure does not overwrite another's message
static void last_error_threads() {
    std::vector<std::thread> th;
    std::vector<int> good(8, 0);
    for (int t = 0; t < 8; ++t)
        th.emplace_back([t, &good] {
            for (int i = 0; i < 200; ++i) {
                uint64_t b, e;
                if (t % 2) {
                    (void)pcs_shard_range(1, 0, 0, &b, &e);
                    good[t] += std::string(pcs_last_error()).find("rank must be") != std::string::npos;
                } else {
                    (void)pcs_set_tuning(99999, 1);
                    good[t] += std::string(pcs_last_error()).find("tuning") != std::string::npos;
                }
            }
        });
    for (auto& x : th) x.join();
    for (int t = 0; t < 8; ++t) CHECK(good[t] == 200);
}

// ABI 4 additions without a device: pcs_abi_version, pcs_service_start_ex's
// argument checks (made before the device is looked up), PCS_TUNE_FAIL_INJECT
// (consumed by the next k host-batch calls, never by skip_verify), and the
// non-aborting C++ forms the INTEGRATION.md §6 fallback is built on
static void abi4_no_device() {
    CHECK(pcs_abi_version() == PCS_ABI_VERSION && PCS_ABI_VERSION >= 4);
    CHECK(pcs_service_start_ex(0, 4, 0) == PCS_ERR_INVALID);
    CHECK(std::strstr(pcs_last_error(), "lines must be") != nullptr);
    CHECK(pcs_service_start_ex(9, 1, 0) == PCS_ERR_INVALID);
    CHECK(pcs_service_start_ex(8, 33, 0) == PCS_ERR_INVALID);
    CHECK(std::strstr(pcs_last_error(), "workgroups must be") != nullptr);
    CHECK(pcs_service_start_ex(2, 0, 0) == PCS_ERR_INVALID);
    CHECK(pcs_service_start_ex(2, 4, 150) == PCS_ERR_INVALID);
    CHECK(pcs_service_start_ex(8, 32, 0) == PCS_ERR_NO_DEVICE);  // 256 workgroups: arguments fine
    CHECK(pcs_counter(PCS_COUNTER_SERVICE_TORN_REQUESTS) == 0);
    CHECK(pcs_get_tuning(PCS_TUNE_SERVICE_MAX_CALLERS) == 2 && pcs_get_tuning(29) == -1);
    CHECK(pcs_get_tuning(PCS_TUNE_FAIL_INJECT) == 0 && pcs_get_tuning(PCS_TUNE_SERVICE_TEAR_TEST) == 0);
    // ABI 5: the re-post drill knob and counter
    CHECK(PCS_ABI_VERSION >= 5 && pcs_get_tuning(PCS_TUNE_SERVICE_REPOST_TEST) == 0);
    CHECK(pcs_counter(PCS_COUNTER_SERVICE_REPOSTS) == 0 && pcs_get_tuning(37) == -1);
    // ABI 6: the slow-exit test knob, the path bits and the thread prepare
    CHECK(PCS_ABI_VERSION >= 6 && pcs_get_tuning(PCS_TUNE_SERVICE_SLOW_EXIT_TEST) == 0);
    CHECK(pcs_get_tuning(PCS_TUNE_ZC_BATCH_EVENT) == 0 && pcs_get_tuning(PCS_TUNE_SYNC_SPIN_US) == 0);
    CHECK(pcs_get_tuning(PCS_TUNE_SERVICE_DEPARTURE) == 1);
    CHECK((pcs_last_path() & ~63) == 0 && pcs_batch_path(nullptr) == 0);
    CHECK(pcs_thread_prepare() == PCS_ERR_NO_DEVICE);
    CHECK(pcs_get_tuning(32) == -1 && pcs_set_tuning(32, 2) == PCS_ERR_INVALID);  // retired (round 5)
    CHECK(pcs_get_tuning(PCS_TUNE_ZC_STAMP_POLL_PAGES) == 256);
    // a huge gate knob is accepted (it acts as 2^20 callers: never closes)
    CHECK(pcs_set_tuning(PCS_TUNE_SERVICE_MAX_CALLERS, INT64_MAX) == PCS_OK);
    CHECK(pcs_set_tuning(PCS_TUNE_SERVICE_MAX_CALLERS, 2) == PCS_OK);

    std::vector<char> page(4096, 0x33);
    const char* cpages[1] = {page.data()};
    char* wpages[1] = {page.data()};
    uint8_t ok[1] = {7};
    size_t fb = 99;
    CHECK(pcs_set_tuning(PCS_TUNE_FAIL_INJECT, 2) == PCS_OK);
    // skip_verify never reaches the GPU and leaves the injections alone
    CHECK(eloqstore::TryValidateChecksums(cpages, 4096, ok, &fb, eloqstore::PageHash::XXH3_64, true) == PCS_OK);
    CHECK(ok[0] == 1 && fb == 1 && pcs_get_tuning(PCS_TUNE_FAIL_INJECT) == 2);
    fb = 99;
    CHECK(eloqstore::TryValidateChecksums(cpages, 4096, ok, &fb) == PCS_ERR_HIP && fb == 99);
    CHECK(std::strstr(eloqstore::LastChecksumError(), "injected failure") != nullptr);
    CHECK(eloqstore::TrySetChecksums(wpages, 4096) == PCS_ERR_HIP);
    CHECK(pcs_get_tuning(PCS_TUNE_FAIL_INJECT) == 0 && page[0] == 0x33);
    // the manifest host calls consume injections too
    CHECK(pcs_set_tuning(PCS_TUNE_FAIL_INJECT, 2) == PCS_OK);
    uint64_t h = 0;
    int valid = 7;
    CHECK(pcs_manifest_checksum_host(page.data(), page.size(), &h) == PCS_ERR_HIP);
    CHECK(pcs_manifest_validate_host(page.data(), page.size(), &valid) == PCS_ERR_HIP && valid == 7);
    CHECK(pcs_get_tuning(PCS_TUNE_FAIL_INJECT) == 0);
    CHECK(pcs_manifest_checksum_host(page.data(), page.size(), &h) == PCS_ERR_NO_DEVICE);
    // injections spent: the plain no-device failure again
    CHECK(eloqstore::TryValidateChecksums(cpages, 4096, ok, &fb) == PCS_ERR_NO_DEVICE);
    CHECK(std::strstr(eloqstore::LastChecksumError(), "no usable HIP device") != nullptr);
    CHECK(eloqstore::TrySetChecksums(wpages, 4096, eloqstore::PageHash::XXH64) == PCS_ERR_NO_DEVICE);
    CHECK(pcs_set_tuning(PCS_TUNE_FAIL_INJECT, -1) == PCS_ERR_INVALID);

    // a batch that could not be created reports why on every call, never aborts
    eloqstore::ChecksumBatch cb;
    CHECK(cb.Status() == PCS_ERR_NO_DEVICE);
    CHECK(cb.TrySubmitValidate(cpages, 4096) == PCS_ERR_NO_DEVICE);
    CHECK(cb.TrySubmitValidate(cpages, 4096, eloqstore::PageHash::XXH3_64, true) == PCS_ERR_NO_DEVICE);
    CHECK(cb.TrySubmitStamp(wpages, 4096) == PCS_ERR_NO_DEVICE);
    CHECK(cb.TryPoll() == PCS_ERR_NO_DEVICE);
}

int main() {
    shard_ranges();
    no_device();
    arguments();
    last_error_threads();
    abi4_no_device();
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("capi_sanitize_test: all checks passed\n");
    return 0;
}
