// service_poll_lab.cpp — validate-service latency against the number of
// request-line polls each polling lane keeps in flight
// (32 /* PCS_TUNE_SERVICE_POLL_DEPTH, retired */ 1 / 2 / 4).  Not part of the product.  One
// thread, a registered 1 GiB pool of 4 KiB pages, random pages per call.
// The depth is read when a service kernel is queued, so each round sets it,
// restarts the service (4 workgroups, one line, 1 ms idle), warms 50 calls
// and times 300 calls per page count (page counts shuffled per repetition);
// rounds cycle the depths (1 2 4 1 2 4 ...), medians over all rounds.
//
// Result (profiles/r05/service_poll_lab_r05k.txt): depth 1 fastest; the knob
// (key 32) and the templated kernel were retired after this run, so this
// lab now builds against raw key 32, which the library refuses.
//
//   make -C tools/lab $PWD/tools/lab/service_poll_lab && ./tools/lab/service_poll_lab [rounds]
#include "eloqstore_pcs.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <vector>

#include "xxh_oracle.h"

#define CHECK(c)                                                                                  \
    do {                                                                                          \
        if (!(c)) {                                                                               \
            std::fprintf(stderr, "%s:%d CHECK(%s) %s\n", __FILE__, __LINE__, #c, pcs_last_error()); \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

int main(int argc, char** argv) {
    using clk = std::chrono::steady_clock;
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 6;
    const size_t P = 4096, NP = size_t(1) << 18;
    char* pool = static_cast<char*>(std::aligned_alloc(4096, NP * P));
    CHECK(pool);
    oracle_fill_pages(pool, P, NP, 0x9011, 0);
    for (size_t i = 0; i < NP; ++i) oracle_set_checksum(pool + i * P, P);
    CHECK(pcs_host_register(pool, NP * P) == PCS_OK);
    const std::vector<size_t> sizes = {1, 6, 32, 128};
    const int depths[] = {1, 2, 4};
    std::map<std::pair<int, size_t>, std::vector<double>> sync_us, async_us;
    std::mt19937_64 rng(3);
    pcs_batch* b = nullptr;
    CHECK(pcs_batch_create(&b) == PCS_OK);
    for (int r = 0; r < rounds * 3; ++r) {
        const int depth = depths[r % 3];
        CHECK(pcs_set_tuning(32 /* PCS_TUNE_SERVICE_POLL_DEPTH, retired */, depth) == PCS_OK);
        CHECK(pcs_service_start_ex(1, 4, 1000) == PCS_OK);
        const uint64_t served0 = pcs_counter(PCS_COUNTER_SERVICE_BATCHES);
        uint64_t calls = 0;
        for (int rep = 0; rep < 350; ++rep) {
            std::vector<size_t> order = sizes;
            std::shuffle(order.begin(), order.end(), rng);
            for (size_t n : order)
                for (int async = 0; async < 2; ++async) {
                    std::vector<const void*> ptrs(n);
                    for (auto& p : ptrs) p = pool + (rng() % NP) * P;
                    std::vector<uint8_t> ok(n);
                    uint64_t fb = 0;
                    const auto t0 = clk::now();
                    if (async) {
                        CHECK(pcs_batch_submit(b, 1, ptrs.data(), P, n, 0) == PCS_OK);
                        int x;
                        while ((x = pcs_batch_poll(b)) == 0) {
                        }
                        CHECK(x == 1);
                    } else {
                        CHECK(pcs_pages_validate_host(ptrs.data(), P, n, 0, ok.data(), &fb) == PCS_OK);
                        CHECK(fb == UINT64_MAX);
                    }
                    const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
                    ++calls;
                    if (rep >= 50) (async ? async_us : sync_us)[{depth, n}].push_back(us);
                }
        }
        CHECK(pcs_counter(PCS_COUNTER_SERVICE_BATCHES) - served0 == calls);
        CHECK(pcs_service_stop() == PCS_OK);
    }
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    auto pct = [](std::vector<double> v, double q) {
        std::sort(v.begin(), v.end());
        return v[std::min(v.size() - 1, (size_t)(q * v.size()))];
    };
    std::printf("depth  pages  sync p50  sync p99  async p50  (us; %d rounds per depth, all served)\n", rounds);
    for (int d : depths)
        for (size_t n : sizes)
            std::printf("%5d  %5zu  %8.2f  %8.2f  %9.2f\n", d, n, med(sync_us[{d, n}]), pct(sync_us[{d, n}], 0.99),
                        med(async_us[{d, n}]));
    pcs_batch_destroy(b);
    CHECK(pcs_set_tuning(32 /* PCS_TUNE_SERVICE_POLL_DEPTH, retired */, 1) == PCS_OK);
    CHECK(pcs_host_unregister(pool) == PCS_OK);
    std::free(pool);
    return 0;
}
