// async_lab.cpp — why is an async zero-copy validate of 192-256 pages ~4.5 us
// slower than the same synchronous call (profiles/r05/crossover_r05e.txt,
// r05f), when at <= 128 pages the two are within 0.3 us?  Not part of the
// product.  One thread, a registered 1 GiB pool of 4 KiB pages, random pages
// per call; per page count, the columns below in a fresh random order every
// repetition, median of 400:
//   sync        pcs_pages_validate_host (thread context, zero-copy)
//   async       pcs_batch_submit + pcs_batch_poll spin, batch A (created first)
//   async_late  the same on batch B, created after the sync path's streams
//   async_wait  batch A, pcs_batch_wait instead of the poll spin
//   stamp_sync / stamp_async  SetChecksums vs SubmitStamp + poll
//   async_noinl batch A with PCS_TUNE_INLINE_LIST = 0 (list read from host)
//   sync_noinl  the same for the sync call
//
//   make -C tools/lab async_lab && ./tools/lab/async_lab
#include "eloqstore_pcs.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "xxh_oracle.h"

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::fprintf(stderr, "%s:%d CHECK(%s) %s\n", __FILE__, __LINE__, #c, pcs_last_error()); \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

int main() {
    using clk = std::chrono::steady_clock;
    const size_t P = 4096, NP = size_t(1) << 18;
    pcs_batch* a = nullptr;
    CHECK(pcs_batch_create(&a) == PCS_OK);  // before anything else makes a stream
    char* pool = static_cast<char*>(std::aligned_alloc(4096, NP * P));
    CHECK(pool);
    oracle_fill_pages(pool, P, NP, 0xA5A5, 0);
    for (size_t i = 0; i < NP; ++i) oracle_set_checksum(pool + i * P, P);
    CHECK(pcs_host_register(pool, NP * P) == PCS_OK);
    std::vector<const void*> warm(8, pool);
    std::vector<uint8_t> okw(8);
    uint64_t fbw;
    CHECK(pcs_pages_validate_host(warm.data(), P, 8, 0, okw.data(), &fbw) == PCS_OK);
    // optionally run the gather path once (its three staging slots each make
    // a stream, as in integration_snippets --crossover): with GPU_MAX_HW_QUEUES
    // = 4 the process then has more streams than hardware queues
    if (std::getenv("ASYNC_LAB_GATHER")) {
        std::vector<char> heap(64 * P);
        for (int i = 0; i < 64; ++i) {
            oracle_fill_pages(heap.data() + i * P, P, 1, 0xBEEF, i);
            oracle_set_checksum(heap.data() + i * P, P);
        }
        std::vector<const void*> hp(64);
        for (int i = 0; i < 64; ++i) hp[i] = heap.data() + i * P;
        std::vector<uint8_t> okh(64);
        uint64_t fbh;
        CHECK(pcs_pages_validate_host(hp.data(), P, 64, 0, okh.data(), &fbh) == PCS_OK && fbh == UINT64_MAX);
        CHECK(pcs_counter(PCS_COUNTER_GATHER_CHUNKS) > 0);
        std::printf("(gather path run first: its staging streams exist)\n");
    }
    pcs_batch* b = nullptr;
    CHECK(pcs_batch_create(&b) == PCS_OK);
    std::mt19937_64 rng(7);
    std::printf("pages  sync  async  async_late  async_wait  async_noinl  sync_noinl  stamp_sync  stamp_async  (us)\n");
    for (size_t n : {64, 128, 160, 192, 256}) {
        std::vector<const void*> ptrs(n);
        std::vector<uint8_t> ok(n);
        uint64_t fb = 0;
        auto fill = [&] {
            for (auto& p : ptrs) p = pool + (rng() % NP) * P;
        };
        auto spin = [&](pcs_batch* x) {
            int r;
            while ((r = pcs_batch_poll(x)) == 0) {
            }
            CHECK(r == 1);
        };
        struct Col {
            const char* name;
            std::function<void()> pre, run, post;
            std::vector<double> us;
        };
        std::vector<Col> cols = {
            {"sync", fill, [&] { CHECK(pcs_pages_validate_host(ptrs.data(), P, n, 0, ok.data(), &fb) == PCS_OK); }, nullptr},
            {"async", fill, [&] { CHECK(pcs_batch_submit(a, 1, ptrs.data(), P, n, 0) == PCS_OK); spin(a); }, nullptr},
            {"async_late", fill, [&] { CHECK(pcs_batch_submit(b, 1, ptrs.data(), P, n, 0) == PCS_OK); spin(b); }, nullptr},
            {"async_wait", fill, [&] { CHECK(pcs_batch_submit(a, 1, ptrs.data(), P, n, 0) == PCS_OK);
                                       CHECK(pcs_batch_wait(a) == PCS_OK); }, nullptr},
            {"async_noinl", [&] { fill(); pcs_set_tuning(PCS_TUNE_INLINE_LIST, 0); },
             [&] { CHECK(pcs_batch_submit(a, 1, ptrs.data(), P, n, 0) == PCS_OK); spin(a); },
             [&] { pcs_set_tuning(PCS_TUNE_INLINE_LIST, 1); }},
            {"sync_noinl", [&] { fill(); pcs_set_tuning(PCS_TUNE_INLINE_LIST, 0); },
             [&] { CHECK(pcs_pages_validate_host(ptrs.data(), P, n, 0, ok.data(), &fb) == PCS_OK); },
             [&] { pcs_set_tuning(PCS_TUNE_INLINE_LIST, 1); }},
            {"stamp_sync", fill, [&] { CHECK(pcs_pages_stamp_host(const_cast<void* const*>(ptrs.data()), P, n, 0) == PCS_OK); }, nullptr},
            {"stamp_async", fill, [&] { CHECK(pcs_batch_submit(a, 2, ptrs.data(), P, n, 0) == PCS_OK); spin(a); }, nullptr},
        };
        std::vector<size_t> order(cols.size());
        for (size_t i = 0; i < order.size(); ++i) order[i] = i;
        for (int r = 0; r < 440; ++r) {
            std::shuffle(order.begin(), order.end(), rng);
            for (size_t k : order) {
                Col& c = cols[k];
                if (c.pre) c.pre();
                const auto t0 = clk::now();
                c.run();
                const auto t1 = clk::now();
                if (c.post) c.post();
                if (r >= 40) c.us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            }
        }
        std::printf("%5zu", n);
        for (Col& c : cols) {
            std::sort(c.us.begin(), c.us.end());
            std::printf("  %.1f", c.us[c.us.size() / 2]);
        }
        std::printf("\n");
    }
    pcs_batch_destroy(a);
    pcs_batch_destroy(b);
    CHECK(pcs_host_unregister(pool) == PCS_OK);
    std::free(pool);
    return 0;
}
