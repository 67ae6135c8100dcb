// service_load.cpp — small read batches under load: the validate service
// against the launch path and the reference loop.  Not part of the product.
//
// EloqStore's most frequent ReadPages batches are small: the scan prefetch
// reads 6 pages by default (types.h:31, scan_task.cpp:215).  T shard threads
// (kv_options.h:29) each validate batches of B random pages of a registered
// 1 GiB pool back to back with the synchronous drop-in call
// (eloqstore::ValidateChecksums), in three modes:
//   launch   the launch path (one zero-copy launch per batch, its own stream
//            per thread);
//   service  the same calls with the validate service on (4 workgroups): one
//            request at a time goes through the device's request line, a call
//            that finds it busy takes the launch path;
//   cpu      the reference's own loop (XXH3_64bits over [8, P) per page,
//            oracle/_ref's build of external/xxhash.c).
// Output per (mode, B, T): batches/s over all threads, pages/s, and per-batch
// latency p50 / p99.
//
//   make -C tools/lab && ./tools/lab/service_load [seconds_per_point]
#include "eloqstore/page_checksum.h"
#include "eloqstore_pcs.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

extern "C" uint64_t XXH3_64bits(const void* input, size_t length);  // oracle/_ref (reference build)

using Clock = std::chrono::steady_clock;

namespace {
constexpr size_t P = 4096;

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Point {
    double batches_per_s = 0, p50_us = 0, p99_us = 0;
    uint64_t batches = 0, bad = 0, min_thread = 0, max_thread = 0;  // batches of the least / most served thread
};

enum Mode { kLaunch, kService, kCpu };

Point run(char* pool, size_t np, Mode mode, size_t B, int T, double secs) {
    std::atomic<uint64_t> batches{0}, bad{0};
    std::vector<std::vector<float>> lat(T);
    std::vector<uint64_t> per(T, 0);
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    Clock::time_point t0, stop;
    std::vector<std::thread> th;
    for (int k = 0; k < T; ++k)
        th.emplace_back([&, k] {
            uint64_t rng = 0x10AD0000ull + (uint64_t)k * 7919 + B;
            std::vector<const char*> ptrs(B);
            std::vector<uint8_t> ok(B);
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) {
            }
            uint64_t n = 0, nbad = 0;
            lat[k].reserve(1 << 16);
            while (Clock::now() < stop) {
                for (auto& p : ptrs) p = pool + (splitmix(rng) % np) * P;
                const auto a = Clock::now();
                if (mode == kCpu) {
                    for (size_t i = 0; i < B; ++i) {
                        uint64_t stored;
                        std::memcpy(&stored, ptrs[i], 8);
                        if (XXH3_64bits(ptrs[i] + 8, P - 8) != stored) {
                            ++nbad;
                            break;
                        }
                    }
                } else if (eloqstore::ValidateChecksums(ptrs, P, ok.data()) != B) {
                    ++nbad;
                }
                const auto b = Clock::now();
                lat[k].push_back((float)std::chrono::duration<double, std::micro>(b - a).count());
                ++n;
            }
            batches.fetch_add(n);
            bad.fetch_add(nbad);
            per[k] = n;
        });
    while (ready.load() < T) {
    }
    t0 = Clock::now();
    stop = t0 + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(secs));
    go.store(true, std::memory_order_release);
    for (auto& t : th) t.join();
    const double el = std::chrono::duration<double>(Clock::now() - t0).count();
    std::vector<float> all;
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    Point r;
    r.batches = batches.load();
    r.batches_per_s = r.batches / el;
    r.p50_us = all.empty() ? 0 : all[all.size() / 2];
    r.p99_us = all.empty() ? 0 : all[std::min(all.size() - 1, all.size() * 99 / 100)];
    r.bad = bad.load();
    r.min_thread = *std::min_element(per.begin(), per.end());
    r.max_thread = *std::max_element(per.begin(), per.end());
    return r;
}
}  // namespace

int main(int argc, char** argv) {
    const double secs = argc > 1 ? std::atof(argv[1]) : 1.0;
    const size_t np = size_t(1) << 18;  // 1 GiB of 4 KiB pages
    char* pool = static_cast<char*>(std::aligned_alloc(4096, np * P));
    if (!pool) return 1;
    uint64_t s = 0xC0FFEE;
    for (size_t i = 0; i < np * P / 8; ++i) {
        const uint64_t w = splitmix(s);
        std::memcpy(pool + i * 8, &w, 8);
    }
    for (size_t i = 0; i < np; ++i) {
        const uint64_t h = XXH3_64bits(pool + i * P + 8, P - 8);
        std::memcpy(pool + i * P, &h, 8);  // EncodeFixed64 (LE)
    }
    eloqstore::RegisterPagePool(pool, np * P);
    std::printf("mode     pages  threads  batches/s  pages/s     p50_us  p99_us  bad  served_share  thread_min  thread_max\n");
    uint64_t total_bad = 0;
    // argv[2]: service stream kinds to run (PCS_TUNE_SERVICE_STREAM digits:
    // 1 highest priority, 0 plain), default "1"
    const char* kinds = argc > 2 ? argv[2] : "1";
    std::vector<int> modes = {kCpu, kLaunch};
    for (const char* k = kinds; *k; ++k) modes.push_back(100 + (*k - '0'));
    for (size_t B : {6, 32, 128})
        for (int mm : modes)
            for (int T : {1, 2, 4, 8, 16}) {
                const Mode m = mm >= 100 ? kService : (Mode)mm;
                if (m == kService) {
                    pcs_set_tuning(PCS_TUNE_SERVICE_STREAM, mm - 100);
                    eloqstore::StartChecksumService(4, 1000);
                }
                const uint64_t served0 = pcs_counter(PCS_COUNTER_SERVICE_BATCHES);
                const Point r = run(pool, np, m, B, T, secs);
                const uint64_t served = pcs_counter(PCS_COUNTER_SERVICE_BATCHES) - served0;
                if (m == kService) eloqstore::StopChecksumService();
                const uint64_t total = r.batches;
                if ((m == kService) != (served > 0)) {
                    std::printf("path check failed: mode %d served %llu\n", (int)m, (unsigned long long)served);
                    return 1;
                }
                total_bad += r.bad;
                char name[16];
                std::snprintf(name, sizeof name, "%s", m == kCpu ? "cpu" : m == kLaunch ? "launch" : "service");
                if (m == kService) std::snprintf(name, sizeof name, "service%d", mm - 100);
                std::printf("%-8s %5zu  %7d  %9.0f  %10.0f  %6.1f  %6.1f  %llu  %12.2f  %10llu  %10llu\n",
                            name, B, T, r.batches_per_s,
                            r.batches_per_s * B, r.p50_us, r.p99_us, (unsigned long long)r.bad,
                            total ? (double)served / (double)total : 0.0, (unsigned long long)r.min_thread,
                            (unsigned long long)r.max_thread);
                std::fflush(stdout);
            }
    eloqstore::UnregisterPagePool(pool);
    std::free(pool);
    return total_bad ? 2 : 0;
}
