// shard_sim.cpp — EloqStore's read and write checksum paths under load.  Not part of the product.
//
// IouringMgr::ReadPages checks up to max_read_pages_batch = 128 pages per
// batch (async_io_manager.cpp:353-366, kv_options.h:18-19), one shard thread
// per core (kv_options.h:29), coroutines yielding while I/O is in flight
// (shard.cpp:67-130).  This harness drives that pattern through the drop-in
// API: T shard threads, each keeping Q batches of 128 pages in flight with
// eloqstore::ChecksumBatch (SubmitValidate, then Poll() from the work loop),
// pages drawn at random from a page pool registered once
// (eloqstore::RegisterPagePool, PagesPool chunks of 1024 pages, page.cpp:95-120),
// so every batch is one zero-copy launch over PCIe.  The same T threads then
// run the reference's own loop: XXH3_64bits over [8, P) per page compared with
// the stored digest (ValidateChecksum, page.cpp:25-31), linked from the
// reference's external/xxhash.c build (oracle/_ref, test infrastructure).
//
// The write path (FlushBatchPages, write_task.cpp:155-167; write batches of
// up to 256 pages, kv_options.h:70) is driven the same way with SubmitStamp
// against the reference's SetChecksum loop.
//
// Output per (T, Q): pages/s, GiB/s, batch latency p50 / p99 (GPU) and
// pages/s, GiB/s (CPU).
//
//   make -C tools/lab && ./tools/lab/shard_sim [seconds_per_point] [pool_GiB]
#include "eloqstore/page_checksum.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" uint64_t XXH3_64bits(const void* input, size_t length);  // oracle/_ref (reference build)

using Clock = std::chrono::steady_clock;
using namespace eloqstore;

namespace {
constexpr size_t P = 4096;
constexpr size_t kChunkPages = 1024;
constexpr size_t kReadBatch = 128;   // max_read_pages_batch (kv_options.h:18-19)
constexpr size_t kWriteBatch = 256;  // write batch (kv_options.h:70)

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Result {
    double pages_per_s = 0, gib_s = 0, p50_us = 0, p99_us = 0;
    uint64_t bad = 0;
};

// write = false: ReadPages validation (SubmitValidate); true: FlushBatchPages
// stamping (SubmitStamp writes the digests into the pool pages).
Result run_gpu(const std::vector<char*>& pool, int T, int Q, double secs, bool write) {
    const size_t kBatch = write ? kWriteBatch : kReadBatch;
    std::atomic<uint64_t> pages{0}, bad{0};
    std::vector<std::vector<float>> lat(T);
    const auto t0 = Clock::now();
    const auto stop = t0 + std::chrono::duration<double>(secs);
    std::vector<std::thread> th;
    for (int k = 0; k < T; ++k)
        th.emplace_back([&, k] {
            uint64_t rng = 0x5EED5EEDull + (uint64_t)k * 7919;
            std::vector<ChecksumBatch> b(Q);
            std::vector<std::vector<char*>> ptrs(Q, std::vector<char*>(kBatch));
            std::vector<Clock::time_point> sub(Q);
            std::vector<bool> busy(Q, false);
            uint64_t done = 0, nbad = 0;
            auto submit = [&](int i) {
                for (auto& p : ptrs[i]) p = pool[splitmix(rng) % pool.size()];
                sub[i] = Clock::now();
                if (write) b[i].SubmitStamp(ptrs[i], P);
                else b[i].SubmitValidate(std::span<const char* const>(ptrs[i].data(), kBatch), P);
                busy[i] = true;
            };
            for (int i = 0; i < Q; ++i) submit(i);
            while (true) {
                bool any = false;
                for (int i = 0; i < Q; ++i) {
                    if (!busy[i]) continue;
                    any = true;
                    if (!b[i].Poll()) continue;
                    const auto now = Clock::now();
                    lat[k].push_back(std::chrono::duration<float, std::micro>(now - sub[i]).count());
                    if (!write) nbad += b[i].FirstBad() != kBatch;
                    done += kBatch;
                    busy[i] = false;
                    if (now < stop) submit(i);
                }
                if (!any) break;
            }
            pages += done;
            bad += nbad;
        });
    for (auto& x : th) x.join();
    const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
    std::vector<float> all;
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    Result r;
    r.pages_per_s = pages / dt;
    r.gib_s = pages * (double)P / dt / (1u << 30);
    r.p50_us = all.empty() ? 0 : all[all.size() / 2];
    r.p99_us = all.empty() ? 0 : all[all.size() * 99 / 100];
    r.bad = bad;
    return r;
}

Result run_cpu(const std::vector<char*>& pool, int T, double secs, bool write) {
    const size_t kBatch = write ? kWriteBatch : kReadBatch;
    std::atomic<uint64_t> pages{0}, bad{0};
    const auto t0 = Clock::now();
    const auto stop = t0 + std::chrono::duration<double>(secs);
    std::vector<std::thread> th;
    for (int k = 0; k < T; ++k)
        th.emplace_back([&, k] {
            uint64_t rng = 0xC0FFEEull + (uint64_t)k * 7919;
            uint64_t done = 0, nbad = 0;
            while (Clock::now() < stop) {
                for (size_t j = 0; j < kBatch; ++j) {  // one batch, page by page (page.cpp:18-31)
                    char* p = pool[splitmix(rng) % pool.size()];
                    const uint64_t h = XXH3_64bits(p + 8, P - 8);
                    if (write) {
                        std::memcpy(p, &h, 8);  // SetChecksum: EncodeFixed64
                    } else {
                        uint64_t stored;
                        std::memcpy(&stored, p, 8);
                        nbad += h != stored;
                    }
                }
                done += kBatch;
            }
            pages += done;
            bad += nbad;
        });
    for (auto& x : th) x.join();
    const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
    Result r;
    r.pages_per_s = pages / dt;
    r.gib_s = pages * (double)P / dt / (1u << 30);
    r.bad = bad;
    return r;
}
}  // namespace

int main(int argc, char** argv) {
    const double secs = argc > 1 ? std::atof(argv[1]) : 2.0;
    const double pool_gib = argc > 2 ? std::atof(argv[2]) : 1.0;
    const size_t chunks = std::max<size_t>(1, (size_t)(pool_gib * (1u << 30) / (kChunkPages * P)));
    std::vector<char*> chunk(chunks), pool;
    uint64_t seed = 1;
    for (auto& c : chunk) {
        c = static_cast<char*>(std::aligned_alloc(4096, kChunkPages * P));
        auto* w = reinterpret_cast<uint64_t*>(c);
        for (size_t i = 0; i < kChunkPages * P / 8; ++i) w[i] = splitmix(seed);
        RegisterPagePool(c, kChunkPages * P);
        for (size_t j = 0; j < kChunkPages; ++j) pool.push_back(c + j * P);
    }
    for (size_t i = 0; i < pool.size(); i += 65536) {  // stamp the pool (SetChecksums, write_task.cpp:155-167)
        const size_t n = std::min<size_t>(65536, pool.size() - i);
        SetChecksums(std::span<char* const>(pool.data() + i, n), P);
    }
    std::printf("pool: %zu pages of %zu B (%.2f GiB) in %zu registered chunks; %.1f s per point\n", pool.size(), P,
                pool.size() * (double)P / (1u << 30), chunks, secs);
    for (bool write : {false, true}) {
        std::printf("%s: batches of %zu pages\n", write ? "write path (SubmitStamp / SetChecksum)"
                                                        : "read path (SubmitValidate / ValidateChecksum)",
                    write ? kWriteBatch : kReadBatch);
        std::printf("%-28s %12s %9s %9s %9s %5s\n", "mode", "pages/s", "GiB/s", "p50 us", "p99 us", "bad");
        for (int T : {1, 2, 4, 8}) {
            for (int Q : {1, 4, 8}) {
                const Result r = run_gpu(pool, T, Q, secs, write);
                std::printf("gpu  T=%d Q=%d                 %12.0f %9.2f %9.1f %9.1f %5llu\n", T, Q, r.pages_per_s,
                            r.gib_s, r.p50_us, r.p99_us, (unsigned long long)r.bad);
                std::fflush(stdout);
            }
            const Result c = run_cpu(pool, T, secs, write);
            std::printf("cpu  T=%d (reference loop)     %12.0f %9.2f %9s %9s %5llu\n", T, c.pages_per_s, c.gib_s, "-",
                        "-", (unsigned long long)c.bad);
            std::fflush(stdout);
        }
    }
    // the pool must still validate after both stamping runs
    std::vector<uint8_t> ok(65536);
    size_t bad = 0;
    for (size_t i = 0; i < pool.size(); i += 65536) {
        const size_t n = std::min<size_t>(65536, pool.size() - i);
        const size_t fb = ValidateChecksums(std::span<const char* const>(pool.data() + i, n), P, ok.data());
        bad += fb != n;
    }
    std::printf("pool re-validated after stamping: %s\n", bad ? "FAILED" : "ok");
    if (bad) return 1;
    for (auto& c : chunk) {
        UnregisterPagePool(c);
        std::free(c);
    }
    return 0;
}
