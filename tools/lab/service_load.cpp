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
//            that finds it busy takes the launch path; `service<k>` runs with
//            the stream kind k (PCS_TUNE_SERVICE_STREAM) and the contention
//            gate off, `gated<k>` with the gate at its default (2 callers);
//   cpu      the reference's own loop (XXH3_64bits over [8, P) per page,
//            oracle/_ref's build of external/xxhash.c).
// Output per (mode, B, T): batches/s over all threads, pages/s, and per-batch
// latency p50 / p99.
//
// Every thread keeps a phase marker (what it is doing, since when); a
// watchdog thread prints the markers and a backtrace of every thread stuck in
// one phase for more than 3 s, then exits, so a stall names its blocking call
// instead of ending in a silent hang.
//
//   make -C tools/lab && ./tools/lab/service_load [seconds_per_point] [kinds] [pages]
#include "eloqstore/page_checksum.h"
#include "eloqstore_pcs.h"

#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>

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

// ---- phase markers + stall watchdog --------------------------------------
enum Phase { kIdle, kPickPages, kValidate, kCpuLoop, kStartService, kStopService, kRegister, kNumPhases };
const char* const kPhaseName[kNumPhases] = {"idle", "pick pages", "ValidateChecksums", "reference loop",
                                            "StartChecksumService", "StopChecksumService", "RegisterPagePool"};
struct Marker {
    std::atomic<int> phase{kIdle};
    std::atomic<int64_t> since_ns{0};
    std::atomic<pthread_t> tid{};
    std::atomic<bool> live{false};
};
constexpr int kMaxMarkers = 64;
Marker g_mark[kMaxMarkers];  // 0: main thread, 1 + k: worker k
int64_t now_ns() { return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count(); }
void mark(int slot, Phase p) {
    g_mark[slot].since_ns.store(now_ns(), std::memory_order_relaxed);
    g_mark[slot].phase.store(p, std::memory_order_release);
}
void mark_thread(int slot) {
    g_mark[slot].tid.store(pthread_self());
    g_mark[slot].live.store(true);
    mark(slot, kIdle);
}
void on_dump(int) {  // async-signal-safe enough for a dying lab: backtrace to stderr
    void* fr[48];
    const int n = backtrace(fr, 48);
    backtrace_symbols_fd(fr, n, 2);
    const char sep[] = "----\n";
    (void)!write(2, sep, sizeof sep - 1);
}
void watchdog() {
    for (;;) {
        std::this_thread::sleep_for(std::chrono::milliseconds(500));
        const int64_t t = now_ns();
        bool stuck = false;
        for (auto& m : g_mark)
            if (m.live.load() && m.phase.load() != kIdle && t - m.since_ns.load() > 3'000'000'000ll) stuck = true;
        if (!stuck) continue;
        std::fprintf(stderr, "STALL: phase markers (thread slot: phase, seconds in it)\n");
        for (int k = 0; k < kMaxMarkers; ++k) {
            Marker& m = g_mark[k];
            if (!m.live.load()) continue;
            const double secs = (t - m.since_ns.load()) / 1e9;
            std::fprintf(stderr, "  slot %d: %s, %.2f s\n", k, kPhaseName[m.phase.load()], secs);
            if (m.phase.load() != kIdle && secs > 3.0) {
                std::fprintf(stderr, "  backtrace of slot %d:\n", k);
                std::fflush(stderr);
                pthread_kill(m.tid.load(), SIGUSR1);
                std::this_thread::sleep_for(std::chrono::milliseconds(200));
            }
        }
        std::fflush(stderr);
        _exit(3);
    }
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
            mark_thread(1 + k);
            uint64_t rng = 0x10AD0000ull + (uint64_t)k * 7919 + B;
            std::vector<const char*> ptrs(B);
            std::vector<uint8_t> ok(B);
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) {
            }
            uint64_t n = 0, nbad = 0;
            lat[k].reserve(1 << 16);
            while (Clock::now() < stop) {
                mark(1 + k, kPickPages);
                for (auto& p : ptrs) p = pool + (splitmix(rng) % np) * P;
                mark(1 + k, mode == kCpu ? kCpuLoop : kValidate);
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
                mark(1 + k, kIdle);
                lat[k].push_back((float)std::chrono::duration<double, std::micro>(b - a).count());
                ++n;
            }
            batches.fetch_add(n);
            bad.fetch_add(nbad);
            per[k] = n;
            g_mark[1 + k].live.store(false);
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
    signal(SIGUSR1, on_dump);
    mark_thread(0);
    std::thread(watchdog).detach();
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
    mark(0, kRegister);
    eloqstore::RegisterPagePool(pool, np * P);
    mark(0, kIdle);
    std::printf("mode     pages  threads  batches/s  pages/s     p50_us  p99_us  bad  served_share  thread_min  thread_max\n");
    uint64_t total_bad = 0;
    // argv[2]: service runs, one letter-digit pair each: s<k> = gate off,
    // g<k> = gate at its default (2 callers), k = PCS_TUNE_SERVICE_STREAM
    // (1 highest priority, 0 plain); L<n> / M<n> / N<n> = n request lines of
    // one / two / four workgroups each, gate at its default, highest-priority
    // stream; default "s1g1".
    // argv[3]: batch sizes, comma-separated (default 6,32,128).
    const char* kinds = argc > 2 ? argv[2] : "s1g1";
    std::vector<int> modes = {kCpu, kLaunch};
    for (const char* k = kinds; k[0] && k[1]; k += 2)
        modes.push_back((k[0] == 'g' ? 200 : k[0] == 'L' ? 300 : k[0] == 'M' ? 400 : k[0] == 'N' ? 500 : 100) +
                        (k[1] - '0'));
    std::vector<size_t> sizes;
    for (const char* b = argc > 3 ? argv[3] : "6,32,128"; *b;) {
        sizes.push_back(std::strtoul(b, const_cast<char**>(&b), 10));
        if (*b == ',') ++b;
    }
    for (size_t B : sizes)
        for (int mm : modes)
            for (int T : {1, 2, 4, 8, 16}) {
                const Mode m = mm >= 100 ? kService : (Mode)mm;
                const bool gated = mm >= 200;
                const int lines = mm >= 300 ? mm % 100 : 1;
                const int wpl = mm >= 500 ? 4 : mm >= 400 ? 2 : mm >= 300 ? 1 : 4;
                if (m == kService) {
                    pcs_set_tuning(PCS_TUNE_SERVICE_STREAM, mm >= 300 ? 1 : mm % 100);
                    pcs_set_tuning(PCS_TUNE_SERVICE_MAX_CALLERS, gated ? 2 : 0);
                    mark(0, kStartService);
                    eloqstore::StartChecksumService(wpl, 1000, lines);
                    mark(0, kIdle);
                }
                const uint64_t served0 = pcs_counter(PCS_COUNTER_SERVICE_BATCHES);
                const Point r = run(pool, np, m, B, T, secs);
                const uint64_t served = pcs_counter(PCS_COUNTER_SERVICE_BATCHES) - served0;
                if (m == kService) {
                    mark(0, kStopService);
                    eloqstore::StopChecksumService();
                    mark(0, kIdle);
                }
                const uint64_t total = r.batches;
                if (m != kService && served > 0) {
                    std::printf("path check failed: mode %d served %llu\n", (int)m, (unsigned long long)served);
                    return 1;
                }
                total_bad += r.bad;
                char name[16];
                std::snprintf(name, sizeof name, "%s", m == kCpu ? "cpu" : "launch");
                if (m == kService)
                    std::snprintf(name, sizeof name, "%s%d", mm >= 300 ? (wpl == 1 ? "L1x" : wpl == 2 ? "L2x" : "L4x")
                                                                    : gated ? "gated" : "service", mm % 100);
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
