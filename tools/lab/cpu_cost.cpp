// cpu_cost.cpp — shard-thread CPU spent per GiB of pages checked, by form.
// Not part of the product.  VERDICT r05 #2: the offload's value for EloqStore
// is the shard-thread CPU it gives back; round 5 derived "~6 cores" from
// throughput ratios and never measured it.
//
// EloqStore validates up to max_read_pages_batch = 128 pages per ReadPages
// batch (async_io_manager.cpp:353-366, kv_options.h:18-19) and stamps up to
// 256 per FlushBatchPages (write_task.cpp:155-167, kv_options.h:70), on shard
// threads whose loop is Submit -> PollComplete -> ExecuteReadyTasks
// (shard.cpp:118-125).  For batches of random 4 KiB pages of a registered
// 1 GiB pool (PagesPool chunks of 1024 pages, page.cpp:95-120), each form
// runs on T shard threads for a fixed time, and every thread reads its own
// CLOCK_THREAD_CPUTIME_ID before and after:
//   ref      the reference loop: XXH3_64bits(page + 8, 4088) per page and the
//            header compare / store (page.cpp:18-31), linked from the
//            reference's own external/xxhash.c (oracle/_ref)
//   sync     ValidateChecksums / SetChecksums, service off: one zero-copy
//            launch per batch, the caller waiting (spinning) on it
//   service  the same with the validate service on (one request line per
//            thread, 4 workgroups each)
//   async    ChecksumBatch: SubmitValidate / SubmitStamp, then Poll() from a
//            work loop that runs ~10 us of other work between polls (Q
//            batches in flight per thread); the checksum's CPU is the
//            thread's CPU minus the other work's, which is calibrated
//            separately with the same clock, and (cross-check) the wall time
//            spent inside the library's calls
//   async_service  the same with the service on (Q lines per thread): a
//            submit is a mailbox write instead of a kernel launch
//   async_service_q1  one batch in flight per thread, so that eight threads
//            fit the service's eight request lines and its gate stays open
//   async_event  async with PCS_TUNE_ZC_BATCH_EVENT = 1 (round 5's event
//            recorded behind every zero-copy batch's kernel)
//   sync_sleep  sync with PCS_TUNE_SYNC_SPIN_US = 30: the caller spins 30 us,
//            then sleeps ~10 us between checks
// Output per form and thread count: GiB/s checked, shard-thread CPU seconds
// per GiB, and the CPU saved per GiB against the reference loop; then the
// cores a GPU frees at its host-fed rate.  Verdict flips are checked: every
// validate must find its pages good (the pool is stamped first).
//
//   make -C tools/lab cpu_cost && ./tools/lab/cpu_cost [seconds_per_point] [json_out]
#include "eloqstore/page_checksum.h"
#include "eloqstore_pcs.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <thread>
#include <vector>

extern "C" uint64_t XXH3_64bits(const void* input, size_t length);  // oracle/_ref (reference build)

using Clock = std::chrono::steady_clock;
using namespace eloqstore;

namespace {
constexpr size_t P = 4096;
constexpr size_t kChunkPages = 1024;

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double thread_cpu_s() {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// ~10 us of "other shard work" (coroutine bodies, index lookups): a fixed
// number of dependent integer steps, calibrated once
uint64_t g_work_iters = 1000;
__attribute__((noinline)) uint64_t other_work(uint64_t seed) {
    uint64_t x = seed;
    for (uint64_t i = 0; i < g_work_iters; ++i) x = x * 0x9E3779B97F4A7C15ull + (x >> 29);
    return x;
}
double calibrate_work() {  // CPU seconds of one other_work call
    for (int r = 0; r < 3; ++r) {
        const double t0 = thread_cpu_s();
        uint64_t sink = 0;
        for (int k = 0; k < 2000; ++k) sink += other_work(k);
        const double per = (thread_cpu_s() - t0) / 2000;
        if (sink == 42) std::puts("");
        g_work_iters = std::max<uint64_t>(16, (uint64_t)(g_work_iters * 10e-6 / per));
    }
    const double t0 = thread_cpu_s();
    uint64_t sink = 0;
    for (int k = 0; k < 20000; ++k) sink += other_work(k);
    const double per = (thread_cpu_s() - t0) / 20000;
    if (sink == 42) std::puts("");
    return per;
}

struct Point {
    std::string form, path;
    int T = 0, Q = 0;
    bool write = false;
    double gib = 0, wall_s = 0, cpu_s = 0, work_cpu_s = 0, in_call_s = 0, served = 0;
    uint64_t bad = 0, polls = 0, work_units = 0;
    double cpu_per_gib() const { return (cpu_s - work_cpu_s) / gib; }
};

Point run(const std::vector<char*>& pool, const std::string& form, int T, int Q, bool write, double secs,
          double work_cpu_per_unit) {
    const size_t kBatch = write ? 256 : 128;
    std::atomic<uint64_t> pages{0}, bad{0}, polls{0}, units{0};
    std::vector<double> cpu(T, 0), in_call(T, 0);
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<std::thread> th;
    for (int k = 0; k < T; ++k)
        th.emplace_back([&, k] {
            uint64_t rng = 0xC0C0ull + (uint64_t)k * 7919 + (write ? 1 : 0);
            pcs_thread_prepare();
            const bool async = form.rfind("async", 0) == 0;
            std::vector<ChecksumBatch> b(async ? Q : 0);
            std::vector<std::vector<char*>> ptrs(std::max(1, Q), std::vector<char*>(kBatch));
            std::vector<uint8_t> ok(kBatch);
            ready.fetch_add(1);
            while (!go.load()) std::this_thread::yield();
            const auto stop = Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(secs));
            const double c0 = thread_cpu_s();
            uint64_t done = 0, nbad = 0, np = 0, nu = 0;
            double ic = 0;
            auto pick = [&](std::vector<char*>& v) {
                for (auto& p : v) p = pool[splitmix(rng) % pool.size()];
            };
            if (form == "ref") {
                while (Clock::now() < stop) {
                    pick(ptrs[0]);
                    for (char* p : ptrs[0]) {  // page.cpp:18-31
                        const uint64_t h = XXH3_64bits(p + 8, P - 8);
                        if (write) {
                            std::memcpy(p, &h, 8);
                        } else {
                            uint64_t s;
                            std::memcpy(&s, p, 8);
                            nbad += h != s;
                        }
                    }
                    done += kBatch;
                }
            } else if (form == "sync" || form == "service" || form == "sync_sleep") {
                while (Clock::now() < stop) {
                    pick(ptrs[0]);
                    if (write) {
                        SetChecksums(ptrs[0], P);
                    } else {
                        const size_t fb = ValidateChecksums(std::span<const char* const>(ptrs[0].data(), kBatch), P,
                                                            ok.data());
                        nbad += fb != kBatch;
                    }
                    done += kBatch;
                }
            } else {  // async: Q batches in flight, ~10 us of other work between polls
                std::vector<bool> busy(Q, false);
                auto submit = [&](int i) {
                    pick(ptrs[i]);
                    const auto t0 = Clock::now();
                    if (write) b[i].SubmitStamp(ptrs[i], P);
                    else b[i].SubmitValidate(std::span<const char* const>(ptrs[i].data(), kBatch), P);
                    ic += std::chrono::duration<double>(Clock::now() - t0).count();
                    busy[i] = true;
                };
                for (int i = 0; i < Q; ++i) submit(i);
                uint64_t sink = 0;
                for (;;) {
                    bool any = false;
                    for (int i = 0; i < Q; ++i) {
                        if (!busy[i]) continue;
                        any = true;
                        const auto t0 = Clock::now();
                        const bool d = b[i].Poll();
                        ic += std::chrono::duration<double>(Clock::now() - t0).count();
                        ++np;
                        if (!d) continue;
                        if (!write) nbad += b[i].FirstBad() != kBatch;
                        done += kBatch;
                        busy[i] = false;
                        if (Clock::now() < stop) submit(i);
                    }
                    if (!any) break;
                    sink += other_work(np);  // the rest of the shard's work loop
                    ++nu;
                }
                if (sink == 42) std::puts("");
            }
            cpu[k] = thread_cpu_s() - c0;
            in_call[k] = ic;
            pages += done;
            bad += nbad;
            polls += np;
            units += nu;
        });
    while (ready.load() < T) std::this_thread::yield();
    const uint64_t s0 = pcs_counter(PCS_COUNTER_SERVICE_BATCHES);
    const auto t0 = Clock::now();
    go = true;
    for (auto& x : th) x.join();
    const double batches = pages.load() / (double)kBatch;
    Point pt;
    pt.form = form;
    pt.T = T;
    pt.Q = form.rfind("async", 0) == 0 ? Q : 0;
    pt.write = write;
    pt.wall_s = std::chrono::duration<double>(Clock::now() - t0).count();
    pt.gib = pages.load() * (double)P / (1u << 30);
    for (int k = 0; k < T; ++k) {
        pt.cpu_s += cpu[k];
        pt.in_call_s += in_call[k];
    }
    pt.work_units = units.load();
    pt.work_cpu_s = units.load() * work_cpu_per_unit;
    pt.bad = bad.load();
    pt.polls = polls.load();
    pt.served = batches > 0 ? (pcs_counter(PCS_COUNTER_SERVICE_BATCHES) - s0) / batches : 0;
    return pt;
}
}  // namespace

int main(int argc, char** argv) {
    const double secs = argc > 1 ? std::atof(argv[1]) : 2.0;
    const char* json_out = argc > 2 ? argv[2] : nullptr;
    const size_t chunks = 256;  // 1 GiB
    std::vector<char*> chunk(chunks), pool;
    uint64_t seed = 1;
    for (auto& c : chunk) {
        c = static_cast<char*>(std::aligned_alloc(4096, kChunkPages * P));
        auto* w = reinterpret_cast<uint64_t*>(c);
        for (size_t i = 0; i < kChunkPages * P / 8; ++i) w[i] = splitmix(seed);
        RegisterPagePool(c, kChunkPages * P);
        for (size_t j = 0; j < kChunkPages; ++j) pool.push_back(c + j * P);
    }
    for (size_t i = 0; i < pool.size(); i += 65536) {
        const size_t n = std::min<size_t>(65536, pool.size() - i);
        SetChecksums(std::span<char* const>(pool.data() + i, n), P);
    }
    const double work_unit = calibrate_work();
    std::printf("pool: %zu registered 4 KiB pages (1 GiB); %.1f s per point; other work: %.2f us CPU per unit "
                "(%llu iterations)\n", pool.size(), secs, work_unit * 1e6, (unsigned long long)g_work_iters);
    std::vector<Point> pts;
    for (bool write : {false, true}) {
        std::printf("%s (batches of %d pages)\n", write ? "write path: stamp" : "read path: validate", write ? 256 : 128);
        std::printf("  %-14s %2s %2s %9s %12s %12s %12s %7s %5s\n", "form", "T", "Q", "GiB/s", "cpu_s/GiB",
                    "in_call/GiB", "saved/GiB", "served", "bad");
        double ref_per_gib = 0;
        for (int T : {1, 8}) {
            for (const char* form : {"ref", "sync", "sync_sleep", "service", "service_d0", "async", "async_event",
                                     "async_service", "async_service_d0", "async_service_q1", "async_service_q1_d0"}) {
                // CPU_COST_FORMS: a comma-separated subset to run (all by default)
                if (const char* only = std::getenv("CPU_COST_FORMS")) {
                    const std::string list = std::string(",") + only + ",";
                    if (list.find(std::string(",") + form + ",") == std::string::npos) continue;
                }
                // "_d0": the same form with the service's departure words off
                // (PCS_TUNE_SERVICE_DEPARTURE = 0: the runtime is asked every 50 us)
                std::string base = form;
                const bool d0 = base.size() > 3 && base.compare(base.size() - 3, 3, "_d0") == 0;
                if (d0) base.resize(base.size() - 3);
                const bool svc = base.find("service") != std::string::npos;
                const bool ev = base == "async_event";
                pcs_set_tuning(PCS_TUNE_ZC_BATCH_EVENT, ev ? 1 : 0);
                pcs_set_tuning(PCS_TUNE_SYNC_SPIN_US, base == "sync_sleep" ? 30 : 0);
                pcs_set_tuning(PCS_TUNE_SERVICE_DEPARTURE, d0 ? 0 : 1);
                const int Q = base == "async_service_q1" ? 1 : 4;
                // a line per request that can be in flight (at most 8 lines)
                static const int max_lines = std::getenv("CPU_COST_MAX_LINES") ? std::atoi(std::getenv("CPU_COST_MAX_LINES")) : 8;
                if (svc) StartChecksumService(base == "service" ? 4 : 2, 1000, std::min(max_lines, base == "service" ? T : T * Q));
                Point pt = run(pool, base.c_str(), T, Q, write, secs, work_unit);
                pt.form = form;
                if (svc) StopChecksumService();
                pt.path = svc ? "service" : std::strcmp(form, "ref") == 0 ? "cpu" : "zero-copy launch";
                if (pt.form == "ref" && T == 1) ref_per_gib = pt.cpu_per_gib();
                std::printf("  %-14s %2d %2d %9.2f %12.4f %12.4f %12.4f %7.3f %5llu\n", form, T, pt.Q,
                            pt.gib / pt.wall_s, pt.cpu_per_gib(), pt.Q ? pt.in_call_s / pt.gib : pt.cpu_per_gib(),
                            ref_per_gib - pt.cpu_per_gib(), pt.served, (unsigned long long)pt.bad);
                std::fflush(stdout);
                if (pt.bad) {
                    std::printf("FAILED: verdicts\n");
                    return 1;
                }
                pts.push_back(pt);
            }
        }
    }
    if (json_out) {
        FILE* f = std::fopen(json_out, "w");
        std::fprintf(f, "{\"work_unit_us\": %.3f, \"points\": [", work_unit * 1e6);
        for (size_t i = 0; i < pts.size(); ++i) {
            const Point& p = pts[i];
            std::fprintf(f, "%s{\"form\": \"%s\", \"path\": \"%s\", \"write\": %s, \"T\": %d, \"Q\": %d, \"GiB\": %.4f, "
                            "\"wall_s\": %.4f, \"cpu_s\": %.4f, \"other_work_cpu_s\": %.4f, \"in_call_s\": %.4f, "
                            "\"GiBps\": %.3f, \"cpu_s_per_GiB\": %.5f, \"served_share\": %.4f, \"polls\": %llu}",
                         i ? ", " : "", p.form.c_str(), p.path.c_str(), p.write ? "true" : "false", p.T, p.Q, p.gib,
                         p.wall_s, p.cpu_s, p.work_cpu_s, p.in_call_s, p.gib / p.wall_s, p.cpu_per_gib(), p.served,
                         (unsigned long long)p.polls);
        }
        std::fprintf(f, "]}\n");
        std::fclose(f);
    }
    for (auto& c : chunk) {
        UnregisterPagePool(c);
        std::free(c);
    }
    std::printf("cpu cost ok\n");
    return 0;
}
