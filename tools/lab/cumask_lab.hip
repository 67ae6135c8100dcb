// cumask_lab.hip — why did a CU-masked service stream hang?  Not part of the
// product.
//
// Round 3 tried the validate service on a CU-masked stream
// (hipExtStreamCreateWithCUMask: a hardware queue of its own, limited to a
// few CUs) and the service_load run hung at the first point with two threads
// (profiles/r03/service_load_cumask_hang.txt ends after "service1 6 1").  The
// product then stopped offering the option; this lab replays the same
// sequence with a phase marker on every thread and a watchdog that, when a
// thread sits in one phase for more than 3 s, prints every marker and the
// stuck threads' backtraces and exits, so the blocking call is named.
//
// Per point (T = 1, 2, 4; CU mask of `cus` CUs or none):
//   start:  create the service stream (CU-masked or plain), hipHostMalloc the
//           mailbox (coherent, mapped)                        [as pcs_service_start]
//   run:    thread 0 posts requests to a resident polling kernel (it leaves
//           after 1 ms idle or 2 ms of life; the host queues the next
//           generation when it cannot be sure one waits); threads 1..T-1 are
//           fresh threads taking the launch path: hipStreamCreate +
//           hipHostMalloc x3 on first use (the library's per-thread staging),
//           then launch + hipStreamSynchronize of a small kernel, for 0.5 s
//   stop:   stop word, hipStreamSynchronize, hipStreamDestroy, hipHostFree
//
//   ./tools/lab/cumask_lab [kind=all] [mode=0] [cus=4]
//     kind: plain | prio (highest-priority stream, the product's default) |
//           cumask | all (plain then cumask, the first run)
//     mode: 0 as above; 1 the launch-path threads create their streams and
//           staging before the service's first kernel; 2 no service kernel
//           at all (the CU-masked stream only exists)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

using Clock = std::chrono::steady_clock;

#define HC(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

namespace {
// ---- phase markers + stall watchdog --------------------------------------
enum Phase {
    kIdle, kStreamCreate, kCuMaskStreamCreate, kHostMalloc, kLaunch, kSync, kPost, kWaitAnswer, kServiceLaunch,
    kStopSync, kStreamDestroy, kHostFree, kNumPhases
};
const char* const kName[kNumPhases] = {"idle", "hipStreamCreate", "hipExtStreamCreateWithCUMask", "hipHostMalloc",
                                       "hipLaunchKernel (launch path)", "hipStreamSynchronize (launch path)",
                                       "post request", "wait for the service's answer",
                                       "hipLaunchKernel (service generation)", "hipStreamSynchronize (service stop)",
                                       "hipStreamDestroy (service stream)", "hipHostFree (mailbox)"};
struct Marker {
    std::atomic<int> phase{kIdle};
    std::atomic<int64_t> since{0};
    std::atomic<pthread_t> tid{};
    std::atomic<bool> live{false};
};
Marker g_mark[16];
int64_t now_ns() { return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count(); }
void mark(int s, Phase p) {
    g_mark[s].since.store(now_ns());
    g_mark[s].phase.store(p);
}
void on_dump(int) {
    void* fr[48];
    const int n = backtrace(fr, 48);
    backtrace_symbols_fd(fr, n, 2);
}
void watchdog() {
    for (;;) {
        std::this_thread::sleep_for(std::chrono::milliseconds(250));
        const int64_t t = now_ns();
        bool stuck = false;
        for (auto& m : g_mark)
            if (m.live && m.phase != kIdle && t - m.since > 3'000'000'000ll) stuck = true;
        if (!stuck) continue;
        std::printf("STALL\n");
        for (int k = 0; k < 16; ++k) {
            if (!g_mark[k].live) continue;
            const double secs = (t - g_mark[k].since) / 1e9;
            std::printf("  thread %d: %s for %.2f s\n", k, kName[g_mark[k].phase.load()], secs);
            std::fflush(stdout);
            if (g_mark[k].phase != kIdle && secs > 3.0) {
                std::fprintf(stderr, "backtrace of thread %d:\n", k);
                pthread_kill(g_mark[k].tid.load(), SIGUSR1);
                std::this_thread::sleep_for(std::chrono::milliseconds(300));
            }
        }
        std::fflush(stdout);
        std::fflush(stderr);
        _exit(3);
    }
}

struct Box {
    alignas(64) uint64_t seq;
    alignas(64) uint64_t stop;
    alignas(64) uint64_t answer;
};

// The service kernel's shape: poll seq, answer, leave on idle / life / stop /
// a newer generation.
__global__ void k_poll(Box* box, uint64_t gen, uint64_t idle_ticks, uint64_t life_ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t born = __builtin_amdgcn_s_memrealtime();
    uint64_t t_last = born, last = gen << 32;
    for (;;) {
        const uint64_t s = __hip_atomic_load(&box->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (s != last) {
            if ((s >> 32) != gen) return;
            last = s;
            if (blockIdx.x == 0) __hip_atomic_store(&box->answer, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            t_last = __builtin_amdgcn_s_memrealtime();
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (__hip_atomic_load(&box->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) || now - t_last > idle_ticks ||
            now - born > life_ticks)
            return;
    }
}

__global__ void k_small(uint64_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint64_t)i * 0x9E3779B97F4A7C15ull;
}

struct Point {
    uint64_t requests = 0, launches = 0;
};

enum Kind { kPlain, kPrio, kCuMask };

Point run_point(int T, Kind kind, int cus, int mode, double secs) {
    // start
    hipStream_t ss;
    mark(0, kind == kCuMask ? kCuMaskStreamCreate : kStreamCreate);
    if (kind == kCuMask) {
        std::vector<uint32_t> mask(8, 0);  // 256 CUs
        for (int c = 0; c < cus; ++c) mask[c / 32] |= 1u << (c % 32);
        HC(hipExtStreamCreateWithCUMask(&ss, (uint32_t)mask.size(), mask.data()));
    } else if (kind == kPrio) {
        int lo = 0, hi = 0;
        HC(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HC(hipStreamCreateWithPriority(&ss, hipStreamNonBlocking, hi));
    } else {
        HC(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
    }
    Box* h = nullptr;
    mark(0, kHostMalloc);
    HC(hipHostMalloc(reinterpret_cast<void**>(&h), sizeof(Box), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(h, 0, sizeof(Box));
    Box* d = nullptr;
    HC(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
    mark(0, kIdle);

    Point pt;
    std::atomic<uint64_t> launches{0};
    std::atomic<int> ready{0};
    auto stop = Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(secs));
    std::vector<std::thread> th;
    for (int k = 1; k < T; ++k)
        th.emplace_back([&, k] {
            g_mark[k].tid = pthread_self();
            g_mark[k].live = true;
            hipStream_t s;
            mark(k, kStreamCreate);
            HC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            void *a, *b, *c;
            mark(k, kHostMalloc);
            HC(hipHostMalloc(&a, 2048, hipHostMallocDefault));
            HC(hipHostMalloc(&b, 2048, hipHostMallocDefault));
            HC(hipHostMalloc(&c, 256, hipHostMallocDefault));
            uint64_t* out = nullptr;
            HC(hipHostGetDevicePointer(reinterpret_cast<void**>(&out), a, 0));
            mark(k, kIdle);
            ready.fetch_add(1);
            uint64_t n = 0;
            while (Clock::now() < stop) {
                mark(k, kLaunch);
                hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, out, 64);
                HC(hipGetLastError());
                mark(k, kSync);
                HC(hipStreamSynchronize(s));
                ++n;
            }
            mark(k, kIdle);
            launches += n;
            HC(hipStreamSynchronize(s));
            HC(hipStreamDestroy(s));
            HC(hipHostFree(a));
            HC(hipHostFree(b));
            HC(hipHostFree(c));
            g_mark[k].live = false;
        });
    // thread 0: the service requests
    if (mode == 1)  // the launch-path threads' streams and staging exist before the first service kernel
        while (ready.load() < T - 1) std::this_thread::yield();
    uint32_t gen = 0, count = 0;
    auto launched = Clock::now() - std::chrono::seconds(1);
    while (mode != 2 && Clock::now() < stop) {
        if (Clock::now() - launched > std::chrono::microseconds(1500)) {
            ++gen;
            count = 0;
            mark(0, kServiceLaunch);
            hipLaunchKernelGGL(k_poll, dim3(4), dim3(256), 0, ss, d, (uint64_t)gen, 100000ull, 200000ull);
            HC(hipGetLastError());
            launched = Clock::now();
        }
        mark(0, kPost);
        const uint64_t seq = (uint64_t)gen << 32 | ++count;
        __atomic_store_n(&h->seq, seq, __ATOMIC_RELEASE);
        mark(0, kWaitAnswer);
        const auto t0 = Clock::now();
        while (__atomic_load_n(&h->answer, __ATOMIC_ACQUIRE) != seq) {
            if (Clock::now() - t0 > std::chrono::milliseconds(2)) {  // the generation left: start the next
                launched = Clock::now() - std::chrono::seconds(1);
                break;
            }
        }
        mark(0, kIdle);
        ++pt.requests;
    }
    for (auto& x : th) x.join();
    pt.launches = launches;
    // stop
    __atomic_store_n(&h->stop, 1, __ATOMIC_RELEASE);
    mark(0, kStopSync);
    HC(hipStreamSynchronize(ss));
    mark(0, kStreamDestroy);
    HC(hipStreamDestroy(ss));
    mark(0, kHostFree);
    HC(hipHostFree(h));
    mark(0, kIdle);
    return pt;
}
}  // namespace

int main(int argc, char** argv) {
    signal(SIGUSR1, on_dump);
    g_mark[0].tid = pthread_self();
    g_mark[0].live = true;
    std::thread(watchdog).detach();
    const char* kind = argc > 1 ? argv[1] : "all";
    const int mode = argc > 2 ? std::atoi(argv[2]) : 0;
    const int cus = argc > 3 ? std::atoi(argv[3]) : 4;
    HC(hipSetDevice(0));
    std::vector<Kind> kinds;
    if (!std::strcmp(kind, "all")) kinds = {kPlain, kCuMask};
    else kinds = {!std::strcmp(kind, "prio") ? kPrio : !std::strcmp(kind, "cumask") ? kCuMask : kPlain};
    const char* const names[] = {"plain", "priority", "cu-masked"};
    for (Kind k : kinds)
        for (int T : {1, 2, 4}) {
            std::printf("%-10s mode %d cus %3d threads %d: ", names[k], mode, k == kCuMask ? cus : 0, T);
            std::fflush(stdout);
            const Point p = run_point(T, k, cus, mode, 0.5);
            std::printf("%8llu service requests, %8llu launch-path kernels\n", (unsigned long long)p.requests,
                        (unsigned long long)p.launches);
            std::fflush(stdout);
        }
    std::printf("cumask lab done\n");
    return 0;
}
