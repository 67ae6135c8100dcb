// service_lab.hip — how low can a small host validate batch go without a
// launch per batch?  (Experiment harness, not part of the product.)
//
// A persistent "service" kernel (G workgroups) polls a mailbox in pinned host
// memory.  The host posts a request (n registered-pool page addresses, then a
// sequence number), the workgroups hash their share of the pages (XXH3, 4 KiB,
// the product's xxh3_page_fixed body) and write each verdict straight into
// the mailbox; the host returns once every verdict has landed (the sentinel
// scheme of the product's zero-copy path).  Timed against the library's
// launch-per-batch zero-copy validate (pcs_pages_validate_host) over the same
// kind of pages: random 4 KiB pages of a 1 GiB registered pool.
//
// Safety: every workgroup leaves the service loop on the host's stop word or
// after kMaxIdlePolls polls without a request (a few seconds), so the grid
// always drains; run under `timeout -k`.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "eloqstore_pcs.h"
#include "xxh3_page.h"

#define HIP_OK(x)                                                                     \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "%s:%d CHECK(%s)\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                 \
        }                                                                 \
    } while (0)

constexpr int kMaxPages = 256;
constexpr uint32_t kPending = 0xA5A5A5A5u;
constexpr uint64_t kQuit = ~0ull;
constexpr uint64_t kMaxIdlePolls = 4u << 20;  // ~4-10 s of idle polling, then the kernel ends itself

struct Mailbox {
    // line 0: the request header; with FAST the poll reads it whole, so a
    // request of <= 6 pages arrives in one PCIe read
    alignas(64) uint64_t seq;   // host: ++ to post a request (written last)
    uint64_t n;
    uint64_t ptrs[kMaxPages];   // device-visible page addresses
    alignas(64) uint64_t stop;  // host: 1 to end the service
    alignas(64) uint32_t ok[kMaxPages];  // verdicts as words: system-scope atomic stores
    alignas(64) uint64_t served;  // kernel: last request finished by workgroup 0 (diagnostic)
    alignas(64) uint64_t alive;   // kernel: set when workgroup 0 starts (diagnostic)
};

// seq0: the sequence number already consumed when the kernel was launched
// (the host may post before the kernel starts running).
template <bool FAST>
__global__ __launch_bounds__(256) void k_service(Mailbox* mb, uint64_t seq0) {
    __shared__ uint64_t s_seq, s_n, s_line[8];
    const pcs::Xxh3Lane L = pcs::make_xxh3_lane(threadIdx.x & 15);
    uint64_t last = seq0;
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&mb->alive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
        if (FAST && threadIdx.x < 8) {
            // 8 lanes read the header line in one instruction per poll
            const uint64_t* line = &mb->seq;
            uint64_t q = kQuit, polls = 0, w = 0;
            for (;;) {
                w = __hip_atomic_load(line + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                const uint64_t cur = __shfl(w, 0, 8);
                if (cur != last) {
                    q = cur;
                    break;
                }
                if (__hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) || ++polls > kMaxIdlePolls)
                    break;
            }
            s_line[threadIdx.x] = w;
            if (threadIdx.x == 0) {
                s_seq = q;
                s_n = q == kQuit ? 0 : s_line[1];
            }
        } else if (!FAST && threadIdx.x == 0) {
            uint64_t q = kQuit, polls = 0;
            for (;;) {
                const uint64_t cur = __hip_atomic_load(&mb->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (cur != last) {
                    q = cur;
                    break;
                }
                if (__hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) || ++polls > kMaxIdlePolls)
                    break;
            }
            s_seq = q;
            s_n = q == kQuit ? 0 : __hip_atomic_load(&mb->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        const uint64_t q = s_seq, n = s_n;
        __syncthreads();  // s_seq / s_n are rewritten by the next poll
        if (q == kQuit) break;  // uniform: every thread read the same word
        last = q;
        // system-scope acquire: the page list and the page bytes are read
        // fresh from host memory, not from this CU's or XCD's caches
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        for (uint64_t pg = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 4); pg < n; pg += (uint64_t)gridDim.x * 16) {
            const uint8_t* page = reinterpret_cast<const uint8_t*>(
                FAST && pg < 6 ? s_line[2 + pg] : __hip_atomic_load(&mb->ptrs[pg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
            uint64_t stored = 0;
            pcs::u32x4 first;
            const uint64_t h = pcs::xxh3_page_fixed<4096, false>(page, L, stored, first);
            if (L.g == 0)
                __hip_atomic_store(&mb->ok[pg], h == stored ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        // push this request's verdict lines out of the XCD's L2 now, not at
        // kernel end (FAST relies on the system-scope stores alone)
        if (!FAST) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (blockIdx.x == 0 && threadIdx.x == 0)
            __hip_atomic_store(&mb->served, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const int G = argc > 1 ? std::atoi(argv[1]) : 4;
    const bool fast = argc > 2 && std::atoi(argv[2]) != 0;
    const size_t P = 4096, NP = size_t(1) << 18;
    char* pool = static_cast<char*>(std::aligned_alloc(4096, NP * P));
    CHECK(pool);
    std::mt19937_64 fill(7);
    for (size_t i = 0; i < NP * P / 8; ++i) reinterpret_cast<uint64_t*>(pool)[i] = fill();
    CHECK(pcs_host_register(pool, NP * P) == PCS_OK);
    {  // stamp every page (library zero-copy path), in 256-page batches
        std::vector<void*> pp(256);
        for (size_t b = 0; b < NP; b += 256) {
            for (size_t i = 0; i < 256; ++i) pp[i] = pool + (b + i) * P;
            CHECK(pcs_pages_stamp_host(pp.data(), P, 256, PCS_XXH3_64) == PCS_OK);
        }
    }
    void* dpool = nullptr;
    HIP_OK(hipHostGetDevicePointer(&dpool, pool, 0));
    Mailbox* mb = nullptr;
    HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&mb), sizeof(Mailbox), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(mb, 0, sizeof(Mailbox));
    Mailbox* dmb = nullptr;
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dmb), mb, 0));

    using clk = std::chrono::steady_clock;
    std::mt19937_64 rng(99);
    const std::vector<size_t> sizes = {1, 2, 4, 6, 8, 16, 32, 48, 64, 128, 256};
    const int kWarm = 30, kReps = 300;

    // (1) the library's launch-per-batch zero-copy validate, before the service runs
    std::vector<double> lib_med;
    for (size_t n : sizes) {
        std::vector<double> t;
        std::vector<const void*> ptrs(n);
        std::vector<uint8_t> ok(n);
        uint64_t fb = 0;
        for (int r = 0; r < kWarm + kReps; ++r) {
            for (size_t i = 0; i < n; ++i) ptrs[i] = pool + (rng() % NP) * P;
            const auto t0 = clk::now();
            CHECK(pcs_pages_validate_host(ptrs.data(), P, n, PCS_XXH3_64, ok.data(), &fb) == PCS_OK);
            const auto t1 = clk::now();
            CHECK(fb == UINT64_MAX);
            if (r >= kWarm) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        lib_med.push_back(median(t));
    }

    // (2) the service kernel
    hipStream_t s;
    HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (fast) hipLaunchKernelGGL(k_service<true>, dim3(G), dim3(256), 0, s, dmb, (uint64_t)0);
    else hipLaunchKernelGGL(k_service<false>, dim3(G), dim3(256), 0, s, dmb, (uint64_t)0);
    HIP_OK(hipGetLastError());
    uint64_t seq = 0;
    auto post_and_wait = [&](size_t n, const std::vector<uint64_t>& dptrs) {
        for (size_t i = 0; i < n; ++i) mb->ptrs[i] = dptrs[i];
        for (size_t i = 0; i < n; ++i) mb->ok[i] = kPending;
        mb->n = n;
        std::atomic_thread_fence(std::memory_order_release);
        __atomic_store_n(&mb->seq, ++seq, __ATOMIC_RELEASE);
        const volatile uint32_t* v = mb->ok;
        size_t at = 0;
        const auto start = clk::now();
        while (at < n) {
            while (at < n && v[at] != kPending) ++at;
            if (at < n && clk::now() - start > std::chrono::seconds(2)) {
                std::fprintf(stderr, "service did not answer request %llu (n=%zu): alive %llu, served %llu, verdicts landed %zu\n",
                             (unsigned long long)seq, n, (unsigned long long)__atomic_load_n(&mb->alive, __ATOMIC_ACQUIRE),
                             (unsigned long long)__atomic_load_n(&mb->served, __ATOMIC_ACQUIRE), at);
                mb->stop = 1;
                std::exit(2);
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    };
    std::printf("service kernel: %d workgroups of 256 threads, %s\n", G,
                fast ? "header line polled whole, no release fence" : "seq polled alone, release fence per request");
    std::printf("pages  launch_per_batch_us  service_us\n");
    for (size_t k = 0; k < sizes.size(); ++k) {
        const size_t n = sizes[k];
        std::vector<double> t;
        std::vector<uint64_t> dptrs(n);
        std::vector<size_t> idx(n);
        for (int r = 0; r < kWarm + kReps; ++r) {
            for (size_t i = 0; i < n; ++i) {
                idx[i] = rng() % NP;
                dptrs[i] = reinterpret_cast<uint64_t>(static_cast<char*>(dpool) + idx[i] * P);
            }
            const bool corrupt = r % 7 == 3;
            const size_t bad = corrupt ? rng() % n : 0;
            if (corrupt) pool[idx[bad] * P + 10] ^= 0x40;
            const auto t0 = clk::now();
            post_and_wait(n, dptrs);
            const auto t1 = clk::now();
            for (size_t i = 0; i < n; ++i) {
                const bool dup_bad = corrupt && idx[i] == idx[bad];
                CHECK(mb->ok[i] == (dup_bad ? 0 : 1));
            }
            if (corrupt) pool[idx[bad] * P + 10] ^= 0x40;
            if (r >= kWarm) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        std::printf("%5zu  %19.1f  %10.1f\n", n, lib_med[k], median(t));
    }
    __atomic_store_n(&mb->stop, 1, __ATOMIC_RELEASE);
    HIP_OK(hipStreamSynchronize(s));
    std::printf("service ended after %llu requests\n", (unsigned long long)mb->served);
    HIP_OK(hipStreamDestroy(s));
    CHECK(pcs_host_unregister(pool) == PCS_OK);
    HIP_OK(hipHostFree(mb));
    std::free(pool);
    std::printf("service_lab ok\n");
    return 0;
}
