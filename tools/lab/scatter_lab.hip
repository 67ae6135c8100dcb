// scatter_lab.hip — what does the stamp's header-write pass pay for?  Not part
// of the product.
//
// The product stamp is the digest kernel into a compact 8-byte array followed
// by k_scatter_stamp: one 8-byte nt store per page header, thread i -> page i
// (DESIGN.md §4.5a).  It costs ~50 us per 1 M x 4 KiB pages, i.e. ~20 G
// header writes/s, or 0.6 TB/s of the 32 B sectors it dirties.  This harness
// separates the possible causes:
//   * write ORDER (does a permutation of the same 1 M addresses spread them
//     over more DRAM banks / channels at once?): linear, random bijection,
//     64-way spread per wave, XCD-contiguous chunks, reversed;
//   * write WIDTH (partial-sector merge or not): 8 B vs a full 32 B sector vs
//     a 64 B line per page (junk bytes past the header: cost probe only);
//   * STRIDE (same 1 M 8-byte writes packed at 64 B .. 4 KiB apart).
// Each scatter is timed inside whole stamps back to back (K x [digest pass +
// scatter]) minus K digest passes alone, so write-back deferred into the next
// launch is charged, and alone right after a full read pass.
//
//   make -C tools/lab scatter_lab && ./tools/lab/scatter_lab [rounds]
#include <hip/hip_runtime.h>

#include "xxh3_page.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

using namespace pcs;
constexpr int P = 4096;

// The product's 4 KiB page body (xxh3_page_fixed<4096>) with the policy of the
// first 256 B of each page (its chunk 0, which holds the header line) as a
// parameter: HEAD_NT = false loads it with the default policy, so the line
// may still sit in L2 / Infinity Cache when the write pass patches it.
template <bool HEAD_NT>
__device__ __forceinline__ uint64_t page4k(const uint8_t* __restrict__ page, const Xxh3Lane& L) {
    const u32x4* base = reinterpret_cast<const u32x4*>(page) + L.g;
    u32x4 d[5][4];
    d[0][0] = ld16<HEAD_NT>(base);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (i || c) d[i][c] = ld16<true>(base + i * 64 + c * 16);
    uint64_t Ae = L.init_e, Ao = L.init_o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint64_t Te, To;
        if (i < 3) {
            xxh3_block_terms<false>(L, d[i], lo64(d[i + 1][0]), 4, Te, To);
            Ae = xxh3_scramble(Ae + Te, L.ks_e);
            Ao = xxh3_scramble(Ao + To, L.ks_o);
        } else {
            xxh3_block_terms<true>(L, d[i], 0, 4, Te, To);
            Ae += Te;
            Ao += To;
        }
    }
    return xxh3_merge(L, Ae, Ao, (uint64_t)(P - 8));
}

// the product's digest pass (16 digests staged per tile, one 128 B nt store)
template <bool HEAD_NT = true>
__global__ __launch_bounds__(256) void k_digest(const uint8_t* __restrict__ pages, uint64_t n,
                                               uint64_t* __restrict__ out) {
    __shared__ uint64_t tile_h[16];
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const int grp = threadIdx.x >> 4;
    const uint64_t pg = t * 16 + grp;
    if (pg < n) {
        uint64_t h;
        if (HEAD_NT) {
            uint64_t stored;
            u32x4 first;
            h = xxh3_page_fixed<P, true>(pages + pg * (uint64_t)P, L, stored, first);
        } else {
            h = page4k<false>(pages + pg * (uint64_t)P, L);
        }
        if (L.g == 0) tile_h[grp] = h;
    }
    __syncthreads();
    const uint64_t i = t * 16 + threadIdx.x;
    if (threadIdx.x < 16 && i < n) st_nt(out + i, tile_h[threadIdx.x]);
}

enum Order : int { kLin = 0, kRand = 1, kSpread = 2, kXcd = 3, kRev = 4 };

// thread k -> page index (n is a power of two)
__device__ __forceinline__ uint64_t order_map(int ord, uint64_t k, uint64_t n) {
    switch (ord) {
        case kRand: return (k * 0x9E3779B1ull) & (n - 1);
        case kSpread: return (k & 63) * (n >> 6) + (k >> 6);
        case kXcd: {
            const uint64_t nb = n / 256;
            return xcd_tile(k / 256, nb) * 256 + (k & 255);
        }
        case kRev: return n - 1 - k;
        default: return k;
    }
}

template <int W>  // bytes written per page: 8, 32 or 64 (past 8: junk, cost probe)
__global__ __launch_bounds__(256) void k_scatter(uint8_t* __restrict__ pages, uint64_t n, uint64_t stride,
                                                const uint64_t* __restrict__ dig, int ord) {
    constexpr int LPP = W >= 16 ? W / 16 : 1;  // lanes per page
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t j = k / LPP;
    if (j >= n) return;
    const uint64_t i = order_map(ord, j, n);
    if (W == 8) {
        st_nt(reinterpret_cast<uint64_t*>(pages + i * stride), dig[i]);
    } else {
        const uint64_t h = dig[i];
        u32x4 v;
        v.x = (uint32_t)h;
        v.y = (uint32_t)(h >> 32);
        v.z = (uint32_t)k;
        v.w = 0;
        st_nt(reinterpret_cast<u32x4*>(pages + i * stride) + (k % LPP), v);
    }
}

// read the page's first 64 B line (default policy), patch the header, write
// the whole line back nt: 4 lanes per page
__global__ __launch_bounds__(256) void k_rmw64(uint8_t* __restrict__ pages, uint64_t n,
                                              const uint64_t* __restrict__ dig, int ord) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t j = k >> 2;
    if (j >= n) return;
    const uint64_t i = order_map(ord, j, n);
    u32x4* dst = reinterpret_cast<u32x4*>(pages + i * P) + (k & 3);
    u32x4 v = *dst;
    if ((k & 3) == 0) {
        const uint64_t h = dig[i];
        v.x = (uint32_t)h;
        v.y = (uint32_t)(h >> 32);
    }
    st_nt(dst, v);
}

__global__ __launch_bounds__(256) void k_read_all(const u32x4* __restrict__ p, uint64_t n16, uint32_t* sink) {
    uint32_t x = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) sink[0] = x;
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

struct Var {
    std::string name;
    int w, ord;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
    const uint64_t n = 1ull << 20, bytes = n * P, ntiles = n / 16;
    uint8_t* pages;
    uint64_t* dig;
    uint32_t* sink;
    CK(hipMalloc(&pages, bytes));
    CK(hipMalloc(&dig, n * 8));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(pages), bytes / 8);
    hipLaunchKernelGGL(k_digest<true>, dim3(ntiles), dim3(256), 0, 0, pages, n, dig);
    CK(hipDeviceSynchronize());

    // parity of the orderings: every order writes the same header set
    for (int ord = 0; ord <= kRev; ++ord) {
        CK(hipMemset(dig, 0, 8));  // page 0's digest := 0 so the check is order-independent
        hipLaunchKernelGGL(k_digest<true>, dim3(ntiles), dim3(256), 0, 0, pages, n, dig);
        hipLaunchKernelGGL(k_scatter<8>, dim3(n / 256), dim3(256), 0, 0, pages, n, (uint64_t)P, dig, ord);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> h(n), d(n);
        CK(hipMemcpy(d.data(), dig, n * 8, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < n; i += 4093) {
            uint64_t v;
            CK(hipMemcpy(&v, pages + i * P, 8, hipMemcpyDeviceToHost));
            bad += v != d[i];
        }
        std::printf("order %d: headers %s\n", ord, bad ? "WRONG" : "ok");
        if (bad) return 1;
    }

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_us = [&](const std::function<void()>& f, int reps) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < reps; ++k) f();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1e3 / reps;
    };
    auto scatter = [&](int w, int ord, uint64_t cnt, uint64_t stride) {
        const uint64_t lanes = cnt * (w >= 16 ? w / 16 : 1);
        const dim3 g((unsigned)((lanes + 255) / 256)), b(256);
        switch (w) {
            case 8: hipLaunchKernelGGL(k_scatter<8>, g, b, 0, 0, pages, cnt, stride, dig, ord); break;
            case 32: hipLaunchKernelGGL(k_scatter<32>, g, b, 0, 0, pages, cnt, stride, dig, ord); break;
            default: hipLaunchKernelGGL(k_scatter<64>, g, b, 0, 0, pages, cnt, stride, dig, ord); break;
        }
    };
    auto digest = [&] { hipLaunchKernelGGL(k_digest<true>, dim3(ntiles), dim3(256), 0, 0, pages, n, dig); };
    auto read_all = [&] {
        hipLaunchKernelGGL(k_read_all, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const u32x4*>(pages),
                           bytes / 16, sink);
    };

    std::vector<Var> vars = {{"8B lin (product)", 8, kLin}, {"8B rand", 8, kRand},   {"8B spread64", 8, kSpread},
                             {"8B xcd", 8, kXcd},           {"8B rev", 8, kRev},     {"32B lin", 32, kLin},
                             {"64B lin", 64, kLin},         {"32B rand", 32, kRand}};
    constexpr int K = 10;
    std::vector<std::vector<double>> whole(vars.size()), alone(vars.size());
    std::vector<double> dig_only;
    for (int r = 0; r < rounds; ++r) {
        dig_only.push_back(time_us(digest, K));
        for (size_t v = 0; v < vars.size(); ++v) {
            const Var& x = vars[v];
            whole[v].push_back(time_us([&] { digest(); scatter(x.w, x.ord, n, P); }, K));
            read_all();
            alone[v].push_back(time_us([&] { scatter(x.w, x.ord, n, P); }, 1));
        }
    }
    auto med = [](std::vector<double> t) {
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    const double d0 = med(dig_only);
    std::printf("# 1 M x 4 KiB pages; whole = K=%d x [digest + scatter] per stamp; cost = whole - digest (%.1f us)\n",
                K, d0);
    std::printf("%-22s %12s %10s %14s\n", "scatter", "whole us", "cost us", "alone us");
    for (size_t v = 0; v < vars.size(); ++v)
        std::printf("%-22s %12.1f %10.1f %14.1f\n", vars[v].name.c_str(), med(whole[v]), med(whole[v]) - d0,
                    med(alone[v]));

    // header line kept cached by the digest pass (default-policy chunk 0)
    {
        auto digestc = [&] { hipLaunchKernelGGL(k_digest<false>, dim3(ntiles), dim3(256), 0, 0, pages, n, dig); };
        auto rmw = [&](int ord) {
            hipLaunchKernelGGL(k_rmw64, dim3((unsigned)(n * 4 / 256)), dim3(256), 0, 0, pages, n, dig, ord);
        };
        // parity of the cached-head digest: same digests as the product body
        hipLaunchKernelGGL(k_digest<true>, dim3(ntiles), dim3(256), 0, 0, pages, n, dig);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> a(n), b(n);
        CK(hipMemcpy(a.data(), dig, n * 8, hipMemcpyDeviceToHost));
        digestc();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), dig, n * 8, hipMemcpyDeviceToHost));
        std::printf("cached-head digest parity: %s\n", a == b ? "ok" : "MISMATCH");
        if (a != b) return 1;
        struct V2 {
            const char* name;
            std::function<void()> f;
        };
        std::vector<V2> v2 = {
            {"digest(nt head) only", digest},
            {"digest(cached head) only", digestc},
            {"cached head + 8B lin", [&] { digestc(); scatter(8, kLin, n, P); }},
            {"cached head + 8B xcd", [&] { digestc(); scatter(8, kXcd, n, P); }},
            {"cached head + rmw64 lin", [&] { digestc(); rmw(kLin); }},
            {"cached head + rmw64 xcd", [&] { digestc(); rmw(kXcd); }},
            {"nt head + rmw64 xcd", [&] { digest(); rmw(kXcd); }},
        };
        std::vector<std::vector<double>> t2(v2.size());
        for (int r = 0; r < rounds; ++r)
            for (size_t v = 0; v < v2.size(); ++v) t2[v].push_back(time_us(v2[v].f, K));
        std::printf("%-28s %12s %10s\n", "whole stamp", "us", "vs digest");
        for (size_t v = 0; v < v2.size(); ++v)
            std::printf("%-28s %12.1f %10.1f\n", v2[v].name, med(t2[v]), med(t2[v]) - d0);
    }

    // Pipelined stamps on two streams: the scatter of stamp k (stream s1)
    // overlaps the digest pass of stamp k + 1 (stream s0); two digest arrays,
    // each reused only after its scatter is done.
    {
        uint64_t* dig2;
        CK(hipMalloc(&dig2, n * 8));
        uint64_t* digs[2] = {dig, dig2};
        hipStream_t s0, s1;
        CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        hipEvent_t dd[2], sd[2], j0, j1;
        for (int b = 0; b < 2; ++b) {
            CK(hipEventCreateWithFlags(&dd[b], hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&sd[b], hipEventDisableTiming));
        }
        CK(hipEventCreate(&j0));
        CK(hipEventCreate(&j1));
        auto pipelined = [&]() {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(j0, s0));
            for (int k = 0; k < K; ++k) {
                const int b = k & 1;
                if (k >= 2) CK(hipStreamWaitEvent(s0, sd[b], 0));
                hipLaunchKernelGGL(k_digest<true>, dim3(ntiles), dim3(256), 0, s0, pages, n, digs[b]);
                CK(hipEventRecord(dd[b], s0));
                CK(hipStreamWaitEvent(s1, dd[b], 0));
                hipLaunchKernelGGL(k_scatter<8>, dim3(n / 256), dim3(256), 0, s1, pages, n, (uint64_t)P, digs[b], kLin);
                CK(hipEventRecord(sd[b], s1));
            }
            CK(hipStreamWaitEvent(s0, sd[(K - 1) & 1], 0));
            CK(hipEventRecord(j1, s0));
            CK(hipEventSynchronize(j1));
            float ms;
            CK(hipEventElapsedTime(&ms, j0, j1));
            return ms * 1e3 / K;
        };
        std::vector<double> tp, ts;
        for (int r = 0; r < rounds; ++r) {
            tp.push_back(pipelined());
            ts.push_back(time_us([&] { digest(); scatter(8, kLin, n, P); }, K));
        }
        std::printf("%-28s %12.1f %10.1f\n", "pipelined 2 streams", med(tp), med(tp) - d0);
        std::printf("%-28s %12.1f %10.1f\n", "serial (product)", med(ts), med(ts) - d0);
        // headers still right after the pipelined stamps
        hipLaunchKernelGGL(k_digest<true>, dim3(ntiles), dim3(256), 0, 0, pages, n, dig);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> d(n);
        CK(hipMemcpy(d.data(), dig, n * 8, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < n; i += 4093) {
            uint64_t v;
            CK(hipMemcpy(&v, pages + i * P, 8, hipMemcpyDeviceToHost));
            bad += v != d[i];
        }
        std::printf("pipelined headers: %s\n", bad ? "WRONG" : "ok");
    }

    // stride probes: 1 M 8-byte nt writes (fewer past 4 KiB), right after a read pass
    std::printf("# stride probe: 8 B nt writes after a full read pass\n%-10s %10s %10s %12s\n", "stride", "writes",
                "us", "ns/write");
    for (uint64_t stride : {64ull, 256ull, 1024ull, 2048ull, 4096ull, 8192ull, 16384ull}) {
        const uint64_t cnt = std::min<uint64_t>(n, bytes / stride);
        std::vector<double> t;
        for (int r = 0; r < rounds; ++r) {
            read_all();
            t.push_back(time_us([&] { scatter(8, kLin, cnt, stride); }, 1));
        }
        const double m = med(t);
        std::printf("%-10llu %10llu %10.1f %12.3f\n", (unsigned long long)stride, (unsigned long long)cnt, m,
                    m * 1e3 / cnt);
    }
    return 0;
}
