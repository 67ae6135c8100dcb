// tail3_lab.hip — where does config 3 (mixed 4/8/16 KiB pages) lose against
// the fixed-size kernels: in the steady state, or in the launch's ramp and
// tail?  Not part of the product.
//
// Instruments the product's descriptor body (k_xxh3_desc: one 16-lane group
// per page, 16-page tiles, XCD-contiguous tile order, 4-block steps) and, for
// reference, the fixed 4 KiB body (k_xxh3_fixed<4096>) with per-block
// wall_clock64 stamps.  Reports block durations, how many blocks are resident
// over time, and the bytes completed per 20 us bin (by block end), i.e. the
// rate profile of one launch: ramp, steady state, tail.
//
//   make -C tools/lab tail3_lab && ./tools/lab/tail3_lab
#include <hip/hip_runtime.h>

#include "xxh3_page.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

struct Stamp {
    uint64_t t0, t1, bytes;
};

template <bool STAMP>
__global__ __launch_bounds__(256) void k_desc(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                             const uint32_t* __restrict__ len, uint64_t n, uint64_t* __restrict__ out,
                                             Stamp* st) {
    uint64_t t0 = 0;
    if (STAMP) t0 = wall_clock64();
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const uint64_t pg = t * 16 + (threadIdx.x >> 4);
    uint32_t P = 0;
    if (pg < n) {
        P = len[pg];
        uint64_t stored = 0;
        const uint64_t h = xxh3_page_rt4<true>(base + off[pg], P, L, stored);
        if (L.g == 0) st_nt(out + pg, h);
    }
    if (STAMP) {
        __shared__ uint32_t tb[16];
        if ((threadIdx.x & 15) == 0) tb[threadIdx.x >> 4] = P;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t b = 0;
            for (int k = 0; k < 16; ++k) b += tb[k];
            st[blockIdx.x] = {t0, (uint64_t)wall_clock64(), b};
        }
    }
}

template <bool STAMP>
__global__ __launch_bounds__(256) void k_fixed(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* __restrict__ out,
                                              Stamp* st) {
    uint64_t t0 = 0;
    if (STAMP) t0 = wall_clock64();
    __shared__ uint64_t tile_h[16];
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const int grp = threadIdx.x >> 4;
    const uint64_t pg = t * 16 + grp;
    if (pg < n) {
        uint64_t stored;
        u32x4 first;
        const uint64_t h = xxh3_page_fixed<4096, true>(pages + pg * 4096ull, L, stored, first);
        if (L.g == 0) tile_h[grp] = h;
    }
    __syncthreads();
    if (threadIdx.x < 16 && t * 16 + threadIdx.x < n) st_nt(out + t * 16 + threadIdx.x, tile_h[threadIdx.x]);
    if (STAMP && threadIdx.x == 0) st[blockIdx.x] = {t0, (uint64_t)wall_clock64(), 16 * 4096};
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void report(const char* name, std::vector<Stamp> h, double tick_us) {
    uint64_t t0 = ~0ull, t1 = 0, bytes = 0;
    for (auto& s : h) t0 = std::min(t0, s.t0), t1 = std::max(t1, s.t1), bytes += s.bytes;
    const double span = (t1 - t0) * tick_us;
    std::vector<double> dur;
    for (auto& s : h) dur.push_back((s.t1 - s.t0) * tick_us);
    std::sort(dur.begin(), dur.end());
    std::printf("== %s: %zu blocks, span %.1f us, %.3f TB/s over the span; block us p10 %.1f p50 %.1f p90 %.1f "
                "p99 %.1f max %.1f\n",
                name, h.size(), span, bytes / span / 1e6, dur[dur.size() / 10], dur[dur.size() / 2],
                dur[dur.size() * 9 / 10], dur[dur.size() * 99 / 100], dur.back());
    const double bin = 20.0;
    const int nb = (int)(span / bin) + 1;
    std::vector<double> done(nb, 0), resident(nb, 0);
    for (auto& s : h) {
        const double a = (s.t0 - t0) * tick_us, b = (s.t1 - t0) * tick_us;
        done[std::min(nb - 1, (int)(b / bin))] += s.bytes;
        for (int k = (int)(a / bin); k <= std::min(nb - 1, (int)(b / bin)); ++k) {
            const double lo = std::max(a, k * bin), hi = std::min(b, (k + 1) * bin);
            if (hi > lo) resident[k] += (hi - lo) / bin;
        }
    }
    // steady = median rate of the bins between the first and last 10 %
    std::vector<double> mid;
    for (int k = nb / 10; k < nb - nb / 10; ++k) mid.push_back(done[k] / bin / 1e6);
    std::sort(mid.begin(), mid.end());
    const double steady = mid.empty() ? 0 : mid[mid.size() / 2];
    std::printf("   steady-state rate (median 20 us bin) %.3f TB/s; span at that rate %.1f us -> ramp+tail cost %.1f us "
                "(%.1f %%)\n",
                steady, bytes / steady / 1e6, span - bytes / steady / 1e6, 100 * (span - bytes / steady / 1e6) / span);
    std::printf("   bin(us)   TB/s  resident_blocks\n");
    for (int k = 0; k < nb; ++k)
        if (k < 6 || k >= nb - 8 || k % 10 == 0)
            std::printf("   %6.0f  %6.3f  %8.0f\n", k * bin, done[k] / bin / 1e6, resident[k]);
}

int main() {
    const uint64_t n = 1 << 20;
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n);
    uint64_t o = 0;
    for (uint64_t p = 0; p < n; ++p) {  // config 3's size rule (tests/workload.py)
        const uint64_t cls = mix((0x5EED0003ull ^ p) + (0x5A5A5A5Aull + 1) * 0x9E3779B97F4A7C15ull) % 3;
        len[p] = 4096u << cls;
        off[p] = o;
        o += len[p];
    }
    const uint64_t bytes3 = o, bytes2 = n * 4096;
    uint8_t* buf;
    uint64_t *d_off, *out;
    uint32_t* d_len;
    Stamp* st;
    CK(hipMalloc(&buf, bytes3));
    CK(hipMalloc(&d_off, n * 8));
    CK(hipMalloc(&d_len, n * 4));
    CK(hipMalloc(&out, n * 8));
    CK(hipMalloc(&st, (n / 16) * sizeof(Stamp)));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(buf), bytes3 / 8);
    CK(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_len, len.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    int wclk = 0;
    CK(hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0));  // kHz
    const double tick_us = 1e3 / wclk;
    const unsigned nt = (unsigned)(n / 16);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {
        for (int which = 0; which < 2; ++which) {
            // un-instrumented timing, then the instrumented run
            float ms = 0;
            for (int k = 0; k < 3; ++k) {
                CK(hipEventRecord(e0, 0));
                if (which == 0) hipLaunchKernelGGL((k_fixed<false>), dim3(nt), dim3(256), 0, 0, buf, n, out, st);
                else hipLaunchKernelGGL((k_desc<false>), dim3(nt), dim3(256), 0, 0, buf, d_off, d_len, n, out, st);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
            }
            if (which == 0) hipLaunchKernelGGL((k_fixed<true>), dim3(nt), dim3(256), 0, 0, buf, n, out, st);
            else hipLaunchKernelGGL((k_desc<true>), dim3(nt), dim3(256), 0, 0, buf, d_off, d_len, n, out, st);
            CK(hipDeviceSynchronize());
            std::vector<Stamp> h(nt);
            CK(hipMemcpy(h.data(), st, nt * sizeof(Stamp), hipMemcpyDeviceToHost));
            const double b = which == 0 ? bytes2 : bytes3;
            std::printf("-- %s: un-instrumented launch %.1f us = %.3f TB/s\n", which == 0 ? "config 2 fixed" : "config 3 desc",
                        ms * 1e3, b / ms / 1e9);
            report(which == 0 ? "config 2 fixed<4096>" : "config 3 desc", h, tick_us);
        }
    }
    return 0;
}
