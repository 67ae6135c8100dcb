// blocksize_lab.hip — workgroup size of the 4 KiB page kernel.  Not part of
// the product.
//
// The product k_xxh3_fixed<4096> runs 256-thread workgroups, one 16-page tile
// each; ramp + tail cost 2-2.7 % of a config-2 launch (tail3_lab).  Larger
// workgroups (32 or 64 pages, 512 / 1024 threads) need fewer dispatches to
// fill the chip; smaller ones (8 pages, 128 threads) free slots sooner in the
// tail.  Same body, same XCD-contiguous tile order, digests checked equal.
//
//   make -C tools/lab blocksize_lab && ./tools/lab/blocksize_lab [rounds]
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

template <int BT>
__global__ __launch_bounds__(BT) void k_fixed_bt(const uint8_t* __restrict__ pages, uint64_t n,
                                                uint64_t* __restrict__ out) {
    constexpr int TP = BT / 16;  // pages per tile
    __shared__ uint64_t tile_h[TP];
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + TP - 1) / TP;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const int grp = threadIdx.x >> 4;
    const uint64_t pg = t * TP + grp;
    if (pg < n) {
        uint64_t stored;
        u32x4 first;
        const uint64_t h = xxh3_page_fixed<4096, true>(pages + pg * 4096ull, L, stored, first);
        if (L.g == 0) tile_h[grp] = h;
    }
    __syncthreads();
    if (threadIdx.x < TP && t * TP + threadIdx.x < n) st_nt(out + t * TP + threadIdx.x, tile_h[threadIdx.x]);
}

// the product's descriptor body (one group per page, 4-block steps) with
// BT / 16 pages per workgroup
template <int BT>
__global__ __launch_bounds__(BT) void k_desc_bt(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                               const uint32_t* __restrict__ len, uint64_t n, uint64_t* __restrict__ out) {
    constexpr int TP = BT / 16;
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + TP - 1) / TP;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const uint64_t pg = t * TP + (threadIdx.x >> 4);
    if (pg < n) {
        uint64_t stored = 0;
        const uint64_t h = xxh3_page_rt4<true>(base + off[pg], len[pg], L, stored);
        if (L.g == 0) st_nt(out + pg, h);
    }
}

static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
    const uint64_t nbig = 1ull << 23;  // config 5: 32 GiB
    uint8_t* pages;
    uint64_t *out, *ref;
    CK(hipMalloc(&pages, nbig * 4096));
    CK(hipMalloc(&out, nbig * 8));
    CK(hipMalloc(&ref, nbig * 8));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(pages), nbig * 512);
    CK(hipDeviceSynchronize());
    struct V {
        std::string name;
        uint64_t n;
        std::function<void()> run;
        std::vector<float> us;
    };
    std::vector<V> vs;
    for (uint64_t n : {uint64_t(1) << 20, nbig}) {
        auto add = [&](int bt, auto kern) {
            char nm[64];
            std::snprintf(nm, sizeof nm, "%s  %4d threads (%2d pages/WG)", n == nbig ? "32 GiB" : " 4 GiB", bt, bt / 16);
            const unsigned g = (unsigned)((n + bt / 16 - 1) / (bt / 16));
            vs.push_back({nm, n, [=] { hipLaunchKernelGGL(kern, dim3(g), dim3(bt), 0, 0, pages, n, out); }, {}});
        };
        add(128, k_fixed_bt<128>);
        add(256, k_fixed_bt<256>);
        add(512, k_fixed_bt<512>);
        add(1024, k_fixed_bt<1024>);
    }
    // config 3 (1 M mixed 4/8/16 KiB pages packed at the start of the buffer)
    const uint64_t n3 = 1 << 20;
    std::vector<uint64_t> off3(n3);
    std::vector<uint32_t> len3(n3);
    uint64_t o3 = 0;
    for (uint64_t p = 0; p < n3; ++p) {
        const uint64_t cls = mix((0x5EED0003ull ^ p) + (0x5A5A5A5Aull + 1) * 0x9E3779B97F4A7C15ull) % 3;
        len3[p] = 4096u << cls;
        off3[p] = o3;
        o3 += len3[p];
    }
    uint64_t* d_off;
    uint32_t* d_len;
    CK(hipMalloc(&d_off, n3 * 8));
    CK(hipMalloc(&d_len, n3 * 4));
    CK(hipMemcpy(d_off, off3.data(), n3 * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_len, len3.data(), n3 * 4, hipMemcpyHostToDevice));
    const double bytes3 = (double)o3 + 8.0 * n3;
    auto add3 = [&](int bt, auto kern) {
        char nm[64];
        std::snprintf(nm, sizeof nm, "config 3 desc %4d threads (%2d pages/WG)", bt, bt / 16);
        const unsigned g = (unsigned)((n3 + bt / 16 - 1) / (bt / 16));
        vs.push_back({nm, 0, [=] { hipLaunchKernelGGL(kern, dim3(g), dim3(bt), 0, 0, pages, d_off, d_len, n3, out); }, {}});
    };
    add3(64, k_desc_bt<64>);
    add3(128, k_desc_bt<128>);
    add3(256, k_desc_bt<256>);
    add3(512, k_desc_bt<512>);
    // parity: every variant's digests equal the 256-thread ones
    for (uint64_t n : {uint64_t(1) << 20, nbig}) {
        hipLaunchKernelGGL(k_fixed_bt<256>, dim3((unsigned)(n / 16)), dim3(256), 0, 0, pages, n, ref);
        for (auto& v : vs)
            if (v.n == n) {
                CK(hipMemset(out, 0, n * 8));
                v.run();
                CK(hipDeviceSynchronize());
                std::vector<uint64_t> a(n), b(n);
                CK(hipMemcpy(a.data(), out, n * 8, hipMemcpyDeviceToHost));
                CK(hipMemcpy(b.data(), ref, n * 8, hipMemcpyDeviceToHost));
                if (a != b) {
                    std::printf("MISMATCH %s\n", v.name.c_str());
                    return 1;
                }
            }
    }
    std::printf("parity: all variants equal\n");
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    constexpr int K = 10;
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            v.run();
            CK(hipEventRecord(e0, 0));
            for (int k = 0; k < K; ++k) v.run();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(ms * 1e3f / K);
        }
    std::printf("%-36s %10s %8s %7s\n", "variant", "med_us", "TB/s", "frac");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double m = v.us[v.us.size() / 2], bytes = v.n ? v.n * 4104.0 : bytes3;
        std::printf("%-36s %10.1f %8.3f %7.4f\n", v.name.c_str(), m, bytes / m / 1e6, bytes / m / 1e6 / 8.0);
    }
    return 0;
}
