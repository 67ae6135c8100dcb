// deferred_stamp_lab.hip — VERDICT r01 #6: a stamp that writes each page's
// 8-byte header from inside the digest kernel, but DEFERRED: a workgroup
// walks several tiles and writes the headers of its previous tile right after
// issuing the current tile's page loads, so the header writes ride behind
// loads already in flight instead of interleaving with a tile's own read
// stream.  Not part of the product.
//
// Variants, config 2 (1 M x 4 KiB), each timed as 10 back-to-back stamps (so
// write-back a variant defers into the next launch is charged):
//   two-pass    the product: digest kernel (one tile per workgroup, staged
//               results) + 8-byte nt scatter
//   inplace     headers written by the digest kernel right after each page
//               is hashed (one tile per workgroup)
//   deferred T  T tiles per workgroup (grid = tiles / T, rounded to a
//               multiple of 8 so a workgroup's tiles stay in its XCD region),
//               tile k-1's headers written after tile k's loads are issued
//   digest      digest kernel only (the floor)
// Every stamp variant is checked: all headers equal the digest kernel's output.
//
//   make -C tools/lab deferred_stamp_lab && ./tools/lab/deferred_stamp_lab [rounds]
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

// the product's 4 KiB body (xxh3_page_fixed<4096>: three full blocks and a
// final block of four chunks, all loaded in one batch), with a hook run after
// the loads are issued and before any is used
template <typename Hook>
__device__ __forceinline__ uint64_t page4k(const uint8_t* page, const Xxh3Lane& L, uint64_t& stored, Hook hook) {
    const u32x4* base = reinterpret_cast<const u32x4*>(page) + L.g;
    u32x4 d[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) d[i][c] = ld16<true>(base + i * 64 + c * 16);
    hook();
    stored = lo64(d[0][0]);
    uint64_t Ae = L.init_e, Ao = L.init_o;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        uint64_t Te, To;
        xxh3_block_terms<false>(L, d[i], lo64(d[i + 1][0]), 4, Te, To);
        Ae = xxh3_scramble(Ae + Te, L.ks_e);
        Ao = xxh3_scramble(Ao + To, L.ks_o);
    }
    uint64_t Te, To;
    xxh3_block_terms<true>(L, d[3], 0, 4, Te, To);
    return xxh3_merge(L, Ae + Te, Ao + To, (uint64_t)(P - 8));
}

__global__ __launch_bounds__(256) void k_digest(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* __restrict__ out) {
    __shared__ uint64_t tile_h[16];
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16, t = xcd_tile(blockIdx.x, ntiles);
    const int grp = threadIdx.x >> 4;
    const uint64_t pg = t * 16 + grp;
    if (pg < n) {
        uint64_t stored;
        const uint64_t h = page4k(pages + pg * (uint64_t)P, L, stored, [] {});
        if (L.g == 0) tile_h[grp] = h;
    }
    __syncthreads();
    if (threadIdx.x < 16 && t * 16 + threadIdx.x < n) st_nt(out + t * 16 + threadIdx.x, tile_h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_scatter(uint8_t* __restrict__ pages, uint64_t n, const uint64_t* __restrict__ dig) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) st_nt(reinterpret_cast<uint64_t*>(pages + i * (uint64_t)P), dig[i]);
}

__global__ __launch_bounds__(256) void k_inplace(uint8_t* __restrict__ pages, uint64_t n) {
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16, t = xcd_tile(blockIdx.x, ntiles);
    const uint64_t pg = t * 16 + (threadIdx.x >> 4);
    if (pg < n) {
        uint64_t stored;
        const uint64_t h = page4k(pages + pg * (uint64_t)P, L, stored, [] {});
        if (L.g == 0) st_nt(reinterpret_cast<uint64_t*>(pages + pg * (uint64_t)P), h);
    }
}

__global__ __launch_bounds__(256) void k_deferred(uint8_t* __restrict__ pages, uint64_t n) {
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    const int grp = threadIdx.x >> 4;
    uint64_t prev = ~0ull, prev_h = 0;  // this group's page of the previous tile
    for (uint64_t t0 = blockIdx.x; t0 < ntiles; t0 += gridDim.x) {  // gridDim % 8 == 0: tiles stay in the XCD region
        const uint64_t pg = xcd_tile(t0, ntiles) * 16 + grp;
        if (pg < n) {
            uint64_t stored;
            const uint64_t h = page4k(pages + pg * (uint64_t)P, L, stored, [&] {
                if (L.g == 0 && prev != ~0ull) st_nt(reinterpret_cast<uint64_t*>(pages + prev * (uint64_t)P), prev_h);
            });
            prev = pg;
            prev_h = h;
        } else if (L.g == 0 && prev != ~0ull) {
            st_nt(reinterpret_cast<uint64_t*>(pages + prev * (uint64_t)P), prev_h);
            prev = ~0ull;
        }
    }
    if (L.g == 0 && prev != ~0ull) st_nt(reinterpret_cast<uint64_t*>(pages + prev * (uint64_t)P), prev_h);
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

__global__ void k_zero_headers(uint8_t* pages, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) *reinterpret_cast<uint64_t*>(pages + i * (uint64_t)P) = 0;
}

__global__ void k_headers(const uint8_t* pages, uint64_t n, uint64_t* hdr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) hdr[i] = *reinterpret_cast<const uint64_t*>(pages + i * (uint64_t)P);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
    const uint64_t n = 1 << 20, ntiles = n / 16;
    uint8_t* pages;
    uint64_t *dig, *ref, *hdr;
    CK(hipMalloc(&pages, n * P));
    CK(hipMalloc(&dig, n * 8));
    CK(hipMalloc(&ref, n * 8));
    CK(hipMalloc(&hdr, n * 8));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(pages), n * P / 8);
    hipLaunchKernelGGL(k_digest, dim3((unsigned)ntiles), dim3(256), 0, 0, pages, n, ref);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> want(n);
    CK(hipMemcpy(want.data(), ref, n * 8, hipMemcpyDeviceToHost));
    struct V {
        std::string name;
        bool stamps;
        std::function<void()> run;
        std::vector<float> us;
    };
    std::vector<V> vs;
    vs.push_back({"two-pass (product)", true, [&] {
                      hipLaunchKernelGGL(k_digest, dim3((unsigned)ntiles), dim3(256), 0, 0, pages, n, dig);
                      hipLaunchKernelGGL(k_scatter, dim3((unsigned)(n / 256)), dim3(256), 0, 0, pages, n, dig);
                  }, {}});
    vs.push_back({"inplace", true, [&] { hipLaunchKernelGGL(k_inplace, dim3((unsigned)ntiles), dim3(256), 0, 0, pages, n); }, {}});
    for (int T : {2, 4, 8, 32, 64}) {
        const unsigned g = (unsigned)((ntiles / T + 7) / 8 * 8);
        vs.push_back({"deferred " + std::to_string(T) + " tiles/WG", true,
                      [=] { hipLaunchKernelGGL(k_deferred, dim3(g), dim3(256), 0, 0, pages, n); }, {}});
    }
    vs.push_back({"digest only (floor)", false,
                  [&] { hipLaunchKernelGGL(k_digest, dim3((unsigned)ntiles), dim3(256), 0, 0, pages, n, dig); }, {}});
    // parity: every stamp leaves every header equal to the digest
    for (auto& v : vs) {
        if (!v.stamps) continue;
        // zero every header first, so a variant that misses a page is caught
        hipLaunchKernelGGL(k_zero_headers, dim3((unsigned)(n / 256)), dim3(256), 0, 0, pages, n);
        v.run();
        hipLaunchKernelGGL(k_headers, dim3((unsigned)(n / 256)), dim3(256), 0, 0, pages, n, hdr);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> got(n);
        CK(hipMemcpy(got.data(), hdr, n * 8, hipMemcpyDeviceToHost));
        if (got != want) {
            std::printf("MISMATCH %s\n", v.name.c_str());
            return 1;
        }
    }
    std::printf("parity: every stamp variant leaves all %llu headers equal to the digests\n", (unsigned long long)n);
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
    std::printf("%-28s %10s %8s\n", "variant (config 2)", "us/stamp", "frac");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double m = v.us[v.us.size() / 2];
        std::printf("%-28s %10.1f %8.4f\n", v.name.c_str(), m, n * (P + 8.0) / m / 1e6 / 8.0);
    }
    return 0;
}
