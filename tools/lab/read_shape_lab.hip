// read_shape_lab.hip — read-only access shapes over 16 KiB pages (4 GiB),
// one workgroup of 16 groups per tile, XCD-contiguous tiles, nt 16-byte
// loads, each group loading 4 KiB per step and folding it before its next
// step (the page kernels' step structure).  Not part of the product.
//
//   G1  one group per page, 16 pages per tile, 4 steps   (k_xxh3_desc on 16 KiB)
//   G2  two groups per page (A: 4 KiB pieces 0, 2; B: 1, 3), 8 pages, 2 steps:
//       each pair reads 8 KiB contiguous per step
//   G4  four groups per page, 4 pages, 1 step             (k_xxh3_split<16384>)
//
// If G2 reads like G4, a descriptor kernel that pairs groups on large pages
// (chain handed between the two groups of a wave) could close config 3's
// 16 KiB gap; if it reads like G1, it cannot.
//
//   make -C tools/lab /root/repo/tools/lab/read_shape_lab && ./tools/lab/read_shape_lab [rounds]
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
constexpr uint64_t P = 16384;

__device__ __forceinline__ uint32_t fold(u32x4 v) { return v.x ^ (v.y * 3u) ^ v.z ^ (v.w + 7u); }

// GPP groups per page; each group reads 4 KiB pieces j = sub, sub + GPP, ...
template <int GPP>
__global__ __launch_bounds__(256) void k_shape(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    constexpr int PPT = 16 / GPP;  // pages per tile
    const int g = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const uint64_t ntiles = (n + PPT - 1) / PPT, t = xcd_tile(blockIdx.x, ntiles);
    const uint64_t pg = t * PPT + grp / GPP;
    const int sub = grp % GPP;
    uint32_t r = 0;
    if (pg < n) {
        for (int j = sub; j < (int)(P / 4096); j += GPP) {
            const u32x4* base = reinterpret_cast<const u32x4*>(pages + pg * P + 4096u * j) + g;
            u32x4 d[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) d[c] = ld16<true>(base + c * 16);
#pragma unroll
            for (int c = 0; c < 16; ++c) r = r * 31u + fold(d[c]);  // waits for the step's loads
        }
    }
    if (r == 0x12345678u) out[blockIdx.x] = r;
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = i * 0x9E3779B97F4A7C15ull;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
    const uint64_t n = (4ull << 30) / P;
    uint8_t* pages;
    uint64_t* out;
    CK(hipMalloc(&pages, n * P));
    CK(hipMalloc(&out, 1 << 24));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(pages), n * P / 8);
    CK(hipDeviceSynchronize());
    struct V {
        std::string name;
        std::function<void()> run;
        std::vector<float> us;
    };
    std::vector<V> vs;
    vs.push_back({"G1 one group per page", [&] { hipLaunchKernelGGL(k_shape<1>, dim3((unsigned)(n / 16)), dim3(256), 0, 0, pages, n, out); }, {}});
    vs.push_back({"G2 two groups per page", [&] { hipLaunchKernelGGL(k_shape<2>, dim3((unsigned)(n / 8)), dim3(256), 0, 0, pages, n, out); }, {}});
    vs.push_back({"G4 four groups per page", [&] { hipLaunchKernelGGL(k_shape<4>, dim3((unsigned)(n / 4)), dim3(256), 0, 0, pages, n, out); }, {}});
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
    std::printf("%-28s %10s %8s %7s\n", "shape (16 KiB pages, 4 GiB)", "med_us", "TB/s", "frac");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double m = v.us[v.us.size() / 2], bytes = (double)n * P;
        std::printf("%-28s %10.1f %8.3f %7.4f\n", v.name.c_str(), m, bytes / m / 1e6, bytes / m / 1e6 / 8.0);
    }
    return 0;
}
