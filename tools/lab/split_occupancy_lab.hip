// split_occupancy_lab.hip — waves per SIMD of the split-page kernel
// (k_xxh3_split<P>, 8-64 KiB pages).  Not part of the product.
//
// The 4 KiB kernel reads at the best plain-read rate found (occupancy_lab);
// the 16 KiB split kernel sits ~1 % below it (0.911 against 0.921 of spec).
// Both run 4 waves per SIMD by their registers (122 / 120 VGPRs).  Here the
// product's split tile (xxh3_split_tile, included from pcs_kernels.hip) runs
// with occupancy capped by dynamic LDS at 2 and 3 waves per SIMD, beside the
// uncapped kernel, on 16 KiB and 64 KiB pages (4 GiB each), interleaved over
// rounds, medians; digests checked equal.
//
//   make -C tools/lab split_occupancy_lab && ./tools/lab/split_occupancy_lab [rounds]
#include "pcs_kernels.hip"

#include <cstdio>
#include <functional>
#include <string>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

using namespace pcs;

template <int P>
__global__ __launch_bounds__(256) void k_split_capped(const uint8_t* __restrict__ pages, uint64_t n,
                                                     uint64_t* __restrict__ out) {
    extern __shared__ uint64_t pad[];
    constexpr int PPB = 16 / (P / 4096);
    __shared__ uint64_t S[64 * 8];
    __shared__ uint64_t C[16];
    __shared__ uint64_t tile_h[16];
    __shared__ uint8_t tile_ok[16];
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + PPB - 1) / PPB;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    xxh3_split_tile<P, true>(
        L,
        [&](int ps) -> const uint8_t* {
            const uint64_t pg = t * PPB + ps;
            return pg < n ? pages + pg * (uint64_t)P : nullptr;
        },
        S, C, tile_h, tile_ok);
    __syncthreads();
    if (threadIdx.x < PPB && t * PPB + threadIdx.x < n) st_nt(out + t * PPB + threadIdx.x, tile_h[threadIdx.x]);
    if (n == 0) pad[threadIdx.x] = 0;
}

__global__ void k_fill_lab(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

size_t pad_for(int o) { return o ? 163840 / o - 8192 : 0; }

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 9;
    const uint64_t bytes = 4ull << 30;
    uint8_t* pages;
    uint64_t *out, *ref;
    CK(hipMalloc(&pages, bytes));
    CK(hipMalloc(&out, (bytes / 8192) * 8));
    CK(hipMalloc(&ref, (bytes / 8192) * 8));
    hipLaunchKernelGGL(k_fill_lab, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(pages), bytes / 8);
    CK(hipDeviceSynchronize());
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_split_capped<16384>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 150000));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_split_capped<65536>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 150000));
    struct V {
        std::string name;
        uint64_t n, P;
        bool base;
        std::function<void()> run;
        std::vector<float> us;
    };
    std::vector<V> vs;
    auto add = [&](uint64_t P, auto kern) {
        const uint64_t n = bytes / P;
        const unsigned g = (unsigned)((n + (16 / (P / 4096)) - 1) / (16 / (P / 4096)));
        for (int o : {0, 2, 3}) {
            char nm[64];
            std::snprintf(nm, sizeof nm, "%2llu KiB split waves/SIMD %s", (unsigned long long)(P >> 10),
                          o ? std::to_string(o).c_str() : "4 (native)");
            const size_t lds = pad_for(o);
            vs.push_back({nm, n, P, o == 0, [=] { hipLaunchKernelGGL(kern, dim3(g), dim3(256), lds, 0, pages, n, out); }, {}});
        }
    };
    add(16384, k_split_capped<16384>);
    add(65536, k_split_capped<65536>);
    for (auto& v : vs) {
        CK(hipMemset(out, 0, v.n * 8));
        v.run();
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        if (v.base) {
            CK(hipMemcpy(ref, out, v.n * 8, hipMemcpyDeviceToDevice));
            continue;
        }
        std::vector<uint64_t> a(v.n), b(v.n);
        CK(hipMemcpy(a.data(), out, v.n * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), ref, v.n * 8, hipMemcpyDeviceToHost));
        if (a != b) {
            std::printf("MISMATCH %s\n", v.name.c_str());
            return 1;
        }
    }
    std::printf("parity: digests equal at every occupancy\n");
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
    std::printf("%-34s %10s %8s %7s\n", "variant", "med_us", "TB/s", "frac");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double m = v.us[v.us.size() / 2], b = v.n * (v.P + 8.0);
        std::printf("%-34s %10.1f %8.3f %7.4f\n", v.name.c_str(), m, b / m / 1e6, b / m / 1e6 / 8.0);
    }
    return 0;
}
