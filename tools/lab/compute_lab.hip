// compute_lab.hip — the VALU ceiling of each hash as the product computes it,
// with no memory traffic.  Not part of the product.
//
// The page kernels are HBM-bound when the hash is cheap enough; this measures
// how fast the chip can run the product's own arithmetic if bytes cost
// nothing: the XXH3 block fold (xxh3_block_terms: 16-lane groups, DPP row
// folds) + scramble per 1 KiB, and the XXH64 quad chunk (xxh64_chunk: two
// serial rounds per lane per 64 B, one DPP quad swap) per 64 B.  Input words
// come from registers, perturbed by the step counter (one XOR per word) so
// nothing is hoisted.  Full occupancy grid, 8 waves per SIMD worth of work.
// Result: bytes hashed per second, to set next to the 8 TB/s HBM peak.
//
//   make -C tools/lab compute_lab && ./tools/lab/compute_lab
#include <hip/hip_runtime.h>

#include "xxh3_page.h"

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

using namespace pcs;

// xxh64 pieces as in pcs_kernels.hip (XXH64_round, xxhash.h:3469-3491)
__device__ __forceinline__ uint64_t rotl64c(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t x64_round(uint64_t acc, uint64_t in) {
    acc += in * kP64_2;
    return rotl64c(acc, 31) * kP64_1;
}
constexpr int kQuadSwap = 2 | (3 << 2) | (0 << 4) | (1 << 6);

// XXH3: each 16-lane group folds 1 KiB blocks (4 chunks of 256 B); steps blocks per group
__global__ __launch_bounds__(256) void k_x3(uint64_t* out, int steps, uint32_t seed) {
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    u32x4 d[5];
    for (int c = 0; c < 5; ++c) d[c] = u32x4{seed + threadIdx.x, seed * 3u + c, seed ^ 0x9E37u, (uint32_t)c};
    uint64_t Ae = L.init_e, Ao = L.init_o;
    for (int s = 0; s < steps; ++s) {
        u32x4 b[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            b[c] = d[c];
            b[c].x ^= (uint32_t)s;
        }
        uint64_t Te, To;
        xxh3_block_terms<false>(L, b, lo64(d[4]) ^ (uint64_t)s, 4, Te, To);
        Ae = xxh3_scramble(Ae + Te, L.ks_e);
        Ao = xxh3_scramble(Ao + To, L.ks_o);
    }
    if ((Ae ^ Ao) == 0x12345) out[blockIdx.x] = Ae;
}

// XXH64: each quad consumes 64 B chunks (2 rounds per lane); steps chunks per quad
__global__ __launch_bounds__(256) void k_x64(uint64_t* out, int steps, uint32_t seed) {
    const int q = threadIdx.x & 3;
    u32x4 d = u32x4{seed + threadIdx.x, seed * 3u, seed ^ 0x9E37u, 7u};
    uint64_t v = kP64_1 + q;
    for (int s = 0; s < steps; ++s) {
        u32x4 e = d;
        e.x ^= (uint32_t)s;
        const uint64_t e0 = lo64(e), e1 = hi64(e);
        const bool sends_e0 = (q == 0) || (q == 3);
        const uint64_t send = sends_e0 ? e0 : e1;
        const uint64_t keep = sends_e0 ? e1 : e0;
        const uint64_t recv = dpp64<kQuadSwap>(send);
        v = x64_round(x64_round(v, q < 2 ? keep : recv), q < 2 ? recv : keep);
    }
    if (v == 0x12345) out[blockIdx.x] = v;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint64_t* out;
    CK(hipMalloc(&out, 1 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int steps = 4096;
    for (int bpc : {4, 8, 16}) {
        const unsigned grid = (unsigned)(cus * bpc);
        float ms3 = 0, ms64 = 0;
        for (int rep = 0; rep < 2; ++rep) {  // second run timed
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_x3, dim3(grid), dim3(256), 0, 0, out, steps, 1u + rep);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms3, e0, e1));
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_x64, dim3(grid), dim3(256), 0, 0, out, steps, 1u + rep);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms64, e0, e1));
        }
        // bytes: XXH3 16 groups x 1 KiB per step per block; XXH64 64 quads x 64 B per step per block
        const double b3 = (double)grid * 16 * 1024 * steps, b64 = (double)grid * 64 * 64 * steps;
        std::printf("blocks/CU %2d: XXH3 fold+scramble %7.2f TB/s (%.2f ms)   XXH64 rounds %7.2f TB/s (%.2f ms)\n", bpc,
                    b3 / ms3 / 1e9, ms3, b64 / ms64 / 1e9, ms64);
    }
    return 0;
}
