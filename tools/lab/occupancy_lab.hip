// occupancy_lab.hip — waves per SIMD of the 4 KiB page kernel and of the
// plain streaming reader.  Not part of the product.
//
// The product's k_xxh3_fixed<4096> uses 120 VGPRs: 4 waves per SIMD.  The
// plain reader built on its structure (k_stream_read) uses 72: 7 waves per
// SIMD, and read 3.4 % SLOWER than the hash kernel under one protocol
// (bench.py ceiling_ab, profiles/r06/bench_r06d.json).  Here both run with
// their occupancy capped by dynamic LDS (blocks per CU = waves per SIMD for a
// 256-thread block: 160 KiB / o bytes each), o = 2 .. their register limit,
// on config 2 (4 GiB) and config 5 (32 GiB), interleaved over rounds,
// medians.  Hash digests are checked equal across occupancies.
//
//   make -C tools/lab occupancy_lab && ./tools/lab/occupancy_lab [rounds]
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

// k_xxh3_fixed<4096, digest, nt> with a full-coverage grid
__global__ __launch_bounds__(256) void k_hash(const uint8_t* __restrict__ pages, uint64_t n,
                                             uint64_t* __restrict__ out) {
    extern __shared__ uint64_t pad[];  // occupancy cap only
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
    if (n == 0) pad[threadIdx.x] = 0;  // never: keeps the array
}

// k_stream_read (pcs_kernels.hip), whole pages only
__global__ __launch_bounds__(256) void k_read(const uint8_t* __restrict__ buf, uint64_t n, uint64_t* __restrict__ out) {
    extern __shared__ uint64_t pad[];
    __shared__ uint64_t tile_h[16];
    const int g = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const uint64_t ntiles = (n + 15) / 16;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const uint64_t pg = t * 16 + grp;
    if (pg < n) {
        const u32x4* base = reinterpret_cast<const u32x4*>(buf + pg * 4096ull) + g;
        u32x4 d[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) d[c] = ld16<true>(base + c * 16);
        uint32_t x = 0, y = 0, z = 0, v = 0;
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            x ^= d[c].x;
            y += d[c].y;
            z ^= d[c].z;
            v += d[c].w;
        }
        uint64_t r = ((uint64_t)(x ^ z) << 32) | (y + v);
        r ^= dpp64<kRowRor1>(r);
        r ^= dpp64<kRowRor2>(r);
        r ^= dpp64<kRowRor4>(r);
        r ^= dpp64<kRowRor8>(r);
        if (g == 0) tile_h[grp] = r;
    }
    __syncthreads();
    if (threadIdx.x < 16 && t * 16 + threadIdx.x < n) st_nt(out + t * 16 + threadIdx.x, tile_h[threadIdx.x]);
    if (n == 0) pad[threadIdx.x] = 0;
}

// k_read with each 16-lane group reading TWO pages (32 dwordx4 loads per lane
// in flight), 32 pages per workgroup; NT: non-temporal (1) or default policy
template <int NPG, bool NT>
__global__ __launch_bounds__(256) void k_read_multi(const uint8_t* __restrict__ buf, uint64_t n,
                                                   uint64_t* __restrict__ out) {
    extern __shared__ uint64_t pad[];
    __shared__ uint64_t tile_h[16 * NPG];
    const int g = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const uint64_t ntiles = (n + 16 * NPG - 1) / (16 * NPG);
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    u32x4 d[NPG][16];
#pragma unroll
    for (int q = 0; q < NPG; ++q) {
        const uint64_t pg = t * 16 * NPG + q * 16 + grp;
        const u32x4* base = reinterpret_cast<const u32x4*>(buf + (pg < n ? pg : 0) * 4096ull) + g;
#pragma unroll
        for (int c = 0; c < 16; ++c) d[q][c] = ld16<NT>(base + c * 16);
    }
#pragma unroll
    for (int q = 0; q < NPG; ++q) {
        uint32_t x = 0, y = 0, z = 0, v = 0;
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            x ^= d[q][c].x;
            y += d[q][c].y;
            z ^= d[q][c].z;
            v += d[q][c].w;
        }
        uint64_t r = ((uint64_t)(x ^ z) << 32) | (y + v);
        r ^= dpp64<kRowRor1>(r);
        r ^= dpp64<kRowRor2>(r);
        r ^= dpp64<kRowRor4>(r);
        r ^= dpp64<kRowRor8>(r);
        if (g == 0) tile_h[q * 16 + grp] = r;
    }
    __syncthreads();
    if (threadIdx.x < 16 * NPG && t * 16 * NPG + threadIdx.x < n) st_nt(out + t * 16 * NPG + threadIdx.x, tile_h[threadIdx.x]);
    if (n == 0) pad[threadIdx.x] = 0;
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

// dynamic LDS per block for o blocks (= waves per SIMD) per CU; 0: no cap
size_t pad_for(int o) { return o ? 163840 / o - 2048 : 0; }

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
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_hash), hipFuncAttributeMaxDynamicSharedMemorySize, 160000));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_read), hipFuncAttributeMaxDynamicSharedMemorySize, 160000));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_read_multi<2, true>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 150000));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_read_multi<1, false>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 150000));
    struct V {
        std::string name;
        uint64_t n;
        bool hash;
        std::function<void()> run;
        std::vector<float> us;
    };
    std::vector<V> vs;
    for (uint64_t n : {uint64_t(1) << 20, nbig}) {
        const unsigned g = (unsigned)(n / 16);
        for (int o : {0, 2, 3, 4}) {
            char nm[64];
            std::snprintf(nm, sizeof nm, "%s hash  waves/SIMD %s", n == nbig ? "32 GiB" : " 4 GiB",
                          o ? std::to_string(o).c_str() : "4 (native)");
            const size_t lds = pad_for(o);
            vs.push_back({nm, n, true, [=] { hipLaunchKernelGGL(k_hash, dim3(g), dim3(256), lds, 0, pages, n, out); }, {}});
        }
        for (int o : {0, 1, 2, 3, 4}) {
            char nm[64];
            std::snprintf(nm, sizeof nm, "%s read  waves/SIMD %s", n == nbig ? "32 GiB" : " 4 GiB",
                          o ? std::to_string(o).c_str() : "7 (native)");
            const size_t lds = pad_for(o);
            vs.push_back({nm, n, false, [=] { hipLaunchKernelGGL(k_read, dim3(g), dim3(256), lds, 0, pages, n, out); }, {}});
        }
        for (int o : {1, 2, 3}) {  // two pages per group: twice the bytes in flight per wave
            char nm[64];
            std::snprintf(nm, sizeof nm, "%s read2 waves/SIMD %d", n == nbig ? "32 GiB" : " 4 GiB", o);
            const size_t lds = pad_for(o);
            const unsigned g2 = (unsigned)(n / 32);
            vs.push_back({nm, n, false,
                          [=] { hipLaunchKernelGGL((k_read_multi<2, true>), dim3(g2), dim3(256), lds, 0, pages, n, out); },
                          {}});
        }
        for (int o : {2, 3}) {  // default cache policy
            char nm[64];
            std::snprintf(nm, sizeof nm, "%s read-cached waves/SIMD %d", n == nbig ? "32 GiB" : " 4 GiB", o);
            const size_t lds = pad_for(o);
            vs.push_back({nm, n, false,
                          [=] { hipLaunchKernelGGL((k_read_multi<1, false>), dim3(g), dim3(256), lds, 0, pages, n, out); },
                          {}});
        }
    }
    for (auto& v : vs) {  // every variant launches; hash digests equal the uncapped ones
        CK(hipMemset(out, 0, v.n * 8));
        v.run();
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        if (!v.hash) continue;
        if (v.name.find("native") != std::string::npos) {
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
    std::printf("parity: hash digests equal at every occupancy\n");
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
        const double m = v.us[v.us.size() / 2], bytes = v.n * 4104.0;
        std::printf("%-36s %10.1f %8.3f %7.4f\n", v.name.c_str(), m, bytes / m / 1e6, bytes / m / 1e6 / 8.0);
    }
    return 0;
}
