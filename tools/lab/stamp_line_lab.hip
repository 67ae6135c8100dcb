// stamp_line_lab.hip — cost of the stamp's write pass.  Not part of the product.
//
// The product stamp (SetChecksum over a batch) runs the digest kernel into a
// compact 8-byte array, then k_scatter_stamp writes 8 bytes into every page
// header: 53 us for 1 M pages after a full read pass.  An
// 8-byte write is a partial line the memory side must merge.  This harness
// asks whether a two-pass stamp that writes WHOLE 64-byte header lines is
// cheaper: pass 1 keeps the page's first 64 bytes (lanes 0-3 of the group
// already hold them) and writes digest + bytes [8, 64) into a compact line
// array; pass 2 copies each 64-byte line over the page's first line.
//
//   digest8      product pass 1 (16 digests staged per tile, one 128 B store)
//   digestline   pass 1 writing 64 B lines (lanes 0-3 of each group, nt)
//   scatter8     product pass 2: one 8-byte nt store per page
//   scatter64    4 lanes per page, 16 B nt stores from the compact lines
//   scatter64p   same with plain stores
//   scatter8p    same with a plain store
//   rmw64        read the page's first line, patch 8 bytes, write it back (nt)
//   rmw64p/32p/128p  the same with plain stores over 64 / 32 / 128 bytes
// Each variant is timed right after a full nt read of the batch (the state
// the product's scatter runs in).  Parity: after the 8-byte stamp and the
// line stamp the first 64 bytes of every checked page must be identical.
//
//   make -C tools/lab && ./tools/lab/stamp_line_lab [rounds]
#include <hip/hip_runtime.h>

#include "xxh3_page.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

template <bool LINE>
__global__ __launch_bounds__(256) void k_digest(const uint8_t* __restrict__ pages, uint64_t n,
                                               uint64_t* __restrict__ out, u32x4* __restrict__ lines) {
    __shared__ uint64_t tile_h[16];
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const int grp = threadIdx.x >> 4;
    const uint64_t pg = t * 16 + grp;
    if (pg < n) {
        uint64_t stored;
        u32x4 first;
        const uint64_t h = xxh3_page_fixed<P, true>(pages + pg * (uint64_t)P, L, stored, first);
        if (LINE) {
            if (L.g == 0) {
                first.x = (uint32_t)h;
                first.y = (uint32_t)(h >> 32);
            }
            if (L.g < 4) st_nt(lines + pg * 4 + L.g, first);
        } else if (L.g == 0) {
            tile_h[grp] = h;
        }
    }
    if (!LINE) {
        __syncthreads();
        const uint64_t i = t * 16 + threadIdx.x;
        if (threadIdx.x < 16 && i < n) st_nt(out + i, tile_h[threadIdx.x]);
    }
}

template <bool NTS>
__global__ __launch_bounds__(256) void k_scatter8(uint8_t* __restrict__ pages, uint64_t n,
                                                 const uint64_t* __restrict__ dig) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint64_t* dst = reinterpret_cast<uint64_t*>(pages + i * P);
        if (NTS) st_nt(dst, dig[i]);
        else *dst = dig[i];
    }
}

template <bool NTS>
__global__ __launch_bounds__(256) void k_scatter64(uint8_t* __restrict__ pages, uint64_t n,
                                                  const u32x4* __restrict__ lines) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i = k >> 2;
    if (i < n) {
        const u32x4 v = __builtin_nontemporal_load(lines + k);
        u32x4* dst = reinterpret_cast<u32x4*>(pages + i * P) + (k & 3);
        if (NTS) st_nt(dst, v);
        else *dst = v;
    }
}

template <bool NTS, int LINE>
__global__ __launch_bounds__(256) void k_rmw(uint8_t* __restrict__ pages, uint64_t n,
                                            const uint64_t* __restrict__ dig) {
    constexpr int LPP = LINE / 16;  // lanes per page
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i = k / LPP;
    if (i < n) {
        u32x4* dst = reinterpret_cast<u32x4*>(pages + i * P) + (k % LPP);
        u32x4 v = *dst;
        if ((k % LPP) == 0) {
            const uint64_t h = dig[i];
            v.x = (uint32_t)h;
            v.y = (uint32_t)(h >> 32);
        }
        if (NTS) st_nt(dst, v);
        else *dst = v;
    }
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

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 9;
    const uint64_t n = 1ull << 20, bytes = n * P, ntiles = n / 16;
    uint8_t *pages, *pages2;
    uint64_t* dig;
    u32x4* lines;
    uint32_t* sink;
    CK(hipMalloc(&pages, bytes));
    CK(hipMalloc(&pages2, bytes));
    CK(hipMalloc(&dig, n * 8));
    CK(hipMalloc(&lines, n * 64));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(pages), bytes / 8);
    CK(hipMemcpy(pages2, pages, bytes, hipMemcpyDeviceToDevice));
    CK(hipDeviceSynchronize());

    // parity: two-pass 8-byte stamp on pages, line stamp on pages2
    hipLaunchKernelGGL(k_digest<false>, dim3(ntiles), dim3(256), 0, 0, pages, n, dig, lines);
    hipLaunchKernelGGL(k_scatter8<true>, dim3(n / 256), dim3(256), 0, 0, pages, n, dig);
    hipLaunchKernelGGL(k_digest<true>, dim3(ntiles), dim3(256), 0, 0, pages2, n, dig, lines);
    hipLaunchKernelGGL(k_scatter64<true>, dim3(n * 4 / 256), dim3(256), 0, 0, pages2, n, lines);
    CK(hipDeviceSynchronize());
    {
        std::vector<uint8_t> a(64), b(64);
        uint64_t bad = 0;
        for (uint64_t i = 0; i < n; i += 997) {
            CK(hipMemcpy(a.data(), pages + i * P, 64, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), pages2 + i * P, 64, hipMemcpyDeviceToHost));
            bad += a != b;
        }
        std::printf("parity (every 997th page, first 64 B): %s\n", bad ? "FAIL" : "ok");
        if (bad) return 1;
    }

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"digest8",   "digestline", "scatter8", "scatter8p", "scatter64", "scatter64p",
                           "rmw64",     "rmw64p",     "rmw32p",   "rmw128p"};
    constexpr int NV = 10;
    std::vector<std::vector<float>> ts(NV);
    for (int r = 0; r < rounds; ++r)
        for (int v = 0; v < NV; ++v) {
            hipLaunchKernelGGL(k_read_all, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const u32x4*>(pages),
                               bytes / 16, sink);
            CK(hipEventRecord(e0, 0));
            const dim3 g4(n * 4 / 256), g2(n * 2 / 256), g8(n * 8 / 256), g1(n / 256), b(256);
            switch (v) {
                case 0: hipLaunchKernelGGL(k_digest<false>, dim3(ntiles), b, 0, 0, pages, n, dig, lines); break;
                case 1: hipLaunchKernelGGL(k_digest<true>, dim3(ntiles), b, 0, 0, pages, n, dig, lines); break;
                case 2: hipLaunchKernelGGL(k_scatter8<true>, g1, b, 0, 0, pages, n, dig); break;
                case 3: hipLaunchKernelGGL(k_scatter8<false>, g1, b, 0, 0, pages, n, dig); break;
                case 4: hipLaunchKernelGGL(k_scatter64<true>, g4, b, 0, 0, pages, n, lines); break;
                case 5: hipLaunchKernelGGL(k_scatter64<false>, g4, b, 0, 0, pages, n, lines); break;
                case 6: hipLaunchKernelGGL((k_rmw<true, 64>), g4, b, 0, 0, pages, n, dig); break;
                case 7: hipLaunchKernelGGL((k_rmw<false, 64>), g4, b, 0, 0, pages, n, dig); break;
                case 8: hipLaunchKernelGGL((k_rmw<false, 32>), g2, b, 0, 0, pages, n, dig); break;
                case 9: hipLaunchKernelGGL((k_rmw<false, 128>), g8, b, 0, 0, pages, n, dig); break;
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts[v].push_back(ms * 1e3f);
        }
    for (int v = 0; v < NV; ++v) {
        auto t = ts[v];
        std::sort(t.begin(), t.end());
        std::printf("  %-12s med %7.1f us  best %7.1f us\n", names[v], t[t.size() / 2], t[0]);
    }

    // Whole stamps back to back (what bench --mode stamp runs): K x (pass 1 +
    // pass 2) between two events, so write-back a pass defers into the next
    // launch is charged too.  Interleaved over rounds.
    constexpr int K = 10;
    const char* pnames[] = {"stamp: digest8 + scatter8 (nt)", "stamp: digest8 + scatter8p",
                            "stamp: digestline + scatter64 (nt)", "stamp: digestline + scatter64p",
                            "stamp: digest8 + rmw64 (nt)", "digest8 only"};
    constexpr int NP = 6;
    std::vector<std::vector<float>> pt(NP);
    for (int r = 0; r < rounds; ++r)
        for (int v = 0; v < NP; ++v) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            const dim3 g4(n * 4 / 256), g1(n / 256), b(256), gt(ntiles);
            for (int k = 0; k < K; ++k) {
                switch (v) {
                    case 0:
                        hipLaunchKernelGGL(k_digest<false>, gt, b, 0, 0, pages, n, dig, lines);
                        hipLaunchKernelGGL(k_scatter8<true>, g1, b, 0, 0, pages, n, dig);
                        break;
                    case 1:
                        hipLaunchKernelGGL(k_digest<false>, gt, b, 0, 0, pages, n, dig, lines);
                        hipLaunchKernelGGL(k_scatter8<false>, g1, b, 0, 0, pages, n, dig);
                        break;
                    case 2:
                        hipLaunchKernelGGL(k_digest<true>, gt, b, 0, 0, pages, n, dig, lines);
                        hipLaunchKernelGGL(k_scatter64<true>, g4, b, 0, 0, pages, n, lines);
                        break;
                    case 3:
                        hipLaunchKernelGGL(k_digest<true>, gt, b, 0, 0, pages, n, dig, lines);
                        hipLaunchKernelGGL(k_scatter64<false>, g4, b, 0, 0, pages, n, lines);
                        break;
                    case 4:
                        hipLaunchKernelGGL(k_digest<false>, gt, b, 0, 0, pages, n, dig, lines);
                        hipLaunchKernelGGL((k_rmw<true, 64>), g4, b, 0, 0, pages, n, dig);
                        break;
                    case 5: hipLaunchKernelGGL(k_digest<false>, gt, b, 0, 0, pages, n, dig, lines); break;
                }
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            pt[v].push_back(ms * 1e3f / K);
        }
    for (int v = 0; v < NP; ++v) {
        auto t = pt[v];
        std::sort(t.begin(), t.end());
        std::printf("  %-36s med %7.1f us/stamp  best %7.1f\n", pnames[v], t[t.size() / 2], t[0]);
    }
    return 0;
}
