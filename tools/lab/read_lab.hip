// read_lab.hip — access-pattern experiments for the page-checksum kernels.
// Not part of the product.  Times read-only variants over 1 M x 4 KiB pages
// (4 GiB) in interleaved rounds (one process, cdna_hip_programming.md §5.4
// rule 24) and prints the median GB/s of each.
//
//   make -C tools/lab        (links the product library for A/B against it)
//   ./tools/lab/read_lab [rounds] [const]
#include <hip/hip_runtime.h>

#include "eloqstore_pcs.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

__device__ __forceinline__ uint32_t fold(u32x4 v) { return v.x ^ (v.y * 3u) ^ v.z ^ (v.w + 7u); }

// A: 16-lane group per page, 4 pages per wave (the product layout)
template <int P, bool NT>
__global__ __launch_bounds__(256) void k_group16(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    const int g = threadIdx.x & 15;
    const uint64_t ngroups = (uint64_t)gridDim.x * 16;
    for (uint64_t pg = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 4; pg < n; pg += ngroups) {
        const u32x4* base = reinterpret_cast<const u32x4*>(pages + pg * P) + g;
        u32x4 d[P / 256];
#pragma unroll
        for (int c = 0; c < P / 256; ++c) d[c] = ld<NT>(base + c * 16);
        uint32_t r = 0;
#pragma unroll
        for (int c = 0; c < P / 256; ++c) r += fold(d[c]);
        if (r == 0x12345678u) out[pg] = r;  // practically never: keeps loads live
    }
}

// A2: as A, but every page writes its 8-byte result (lane 0 of the group),
// or (STAGED) the block's 16 results are staged in LDS and written by 16 lanes
// of wave 0 as one 128-byte store.
template <int P, bool STAGED>
__global__ __launch_bounds__(256) void k_group16_store(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    __shared__ uint64_t res[16];
    const int g = threadIdx.x & 15;
    const uint64_t pg = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    uint32_t r = 0;
    if (pg < n) {
        const u32x4* base = reinterpret_cast<const u32x4*>(pages + pg * P) + g;
        u32x4 d[P / 256];
#pragma unroll
        for (int c = 0; c < P / 256; ++c) d[c] = ld<true>(base + c * 16);
#pragma unroll
        for (int c = 0; c < P / 256; ++c) r += fold(d[c]);
    }
    if constexpr (STAGED) {
        if (g == 0) res[threadIdx.x >> 4] = r;
        __syncthreads();
        const uint64_t first = (uint64_t)blockIdx.x * 16;
        if (threadIdx.x < 16 && first + threadIdx.x < n) out[first + threadIdx.x] = res[threadIdx.x];
    } else {
        if (g == 0 && pg < n) out[pg] = r;
    }
}

// A3: each block hashes 16*M contiguous pages (M rounds of 16), keeps the
// results in LDS and writes them as one 128*M-byte burst at the end.
template <int P, int M, bool NTST>
__global__ __launch_bounds__(256) void k_group16_batchstore(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    __shared__ uint64_t res[16 * M];
    const int g = threadIdx.x & 15;
    const uint64_t first = (uint64_t)blockIdx.x * 16 * M;
    for (int m = 0; m < M; ++m) {
        const uint64_t pg = first + m * 16 + (threadIdx.x >> 4);
        uint32_t r = 0;
        if (pg < n) {
            const u32x4* base = reinterpret_cast<const u32x4*>(pages + pg * P) + g;
            u32x4 d[P / 256];
#pragma unroll
            for (int c = 0; c < P / 256; ++c) d[c] = ld<true>(base + c * 16);
#pragma unroll
            for (int c = 0; c < P / 256; ++c) r += fold(d[c]);
        }
        if (g == 0) res[m * 16 + (threadIdx.x >> 4)] = r;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 16 * M; i += 256)
        if (first + i < n) {
            if constexpr (NTST) __builtin_nontemporal_store(res[i], out + first + i);
            else out[first + i] = res[i];
        }
}

// A4: group16 nt, non-persistent, with the block -> tile map remapped so the
// blocks that share an XCD (b % 8 equal) stream one contiguous 1/8 of the
// buffer (cdna_hip_programming.md T1) instead of interleaving 64 KiB tiles.
template <int P>
__global__ __launch_bounds__(256) void k_group16_xcd(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    const uint64_t nb = gridDim.x, b = blockIdx.x;
    const uint64_t q = nb / 8, tile = (b % 8) * q + b / 8;  // nb % 8 == 0 here
    const int g = threadIdx.x & 15;
    const uint64_t pg = tile * 16 + (threadIdx.x >> 4);
    if (pg >= n) return;
    const u32x4* base = reinterpret_cast<const u32x4*>(pages + pg * P) + g;
    u32x4 d[P / 256];
#pragma unroll
    for (int c = 0; c < P / 256; ++c) d[c] = ld<true>(base + c * 16);
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < P / 256; ++c) r += fold(d[c]);
    if (r == 0x12345678u) out[pg] = r;
}

// B: one page per wave, 1 KiB contiguous per wave-instruction
template <int P, bool NT>
__global__ __launch_bounds__(256) void k_wavepage(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    for (uint64_t pg = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; pg < n; pg += nwaves) {
        const u32x4* base = reinterpret_cast<const u32x4*>(pages + pg * P) + lane;
        u32x4 d[P / 1024];
#pragma unroll
        for (int c = 0; c < P / 1024; ++c) d[c] = ld<NT>(base + c * 64);
        uint32_t r = 0;
#pragma unroll
        for (int c = 0; c < P / 1024; ++c) r += fold(d[c]);
        if (r == 0x12345678u) out[pg] = r;
    }
}

// C: canonical linear grid-stride, U loads in flight per lane
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_linear(const uint8_t* __restrict__ buf, uint64_t nvec, uint64_t* out) {
    const u32x4* v = reinterpret_cast<const u32x4*>(buf);
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint32_t r = 0;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = ld<NT>(v + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) r += fold(d[u]);
    }
    for (; i < nvec; i += stride) r += fold(ld<NT>(v + i));
    if (r == 0x12345678u) out[0] = r;
}

// D: 16-lane group per page, but the 4 pages of a wave are page-interleaved so
// that one wave-instruction reads 1 KiB contiguous: wave w owns pages
// 4w..4w+3 and lane l reads page 4w + (c*4 + l/16)/16 ... (contiguous 1 KiB:
// instruction i covers bytes [i*1024, i*1024+1024) of the wave's 16 KiB span)
template <bool NT>
__global__ __launch_bounds__(256) void k_group16_contig(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    constexpr int P = 4096;
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    for (uint64_t w = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; w * 4 < n; w += nwaves) {
        const u32x4* base = reinterpret_cast<const u32x4*>(pages + w * 4 * P) + lane;
        u32x4 d[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) d[i] = ld<NT>(base + i * 64);
        uint32_t r = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) r += fold(d[i]);
        if (r == 0x12345678u) out[w] = r;
    }
}

// E: LDS-DMA (global_load_lds_dwordx4) staging of each group's page, 16 KiB
// per wave per step, then LDS reads.  One wave per block slice.
template <bool NT>
__global__ __launch_bounds__(256) void k_glds(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    constexpr int P = 4096;
    __shared__ __attribute__((aligned(16))) uint8_t lds[4][4 * P];  // 64 KiB: 16 KiB per wave
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    for (uint64_t w = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; w * 4 < n; w += nwaves) {
        const uint8_t* src = pages + w * 4 * P + lane * 16;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(src + i * 1024), (void __attribute__((address_space(3)))*)(&lds[wv][i * 1024]), 16, 0, NT ? 2 : 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t r = 0;
        const u32x4* l = reinterpret_cast<const u32x4*>(&lds[wv][0]) + lane;
#pragma unroll
        for (int i = 0; i < 16; ++i) r += fold(l[i * 64]);
        if (r == 0x12345678u) out[w] = r;
        __builtin_amdgcn_wave_barrier();
    }
}

// F: XXH64 pattern: one quad per page, 16 pages per wave, 64 B per page per
// wave-instruction, U chunks in flight per lane.
template <int P, bool NT, int U>
__global__ __launch_bounds__(256) void k_quad64(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    const int q = threadIdx.x & 3;
    const uint64_t nq = (uint64_t)gridDim.x * 64;
    for (uint64_t pg = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 2; pg < n; pg += nq) {
        const u32x4* base = reinterpret_cast<const u32x4*>(pages + pg * P) + q;
        uint32_t r = 0;
        for (int k = 0; k < P / 64; k += U) {
            u32x4 d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) d[u] = ld<NT>(base + 4 * (k + u));
#pragma unroll
            for (int u = 0; u < U; ++u) r += fold(d[u]);
        }
        if (r == 0x12345678u) out[pg] = r;
    }
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + 12345;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

__global__ void k_spin(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
}

struct Variant {
    std::string name;
    std::function<void(hipStream_t)> run;
    std::vector<float> ms;
};

// G: 64 KiB pages, one workgroup per page: group j reads the page's 4 KiB
// slice j (the shape of a split long-page hash: block sums in parallel, one
// short serial chain per page).
template <bool NT>
__global__ __launch_bounds__(256) void k_wg_page64k(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    const int g = threadIdx.x & 15, j = threadIdx.x >> 4;
    for (uint64_t pg = blockIdx.x; pg < n; pg += gridDim.x) {
        const u32x4* base = reinterpret_cast<const u32x4*>(pages + pg * 65536 + j * 4096) + g;
        u32x4 d[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) d[c] = ld<NT>(base + c * 16);
        uint32_t r = 0;
#pragma unroll
        for (int c = 0; c < 16; ++c) r += fold(d[c]);
        if (r == 0x12345678u) out[pg] = r;
    }
}

// A5: product-like 64 KiB: 16-lane group per page, 4 KiB batches in sequence.
template <bool NT>
__global__ __launch_bounds__(256) void k_group16_big(const uint8_t* __restrict__ pages, uint64_t n, uint64_t* out) {
    const int g = threadIdx.x & 15;
    const uint64_t ngroups = (uint64_t)gridDim.x * 16;
    for (uint64_t pg = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 4; pg < n; pg += ngroups) {
        uint32_t r = 0;
        for (int b = 0; b < 16; ++b) {
            const u32x4* base = reinterpret_cast<const u32x4*>(pages + pg * 65536 + b * 4096) + g;
            u32x4 d[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) d[c] = ld<NT>(base + c * 16);
#pragma unroll
            for (int c = 0; c < 16; ++c) r += fold(d[c]);
        }
        if (r == 0x12345678u) out[pg] = r;
    }
}

// Stamp pass-2 variants: write each page's 8-byte digest into its header.
// W = bytes written per page (8/16/32: from the digest + zeros would corrupt,
// so W > 8 re-reads the line first: read W bytes, patch 8, write W).
template <int W, bool NTST>
__global__ __launch_bounds__(256) void k_scatter(uint8_t* __restrict__ pages, uint64_t P, uint64_t n,
                                                 const uint64_t* __restrict__ dig) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t* dst = reinterpret_cast<uint64_t*>(pages + i * P);
    if constexpr (W == 8) {
        if constexpr (NTST) __builtin_nontemporal_store(dig[i], dst);
        else *dst = dig[i];
    } else {
        uint64_t line[W / 8];
#pragma unroll
        for (int k = 0; k < W / 8; ++k) line[k] = dst[k];
        line[0] = dig[i];
#pragma unroll
        for (int k = 0; k < W / 8; ++k) {
            if constexpr (NTST) __builtin_nontemporal_store(line[k], dst + k);
            else dst[k] = line[k];
        }
    }
}

// one wave per 64 pages, but lanes cooperate: lane l writes 8 B of page
// (base + l / (W/8)) so each page's W-byte header is one contiguous store
// group (W > 8 re-reads the header first).
template <int W>
__global__ __launch_bounds__(256) void k_scatter_coop(uint8_t* __restrict__ pages, uint64_t P, uint64_t n,
                                                      const uint64_t* __restrict__ dig) {
    constexpr int L = W / 8;  // lanes per page
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i = t / L;
    const int k = (int)(t % L);
    if (i >= n) return;
    uint64_t* dst = reinterpret_cast<uint64_t*>(pages + i * P) + k;
    const uint64_t v = k == 0 ? dig[i] : *dst;
    __builtin_nontemporal_store(v, dst);
}

static int main_stamp(int rounds) {
    const uint64_t P = 4096, n = 1 << 20, bytes = n * P;
    uint8_t* pages;
    uint64_t* dig;
    CK(hipMalloc(&pages, bytes));
    CK(hipMalloc(&dig, n * 8));
    if (pcs_gen_pages_dev(pages, P, n, 0x5EED0002, 0, nullptr)) std::exit(2);
    if (pcs_pages_digest_dev(pages, P, n, 0, dig, nullptr)) std::exit(2);
    CK(hipDeviceSynchronize());
    hipStream_t s;
    CK(hipStreamCreate(&s));
    struct V { std::string name; std::function<void(hipStream_t)> run; std::vector<float> ms; };
    std::vector<V> vs;
    auto add = [&](std::string name, std::function<void(hipStream_t)> f) { vs.push_back({name, f, {}}); };
    const unsigned g1 = (unsigned)((n + 255) / 256);
    add("scatter 8B plain", [=](hipStream_t st) { hipLaunchKernelGGL((k_scatter<8, false>), dim3(g1), dim3(256), 0, st, pages, P, n, dig); });
    add("scatter 8B nt", [=](hipStream_t st) { hipLaunchKernelGGL((k_scatter<8, true>), dim3(g1), dim3(256), 0, st, pages, P, n, dig); });
    add("scatter 32B rmw nt", [=](hipStream_t st) { hipLaunchKernelGGL((k_scatter<32, true>), dim3(g1), dim3(256), 0, st, pages, P, n, dig); });
    add("scatter 64B rmw nt", [=](hipStream_t st) { hipLaunchKernelGGL((k_scatter<64, true>), dim3(g1), dim3(256), 0, st, pages, P, n, dig); });
    add("scatter 64B rmw plain", [=](hipStream_t st) { hipLaunchKernelGGL((k_scatter<64, false>), dim3(g1), dim3(256), 0, st, pages, P, n, dig); });
    add("coop 32B", [=](hipStream_t st) { hipLaunchKernelGGL((k_scatter_coop<32>), dim3(g1 * 4), dim3(256), 0, st, pages, P, n, dig); });
    add("coop 64B", [=](hipStream_t st) { hipLaunchKernelGGL((k_scatter_coop<64>), dim3(g1 * 8), dim3(256), 0, st, pages, P, n, dig); });
    add("coop 128B", [=](hipStream_t st) { hipLaunchKernelGGL((k_scatter_coop<128>), dim3(g1 * 16), dim3(256), 0, st, pages, P, n, dig); });
    add("PRODUCT pcs_pages_stamp_dev (two-pass)", [=](hipStream_t st) { pcs_pages_stamp_dev(pages, P, n, 0, (pcs_stream_t)st); });
    add("PRODUCT pcs_pages_digest_dev", [=](hipStream_t st) { pcs_pages_digest_dev(pages, P, n, 0, dig, (pcs_stream_t)st); });
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    uint8_t* okd;
    uint64_t* fbd;
    CK(hipMalloc(&okd, n));
    CK(hipMalloc(&fbd, 8));
    for (auto& v : vs) {  // warm, and check every variant leaves all pages valid
        v.run(s);
        CK(hipStreamSynchronize(s));
        if (pcs_pages_validate_dev(pages, P, n, 0, okd, fbd, (pcs_stream_t)s)) std::exit(2);
        uint64_t f = 0;
        CK(hipMemcpyAsync(&f, fbd, 8, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        std::printf("after %-38s first_bad = %s\n", v.name.c_str(), f == ~0ull ? "none" : std::to_string(f).c_str());
    }
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 200000LL);
            CK(hipEventRecord(a, s));
            v.run(s);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            v.ms.push_back(ms);
            if (r < 2) {
                if (pcs_pages_validate_dev(pages, P, n, 0, okd, fbd, (pcs_stream_t)s)) std::exit(2);
                uint64_t f = 0;
                CK(hipMemcpyAsync(&f, fbd, 8, hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                if (f != ~0ull) std::printf("round %d after %s: first_bad = %llu\n", r, v.name.c_str(), (unsigned long long)f);
            }
        }
    CK(hipGetLastError());
    // the pages must still validate after all the header rewrites
    uint8_t* ok;
    uint64_t* fb;
    CK(hipMalloc(&ok, n));
    CK(hipMalloc(&fb, 8));
    if (pcs_pages_validate_dev(pages, P, n, 0, ok, fb, (pcs_stream_t)s)) std::exit(2);
    uint64_t fbh = 0;
    CK(hipMemcpyAsync(&fbh, fb, 8, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    if (fbh != ~0ull) {  // which pages, and what do their headers hold?
        std::vector<uint8_t> okh(n);
        CK(hipMemcpy(okh.data(), ok, n, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t k = 0; k < n; ++k) bad += okh[k] == 0;
        uint64_t hdr = 0, d = 0;
        CK(hipMemcpy(&hdr, pages + fbh * P, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&d, dig + fbh, 8, hipMemcpyDeviceToHost));
        std::printf("bad pages: %zu; page %llu header %016llx dig %016llx\n", bad, (unsigned long long)fbh,
                    (unsigned long long)hdr, (unsigned long long)d);
    }
    std::printf("validate after rewrites: first_bad = %s\n", fbh == ~0ull ? "none" : std::to_string(fbh).c_str());
    std::printf("%-40s %9s\n", "variant (1 M x 4 KiB headers)", "med_us");
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        std::printf("%-40s %9.1f\n", v.name.c_str(), v.ms[v.ms.size() / 2] * 1e3);
    }
    return 0;
}

struct Variant;
static int main_big(int rounds);

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
    if (argc > 2 && std::string(argv[2]) == "big") return main_big(rounds);
    if (argc > 2 && std::string(argv[2]) == "stamp") return main_stamp(rounds);
    const uint64_t P = 4096, n = 1 << 20, bytes = n * P;
    uint8_t* pages;
    uint64_t* out;
    CK(hipMalloc(&pages, bytes));
    CK(hipMalloc(&out, n * 8));
    const bool random = !(argc > 2 && std::string(argv[2]) == "const");
    const bool gen = argc > 2 && std::string(argv[2]) == "gen";
    if (gen) {
        if (pcs_gen_pages_dev(pages, P, n, 0x5EED0002, 0, nullptr)) std::exit(2);
        CK(hipDeviceSynchronize());
    } else if (random) {
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(pages), bytes / 8);
        CK(hipDeviceSynchronize());
    } else {
        CK(hipMemset(pages, 0x5A, bytes));
    }
    std::printf("data: %s\n", gen ? "pcs_gen_pages_dev pages" : random ? "random (splitmix64)" : "constant 0x5A");
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipStream_t s;
    CK(hipStreamCreate(&s));

    std::vector<Variant> vs;
    auto add = [&](std::string name, std::function<void(hipStream_t)> f) { vs.push_back({name, f, {}}); };
    for (int bpc : {4, 8, 16, 32}) {
        const unsigned grid = cus * bpc;
        add("group16 plain bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_group16<4096, false>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("group16 nt    bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_group16<4096, true>), dim3(grid), dim3(256), 0, st, pages, n, out); });
    }
    {
        const unsigned grid = (unsigned)(n / 16);
        add("group16 plain nonpersistent", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16<4096, false>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("group16 nt    nonpersistent", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16<4096, true>), dim3(grid), dim3(256), 0, st, pages, n, out); });
    }
    for (int bpc : {8, 16}) {
        const unsigned grid = cus * bpc;
        add("wavepage plain bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_wavepage<4096, false>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("wavepage nt    bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_wavepage<4096, true>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("contig16 plain bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_contig<false>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("contig16 nt    bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_contig<true>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("linear U4 plain bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_linear<4, false>), dim3(grid), dim3(256), 0, st, pages, bytes / 16, out); });
        add("linear U4 nt    bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_linear<4, true>), dim3(grid), dim3(256), 0, st, pages, bytes / 16, out); });
        add("linear U8 nt    bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_linear<8, true>), dim3(grid), dim3(256), 0, st, pages, bytes / 16, out); });
    }
    {
        const unsigned grid = (unsigned)(n / 64);
        add("quad64 nt U8 nonpersistent", [=](hipStream_t st) { hipLaunchKernelGGL((k_quad64<4096, true, 8>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("quad64 plain U8 nonpersistent", [=](hipStream_t st) { hipLaunchKernelGGL((k_quad64<4096, false, 8>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("quad64 nt U16 nonpersistent", [=](hipStream_t st) { hipLaunchKernelGGL((k_quad64<4096, true, 16>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("quad64 nt U4 nonpersistent", [=](hipStream_t st) { hipLaunchKernelGGL((k_quad64<4096, true, 4>), dim3(grid), dim3(256), 0, st, pages, n, out); });
    }
    add("group16 nt store-per-page", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_store<4096, false>), dim3(n / 16), dim3(256), 0, st, pages, n, out); });
    add("group16 nt store-staged128", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_store<4096, true>), dim3(n / 16), dim3(256), 0, st, pages, n, out); });
    add("batchstore M=4", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_batchstore<4096, 4, false>), dim3(n / 64), dim3(256), 0, st, pages, n, out); });
    add("batchstore M=16", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_batchstore<4096, 16, false>), dim3(n / 256), dim3(256), 0, st, pages, n, out); });
    add("batchstore M=64", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_batchstore<4096, 64, false>), dim3(n / 1024), dim3(256), 0, st, pages, n, out); });
    add("batchstore M=16 nt-store", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_batchstore<4096, 16, true>), dim3(n / 256), dim3(256), 0, st, pages, n, out); });
    add("batchstore M=1 nt-store", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_batchstore<4096, 1, true>), dim3(n / 16), dim3(256), 0, st, pages, n, out); });
    add("group16 nt xcd-contiguous tiles", [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_xcd<4096>), dim3(n / 16), dim3(256), 0, st, pages, n, out); });
    add("PRODUCT pcs_pages_validate_dev xxh3", [=](hipStream_t st) { pcs_pages_validate_dev(pages, 4096, n, 0, reinterpret_cast<uint8_t*>(out), out + n / 2, (pcs_stream_t)st); });
    add("PRODUCT pcs_pages_stamp_dev xxh3", [=](hipStream_t st) { pcs_pages_stamp_dev(pages, 4096, n, 0, (pcs_stream_t)st); });
    add("PRODUCT pcs_stream_read_dev", [=](hipStream_t st) { pcs_stream_read_dev(pages, 4096 * n, out, (pcs_stream_t)st); });
    add("PRODUCT pcs_pages_digest_dev xxh3", [=](hipStream_t st) { pcs_pages_digest_dev(pages, 4096, n, 0, out, (pcs_stream_t)st); });
    add("PRODUCT pcs_pages_digest_dev xxh64", [=](hipStream_t st) { pcs_pages_digest_dev(pages, 4096, n, 1, out, (pcs_stream_t)st); });
    for (int bpc : {2, 4}) {
        const unsigned grid = cus * bpc;
        add("glds plain bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_glds<false>), dim3(grid), dim3(256), 0, st, pages, n, out); });
        add("glds nt    bpc=" + std::to_string(bpc), [=](hipStream_t st) { hipLaunchKernelGGL((k_glds<true>), dim3(grid), dim3(256), 0, st, pages, n, out); });
    }

    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto& v : vs) v.run(s);  // warm
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 200000LL);  // GPU busy while we enqueue
            CK(hipEventRecord(a, s));
            v.run(s);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            v.ms.push_back(ms);
        }
    CK(hipGetLastError());
    std::printf("%-34s %9s %9s %9s\n", "variant", "med_ms", "GB/s", "best GB/s");
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2];
        std::printf("%-34s %9.4f %9.1f %9.1f\n", v.name.c_str(), med, bytes / (med * 1e-3) / 1e9,
                    bytes / (v.ms[0] * 1e-3) / 1e9);
    }
    return 0;
}

// 64 KiB pages x 256 K = 16 GiB (config 4): is the product's shortfall there
// the access pattern or the buffer size?
static int main_big(int rounds) {
    const uint64_t P = 65536, n = 1 << 18, bytes = n * P;
    uint8_t* pages;
    uint64_t* out;
    CK(hipMalloc(&pages, bytes));
    CK(hipMalloc(&out, n * 16 * 8));
    if (pcs_gen_pages_dev(pages, P, n, 0x5EED0004, 0, nullptr)) std::exit(2);
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    struct V { std::string name; std::function<void(hipStream_t)> run; uint64_t bytes; std::vector<float> ms; };
    std::vector<V> vs;
    auto add = [&](std::string name, uint64_t b, std::function<void(hipStream_t)> f) { vs.push_back({name, f, b, {}}); };
    add("4K-page group16 nt over 16 GiB", bytes, [=](hipStream_t st) { hipLaunchKernelGGL((k_group16<4096, true>), dim3(n * 16 / 16), dim3(256), 0, st, pages, n * 16, out); });
    add("4K-page group16 nt over 4 GiB", bytes / 4, [=](hipStream_t st) { hipLaunchKernelGGL((k_group16<4096, true>), dim3(n * 4 / 16), dim3(256), 0, st, pages, n * 4, out); });
    add("4K-page xcd tiles over 16 GiB", bytes, [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_xcd<4096>), dim3(n), dim3(256), 0, st, pages, n * 16, out); });
    for (int bpc : {8, 16})
        add("linear U8 nt bpc=" + std::to_string(bpc), bytes, [=](hipStream_t st) { hipLaunchKernelGGL((k_linear<8, true>), dim3(cus * bpc), dim3(256), 0, st, pages, bytes / 16, out); });
    for (int bpc : {4, 8, 16})
        add("group16-big nt bpc=" + std::to_string(bpc), bytes, [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_big<true>), dim3(cus * bpc), dim3(256), 0, st, pages, n, out); });
    add("group16-big nt nonpersistent", bytes, [=](hipStream_t st) { hipLaunchKernelGGL((k_group16_big<true>), dim3(n / 16), dim3(256), 0, st, pages, n, out); });
    for (int bpc : {4, 8})
        add("wg-per-page nt bpc=" + std::to_string(bpc), bytes, [=](hipStream_t st) { hipLaunchKernelGGL((k_wg_page64k<true>), dim3(cus * bpc), dim3(256), 0, st, pages, n, out); });
    add("wg-per-page nt nonpersistent", bytes, [=](hipStream_t st) { hipLaunchKernelGGL((k_wg_page64k<true>), dim3(n), dim3(256), 0, st, pages, n, out); });
    add("wg-per-page plain nonpersistent", bytes, [=](hipStream_t st) { hipLaunchKernelGGL((k_wg_page64k<false>), dim3(n), dim3(256), 0, st, pages, n, out); });
    add("PRODUCT pcs_stream_read_dev 64K", bytes, [=](hipStream_t st) { pcs_stream_read_dev(pages, P * n, out, (pcs_stream_t)st); });
    add("PRODUCT pcs_pages_digest_dev xxh3 64K", bytes, [=](hipStream_t st) { pcs_pages_digest_dev(pages, P, n, 0, out, (pcs_stream_t)st); });
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto& v : vs) v.run(s);
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 200000LL);
            CK(hipEventRecord(a, s));
            v.run(s);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            v.ms.push_back(ms);
        }
    CK(hipGetLastError());
    std::printf("%-40s %9s %9s %9s\n", "variant (64 KiB pages, 16 GiB)", "med_ms", "GB/s", "best GB/s");
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2];
        std::printf("%-40s %9.4f %9.1f %9.1f\n", v.name.c_str(), med, v.bytes / (med * 1e-3) / 1e9, v.bytes / (v.ms[0] * 1e-3) / 1e9);
    }
    return 0;
}
