// pcs_kernels.hip — hand-written CDNA4 (gfx950) kernels for EloqStore's page
// checksum path: XXH3_64bits(page + 8, P - 8) / XXH64(page + 8, P - 8, 0) over
// many independent pages per launch (reference call sites:
// src/storage/page.cpp:18-31, src/async_io_manager.cpp:239-244 / 353-366,
// src/tasks/write_task.cpp:58-79).
//
// Work decomposition:
//
//   XXH3 long path — one 16-lane DPP row ("group") per page, 4 pages per wave.
//     Chunk c of a 1 KiB input block is 256 page bytes; lane g of the group
//     loads page bytes [blk*1024 + 256c + 16g, +16) with one global_load_dwordx4,
//     so a wave-instruction reads four fully-used 256 B segments.  Inside an
//     XXH3 block the accumulator updates are pure mod-2^64 sums (xxhash.h:5778-
//     5817), so each lane folds its words into four partial sums and a block
//     needs one cross-lane reduction: a DPP row_ror:15 exchange (page words sit
//     one u64 ahead of the 8-byte-offset hashed stripes) plus row_ror 4/8 folds.
//     The per-block scramble (xxhash.h:5827-5856) runs redundantly on every lane
//     for the accumulator pair (2p, 2p+1), p = g & 3; the merge (xxhash.h:6029-
//     6062) folds the four pairs with row_ror 1/2.
//   XXH64 — one quad per page (lane a owns accumulator a), 16 pages per wave;
//     the serial round chain of each accumulator stays in one lane.
//   Generic — one lane per input range, any length (all XXH3 length classes,
//     xxhash.h:4641-4856), for odd-sized descriptors and raw ranges.
#include "xxh3_page.h"
#include "eloqstore_pcs_internal.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <atomic>
#include <mutex>
#include <vector>

namespace pcs {

// Block tile = 16 consecutive pages (one per group).  The loop runs over
// tiles, so its trip count is uniform across the block and the barriers below
// cannot diverge.  Digest / verdict mode stages the tile's 16 results in LDS
// and writes them as one coalesced non-temporal store (128 B of digests or
// 16 B of verdicts) instead of 16 scattered 8-byte stores.
//
// When the grid covers every tile once, tiles are renumbered so that each
// XCD streams chunks of 64 consecutive tiles, the eight XCDs on adjacent
// chunks (xcd_tile, xxh3_page.h): +7.5 % on config 2 against dispatch order,
// and free of the placement dependence of one contiguous eighth per XCD.
//
// Digest and validate only: a stamp (SetChecksum) is this kernel's digest
// pass followed by k_scatter_stamp (pages_impl), because header writes
// interleaved with the read stream cost 20 % at every rewrite width
// (the in-place forms were retired in round 2).
template <int P, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_xxh3_fixed(const uint8_t* __restrict__ pages, uint64_t n,
                                                   uint64_t* __restrict__ out, uint8_t* __restrict__ ok,
                                                   unsigned long long* first_bad) {
    static_assert(MODE != kStamp, "stamps run as digest + k_scatter_stamp");
    __shared__ uint64_t tile_h[16];
    __shared__ uint8_t tile_ok[16];
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const int grp = threadIdx.x >> 4;
    const uint64_t ntiles = (n + 15) / 16;
    const bool remap = gridDim.x == ntiles;
    for (uint64_t t0 = blockIdx.x; t0 < ntiles; t0 += gridDim.x) {
        const uint64_t t = remap ? xcd_tile(t0, ntiles) : t0;
        const uint64_t pg = t * 16 + grp;
        if (pg < n) {
            const uint8_t* page = pages + pg * (uint64_t)P;
            uint64_t stored = 0;
            u32x4 first;
            const uint64_t h = xxh3_page_fixed<P, NT>(page, L, stored, first);
            if (L.g == 0) {
                tile_h[grp] = h;
                tile_ok[grp] = (h == stored) ? 1 : 0;
            }
        }
        __syncthreads();
        const uint64_t i = t * 16 + threadIdx.x;
        if (threadIdx.x < 16 && i < n) {
            if (MODE == kDigest || out) st_nt(out + i, tile_h[threadIdx.x]);
            if (MODE == kValidate) st_nt(ok + i, tile_ok[threadIdx.x]);
        }
        if (MODE == kValidate && first_bad && threadIdx.x == 0) {
            // one note per tile: its smallest failing page
            for (int k = 0; k < 16 && t * 16 + k < n; ++k)
                if (!tile_ok[k]) {
                    note_bad(first_bad, t * 16 + k);
                    break;
                }
        }
        __syncthreads();
    }
}

// Split pages (P = 8, 16, 32 or 64 KiB): G = P / 4096 groups share a page,
// group j loading its 4 KiB slice (blocks 4j .. 4j+3) at once, so a
// workgroup streams 64 KiB of contiguous page bytes instead of 16 separate
// pages.  XXH3's long loop is acc <- scramble(acc + S_b) over block sums S_b
// that depend on the data only (xxhash.h:5988-6017), so the groups compute
// their S_b in parallel into LDS and one group per page then runs the short
// serial chain (the long-range kernel's scheme, k_xxh3_long).  A slice's last
// block needs the next slice's first word (its carry); it is left out of the
// group's sum and added by the chain from the word the next group publishes.
// One tile of the split scheme: PPB = 16 / G pages, group grp = (page slot ps,
// slice j).  page_at(ps) gives the page's address (nullptr: no page in that
// slot).  S holds PPB * P/1024 block-sum records of 4 pairs x 2 u64 (512 u64),
// C the 16 slice carry words.  On return (after one block barrier) the page
// digests and verdicts are in tile_h / tile_ok[ps]; the caller must barrier
// before reading them.
template <int P, bool NT, typename PageAt>
__device__ __forceinline__ void xxh3_split_tile(const Xxh3Lane& L, PageAt page_at, uint64_t* S, uint64_t* C,
                                                uint64_t* tile_h, uint8_t* tile_ok) {
    static_assert(P % 4096 == 0 && P >= 8192 && P <= 65536, "split pages are 8..64 KiB");
    constexpr int G = P / 4096;       // groups per page
    constexpr int NB = P / 1024 - 1;  // full blocks (xxhash.h:5996); block NB is the final one, 4 chunks
    constexpr int NB1 = NB + 1;
    const int grp = threadIdx.x >> 4, ps = grp / G, j = grp % G, p = L.g & 3;
    const uint8_t* page = page_at(ps);
    uint64_t stored = 0;
    if (page) {
        const u32x4* base = reinterpret_cast<const u32x4*>(page + 4096u * j) + L.g;
        u32x4 d[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) d[i][c] = ld16<NT>(base + i * 64 + c * 16);
        stored = lo64(d[0][0]);
        if (L.g == 0) C[ps * G + j] = lo64(d[0][0]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint64_t Te, To;
            if (i < 3) xxh3_block_terms<false>(L, d[i], lo64(d[i + 1][0]), 4, Te, To);
            else if (j < G - 1) xxh3_block_terms<false, true>(L, d[i], 0, 4, Te, To);
            else xxh3_block_terms<true>(L, d[i], 0, 4, Te, To);
            if (L.g < 4) {
                uint64_t* r = S + ((ps * NB1 + 4 * j + i) * 4 + p) * 2;
                r[0] = Te;
                r[1] = To;
            }
        }
    }
    __syncthreads();
    if (j == 0 && page) {
        const uint64_t k22 = c_keys.acc[22];  // key of a block's last input word (stripe 15, lane 7)
        const uint64_t* Sp = S + (ps * NB1 * 4 + p) * 2;
        uint64_t Ae = L.init_e, Ao = L.init_o;
#pragma unroll 4
        for (int b = 0; b < NB; ++b) {
            uint64_t Te = Sp[b * 8], To = Sp[b * 8 + 1];
            if ((b & 3) == 3 && p == 3) {  // slice boundary: add the carry word's terms
                const uint64_t cw = C[ps * G + ((b + 1) >> 2)];
                Te += cw;
                To += mul32x32(cw ^ k22);
            }
            Ae = xxh3_scramble(Ae + Te, L.ks_e);
            Ao = xxh3_scramble(Ao + To, L.ks_o);
        }
        const uint64_t h = xxh3_merge(L, Ae + Sp[NB * 8], Ao + Sp[NB * 8 + 1], (uint64_t)(P - 8));
        if (L.g == 0) {
            tile_h[ps] = h;
            tile_ok[ps] = (h == stored) ? 1 : 0;
        }
    }
}

template <int P, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_xxh3_split(const uint8_t* __restrict__ pages, uint64_t n,
                                                   uint64_t* __restrict__ out, uint8_t* __restrict__ ok,
                                                   unsigned long long* first_bad) {
    constexpr int PPB = 16 / (P / 4096);  // pages per 256-thread block
    __shared__ uint64_t S[64 * 8];        // block sums per accumulator pair (even, odd)
    __shared__ uint64_t C[16];            // first input word of each slice (the previous block's carry)
    __shared__ uint64_t tile_h[16];
    __shared__ uint8_t tile_ok[16];
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + PPB - 1) / PPB;
    const bool remap = gridDim.x == ntiles;
    for (uint64_t t0 = blockIdx.x; t0 < ntiles; t0 += gridDim.x) {
        const uint64_t t = remap ? xcd_tile(t0, ntiles) : t0;
        xxh3_split_tile<P, NT>(
            L,
            [&](int ps) -> const uint8_t* {
                const uint64_t pg = t * PPB + ps;
                return pg < n ? pages + pg * (uint64_t)P : nullptr;
            },
            S, C, tile_h, tile_ok);
        __syncthreads();
        const uint64_t i0 = t * PPB;
        if (threadIdx.x < PPB && i0 + threadIdx.x < n) {
            if (MODE == kDigest || out) st_nt(out + i0 + threadIdx.x, tile_h[threadIdx.x]);
            if (MODE == kValidate) st_nt(ok + i0 + threadIdx.x, tile_ok[threadIdx.x]);
        }
        if (MODE == kValidate && first_bad && threadIdx.x == 0) {
            for (int k = 0; k < PPB && i0 + k < n; ++k)
                if (!tile_ok[k]) {
                    note_bad(first_bad, i0 + k);
                    break;
                }
        }
        // the next tile's writes to S / tile_h wait for everyone's reads here
        __syncthreads();
    }
}

// Fixed stride, run-time page size.  BODY 0 / 1: the chunked body one block
// or four blocks per step (P % 256 == 0, 16-byte-aligned pages); BODY 2: the
// any-size body (any P >= 249, any alignment).
template <int MODE, bool NT, int BODY>
__global__ __launch_bounds__(256) void k_xxh3_stride(const uint8_t* __restrict__ pages, uint32_t P, uint64_t n,
                                                    uint64_t* __restrict__ out, uint8_t* __restrict__ ok,
                                                    unsigned long long* first_bad) {
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    const bool remap = gridDim.x == ntiles;
    for (uint64_t t0 = blockIdx.x; t0 < ntiles; t0 += gridDim.x) {
        const uint64_t pg = (remap ? xcd_tile(t0, ntiles) : t0) * 16 + (threadIdx.x >> 4);
        if (pg >= n) continue;
        const uint8_t* page = pages + pg * (uint64_t)P;
        uint64_t stored = 0;
        const uint64_t h = BODY == 2   ? xxh3_page_any<NT>(page, P, L, stored)
                           : BODY == 1 ? xxh3_page_rt4<NT>(page, P, L, stored)
                                       : xxh3_page_rt<NT>(page, P, L, stored);
        if (L.g == 0) emit(MODE, pg, h, stored, const_cast<uint8_t*>(page), out, ok, first_bad);
    }
}

// Page list: page pg is the absolute address ptrs[pg], all of size P
// (P % 256 == 0, 16-byte aligned; checked by the caller).  Used for pool pages
// in registered host memory, read in place over PCIe (zero-copy): the list
// and the results live in pinned host memory too, so a batch is one launch.
// PF > 0 uses the compile-time page size (a 4 KiB page is then one batch of
// loads: one PCIe round trip instead of one per 1 KiB block).
template <int MODE, int PF, typename PageAt>
__device__ __forceinline__ void xxh3_list_body(PageAt page_at, uint32_t P, uint64_t n, uint64_t* __restrict__ out,
                                               uint8_t* __restrict__ ok) {
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    for (uint64_t t = blockIdx.x; t < (n + 15) / 16; t += gridDim.x) {
        const uint64_t pg = t * 16 + (threadIdx.x >> 4);
        if (pg >= n) continue;
        const uint8_t* page = page_at(pg);
        uint64_t stored = 0;
        uint64_t h;
        if constexpr (PF > 0) {
            u32x4 first;
            h = xxh3_page_fixed<PF, false>(page, L, stored, first);
        } else {
            h = xxh3_page_rt4<false>(page, P, L, stored);
        }
        if (L.g == 0) {
            if (MODE == kStamp && ok) {
                // small stamp batches: a done byte per page that the host
                // polls instead of the completion signal.  The header and
                // the done byte are system-scope stores, the byte released
                // after the header, as the validate service writes them.
                // With the header as a non-temporal store behind a release
                // fence, the host saw the done byte before the header ~1 in
                // 10^5 stamps under eight threads (service_threads_test
                // --soak, profiles/r05/soak_bisect.txt).
                __hip_atomic_store(reinterpret_cast<uint64_t*>(const_cast<uint8_t*>(page)), h, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                // the digest word an async stamp batch returns: system-scope
                // too, since the host reads it as soon as the done byte lands
                if (out) __hip_atomic_store(out + pg, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(ok + pg, (uint8_t)1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                emit(MODE, pg, h, stored, const_cast<uint8_t*>(page), out, ok, nullptr);
            }
        }
    }
}

template <int MODE, int PF>
__global__ __launch_bounds__(256) void k_xxh3_list(const uint64_t* __restrict__ ptrs, uint32_t P, uint64_t n,
                                                  uint64_t* __restrict__ out, uint8_t* __restrict__ ok) {
    xxh3_list_body<MODE, PF>([=](uint64_t pg) { return reinterpret_cast<const uint8_t*>(ptrs[pg]); }, P, n, out, ok);
}

// Small batches (a ReadPages / FlushBatchPages batch is <= 256 pages,
// kv_options.h:18-19, 70) carry the page list in the kernel arguments: the
// waves then go straight to the pages instead of first fetching the list
// from host memory, one PCIe round trip less.
constexpr int kInlinePages = 256;
struct InlineList {
    uint64_t p[kInlinePages];
};

template <int MODE, int PF>
__global__ __launch_bounds__(256) void k_xxh3_list_inl(InlineList list, uint32_t P, uint64_t n,
                                                      uint64_t* __restrict__ out, uint8_t* __restrict__ ok) {
    xxh3_list_body<MODE, PF>([&](uint64_t pg) { return reinterpret_cast<const uint8_t*>(list.p[pg]); }, P, n, out,
                             ok);
}

// ---------------------------------------------------------------------------
// XXH64 page hash, one quad per page (lane a = accumulator a)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t xxh64_init(int a) {
    // XXH64_initAccs with seed 0 (xxhash.h:3521-3528)
    return a == 0 ? kP64_1 + kP64_2 : a == 1 ? kP64_2 : a == 2 ? 0ull : (uint64_t)0 - kP64_1;
}

__device__ __forceinline__ uint64_t ld64(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}

// XXH64_finalize (xxhash.h:3611-3634) over the (len & 31) bytes at tail.
__device__ __forceinline__ uint64_t xxh64_tail(uint64_t h, const uint8_t* tail, uint64_t len) {
    uint32_t rem = (uint32_t)(len & 31);
    for (; rem >= 8; rem -= 8, tail += 8) {
        h ^= xxh64_round(0, ld64(tail));
        h = rotl64(h, 27) * kP64_1 + kP64_4;
    }
    if (rem >= 4) {
        h ^= (uint64_t)ld32(tail) * kP64_1;
        h = rotl64(h, 23) * kP64_2 + kP64_3;
        rem -= 4;
        tail += 4;
    }
    for (; rem > 0; --rem, ++tail) {
        h ^= (uint64_t)(*tail) * kP64_5;
        h = rotl64(h, 11) * kP64_1;
    }
    return xxh64_avalanche(h);
}

// XXH64_mergeAccs (xxhash.h:3573-3593) for a quad whose lane a holds acc a.
__device__ __forceinline__ uint64_t xxh64_quad_merge(uint64_t v) {
    const uint64_t v0 = dpp64<quad_bcast(0)>(v);
    const uint64_t v1 = dpp64<quad_bcast(1)>(v);
    const uint64_t v2 = dpp64<quad_bcast(2)>(v);
    const uint64_t v3 = dpp64<quad_bcast(3)>(v);
    uint64_t h = rotl64(v0, 1) + rotl64(v1, 7) + rotl64(v2, 12) + rotl64(v3, 18);
    h = (h ^ xxh64_round(0, v0)) * kP64_1 + kP64_4;
    h = (h ^ xxh64_round(0, v1)) * kP64_1 + kP64_4;
    h = (h ^ xxh64_round(0, v2)) * kP64_1 + kP64_4;
    h = (h ^ xxh64_round(0, v3)) * kP64_1 + kP64_4;
    return h;
}

// Page convention: XXH64 over [8, P).  Needs 8-byte aligned page, P % 8 == 0,
// P >= 40 (so the hashed length is >= 32 and the 4-accumulator loop runs).
constexpr int kX64Unroll = 16;
// Segments in flight per LDS-kernel step (profiles/r01/x64_depth_lab.txt).  Round 5
// (profiles/r05/x64_depth3_lab_r05z.txt): depth 3 (124 VGPRs, 4 waves per SIMD)
// is -3.2 % on config 3 and +0.9 % on config 2, depth 4 -10.3 % / +0.5 %; 2 stays.
constexpr int kX64LdsDepth = 2;
template <bool NT>
__device__ __forceinline__ uint64_t ld8(const uint64_t* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ uint64_t xxh64_page(const uint8_t* __restrict__ page, uint32_t P, int a,
                                               uint64_t& stored) {
    const uint64_t len = P - 8;
    const uint32_t ns = (uint32_t)(len / 32);
    const uint64_t* w = reinterpret_cast<const uint64_t*>(page + 8) + a;
    stored = *reinterpret_cast<const uint64_t*>(page);
    uint64_t v = xxh64_init(a);
    uint32_t s = 0;
    for (; s + kX64Unroll <= ns; s += kX64Unroll) {
        uint64_t x[kX64Unroll];
#pragma unroll
        for (int u = 0; u < kX64Unroll; ++u) x[u] = ld8<NT>(w + 4 * (s + u));
#pragma unroll
        for (int u = 0; u < kX64Unroll; ++u) v = xxh64_round(v, x[u]);
    }
    for (; s < ns; ++s) v = xxh64_round(v, ld8<NT>(w + 4 * s));
    const uint64_t h = xxh64_quad_merge(v) + len;
    return xxh64_tail(h, page + 8 + 32 * (uint64_t)ns, len);
}

// XXH64 chunk arithmetic for 64-byte pieces (page_size % 64 == 0, 16-byte
// aligned page), used by k_xxh64_lds below.
//
// Lane q of a quad holds page bytes [64k + 16q, +16) of chunk k — page words
// 8k + 2q (half e0) and 8k + 2q + 1 (e1).  XXH64 stripe s covers page words
// 4s+1 .. 4s+4 and accumulator a consumes page word 4s + a + 1.  Accumulators are placed as
// lane q -> acc {0, 1, 3, 2}[q]; acc 3 runs one stripe behind (stripes 2k-1
// and 2k per chunk).  Then each lane needs its own half of one word and its
// partner's (q ^ 2) other half:
//   lane 0 (acc 0): own e1 (stripe 2k),   partner e1 (2k+1)
//   lane 1 (acc 1): own e0 (2k),          partner e0 (2k+1)
//   lane 2 (acc 3): partner e0 (2k-1),    own e0 (2k)
//   lane 3 (acc 2): partner e1 (2k),      own e1 (2k+1)
// i.e. one DPP quad_perm [2,3,0,1] exchange of a selected half per chunk.
// acc 3 skips stripe -1 (page word 0 is the stored digest); in the last
// chunk accs 0-2 skip stripe 2k+1, which is the 24-byte tail (page words
// P/8-3 .. P/8-1: lane 2 e1, lane 3 e0, lane 3 e1), consumed after the merge
// (xxhash.h:3537-3566, 3611-3634).
constexpr int kQuadSwap = 2 | (3 << 2) | (0 << 4) | (1 << 6);  // quad_perm [2,3,0,1]

template <bool SKIP>
__device__ __forceinline__ void xxh64_chunk(uint64_t& v, u32x4 d, int q, bool skip_first, bool skip_second) {
    const uint64_t e0 = lo64(d), e1 = hi64(d);
    const bool sends_e0 = (q == 0) || (q == 3);
    const uint64_t send = sends_e0 ? e0 : e1;
    const uint64_t keep = sends_e0 ? e1 : e0;
    const uint64_t recv = dpp64<kQuadSwap>(send);
    const uint64_t first = q < 2 ? keep : recv;
    const uint64_t second = q < 2 ? recv : keep;
    if constexpr (SKIP) {
        const uint64_t v1 = xxh64_round(v, first);
        v = skip_first ? v : v1;
        const uint64_t v2 = xxh64_round(v, second);
        v = skip_second ? v : v2;
    } else {
        v = xxh64_round(xxh64_round(v, first), second);
    }
}

__device__ __forceinline__ bool xxh64_lines_ok(uint64_t off, uint32_t P) {
    return (P % 64u) == 0 && P >= 128u && (off % 16u) == 0;
}

// XXH64 with the 16-lane load pattern, words handed to quads through LDS.
//
// A wave owns 16 pages.  Loads use the XXH3 layout: for 256-byte segment c,
// wave-instruction ii has row r (lanes 16r..16r+15) load page 4ii + r, lane t
// of the row taking bytes [256c + 16t, +16): four fully used 256 B pieces per
// instruction (the quad-per-page layout reads 64 B pieces, 2x the L2 requests
// per byte, measured ~10 % slower).  The quad that hashes page 4i + r sits in
// the same row r at position i (lanes 16r + 4i + q), so a page's bytes never
// leave its row.  Through LDS, quad lane q takes 16-byte slot 4k + q of the
// segment for chunk 4c + k; the slot is stored at (slot + 4i) mod 16, which
// puts the 16 lanes of every ds_read_b128 lane group on 16 distinct 16-byte
// bank slots (MI355X_MICROARCH.md §LDS: groups {0-3,12-15,20-27}, ...) and
// keeps each 8-lane ds_write_b128 group contiguous.  The chunk arithmetic is
// xxh64_chunk above (quad DPP exchange), unchanged.
// offshape (descriptor batches): a descriptor off the line shape makes the
// kernel store call_id there, and the generic pass that follows runs only
// when it finds this call's id (config 3 has no such page: the pass used to
// read every descriptor for nothing, 6.3 us per call).
// ADDR selects where page pg lives: kAddrStride base + pg * Pfixed,
// kAddrDesc base + off[pg] (length len[pg]), kAddrList the absolute address
// off[pg] (length Pfixed; registered host pages, zero-copy).
enum Addr : int { kAddrStride = 0, kAddrDesc = 1, kAddrList = 2 };

// DEPTH segments are loaded before the first of them is hashed (DEPTH x 4 KiB
// per wave in flight).
// WPB waves per workgroup (PCS_TUNE_XXH64_WAVES): a workgroup owns 16 * WPB
// consecutive pages.  Sorting a tile's pages by size before handing them to
// the waves measured 4 % slower on config 3 (profiles/r01/x64_sort_lab.txt:
// the block is held until its all-16 KiB wave ends) and was retired in round 2.
template <int MODE, bool NT, int ADDR, int DEPTH, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) void k_xxh64_lds(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ len, uint32_t Pfixed, uint64_t n,
                                                       uint64_t* __restrict__ out, uint8_t* __restrict__ ok,
                                                       unsigned long long* first_bad,
                                                       unsigned long long* offshape, uint64_t call_id) {
    __shared__ __attribute__((aligned(16))) u32x4 lds[WPB][16][16];  // [wave][page slot][16 B slot]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r = lane >> 4, t = lane & 15;        // loader role
    const int i = (lane >> 2) & 3, q = lane & 3;   // hasher role: page 4i + r, quad lane q
    const int a = q == 2 ? 3 : q == 3 ? 2 : q;
    constexpr uint64_t kTile = 16 * WPB;
    const uint64_t ntiles = (n + kTile - 1) / kTile;
    const bool remap = gridDim.x == ntiles;
    for (uint64_t t0 = blockIdx.x; t0 < ntiles; t0 += gridDim.x) {
        const uint64_t T = (remap ? xcd_tile_eighths(t0, ntiles) : t0) * kTile;
        // page in wave slot j (0..15) of this wave
        auto page_at = [&](int j) -> uint64_t { return T + wv * 16 + j; };
        // loader pages (4ii + r) and hasher page (4i + r)
        const uint8_t* lp[4];
        uint32_t lP[4];
        uint32_t segs = 0;  // segments this wave must walk (max over its pages)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
            const uint64_t pg = page_at(4 * ii + r);
            uint32_t P = 0;
            const uint8_t* p = nullptr;
            if (pg < n) {
                if (ADDR == kAddrDesc) {
                    const uint64_t o = off[pg];
                    const uint32_t L = len[pg];
                    if (xxh64_lines_ok(o, L)) { P = L; p = base + o; }
                    else if (offshape) *offshape = call_id;  // left to k_generic_desc: it must run
                } else if (ADDR == kAddrList) {
                    P = Pfixed;
                    p = reinterpret_cast<const uint8_t*>(off[pg]);
                } else {
                    P = Pfixed;
                    p = base + pg * (uint64_t)Pfixed;
                }
            }
            lp[ii] = p;
            lP[ii] = P;
        }
        const uint64_t hp = page_at(4 * i + r);
        uint32_t Ph = 0;
        const uint8_t* hptr = nullptr;
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
            if (ii == i) { Ph = lP[ii]; hptr = lp[ii]; }
        {
            uint32_t m = 0;
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) m = max(m, lP[ii]);
            // wave-wide maximum so every lane walks the same segment count
            m = max(m, (uint32_t)__shfl_xor((int)m, 16));
            m = max(m, (uint32_t)__shfl_xor((int)m, 32));
            segs = (m + 255) / 256;
        }
        const int K = (int)(Ph / 64);
        uint64_t v = xxh64_init(a), stored = 0;
        u32x4 last = {0, 0, 0, 0};
        for (uint32_t c0 = 0; c0 < segs; c0 += DEPTH) {
            u32x4 d[DEPTH][4];
#pragma unroll
            for (int j = 0; j < DEPTH; ++j)
#pragma unroll
                for (int ii = 0; ii < 4; ++ii)
                    if (256 * (c0 + j) + 16 * t < lP[ii])
                        d[j][ii] = ld16<NT>(reinterpret_cast<const u32x4*>(lp[ii] + 256 * (c0 + j)) + t);
#pragma unroll
            for (int j = 0; j < DEPTH; ++j) {
                const uint32_t c = c0 + j;
                if (c >= segs) break;  // wave-uniform
#pragma unroll
                for (int ii = 0; ii < 4; ++ii)
                    if (256 * c + 16 * t < lP[ii]) lds[wv][4 * ii + r][(t + 4 * ii) & 15] = d[j][ii];
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int kk = 4 * (int)c + k;
                    if (kk < K) {
                        const u32x4 e = lds[wv][4 * i + r][(4 * k + q + 4 * i) & 15];
                        if (kk == 0) stored = dpp64<quad_bcast(0)>(lo64(e));
                        if (kk == 0 || kk == K - 1)
                            xxh64_chunk<true>(v, e, q, q == 2 && kk == 0, q != 2 && kk == K - 1);
                        else xxh64_chunk<false>(v, e, q, false, false);
                        if (kk == K - 1) last = e;
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (K > 0) {
            const uint64_t v0 = dpp64<quad_bcast(0)>(v);
            const uint64_t v1 = dpp64<quad_bcast(1)>(v);
            const uint64_t v2 = dpp64<quad_bcast(3)>(v);
            const uint64_t v3 = dpp64<quad_bcast(2)>(v);
            uint64_t h = rotl64(v0, 1) + rotl64(v1, 7) + rotl64(v2, 12) + rotl64(v3, 18);
            h = (h ^ xxh64_round(0, v0)) * kP64_1 + kP64_4;
            h = (h ^ xxh64_round(0, v1)) * kP64_1 + kP64_4;
            h = (h ^ xxh64_round(0, v2)) * kP64_1 + kP64_4;
            h = (h ^ xxh64_round(0, v3)) * kP64_1 + kP64_4;
            h += (uint64_t)(Ph - 8);
            const uint64_t t0w = dpp64<quad_bcast(2)>(hi64(last));
            const uint64_t t1w = dpp64<quad_bcast(3)>(lo64(last));
            const uint64_t t2w = dpp64<quad_bcast(3)>(hi64(last));
            h ^= xxh64_round(0, t0w);
            h = rotl64(h, 27) * kP64_1 + kP64_4;
            h ^= xxh64_round(0, t1w);
            h = rotl64(h, 27) * kP64_1 + kP64_4;
            h ^= xxh64_round(0, t2w);
            h = rotl64(h, 27) * kP64_1 + kP64_4;
            h = xxh64_avalanche(h);
            if (q == 0) emit(MODE, hp, h, stored, const_cast<uint8_t*>(hptr), out, ok, first_bad);
        }
    }
}

// Pages off the 64-byte-piece shape (P % 64 != 0 or 8-byte-aligned only): one
// quad per page, lane a reading accumulator a's words (xxh64_page).  The quad
// layout for line-shaped pages (each quad loading its own 64 B pieces, 80 % of
// spec) was retired in round 2 for k_xxh64_lds.
template <int MODE>
__global__ __launch_bounds__(256) void k_xxh64_stride(const uint8_t* __restrict__ pages, uint32_t P, uint64_t n,
                                                     uint64_t* __restrict__ out, uint8_t* __restrict__ ok,
                                                     unsigned long long* first_bad) {
    const int a = threadIdx.x & 3;
    const uint64_t ntiles = (n + 63) / 64;
    const bool remap = gridDim.x == ntiles;
    for (uint64_t t0 = blockIdx.x; t0 < ntiles; t0 += gridDim.x) {
        const uint64_t pg = (remap ? xcd_tile_eighths(t0, ntiles) : t0) * 64 + (threadIdx.x >> 2);
        if (pg >= n) continue;
        const uint8_t* page = pages + pg * (uint64_t)P;
        uint64_t stored = 0;
        const uint64_t h = xxh64_page<false>(page, P, a, stored);
        if (a == 0) emit(MODE, pg, h, stored, const_cast<uint8_t*>(page), out, ok, first_bad);
    }
}

// long raw-range shape (k_xxh3_long, below); the lane kernel skips these
constexpr int kLongWin = 64;             // blocks per window (64 KiB of input)
constexpr uint32_t kLongMin = 2048;      // shorter ranges stay on the lane kernel
constexpr int kQuadSwap1 = 1 | (0 << 2) | (3 << 4) | (2 << 6);  // quad_perm [1,0,3,2]

__device__ __forceinline__ bool xxh3_long_ok(const uint8_t* p, uint32_t L) {
    return L >= kLongMin && ((uintptr_t)p % 8u) == 0;
}

// ---------------------------------------------------------------------------
// generic single-lane XXH3_64bits / XXH64 over any byte range (any alignment)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t rrmxmx(uint64_t h, uint64_t len) {  // xxhash.h:4595-4603
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= kMX2;
    h ^= (h >> 35) + len;
    h *= kMX2;
    return h ^ (h >> 28);
}

// XXH3_mix16B, seed 0 (xxhash.h:4740-4763); SOFF is a compile-time secret offset
__device__ __forceinline__ uint64_t mix16(const uint8_t* in, uint64_t k0, uint64_t k1) {
    return mul_fold64(ld64(in) ^ k0, ld64(in + 8) ^ k1);
}

// XXH3_64bits for len <= 240 (the short and mid-size classes)
__device__ __forceinline__ uint64_t xxh3_short(const uint8_t* in, uint64_t len) {
    if (len <= 16) {  // XXH3_len_0to16_64b, :4696-4704
        if (len > 8) {
            const uint64_t lo = ld64(in) ^ (secret64(24) ^ secret64(32));
            const uint64_t hi = ld64(in + len - 8) ^ (secret64(40) ^ secret64(48));
            const uint64_t acc = len + __builtin_bswap64(lo) + hi + mul_fold64(lo, hi);
            return xxh3_avalanche(acc);
        }
        if (len >= 4) {
            const uint64_t in1 = ld32(in), in2 = ld32(in + len - 4);
            const uint64_t keyed = (in2 + (in1 << 32)) ^ (secret64(8) ^ secret64(16));
            return rrmxmx(keyed, len);
        }
        if (len > 0) {
            const uint32_t combined = ((uint32_t)in[0] << 16) | ((uint32_t)in[len >> 1] << 24) |
                                      (uint32_t)in[len - 1] | ((uint32_t)len << 8);
            return xxh64_avalanche((uint64_t)combined ^ (uint64_t)(secret32(0) ^ secret32(4)));
        }
        return xxh64_avalanche(secret64(56) ^ secret64(64));
    }
    if (len <= 128) {  // XXH3_len_17to128_64b, :4766-4799
        uint64_t acc = len * kP64_1;
        const int rounds = (int)((len - 1) / 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i > rounds) break;
            acc += mix16(in + 16 * i, secret64(32 * i), secret64(32 * i + 8));
            acc += mix16(in + len - 16 * (i + 1), secret64(32 * i + 16), secret64(32 * i + 24));
        }
        return xxh3_avalanche(acc);
    }
    {  // XXH3_len_129to240_64b, :4802-4856 (len <= 240 here)
        uint64_t acc = len * kP64_1;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += mix16(in + 16 * i, secret64(16 * i), secret64(16 * i + 8));
        acc = xxh3_avalanche(acc);
        uint64_t tail = mix16(in + len - 16, secret64(119), secret64(127));
        const int rounds = (int)(len / 16);
#pragma unroll
        for (int i = 8; i < 15; ++i) {
            if (i >= rounds) break;
            tail += mix16(in + 16 * i, secret64(16 * (i - 8) + 3), secret64(16 * (i - 8) + 11));
        }
        return xxh3_avalanche(acc + tail);
    }
}

__device__ uint64_t xxh3_any(const uint8_t* in, uint64_t len) {
    if (len <= 240) return xxh3_short(in, len);
    // long input, scalar (xxhash.h:5988-6081)
    uint64_t acc[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) acc[l] = c_init_acc[l];
    const uint64_t blocks = (len - 1) / 1024;
    auto stripe = [&](const uint8_t* p, int koff, bool last) {
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            const uint64_t v = ld64(p + 8 * l);
            const uint64_t k = v ^ (last ? c_keys.last[l] : c_keys.acc[koff + l]);
            acc[l ^ 1] += v;
            acc[l] += mul32x32(k);
        }
    };
    for (uint64_t b = 0; b < blocks; ++b) {
        for (int s = 0; s < 16; ++s) stripe(in + 1024 * b + 64 * s, s, false);
#pragma unroll
        for (int l = 0; l < 8; ++l) acc[l] = xxh3_scramble(acc[l], c_keys.scr[l]);
    }
    const int ns = (int)(((len - 1) - 1024 * blocks) / 64);
    for (int s = 0; s < ns; ++s) stripe(in + 1024 * blocks + 64 * s, s, false);
    stripe(in + len - 64, 0, true);
    uint64_t r = len * kP64_1;
#pragma unroll
    for (int i = 0; i < 4; ++i) r += mul_fold64(acc[2 * i] ^ c_keys.merge[2 * i], acc[2 * i + 1] ^ c_keys.merge[2 * i + 1]);
    return xxh3_avalanche(r);
}

__device__ uint64_t xxh64_any(const uint8_t* p, uint64_t len, uint64_t seed) {  // xxhash.h:3655-3673
    uint64_t h;
    const uint8_t* q = p;
    if (len >= 32) {
        uint64_t v[4] = {seed + kP64_1 + kP64_2, seed + kP64_2, seed, seed - kP64_1};
        const uint64_t ns = len / 32;
        for (uint64_t s = 0; s < ns; ++s, q += 32)
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = xxh64_round(v[i], ld64(q + 8 * i));
        h = rotl64(v[0], 1) + rotl64(v[1], 7) + rotl64(v[2], 12) + rotl64(v[3], 18);
#pragma unroll
        for (int i = 0; i < 4; ++i) h = (h ^ xxh64_round(0, v[i])) * kP64_1 + kP64_4;
    } else {
        h = seed + kP64_5;
    }
    return xxh64_tail(h + len, q, len);
}

// One lane per range.  SKIP = 8 applies the page convention (hash [8, len),
// stored digest in [0, 8)); SKIP = 0 hashes the raw range.  With FILTER set,
// ranges the fast kernels handle are skipped.
template <int MODE>
__device__ __forceinline__ void generic_one(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                            const uint32_t* __restrict__ len, uint64_t i, int algo, uint64_t seed,
                                            int skip, uint64_t* __restrict__ out, uint8_t* __restrict__ ok,
                                            unsigned long long* first_bad) {
    const uint64_t o = off[i];
    const uint32_t L = len[i];
    const uint8_t* p = base + o;
    if ((uint32_t)skip > L) {  // page shorter than its digest header: never valid
        if (MODE == kValidate) {
            ok[i] = 0;
            if (out) out[i] = 0;
            if (first_bad) note_bad(first_bad, i);
        } else if (MODE == kDigest) {
            out[i] = 0;
        }
        return;
    }
    const uint64_t h = algo == 0 ? xxh3_any(p + skip, L - skip) : xxh64_any(p + skip, L - skip, seed);
    const uint64_t stored = skip ? ld64(p) : 0;
    if (MODE == kStamp) {
        __builtin_memcpy(const_cast<uint8_t*>(p), &h, 8);
        if (out) out[i] = h;
    } else {
        emit(MODE, i, h, stored, nullptr, out, ok, first_bad);
    }
}

// Descriptor batch (mixed sizes), one group per page, every shape: pages on
// the 256-byte chunk grid at 16-byte offsets take the chunked body, other
// long-path pages (P >= 249) the any-size body, shorter ones one lane of the
// group (xxh3_short).  So no generic pass follows.  (In the earlier
// grid-stride form the any-size branch cost 1.2 %, 152 against 136 VGPRs,
// profiles/r02/desc_any_lab.txt; one tile per workgroup compiles all three
// branches in 126.)  Measured alternatives, all
// bit-exact and all slower on config 3: 4 KiB slices dealt
// to the groups in rounds (-8 %), byte-budget slice windows (-12..-30 %),
// per-tile size sort (+-1 %), LPT page pairs (-2 %), a 128-VGPR cap (-0.3 %);
// round 2 (commit 99804f2): pages dealt to a wave's groups as they free up
// (+-1 %), a wave's pages as a stream of adjacent 4 KiB slices (-5..-8 %).
// One workgroup per tile, grid = tiles (no grid-stride loop): 125 VGPRs and
// 4 waves per SIMD, against 136 and 3 for the same body inside a grid-stride
// loop: +1.1 % digest / +0.8 % validate on config 3
// (profiles/r02/desc_tp_lab.txt, list 1 vs 0).  Loading the next tile's
// descriptors ahead with 2 or 4 tiles per workgroup was slower (-0.4..-2.7 %).
template <int MODE, bool NT, bool B4>
__global__ __launch_bounds__(256) void k_xxh3_desc(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                  const uint32_t* __restrict__ len, uint64_t n,
                                                  uint64_t* __restrict__ out, uint8_t* __restrict__ ok,
                                                  unsigned long long* first_bad) {
    __shared__ uint64_t tile_h[16];
    __shared__ uint8_t tile_st[16];  // 0 bad, 1 good, 2 not this kernel's page
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);  // the launch covers every tile once
    // results staged per tile: one coalesced store per tile instead of 16
    // scattered 8-byte (1-byte) stores inside the read stream, +1.0-1.7 % on
    // config 3 (profiles/r02/desc_staged_lab.txt); stamps write headers
    constexpr bool staged = MODE != kStamp;
    const int grp = threadIdx.x >> 4;
    const uint64_t pg = t * 16 + grp;
    uint8_t st = 2;
    if (pg < n) {
        const uint64_t o = off[pg];
        const uint32_t P = len[pg];
        if (xxh3_fast_ok(o, P)) {
            const uint8_t* page = base + o;
            uint64_t stored = 0;
            const uint64_t h = B4 ? xxh3_page_rt4<NT>(page, P, L, stored) : xxh3_page_rt<NT>(page, P, L, stored);
            if (!staged) {
                if (L.g == 0) emit(MODE, pg, h, stored, const_cast<uint8_t*>(page), out, ok, first_bad);
            } else {
                st = h == stored ? 1 : 0;
                if (L.g == 0) tile_h[grp] = h;
            }
        } else if (xxh3_group_ok(P)) {  // off the chunk grid or unaligned: the any-size body
            const uint8_t* page = base + o;
            uint64_t stored = 0;
            const uint64_t h = xxh3_page_any<NT>(page, P, L, stored);
            if (!staged) {
                if (L.g == 0) emit(MODE, pg, h, stored, const_cast<uint8_t*>(page), out, ok, first_bad);
            } else {
                st = h == stored ? 1 : 0;
                if (L.g == 0) tile_h[grp] = h;
            }
        } else if (L.g == 0) {  // shorter than the long path: one lane, results written directly
            if (P < 8) {  // shorter than its header: never valid (as generic_one)
                if (MODE == kValidate) {
                    ok[pg] = 0;
                    if (out) out[pg] = 0;
                    if (first_bad) note_bad(first_bad, pg);
                } else if (MODE == kDigest) {
                    out[pg] = 0;
                }
            } else {
                const uint8_t* page = base + o;
                const uint64_t h = xxh3_short(page + 8, P - 8);
                if (MODE != kStamp) emit(MODE, pg, h, ld64(page), nullptr, out, ok, first_bad);
            }
        }
    }
    if (staged) {
        if (L.g == 0) tile_st[grp] = st;
        __syncthreads();
        const uint64_t i = t * 16 + threadIdx.x;
        const int s = threadIdx.x < 16 && i < n ? tile_st[threadIdx.x] : 2;
        if (s != 2) {
            if (MODE == kDigest || out) st_nt(out + i, tile_h[threadIdx.x]);
            if (MODE == kValidate) st_nt(ok + i, (uint8_t)s);
        }
        if (MODE == kValidate && first_bad && threadIdx.x == 0) {
            for (int k = 0; k < 16 && t * 16 + k < n; ++k)
                if (tile_st[k] == 0) {
                    note_bad(first_bad, t * 16 + k);
                    break;
                }
        }
    }
}

// One lane per range.  SKIP = 8 applies the page convention (hash [8, len),
// stored digest in [0, 8)); SKIP = 0 hashes the raw range.  FILTER 1: XXH64
// pages k_xxh64_lds took are skipped, and with `gate` the whole pass exits
// unless k_xxh64_lds stored this call's id there (it found an off-shape
// page); FILTER 2: raw XXH3 ranges k_xxh3_long took are skipped.  (XXH3 descriptor pages never come here: k_xxh3_desc
// takes every shape.)
template <int MODE>
__global__ __launch_bounds__(256) void k_generic_desc(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                     const uint32_t* __restrict__ len, uint64_t n, int algo,
                                                     uint64_t seed, int skip, int filter, uint64_t* __restrict__ out,
                                                     uint8_t* __restrict__ ok, unsigned long long* first_bad,
                                                     const unsigned long long* gate, uint64_t call_id) {
    if (gate && *gate != call_id) return;  // the fast kernel left no page to this pass
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (filter == 1 && algo == 1 && xxh64_lines_ok(off[i], len[i])) continue;
        if (filter == 2 && xxh3_long_ok(base + off[i], len[i])) continue;
        generic_one<MODE>(base, off, len, i, algo, seed, skip, out, ok, first_bad);
    }
}

// ---------------------------------------------------------------------------
// XXH3 over long raw ranges: one workgroup per range
// ---------------------------------------------------------------------------
// For a single long input (a manifest chunk of up to 1 MiB,
// root_meta.cpp:150-174; a whole object) the page kernels' one-group-per-input
// mapping leaves the GPU idle.  XXH3's long loop (xxhash.h:5988-6017) is a
// chain acc <- scramble(acc + S_b) over 1 KiB blocks whose block sums S_b are
// independent, so the 16 groups of a workgroup compute S_b for a window of
// 64 blocks in parallel into LDS and 8 lanes then run the short serial
// scramble chain over the window.
//
// Lane g of a group loads words g + 16j (j < 8) of a block: 128 contiguous
// bytes per group-instruction.  Word w = g + 16j has stripe s = g/8 + 2j and
// accumulator lane l = g & 7, so a lane's multiply terms all go to acc[l] and
// its raw words to acc[l ^ 1]: one quad_perm swap and one row_ror:8 fold give
// each lane l < 8 the block sum of acc[l].

// block sum for the lane's accumulator l = g & 7 (valid in lanes 0..7)
__device__ __forceinline__ uint64_t xxh3_long_block(const uint64_t* __restrict__ blk, int g, int nstripes) {
    const int l = g & 7;
    uint64_t w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = (g / 8 + 2 * j < nstripes) ? blk[g + 16 * j] : 0;
    uint64_t M = 0, R = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int s = g / 8 + 2 * j;
        if (s < nstripes) {
            M += mul32x32(w[j] ^ c_keys.acc[s + l]);
            R += w[j];
        }
    }
    uint64_t T = M + dpp64<kQuadSwap1>(R);
    T += dpp64<kRowRor8>(T);
    return T;
}

__global__ __launch_bounds__(256) void k_xxh3_long(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                  const uint32_t* __restrict__ len, uint64_t n,
                                                  uint64_t* __restrict__ out) {
    __shared__ uint64_t S[kLongWin][8];
    const int tid = threadIdx.x, g = tid & 15, grp = tid >> 4;
    for (uint64_t r = blockIdx.x; r < n; r += gridDim.x) {
        const uint8_t* in8 = base + off[r];
        const uint32_t L = len[r];
        if (!xxh3_long_ok(in8, L)) continue;  // uniform over the workgroup
        const uint64_t* in = reinterpret_cast<const uint64_t*>(in8);
        const uint32_t nb = (L - 1) / 1024;
        uint64_t acc = tid < 8 ? c_init_acc[tid] : 0;  // threads 0..7 own acc[tid]
        for (uint32_t w0 = 0; w0 < nb; w0 += kLongWin) {
            const int nw = (int)min((uint32_t)kLongWin, nb - w0);
#pragma unroll
            for (int i = 0; i < kLongWin / 16; ++i) {
                const int b = grp + 16 * i;
                if (b < nw) {
                    const uint64_t T = xxh3_long_block(in + (size_t)(w0 + b) * 128, g, 16);
                    if (g < 8) S[b][g] = T;
                }
            }
            __syncthreads();
            if (tid < 8)
                for (int b = 0; b < nw; ++b) acc = xxh3_scramble(acc + S[b][tid], c_keys.scr[tid]);
            __syncthreads();
        }
        if (grp == 0) {
            const int nst = (int)(((L - 1) - 1024 * nb) / 64);
            uint64_t T = xxh3_long_block(in + (size_t)nb * 128, g, nst);
            // last stripe at input + L - 64, keyed with secret + 121 (xxhash.h:6013-6015)
            uint64_t M = 0, R = 0;
            if (g < 8) {
                const uint64_t v = ld64(in8 + L - 64 + 8 * g);
                M = mul32x32(v ^ c_keys.last[g]);
                R = v;
            }
            T += M + dpp64<kQuadSwap1>(R);
            acc += T;
            // mergeAccs (xxhash.h:6029-6052): even lanes fold pairs (l, l + 1)
            const uint64_t nxt = dpp64<kRowRor15>(acc);
            uint64_t m = (g < 8 && (g & 1) == 0) ? mul_fold64(acc ^ c_keys.merge[g], nxt ^ c_keys.merge[g + 1]) : 0;
            m += dpp64<kRowRor2>(m);
            m += dpp64<kRowRor4>(m);  // lane 0..7: m0+m2+m4+m6 (lanes 0,2,4,6 of 0..7)
            if (g == 6) out[r] = xxh3_avalanche((uint64_t)L * kP64_1 + m);
        }
        __syncthreads();
    }
}

// Manifest record aggregate (ManifestBuilder::CalcChecksum, root_meta.cpp:150-174):
// chunk digests folded serially, agg = rotl(agg, 1) ^ h; agg *= 0x9e3779b97f4a7c15.
// ---------------------------------------------------------------------------
// Manifest checksum, wide form: few long chunks (ManifestBuilder::CalcChecksum,
// root_meta.cpp:150-174, 1 MiB per chunk)
// ---------------------------------------------------------------------------
// One workgroup per chunk (k_xxh3_long) leaves a small manifest on a handful
// of CUs: a 1 MiB record took 121 us.  Here the block sums of all chunks are
// computed by 16-block windows spread over the whole GPU (k_manifest_sums),
// then one workgroup per chunk loads its sums into LDS and runs the serial
// scramble chain and the tail (k_manifest_chain).  The chain itself
// (P/1024 - 1 dependent 64x32-bit scrambles) is the floor: ~20-30 us per
// 1 MiB chunk.
constexpr uint32_t kManifestChunk = 1u << 20;  // kCheckSumBatchSize, root_meta.cpp:157
constexpr int kChunkBlocks = kManifestChunk / 1024;
// With 16-byte block-sum loads (k_manifest_sums16), chains staged in LDS
// halves and the scalar fold, the wide form wins at every size, 1 GiB
// included (283 vs 305 us; it lost above 256 chunks before, 380 vs 332 us;
// profiles/r01/manifest_lab.txt).

__device__ __forceinline__ uint32_t manifest_chunk_len(uint64_t total, uint64_t c) {
    return (uint32_t)min((uint64_t)kManifestChunk, total - c * kManifestChunk);
}

__global__ __launch_bounds__(256) void k_manifest_sums(const uint8_t* __restrict__ content, uint64_t total,
                                                      uint64_t* __restrict__ S) {
    const uint64_t c = blockIdx.y;
    const uint32_t L = manifest_chunk_len(total, c);
    if (L < kLongMin) return;  // a short last chunk is hashed whole by the chain kernel
    const int g = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const uint32_t nb = (L - 1) / 1024;
    const uint32_t b = blockIdx.x * 16 + grp;
    if (b >= nb) return;
    const uint64_t* in = reinterpret_cast<const uint64_t*>(content + c * kManifestChunk);
    const uint64_t T = xxh3_long_block(in + (size_t)b * 128, g, 16);
    if (g < 8) S[(c * kChunkBlocks + b) * 8 + g] = T;
}

// The same block sums with 16-byte loads (content 16-byte aligned).  Lane g
// of a 16-lane group holds words 2g and 2g + 1 of each 256-byte chunk cc of a
// 1 KiB block: stripe 4cc + g/4, accumulator lanes 2(g & 3) and 2(g & 3) + 1
// (the page kernels' layout without their one-word page offset).  Word 2g
// adds its multiply term to the even accumulator of pair g & 3 and its raw
// value to the odd one; word 2g + 1 the other way round (xxhash.h:5778-5817).
// Two row rotations (4, 8) finish the block sum of each pair.  A group
// folds four consecutive blocks (16 loads in flight per lane).
constexpr int kSums16Blocks = 4;  // 1 KiB blocks per group
__global__ __launch_bounds__(256) void k_manifest_sums16(const uint8_t* __restrict__ content, uint64_t total,
                                                        uint64_t* __restrict__ S) {
    // workgroups in the page kernels' tile order over (chunk, 64 KiB window):
    // 1 GiB 292.6 -> 284.0 us against dispatch order (profiles/r03/manifest_order_ab.txt)
    const uint64_t lin = (uint64_t)blockIdx.y * gridDim.x + blockIdx.x;
    const uint64_t t = xcd_tile(lin, (uint64_t)gridDim.x * gridDim.y);
    const uint64_t c = t / gridDim.x;
    const uint32_t bx = (uint32_t)(t % gridDim.x);
    const uint32_t L = manifest_chunk_len(total, c);
    if (L < kLongMin) return;  // a short last chunk is hashed whole by the chain kernel
    const int g = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const uint32_t nb = (L - 1) / 1024;
    const uint32_t b0 = (bx * 16 + grp) * kSums16Blocks;
    if (b0 >= nb) return;
    uint64_t key[4][2];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int jb = 32 * cc + 2 * g + e;  // word of the block: stripe jb / 8, lane jb % 8
            key[cc][e] = c_keys.acc[(jb >> 3) + (jb & 7)];
        }
    const u32x4* in = reinterpret_cast<const u32x4*>(content + c * kManifestChunk + (size_t)b0 * 1024) + g;
    u32x4 d[kSums16Blocks][4];
#pragma unroll
    for (int i = 0; i < kSums16Blocks; ++i)
#pragma unroll
        for (int cc = 0; cc < 4; ++cc)
            if (b0 + i < nb) d[i][cc] = ld16<true>(in + i * 64 + cc * 16);
#pragma unroll
    for (int i = 0; i < kSums16Blocks; ++i) {
        if (b0 + i >= nb) break;
        uint64_t E = 0, O = 0;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            const uint64_t w0 = lo64(d[i][cc]), w1 = hi64(d[i][cc]);
            E += mul32x32(w0 ^ key[cc][0]) + w1;
            O += mul32x32(w1 ^ key[cc][1]) + w0;
        }
        E += dpp64<kRowRor4>(E);
        E += dpp64<kRowRor8>(E);
        O += dpp64<kRowRor4>(O);
        O += dpp64<kRowRor8>(O);
        if (g < 4) {
            uint64_t* r = S + (c * kChunkBlocks + b0 + i) * 8 + 2 * g;
            r[0] = E;  // plain stores: the chain kernel reads them back from cache
            r[1] = O;  // (nt: sums 182 -> 186 us, chains 55 -> 74 us at 1 GiB)
        }
    }
}

__global__ __launch_bounds__(256) void k_manifest_chain(const uint8_t* __restrict__ content, uint64_t total,
                                                       const uint64_t* __restrict__ S, uint64_t* __restrict__ h) {
    // The chunk's block sums pass through LDS in halves of 512 blocks (32 KiB),
    // so five workgroups fit a CU and 1,024 chains run in one round (a whole
    // 64 KiB chunk of sums allowed two per CU).
    constexpr uint32_t kHalf = kChunkBlocks / 2;
    __shared__ uint64_t sums[kHalf][8];
    const uint64_t c = blockIdx.x;
    const uint32_t L = manifest_chunk_len(total, c);
    const uint8_t* in8 = content + c * kManifestChunk;
    const int tid = threadIdx.x, g = tid & 15;
    if (L < kLongMin) {
        if (tid == 0) h[c] = xxh3_any(in8, L);
        return;
    }
    const uint32_t nb = (L - 1) / 1024;
    uint64_t acc = tid < 8 ? c_init_acc[tid] : 0;
    for (uint32_t h0 = 0; h0 < nb; h0 += kHalf) {  // trip count uniform across the workgroup
        const uint32_t hn = min(kHalf, nb - h0);
        const u32x4* src = reinterpret_cast<const u32x4*>(S + (c * kChunkBlocks + h0) * 8);
        u32x4* dst = reinterpret_cast<u32x4*>(&sums[0][0]);
        for (uint32_t i = tid; i < hn * 4; i += blockDim.x) dst[i] = src[i];  // hn blocks x 64 B
        __syncthreads();
        if (tid < 8) {
            const uint64_t key = c_keys.scr[tid];
            uint32_t b = 0;
            for (; b + 8 <= hn; b += 8) {  // sums do not depend on acc: read 8 ahead
                uint64_t v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = sums[b + k][tid];
#pragma unroll
                for (int k = 0; k < 8; ++k) acc = xxh3_scramble(acc + v[k], key);
            }
            for (; b < hn; ++b) acc = xxh3_scramble(acc + sums[b][tid], key);
        }
        __syncthreads();  // sums is refilled by the next half
    }
    if (tid >= 64) return;
    if (tid < 16) {  // tail block, last stripe and merge, as in k_xxh3_long
        const uint64_t* in = reinterpret_cast<const uint64_t*>(in8);
        const int nst = (int)(((L - 1) - 1024 * nb) / 64);
        uint64_t T = xxh3_long_block(in + (size_t)nb * 128, g, nst);
        uint64_t M = 0, R = 0;
        if (g < 8) {
            const uint64_t v = ld64(in8 + L - 64 + 8 * g);
            M = mul32x32(v ^ c_keys.last[g]);
            R = v;
        }
        T += M + dpp64<kQuadSwap1>(R);
        acc += T;
        const uint64_t nxt = dpp64<kRowRor15>(acc);
        uint64_t m = (g < 8 && (g & 1) == 0) ? mul_fold64(acc ^ c_keys.merge[g], nxt ^ c_keys.merge[g + 1]) : 0;
        m += dpp64<kRowRor2>(m);
        m += dpp64<kRowRor4>(m);
        if (g == 6) h[c] = xxh3_avalanche((uint64_t)L * kP64_1 + m);
    }
}

// The fold is a serial chain over the chunk digests.  One wave loads 64
// digests at a time (the next batch in flight while this one is folded) and
// walks them with readlane, so the chain waits on multiplies, not on a global
// load per chunk (1,024 chunks: 64-75 us -> see profiles/r01/manifest_lab.txt).
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}
__global__ __launch_bounds__(64) void k_manifest_fold(const uint64_t* __restrict__ chunk_h, uint64_t nchunks,
                                                     uint64_t* __restrict__ out) {
    const int lane = threadIdx.x;
    uint64_t agg = 0;
    uint64_t cur = (uint64_t)lane < nchunks ? chunk_h[lane] : 0;
    for (uint64_t b = 0; b < nchunks; b += 64) {
        const uint64_t nb = b + 64 + (uint64_t)lane;
        const uint64_t nxt = nb < nchunks ? chunk_h[nb] : 0;
        const int m = (int)min<uint64_t>(64, nchunks - b);
        // rotl by shifts, not rotl64: the rotate would be a VALU v_alignbit and a
        // round trip out of the scalar unit on every step of the chain
        if (m == 64) {
#pragma unroll 16
            for (int k = 0; k < 64; ++k) agg = (((agg << 1) | (agg >> 63)) ^ readlane64(cur, k)) * 0x9e3779b97f4a7c15ull;
        } else {
            for (int k = 0; k < m; ++k) agg = (((agg << 1) | (agg >> 63)) ^ readlane64(cur, k)) * 0x9e3779b97f4a7c15ull;
        }
        cur = nxt;
    }
    if (lane == 0) *out = agg;
}

__global__ void k_make_chunks(uint64_t total, uint64_t chunk, uint64_t n, uint64_t* __restrict__ off,
                              uint32_t* __restrict__ len) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        off[i] = i * chunk;
        len[i] = (uint32_t)min(chunk, total - i * chunk);
    }
}

// ---------------------------------------------------------------------------
// workload generation / corruption / read-ceiling (benchmark + test tooling)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix_word(uint64_t seed, uint64_t page, uint64_t w) {
    uint64_t z = (seed ^ page) + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_gen_pages(uint64_t* __restrict__ pages, uint64_t words_per_page, uint64_t n,
                                                  uint64_t seed, uint64_t first_page) {
    for (uint64_t p = blockIdx.x; p < n; p += gridDim.x) {
        uint64_t* dst = pages + p * words_per_page;
        for (uint64_t w = threadIdx.x; w < words_per_page; w += blockDim.x)
            dst[w] = splitmix_word(seed, first_page + p, w);
    }
}

__global__ __launch_bounds__(256) void k_gen_desc(uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                 const uint32_t* __restrict__ len, uint64_t n, uint64_t seed,
                                                 uint64_t first_page) {
    for (uint64_t p = blockIdx.x; p < n; p += gridDim.x) {
        uint8_t* dst = base + off[p];
        const uint32_t L = len[p];
        for (uint32_t w = threadIdx.x; w * 8u < L; w += blockDim.x) {
            const uint64_t v = splitmix_word(seed, first_page + p, w);
            const uint32_t nb = (L - w * 8u) < 8u ? (L - w * 8u) : 8u;
            if (nb == 8 && ((off[p] & 7) == 0)) *reinterpret_cast<uint64_t*>(dst + 8u * w) = v;
            else
                for (uint32_t b = 0; b < nb; ++b) dst[8u * w + b] = (uint8_t)(v >> (8 * b));
        }
    }
}

__global__ void k_flip_byte(uint8_t* pages, uint64_t P, uint64_t n, uint64_t every, uint64_t byte_off) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t p = k * every;
    if (p < n) pages[p * P + byte_off] ^= 0xFF;
}

// Second pass of a two-pass stamp: page i bytes [0, 8) = digest[i], one
// non-temporal store per page.  A plain store makes this kernel faster (33 vs
// 55 us for 1 M headers) but leaves the lines dirty in cache, and their
// write-back then lands inside the next launch: back-to-back stamps took 711
// us each with plain stores against 644 us with nt.  Whole 64-byte header
// lines from a compact copy (pass 1 keeping the page's first line) cost more
// in pass 1 than they save here (725-745 us per stamp;
// tools/lab/stamp_line_lab.hip, profiles/r01/stamp_line_lab.txt).
__global__ __launch_bounds__(256) void k_scatter_stamp(uint8_t* __restrict__ pages, uint64_t P, uint64_t n,
                                                      const uint64_t* __restrict__ dig) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t* p = pages + i * P;
    if (((uintptr_t)p & 7) == 0) st_nt(reinterpret_cast<uint64_t*>(p), dig[i]);
    else __builtin_memcpy(p, &dig[i], 8);  // odd page sizes / unaligned batches
}

// descriptor form of the header pass: page i at base + off[i], len[i] bytes
// (pages shorter than the 8-byte header are left alone, as the digest pass
// leaves them)
__global__ __launch_bounds__(256) void k_scatter_stamp_desc(uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                           const uint32_t* __restrict__ len, uint64_t n,
                                                           const uint64_t* __restrict__ dig) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && len[i] >= 8) {
        uint8_t* p = base + off[i];
        if (((uintptr_t)p & 7) == 0) st_nt(reinterpret_cast<uint64_t*>(p), dig[i]);
        else __builtin_memcpy(p, &dig[i], 8);
    }
}

// Streaming-read ceiling, built on k_xxh3_fixed<4096>'s exact
// structure (round 5's 64 KiB-window reader ran ~4 % below
// the hash kernel it was meant to bound): 256-thread blocks of 16 four-KiB
// "pages", a 16-lane group each, loading xxh3_page_fixed<4096>'s chunks in its
// order (chunk 0, then the other 15 dwordx4 non-temporal loads, all issued
// before any is used), xcd_tile order over a grid that covers every tile
// once, and the tile's 16 results staged in LDS and written as one 128-byte
// non-temporal store.  Only the hash is gone: each lane folds its 16 pieces
// with xor/add and the group xor-reduces them into the page's word.
// Occupancy: with 72 VGPRs this body would run 7 waves per SIMD and read
// 3-4 % slower than the hash kernel (4 waves, 120 VGPRs); over 1-7 waves per
// SIMD a plain read of 4 KiB pages is fastest at 2 (7.40 TB/s on 4 GiB, 7.42
// on 32 GiB: tools/lab/occupancy_lab.hip, profiles/r06/occupancy_lab_r06e.txt),
// so run_stream_read caps it there with dynamic LDS (kStreamLdsPad bytes per
// workgroup: two workgroups per CU).  The ceiling is the best plain read of
// these bytes found, not the reader at one arbitrary occupancy.
constexpr uint64_t kStreamPage = 4096;
constexpr size_t kStreamLdsPad = 163840 / 2 - 2048;
__global__ __launch_bounds__(256) void k_stream_read(const uint8_t* __restrict__ buf, uint64_t bytes,
                                                    uint64_t* __restrict__ out) {
    extern __shared__ uint64_t occupancy_pad[];  // allocated for the cap, never used
    __shared__ uint64_t tile_h[16];
    const int g = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const uint64_t npages = (bytes + kStreamPage - 1) / kStreamPage;
    const uint64_t ntiles = (npages + 15) / 16;
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const uint64_t pg = t * 16 + grp;
    if (pg < npages) {
        const u32x4* base = reinterpret_cast<const u32x4*>(buf + pg * kStreamPage) + g;
        const uint64_t lim = bytes - pg * kStreamPage;  // bytes of this page (whole pages: >= 4096)
        u32x4 d[16];
        if (lim >= kStreamPage) {
#pragma unroll
            for (int c = 0; c < 16; ++c) d[c] = ld16<true>(base + c * 16);
        } else {
#pragma unroll
            for (int c = 0; c < 16; ++c)
                d[c] = 256u * c + 16u * g + 16 <= lim ? ld16<true>(base + c * 16) : u32x4{0, 0, 0, 0};
        }
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
    const uint64_t i = t * 16 + threadIdx.x;
    if (threadIdx.x < 16 && i < npages) st_nt(out + i, tile_h[threadIdx.x]);
    if (bytes == 0) occupancy_pad[threadIdx.x] = 0;  // never taken (bytes >= 16): keeps the array
}

// ---------------------------------------------------------------------------
// launch plumbing
// ---------------------------------------------------------------------------
namespace {

int g_cu_count[64];
std::once_flag g_cu_once[64];

int cu_count() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    std::call_once(g_cu_once[dev], [dev] {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        g_cu_count[dev] = cus;
    });
    return g_cu_count[dev];
}

// Grid for a grid-stride kernel: enough 256-thread blocks to cover the work,
// capped at blocks_per_cu resident blocks per CU.
unsigned grid_for(uint64_t units, unsigned units_per_block, unsigned blocks_per_cu) {
    const uint64_t need = (units + units_per_block - 1) / units_per_block;
    const uint64_t cap = (uint64_t)cu_count() * blocks_per_cu;
    return (unsigned)(need < cap ? (need ? need : 1) : cap);
}

constexpr unsigned kBlock = 256;
constexpr unsigned kBlocksPerCu = 8;  // grid-stride cap for the auxiliary kernels

// Device scratch for multi-kernel operations (two-pass stamp, manifest
// chunk tables), fenced by events instead of the stream-ordered allocator.
// hipMallocAsync / hipFreeAsync scratch was measured to lose writes: a stamp
// enqueued while the GPU was still busy left 7 % of the page headers zero
// (tools/lab/read_lab.hip "stamp", profiles/r01/stamp_lab.txt).  A buffer
// here is handed out only when the event recorded after its last use has
// completed, so concurrent streams and host threads never share one in
// flight.  Buffers are kept for reuse (bounded by the number of operations
// in flight at once).
class ScratchPool {
public:
    hipError_t acquire(size_t bytes, void** out, int* id) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        // Oversized idle buffers given back here are freed after the mutex is
        // released: hipFree synchronises the device, and other threads'
        // acquire/release calls must not wait behind it.
        std::vector<void*> to_free;
        e = acquire_locked(dev, bytes, out, id, to_free);
        for (void* p : to_free) (void)hipFree(p);
        return e;
    }
    // The buffer becomes reusable once the work queued on s so far completes.
    hipError_t release(int id, hipStream_t s) {
        std::lock_guard<std::mutex> lk(mu_);
        Buf& b = bufs_[(size_t)id];
        const hipError_t e = hipEventRecord(b.done, s);
        b.busy = false;
        return e;
    }

private:
    hipError_t acquire_locked(int dev, size_t bytes, void** out, int* id, std::vector<void*>& to_free) {
        hipError_t e = hipSuccess;
        std::lock_guard<std::mutex> lk(mu_);
        int empty = -1;
        for (size_t i = 0; i < bufs_.size(); ++i) {
            Buf& b = bufs_[i];
            if (b.dev != dev || b.busy) continue;
            if (!b.p) {
                empty = (int)i;
                continue;
            }
            const hipError_t q = hipEventQuery(b.done);
            if (q == hipErrorNotReady) continue;
            if (q != hipSuccess) return q;
            // An idle buffer above kKeepBytes serves only a request of at least
            // half its size; any other request gives it back, so one large
            // manifest or stamp does not pin its scratch for the process life.
            const bool fits = b.bytes >= bytes && (b.bytes <= kKeepBytes || 2 * bytes >= b.bytes);
            if (!fits) {
                if (b.bytes > kKeepBytes) {
                    to_free.push_back(b.p);
                    b.p = nullptr;
                    b.bytes = 0;
                    if (empty < 0) empty = (int)i;
                }
                continue;
            }
            b.busy = true;
            *out = b.p;
            *id = (int)i;
            return hipSuccess;
        }
        Buf b;
        b.dev = dev;
        b.bytes = std::max<size_t>(bytes, 1u << 20);
        if ((e = hipMalloc(&b.p, b.bytes)) != hipSuccess) return e;
        b.busy = true;
        if (empty >= 0) {
            b.done = bufs_[(size_t)empty].done;
            bufs_[(size_t)empty] = b;
            *id = empty;
        } else {
            if ((e = hipEventCreateWithFlags(&b.done, hipEventDisableTiming)) != hipSuccess) {
                (void)hipFree(b.p);
                return e;
            }
            bufs_.push_back(b);
            *id = (int)bufs_.size() - 1;
        }
        *out = b.p;
        return hipSuccess;
    }

    static constexpr size_t kKeepBytes = 256u << 20;  // larger idle buffers are freed, not kept
    struct Buf {
        void* p = nullptr;
        size_t bytes = 0;
        hipEvent_t done = nullptr;
        int dev = 0;
        bool busy = false;
    };
    std::mutex mu_;
    std::vector<Buf> bufs_;
};
ScratchPool g_scratch;

// RAII lease of a scratch buffer for the work enqueued on one stream.
struct ScratchLease {
    void* p = nullptr;
    int id = -1;
    hipStream_t s;
    explicit ScratchLease(hipStream_t st) : s(st) {}
    hipError_t get(size_t bytes) { return g_scratch.acquire(bytes, &p, &id); }
    ~ScratchLease() {
        if (id >= 0) (void)g_scratch.release(id, s);
    }
};

bool is_pow2_page(uint64_t P) { return P >= 256 && P <= 65536 && (P & (P - 1)) == 0; }

// Process-unique launch ids for the off-shape flag word (k_xxh64_lds ->
// k_generic_desc): a random start, so a scratch word's stale contents (an
// older id, or whatever a fresh allocation holds) never match a new one.
uint64_t next_call_id() {
    static std::atomic<uint64_t> next{[] {
        uint64_t x = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^ 0x9E3779B97F4A7C15ull;
        x ^= x >> 33;
        x *= 0xFF51AFD7ED558CCDull;
        return x ^ (x >> 33);
    }()};
    return next.fetch_add(1, std::memory_order_relaxed);
}

}  // namespace

// ---------------------------------------------------------------------------
// tuning knobs (pcs_set_tuning): read at every launch
// ---------------------------------------------------------------------------
namespace {
constexpr int kTuneKeys = 37;
// Keys retired in round 2 with the variants they selected (measured slower,
// DESIGN.md §4): 4 XXH64 nt loads, 5 in-place stamp width, 10 descriptor tile
// sort, 12 descriptor slices, 14 XXH64 descriptor sort; round-2 experiments
// (commit 99804f2): 16 pages dealt to a wave's groups as they free up (+-1 %,
// profiles/r02/desc_wave_lab.txt), 17 pipelined split tiles (-2..-22 %,
// split_pipe_lab.txt), 18 plain result stores (+-0.2 %, result_store_lab.txt),
// 19 descriptor pages as a slice stream (-5..-8 %, desc_slices_lab.txt),
// 20 4 KiB-aligned descriptor steps (+-0.2 %, aligned_steps_lab.txt), 21 the
// descriptor body at 4 waves per SIMD (-0.6..-2.3 %, desc_lean_lab.txt);
// round 3: 22 the XXH64 direct-to-LDS segment ring (config 3 -0.8..-34 %,
// profiles/r03/x64_glds_ab_*.txt), 25 XXH64 tile-order chunks (no gain, a lab
// knob in commit 01e849b); round 5: 32 service polls kept in flight (+0.7 to
// +2.8 us per request, profiles/r05/service_poll_lab_r05k.txt).  Setting one
// fails.
constexpr bool kRetired[kTuneKeys] = {false, false, false, false, true, true, false, false, false, false, true,  false,
                                      true,  false, true,  false, true,  true,  true,  true,  true,  true,  true,  false,
                                      false, true,  false, false, false, true,  false, false, true,  false,
                                      false, false, false};
std::atomic<int64_t> g_tune[kTuneKeys] = {0, /*xxh3 blocks/CU*/ 0, /*xxh64 blocks/CU*/ 0, /*xxh3 nt*/ 1,
                                          /*retired*/ 0, /*retired*/ 0, /*xxh64 LDS depth (2/3/4/5 -> 1/2/4/3)*/ 0,
                                          /*zero copy*/ 1, /*xxh3 run-time size: 4-block batches*/ 1,
                                          /*xxh3 split pages from this size (0 = never)*/ 8192,
                                          /*retired*/ 0,
                                          /*zero-copy page list in kernel arguments*/ 1,
                                          /*retired*/ 0,
                                          /*manifest: wide block sums + chain kernel*/ 1,
                                          /*retired*/ 0,
                                          /*xxh64 LDS kernel: waves per workgroup (1, 2; else 4)*/ 4,
                                          /*retired*/ 0, /*retired*/ 0, /*retired*/ 0, /*retired*/ 0,
                                          /*retired*/ 0,
                                          /*retired*/ 0,
                                          /*retired (round 3: XXH64 direct-to-LDS ring)*/ 0,
                                          /*zero-copy validate: completion from the verdicts themselves*/ 1,
                                          /*validate service stream: 1 highest priority, 0 plain*/ 1,
                                          /*retired (round 3 lab: XXH64 tile-order chunks)*/ 0,
                                          /*test only: validate service torn-line drill, microseconds*/ 0,
                                          /*test only: host-batch calls left to fail*/ 0,
                                          /*validate service contention gate: callers (0 = off)*/ 2,
                                          /*retired (round 4 lab: XXH64 equal-byte runs)*/ 0,
                                          /*test only: service requests left to post as a stale partial answer*/ 0,
                                          /*zero-copy XXH3 stamps: done-byte completion up to this many pages*/ 256,
                                          /*retired (round 5 lab: service polls in flight)*/ 0,
                                          /*test only: service kernels serve nothing and leave this many us late*/ 0,
                                          /*zero-copy batches completing from their verdicts: event behind the kernel*/ 0,
                                          /*sync host calls: microseconds of spinning before sleeping between checks (0 = spin)*/ 0,
                                          /*validate service: polls read the kernel's departure words*/ 1};
}
int set_tuning(int key, int64_t value) {
    if (key <= 0 || key >= kTuneKeys || kRetired[key] || value < 0) return -1;
    g_tune[key].store(value, std::memory_order_relaxed);
    return 0;
}
bool take_tuning(int key) {
    if (key <= 0 || key >= kTuneKeys || kRetired[key]) return false;
    int64_t v = g_tune[key].load(std::memory_order_relaxed);
    while (v > 0)
        if (g_tune[key].compare_exchange_weak(v, v - 1, std::memory_order_relaxed)) return true;
    return false;
}
int64_t get_tuning(int key) {
    return (key <= 0 || key >= kTuneKeys || kRetired[key]) ? -1 : g_tune[key].load(std::memory_order_relaxed);
}

namespace {
// Page kernels: the knob caps the grid at that many 256-thread blocks per CU
// (grid-stride loop beyond); 0 = auto.  Auto launches one block per 16 (XXH3)
// / 64 (XXH64) pages for pages up to 16 KiB and caps at 8 blocks per CU for
// larger pages (measured, profiles/r01_kernel_lab.txt).
unsigned page_grid(uint64_t n, unsigned pages_per_block, int key, uint64_t page_size = 0) {
    int64_t bpc = g_tune[key].load(std::memory_order_relaxed);
    if (bpc == 0) bpc = page_size > 16384 ? 8 : (int64_t)1 << 30;
    const uint64_t need = (n + pages_per_block - 1) / pages_per_block;
    const uint64_t cap = std::min<uint64_t>((uint64_t)cu_count() * (uint64_t)bpc, 0x7FFFFFFFull);
    return (unsigned)(need < cap ? (need ? need : 1) : cap);
}
bool use_nt() { return g_tune[3].load(std::memory_order_relaxed) != 0; }
// Fixed-size XXH3 pages hashed by k_xxh3_split (PCS_TUNE_XXH3_SPLIT_PAGES).
bool split_pages(uint64_t P) {
    const int64_t split = g_tune[9].load(std::memory_order_relaxed);
    return split > 0 && P >= (uint64_t)split && P >= 8192 && P <= 65536 && (P & (P - 1)) == 0;
}
bool rt_batch4() { return g_tune[8].load(std::memory_order_relaxed) != 0; }

// XXH64 LDS kernel launch with the segment depth from PCS_TUNE_XXH64_LAYOUT
// (0 or 1 = default depth, 2/3/4/5 = depth 1/2/4/3) and the waves per workgroup
// from PCS_TUNE_XXH64_WAVES.
template <int MODE, bool NT, int ADDR>
void launch_xxh64_lds(unsigned grid, hipStream_t s, const uint8_t* base, const uint64_t* off, const uint32_t* len,
                      uint32_t P, uint64_t n, uint64_t* out, uint8_t* ok, unsigned long long* fb,
                      unsigned long long* offshape = nullptr, uint64_t call_id = 0) {
    const int64_t lay = g_tune[6].load(std::memory_order_relaxed);
    const int depth = lay == 2 ? 1 : lay == 3 ? 2 : lay == 4 ? 4 : lay == 5 ? 3 : kX64LdsDepth;
    const int64_t wpb = g_tune[15].load(std::memory_order_relaxed);
    if (wpb == 1 || wpb == 2) {
        // one workgroup per 16 * wpb pages, every tile covered once
        const unsigned g = (unsigned)std::min<uint64_t>((n + 16 * wpb - 1) / (16 * wpb), 0x7FFFFFFFull);
#define LW(D, W) hipLaunchKernelGGL((k_xxh64_lds<MODE, NT, ADDR, D, W>), dim3(g), dim3(64 * W), 0, s, base, off, len, P, n, out, ok, fb, offshape, call_id)
        if (wpb == 1) {
            if (depth == 1) LW(1, 1);
            else if (depth == 2) LW(2, 1);
            else if (depth == 3) LW(3, 1);
            else LW(4, 1);
        } else {
            if (depth == 1) LW(1, 2);
            else if (depth == 2) LW(2, 2);
            else if (depth == 3) LW(3, 2);
            else LW(4, 2);
        }
#undef LW
        return;
    }
#define L(D) hipLaunchKernelGGL((k_xxh64_lds<MODE, NT, ADDR, D>), dim3(grid), dim3(kBlock), 0, s, base, off, len, P, n, out, ok, fb, offshape, call_id)
    if (depth == 1) L(1);
    else if (depth == 2) L(2);
    else if (depth == 3) L(3);
    else L(4);
#undef L
}

template <int MODE, bool NT>
hipError_t launch_xxh3_pages(uint64_t P, const uint8_t* pages, uint64_t n, uint64_t* out, uint8_t* ok,
                             unsigned long long* fb, hipStream_t s) {
    const unsigned grid = page_grid(n, kBlock / 16, 1, P);  // kBlock/16 = one 16-page tile per block
    if (P % 256 != 0) {  // off the chunk grid: the any-size body
        hipLaunchKernelGGL((k_xxh3_stride<MODE, NT, 2>), dim3(grid), dim3(kBlock), 0, s, pages, (uint32_t)P, n, out, ok,
                           fb);
        return hipGetLastError();
    }
    if ((uintptr_t)pages % 16 != 0) {
        // on the grid but not 16-byte aligned: the chunked run-time-size body
        // reads unaligned 16-byte pieces at ~6 TB/s (4 KiB pages at base + 8),
        // the any-size body's 8-byte final-block loads at ~4.5
        hipLaunchKernelGGL((k_xxh3_stride<MODE, NT, 1>), dim3(grid), dim3(kBlock), 0, s, pages, (uint32_t)P, n, out, ok,
                           fb);
        return hipGetLastError();
    }
    if (split_pages(P)) {
        const uint64_t ppb = 16 / (P / 4096);
        const uint64_t need = (n + ppb - 1) / ppb;
        const unsigned g = (unsigned)std::min<uint64_t>(need, 0x7FFFFFFFull);
        switch (P) {
#define CASE(SZ) \
    case SZ: hipLaunchKernelGGL((k_xxh3_split<SZ, MODE, NT>), dim3(g), dim3(kBlock), 0, s, pages, n, out, ok, fb); break;
            CASE(8192) CASE(16384) CASE(32768) CASE(65536)
#undef CASE
        }
        return hipGetLastError();
    }
    switch (P) {
#define CASE(SZ)                                                                                             \
    case SZ:                                                                                                 \
        hipLaunchKernelGGL((k_xxh3_fixed<SZ, MODE, NT>), dim3(grid), dim3(kBlock), 0, s, pages, n, out, ok, fb);     \
        break;
        CASE(256) CASE(512) CASE(1024) CASE(2048) CASE(4096) CASE(8192) CASE(16384) CASE(32768) CASE(65536)
#undef CASE
        default:
            if (rt_batch4())
                hipLaunchKernelGGL((k_xxh3_stride<MODE, NT, 1>), dim3(grid), dim3(kBlock), 0, s, pages, (uint32_t)P,
                                   n, out, ok, fb);
            else
                hipLaunchKernelGGL((k_xxh3_stride<MODE, NT, 0>), dim3(grid), dim3(kBlock), 0, s, pages, (uint32_t)P,
                                   n, out, ok, fb);
    }
    return hipGetLastError();
}

}  // namespace

// Fixed-stride pages.  Shape checks are done by the caller (capi).
template <int MODE>
static hipError_t pages_impl(int algo, const uint8_t* pages, uint64_t P, uint64_t n, uint64_t* out, uint8_t* ok,
                             unsigned long long* fb, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const bool aligned16 = ((uintptr_t)pages % 16) == 0;
    const bool aligned8 = ((uintptr_t)pages % 8) == 0;
    // XXH3: the chunked kernels on the 256-byte grid at 16-byte alignment, the
    // any-size body (k_xxh3_stride<..., 2>) for every other long-path size
    if (algo == 0 && P >= 249 && P <= 0xFFFFFFFFull) {
        if constexpr (MODE == kStamp) {
            // two-pass stamp: digests into a compact array (the fast digest
            // kernel), then one scattered 8-byte write per page
            uint64_t* dig = out;
            hipError_t e = hipSuccess;
            ScratchLease scratch(s);
            if (!dig) {
                e = scratch.get(n * 8);
                dig = static_cast<uint64_t*>(scratch.p);
            }
            if (e == hipSuccess)
                e = use_nt() ? launch_xxh3_pages<kDigest, true>(P, pages, n, dig, nullptr, nullptr, s)
                             : launch_xxh3_pages<kDigest, false>(P, pages, n, dig, nullptr, nullptr, s);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_scatter_stamp, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                                   const_cast<uint8_t*>(pages), P, n, dig);
                e = hipGetLastError();
            }
            return e;
        } else {
            return use_nt() ? launch_xxh3_pages<MODE, true>(P, pages, n, out, ok, fb, s)
                            : launch_xxh3_pages<MODE, false>(P, pages, n, out, ok, fb, s);
        }
    }
    if (algo == 1 && aligned8 && P % 8 == 0 && P >= 40 && P <= 0xFFFFFFFFull) {
        const bool lines = aligned16 && P % 64 == 0 && P >= 128;
        if (lines) {
            // one workgroup per 64 pages at every page size: the large-page
            // cap of page_grid (8 per CU) cost the LDS kernel 7-8 % on 64 KiB
            // pages (profiles/r01/x64_depth_lab.txt, x64_waves_lab.txt)
            const unsigned lgrid = page_grid(n, kBlock / 4, 2);
            if (use_nt()) launch_xxh64_lds<MODE, true, kAddrStride>(lgrid, s, pages, nullptr, nullptr, (uint32_t)P, n, out, ok, fb);
            else launch_xxh64_lds<MODE, false, kAddrStride>(lgrid, s, pages, nullptr, nullptr, (uint32_t)P, n, out, ok, fb);
            return hipGetLastError();
        }
        const unsigned grid = page_grid(n, kBlock / 4, 2, P);
        hipLaunchKernelGGL((k_xxh64_stride<MODE>), dim3(grid), dim3(kBlock), 0, s, pages, (uint32_t)P, n, out, ok, fb);
        return hipGetLastError();
    }
    return hipErrorNotSupported;  // caller falls back to the descriptor path
}

__global__ void k_uniform_desc(uint64_t P, uint64_t n, uint64_t* __restrict__ off, uint32_t* __restrict__ len) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        off[i] = i * P;
        len[i] = (uint32_t)P;
    }
}

hipError_t run_pages(int mode, int algo, const uint8_t* pages, uint64_t P, uint64_t n, uint64_t* out, uint8_t* ok,
                     unsigned long long* fb, hipStream_t s) {
    hipError_t e;
    switch (mode) {
        case kDigest: e = pages_impl<kDigest>(algo, pages, P, n, out, ok, fb, s); break;
        case kValidate: e = pages_impl<kValidate>(algo, pages, P, n, out, ok, fb, s); break;
        default: e = pages_impl<kStamp>(algo, pages, P, n, out, ok, fb, s); break;
    }
    if (e != hipErrorNotSupported) return e;
    // Odd shape (unaligned base, page size off the fast kernels): the same
    // pages as a descriptor batch (off = i * P, len = P) built on the device.
    ScratchLease scratch(s);
    if ((e = scratch.get(n * 12)) != hipSuccess) return e;
    uint64_t* off = static_cast<uint64_t*>(scratch.p);
    uint32_t* len = reinterpret_cast<uint32_t*>(off + n);
    hipLaunchKernelGGL(k_uniform_desc, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, n, off, len);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return run_desc(mode, algo, pages, off, len, n, 8, 0, out, ok, fb, s);
}

hipError_t scratch_acquire(size_t bytes, void** out, int* id) { return g_scratch.acquire(bytes, out, id); }
hipError_t scratch_release(int id, hipStream_t s) { return g_scratch.release(id, s); }

template <int MODE>
static hipError_t desc_impl(int algo, const uint8_t* base, const uint64_t* off, const uint32_t* len, uint64_t n,
                            int skip, uint64_t seed, uint64_t* out, uint8_t* ok, unsigned long long* fb,
                            hipStream_t s) {
    if (n == 0) return hipSuccess;
    if constexpr (MODE == kStamp) {
        if (skip == 8 && seed == 0) {
            // two-pass stamp, as for fixed-size pages: digests of every page
            // into a compact array (the descriptor digest kernels), then one
            // 8-byte header write per page.  Against headers written by the
            // digest kernel inside its read stream: +2.5 % (XXH3) and +7.1 %
            // (XXH64) on config 3 (profiles/r02/desc_stamp_lab.txt).
            uint64_t* dig = out;
            ScratchLease scratch(s);
            hipError_t e = hipSuccess;
            if (!dig) {
                e = scratch.get(n * 8);
                dig = static_cast<uint64_t*>(scratch.p);
            }
            if (e == hipSuccess) e = desc_impl<kDigest>(algo, base, off, len, n, skip, seed, dig, nullptr, nullptr, s);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_scatter_stamp_desc, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                                   const_cast<uint8_t*>(base), off, len, n, dig);
                e = hipGetLastError();
            }
            return e;
        }
    }
    if (skip == 8 && seed == 0) {
        // fast kernels for conforming pages, generic lanes for the rest
        if (algo == 0) {
            // one workgroup per 16-page tile, every tile covered once
            const uint64_t ntiles = (n + 15) / 16;
            if (ntiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
            const unsigned grid = (unsigned)ntiles;
#define L(NT_, B4_) \
    hipLaunchKernelGGL((k_xxh3_desc<MODE, NT_, B4_>), dim3(grid), dim3(kBlock), 0, s, base, off, len, n, out, ok, fb)
            if (use_nt()) {
                if (rt_batch4()) L(true, true);
                else L(true, false);
            } else {
                if (rt_batch4()) L(false, true);
                else L(false, false);
            }
#undef L
            // every page is the descriptor kernel's (fast body, any-size body,
            // short pages on one lane): no generic pass, which cost 4.7-5.2 us
            // per call on config 3 (profiles/r02d_sweep.json, r02e_sweep.json)
            return hipGetLastError();
        } else {
            // Pages off the line shape (usually none) are left to the generic
            // lanes below.  A separate quad-per-page pass over the
            // descriptors for them cost 9.7 us per call on config 3 even when
            // it found nothing to do (profiles/r02a_sweep.json); the generic
            // pass itself, reading every descriptor, 6.3 us
            // (profiles/r03/r03k_kernel_stats.csv).  Now the LDS kernel
            // stores this call's id in a scratch word when it leaves a page
            // behind, and the generic pass exits at once unless it finds it.
            ScratchLease flag(s);
            hipError_t e = flag.get(sizeof(unsigned long long));
            if (e != hipSuccess) return e;
            auto* word = static_cast<unsigned long long*>(flag.p);
            const uint64_t id = next_call_id();
            const unsigned grid = page_grid(n, kBlock / 4, 2);
            if (use_nt()) launch_xxh64_lds<MODE, true, kAddrDesc>(grid, s, base, off, len, 0u, n, out, ok, fb, word, id);
            else launch_xxh64_lds<MODE, false, kAddrDesc>(grid, s, base, off, len, 0u, n, out, ok, fb, word, id);
            e = hipGetLastError();
            if (e != hipSuccess) return e;
            // one block per CU: when every page conforms (the usual case)
            // each block only reads the flag and leaves (a full-size grid
            // took 4.3 us to do that, profiles/r04b_sweep.json); rare
            // off-shape pages take the grid-stride loop
            const unsigned ggrid = std::min(grid_for(n, kBlock, kBlocksPerCu), (unsigned)cu_count());
            hipLaunchKernelGGL((k_generic_desc<MODE>), dim3(ggrid), dim3(kBlock), 0, s, base, off, len, n, algo, seed,
                               skip, 1, out, ok, fb, word, id);
            return hipGetLastError();
        }
    }
    int filter = 0;
    if (MODE == kDigest && algo == 0 && skip == 0) {
        // raw XXH3 ranges: long ones get a workgroup each
        const unsigned lgrid = grid_for(n, 1, 8);
        hipLaunchKernelGGL(k_xxh3_long, dim3(lgrid), dim3(kBlock), 0, s, base, off, len, n, out);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        filter = 2;
    }
    const unsigned grid = grid_for(n, kBlock, kBlocksPerCu);
    hipLaunchKernelGGL((k_generic_desc<MODE>), dim3(grid), dim3(kBlock), 0, s, base, off, len, n, algo, seed, skip,
                       filter, out, ok, fb, nullptr, 0ull);
    return hipGetLastError();
}

hipError_t run_manifest(const uint8_t* content, uint64_t len, uint64_t* out, hipStream_t s) {
    constexpr uint64_t kChunk = kManifestChunk;
    if (len == 0) return hipMemsetAsync(out, 0, 8, s);
    const uint64_t n = (len + kChunk - 1) / kChunk;
    if (((uintptr_t)content % 8) == 0 && g_tune[13].load(std::memory_order_relaxed) != 0) {
        // wide form: block sums over the whole GPU, then one chain per chunk
        ScratchLease scratch(s);  // block sums (64 KiB per chunk) + chunk digests
        hipError_t e = scratch.get(n * kChunkBlocks * 64 + n * 8);
        if (e != hipSuccess) return e;
        uint64_t* S = static_cast<uint64_t*>(scratch.p);
        uint64_t* h = S + n * kChunkBlocks * 8;
        if ((uintptr_t)content % 16 == 0)
            hipLaunchKernelGGL(k_manifest_sums16, dim3(kChunkBlocks / (16 * kSums16Blocks), (unsigned)n), dim3(256), 0, s,
                               content, len, S);
        else
            hipLaunchKernelGGL(k_manifest_sums, dim3(kChunkBlocks / 16, (unsigned)n), dim3(256), 0, s, content, len, S);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(k_manifest_chain, dim3((unsigned)n), dim3(256), 0, s, content, len, S, h);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(k_manifest_fold, dim3(1), dim3(64), 0, s, h, n, out);
        return hipGetLastError();
    }
    ScratchLease scratch(s);  // chunk offsets, lengths and digests
    hipError_t e = scratch.get(n * 20);
    if (e != hipSuccess) return e;
    uint64_t* off = static_cast<uint64_t*>(scratch.p);
    uint64_t* h = off + n;
    uint32_t* ln = reinterpret_cast<uint32_t*>(h + n);
    {
        hipLaunchKernelGGL(k_make_chunks, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, len, kChunk, n, off, ln);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = desc_impl<kDigest>(0, content, off, ln, n, 0, 0, h, nullptr, nullptr, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_manifest_fold, dim3(1), dim3(64), 0, s, h, n, out);
        e = hipGetLastError();
    }
    return e;
}

hipError_t run_desc(int mode, int algo, const uint8_t* base, const uint64_t* off, const uint32_t* len, uint64_t n,
                    int skip, uint64_t seed, uint64_t* out, uint8_t* ok, unsigned long long* fb, hipStream_t s) {
    switch (mode) {
        case kDigest: return desc_impl<kDigest>(algo, base, off, len, n, skip, seed, out, ok, fb, s);
        case kValidate: return desc_impl<kValidate>(algo, base, off, len, n, skip, seed, out, ok, fb, s);
        default: return desc_impl<kStamp>(algo, base, off, len, n, skip, seed, out, ok, fb, s);
    }
}

hipError_t run_list(int mode, int algo, const uint64_t* ptrs, const uint64_t* host_ptrs, uint64_t P, uint64_t n,
                    uint64_t* out, uint8_t* ok, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (!list_shape_ok(algo, P)) return hipErrorNotSupported;
    if (algo == 0) {
        const unsigned grid = (unsigned)std::min<uint64_t>((n + 15) / 16, (uint64_t)cu_count() * kBlocksPerCu);
        const bool inl = host_ptrs && n <= (uint64_t)kInlinePages && g_tune[11].load(std::memory_order_relaxed) != 0;
        InlineList list;
        if (inl) std::memcpy(list.p, host_ptrs, n * 8);
#define LAUNCH(M, PF)                                                                                                \
    do {                                                                                                             \
        if (inl)                                                                                                     \
            hipLaunchKernelGGL((k_xxh3_list_inl<M, PF>), dim3(grid), dim3(kBlock), 0, s, list, (uint32_t)P, n, out, ok); \
        else                                                                                                         \
            hipLaunchKernelGGL((k_xxh3_list<M, PF>), dim3(grid), dim3(kBlock), 0, s, ptrs, (uint32_t)P, n, out, ok);  \
    } while (0)
#define BY_SIZE(M)                                    \
    switch (P) {                                      \
        case 4096: LAUNCH(M, 4096); break;            \
        case 8192: LAUNCH(M, 8192); break;            \
        case 16384: LAUNCH(M, 16384); break;          \
        default: LAUNCH(M, 0);                        \
    }
        if (mode == kDigest) BY_SIZE(kDigest)
        else if (mode == kValidate) BY_SIZE(kValidate)
        else BY_SIZE(kStamp)
#undef BY_SIZE
#undef LAUNCH
    } else {
        const unsigned grid = (unsigned)std::min<uint64_t>((n + 63) / 64, (uint64_t)cu_count() * kBlocksPerCu);
        // deepest pipeline: over PCIe every segment is a round trip
#define LAUNCH(M)                                                                                              \
    hipLaunchKernelGGL((k_xxh64_lds<M, false, kAddrList, 4>), dim3(grid), dim3(kBlock), 0, s, nullptr, ptrs, nullptr, \
                       (uint32_t)P, n, out, ok, nullptr, nullptr, 0ull)
        if (mode == kDigest) LAUNCH(kDigest);
        else if (mode == kValidate) LAUNCH(kValidate);
        else LAUNCH(kStamp);
#undef LAUNCH
    }
    return hipGetLastError();
}

hipError_t run_gen_pages(uint8_t* pages, uint64_t P, uint64_t n, uint64_t seed, uint64_t first, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned grid = grid_for(n, 1, 16);
    hipLaunchKernelGGL(k_gen_pages, dim3(grid), dim3(kBlock), 0, s, reinterpret_cast<uint64_t*>(pages), P / 8, n, seed,
                       first);
    return hipGetLastError();
}

hipError_t run_gen_desc(uint8_t* base, const uint64_t* off, const uint32_t* len, uint64_t n, uint64_t seed,
                        uint64_t first, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned grid = grid_for(n, 1, 16);
    hipLaunchKernelGGL(k_gen_desc, dim3(grid), dim3(kBlock), 0, s, base, off, len, n, seed, first);
    return hipGetLastError();
}

hipError_t run_flip(uint8_t* pages, uint64_t P, uint64_t n, uint64_t every, uint64_t byte_off, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t count = (n + every - 1) / every;
    const unsigned grid = (unsigned)((count + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_flip_byte, dim3(grid), dim3(kBlock), 0, s, pages, P, n, every, byte_off);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Pre-armed validate service (pcs_service_*, SURVEY.md §8f-1: small
// ReadPages batches).  A launch per host batch costs ~14 µs before its first
// page is read; here a kernel stays resident between requests, polling the
// request line in pinned host memory, so a request finds it waiting: ~7.5 µs
// for one page (tools/lab/service_lab.hip, profiles/r03/service_lab.txt).
// The kernel leaves after idle_ticks without a request and, between
// requests, once it has lived life_ticks, so a device-synchronising call
// elsewhere in the process waits at most that long (a grid that never leaves
// blocks such calls for as long as requests keep coming); the
// host starts the next generation of it when it can no longer be sure one is
// waiting.  A kernel serves only requests of its own generation (the high 32
// bits of seq), so a late kernel of an earlier generation never serves a
// request twice, and leaves as soon as the box names a newer one, so the next
// kernel (queued behind it on the stream) starts at once.  Workgroup w
// serves request line w / wpl, as the (w % wpl)-th of the line's wpl
// workgroups.  18 of its lanes poll: 16 load the line's request words (seq,
// n, page_size, check, ptrs[0..12), eloqstore_pcs_internal.h) and two the
// box's stop and gen words, one 8-byte load each.  Those loads are separate,
// so a poll can see the new seq beside an older request's words: the
// workgroup serves a request only when the 15 words' mixes add up to the
// check word the host wrote with them, and otherwise reads the line again (a
// torn view of one request is ignored, never served).  A request of another
// generation is not this kernel's (the host re-posts it once its own kernel
// has left).  Then the polling lanes run a system-scope acquire (pages and
// ptrs[12..n) are read fresh from host memory, ordered after the seq that
// announced them), and the workgroup hashes pages j * 16 + group, stride
// wpl * 16 (the run-time-size XXH3 body: registered 16-byte-aligned pages,
// page_size % 256 == 0), storing each verdict word system-scope, which
// reaches host memory without a release fence.  A stamp request (high half
// of the page-size word) stores the digest into the page header instead and
// then a done word, released after it.
// One poll of the line in flight per lane.  Keeping 2 or 4 in flight (each
// lane issuing its next load before examining the previous one) measured
// +0.7 / +2.8 us per request (round 5, profiles/r05/service_poll_lab_r05k.txt):
// the acquire that follows a served poll waits for the newer polls still in
// flight, one more PCIe round trip on every request.
//
// exit_ticks (test only, PCS_TUNE_SERVICE_SLOW_EXIT_TEST): nonzero makes the
// kernel a slow leaver for the non-blocking-poll test: it serves no request
// and, once it has decided to leave, stays that many ticks longer.
__global__ __launch_bounds__(256) void k_service(ServiceBox* box, int wpl, uint64_t gen, uint64_t idle_ticks,
                                                 uint64_t life_ticks, uint64_t exit_ticks) {
    constexpr int W = kServiceLineWords;
    __shared__ uint64_t s_line[W];
    __shared__ int s_go;
    ServiceLine* line = &box->line[blockIdx.x / wpl];
    const int j = blockIdx.x % wpl;
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t born = __builtin_amdgcn_s_memrealtime();
    uint64_t t_last = born;
    uint64_t last = 0;  // the last seq this workgroup served
    uint64_t torn_noted = 0;
    for (;;) {
        if (threadIdx.x < W + 2) {
            const uint64_t* src = threadIdx.x < W ? &line->seq + threadIdx.x : &box->stop + (threadIdx.x - W);
            uint64_t w = 0;
            int go = 0;
            for (;;) {
                w = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                const uint64_t w0 = __shfl(w, 0, 32);
                // stop, or a newer generation queued behind this kernel
                if (__shfl(w, W, 32) != 0 || __shfl(w, W + 1, 32) != gen) break;
                if (w0 != last && (w0 >> 32) == gen && exit_ticks == 0) {
                    uint64_t m = threadIdx.x == kServiceCheckWord || threadIdx.x >= W ? 0 : service_word_mix(w, threadIdx.x);
#pragma unroll
                    for (int d = 1; d < W; d <<= 1) m += __shfl_xor(m, d, W);
                    // lane 0's sum for all 18 lanes, so every decision below is uniform
                    if (__shfl(m, 0, 32) == __shfl(w, kServiceCheckWord, 32)) {
                        go = 1;
                        break;
                    }
                    // torn: seq is new, some word is not yet this request's
                    if (j == 0 && threadIdx.x == 0 && torn_noted != w0) {
                        torn_noted = w0;
                        __hip_atomic_store(&line->torn_seq, w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                if (now - t_last > idle_ticks || now - born > life_ticks) break;
            }
            // acquire here, in the lanes whose loads saw the new seq; the
            // barrier then orders every lane's reads after it
            if (go) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            if (threadIdx.x < W) s_line[threadIdx.x] = w;
            if (threadIdx.x == 0) s_go = go;
        }
        __syncthreads();
        if (!s_go) {  // uniform per workgroup: idle, lifetime, stop or a newer generation
            if (exit_ticks) {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                while (__builtin_amdgcn_s_memrealtime() - t0 < exit_ticks) __builtin_amdgcn_s_sleep(127);
            }
            // Departure: each wave's verdict and header stores complete at
            // system scope, then one word says this workgroup has gone, so a
            // host that sees it may re-arm the line (no store of this
            // generation can land in it any more).
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __syncthreads();
            if (threadIdx.x == 0)
                __hip_atomic_store(&box->departed[blockIdx.x], (uint32_t)gen, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        last = s_line[0];
        const uint64_t n = s_line[1];
        const uint32_t P = (uint32_t)s_line[2];
        const bool stamp = (s_line[2] >> 32) != 0;  // kServiceStamp: write the digest into the header
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        for (uint64_t pg = (uint64_t)j * 16 + (threadIdx.x >> 4); pg < n; pg += (uint64_t)wpl * 16) {
            const uint64_t a = pg < (uint64_t)kServiceLinePtrs
                                   ? s_line[4 + pg]  // came with the checked poll
                                   : __hip_atomic_load(&line->ptrs[pg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            uint64_t stored = 0;
            const uint64_t h = xxh3_page_rt4<false>(reinterpret_cast<const uint8_t*>(a), P, L, stored);
            if (L.g == 0) {
                if (stamp) {
                    // the header, then the done word released after it: the
                    // host sees the word only once the header has landed
                    __hip_atomic_store(reinterpret_cast<uint64_t*>(a), h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(&line->ok[pg], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                } else {
                    __hip_atomic_store(&line->ok[pg], h == stored ? 1u : 0u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
        __syncthreads();  // every lane has read s_line and s_go before the next poll rewrites them
        t_last = __builtin_amdgcn_s_memrealtime();  // the idle clock starts after this workgroup's verdicts
    }
}

hipError_t run_service(ServiceBox* d_box, int lines, int wpl, uint32_t gen, uint64_t idle_ticks, uint64_t life_ticks,
                       uint64_t exit_ticks, hipStream_t s) {
    if (lines < 1 || lines > kServiceMaxLines || wpl < 1 || lines * wpl > kServiceMaxWorkgroups) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_service, dim3((unsigned)(lines * wpl)), dim3(kBlock), 0, s, d_box, wpl, (uint64_t)gen,
                       idle_ticks, life_ticks, exit_ticks);
    return hipGetLastError();
}

hipError_t run_stream_read(const uint8_t* buf, uint64_t bytes, uint64_t* out, hipStream_t s) {
    if (bytes < 16) return hipSuccess;
    const uint64_t ntiles = ((bytes + kStreamPage - 1) / kStreamPage + 15) / 16;
    if (ntiles > 0x7FFFFFFFull) return hipErrorNotSupported;
    static std::once_flag once;
    static hipError_t attr = hipSuccess;
    std::call_once(once, [] {
        attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_stream_read),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStreamLdsPad);
    });
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(k_stream_read, dim3((unsigned)ntiles), dim3(kBlock), kStreamLdsPad, s, buf,
                       bytes & ~uint64_t(15), out);
    return hipGetLastError();
}

}  // namespace pcs
