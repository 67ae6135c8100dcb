// xxh3_page.h — the XXH3-64 page body shared by the product kernels
// (pcs_kernels.hip) and the experiment harnesses (tools/lab/*.hip): key
// tables, per-lane state, block folding, whole-page loops and the XCD tile
// order.  Reference arithmetic: external/xxhash.h:5778-6081 (hashLong_64b),
// page convention src/storage/page.cpp:18-31.
#pragma once

#include "xxh_device.h"

namespace pcs {

// ---------------------------------------------------------------------------
// secret-derived key tables (all offsets fixed by xxhash.h)
// ---------------------------------------------------------------------------
struct KeyTables {
    uint64_t acc[24];   // secret + 8k       accumulate (stripe s, lane l -> k = s + l), :5801
    uint64_t last[8];   // secret + 121 + 8l last stripe (XXH_SECRET_LASTACC_START 7), :6013-6015
    uint64_t scr[8];    // secret + 128 + 8l scramble (secret + secretSize - 64), :5996
    uint64_t merge[8];  // secret + 11 + 8m  mergeAccs (XXH_SECRET_MERGEACCS_START), :6056-6061
};
constexpr KeyTables make_tables() {
    KeyTables t{};
    for (int k = 0; k < 24; ++k) t.acc[k] = secret64(8 * k);
    for (int l = 0; l < 8; ++l) t.last[l] = secret64(121 + 8 * l);
    for (int l = 0; l < 8; ++l) t.scr[l] = secret64(128 + 8 * l);
    for (int m = 0; m < 8; ++m) t.merge[m] = secret64(11 + 8 * m);
    return t;
}
__constant__ KeyTables c_keys = make_tables();

// XXH3_INIT_ACC (xxhash.h:6064-6065)
__constant__ uint64_t c_init_acc[8] = {kP32_3, kP64_1, kP64_2, kP64_3, kP64_4, kP32_2, kP64_5, kP32_1};

enum Mode : int { kDigest = 0, kValidate = 1, kStamp = 2 };

// Native 16-byte vector (global_load_dwordx4).  NT selects the non-temporal
// cache policy: every page byte is read exactly once, and the nt stream
// measured +15 % over default-policy loads on this layout (tools/lab/read_lab.hip,
// profiles/r01_read_lab.txt).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
__device__ __forceinline__ uint64_t lo64(u32x4 v) { return ((uint64_t)v.y << 32) | v.x; }
__device__ __forceinline__ uint64_t hi64(u32x4 v) { return ((uint64_t)v.w << 32) | v.z; }

// Per-page output for every kernel: digest array, verdict array + first bad
// index, or the digest stamped little-endian into page bytes [0, 8).  Stores
// are non-temporal: a plain 8-byte result store per page interleaved with the
// page read stream cost ~5 % of read bandwidth, an nt store ~1-2 %
// (profiles/r01/read_lab_stores.txt).
template <typename T>
__device__ __forceinline__ void st_nt(T* p, T v) { __builtin_nontemporal_store(v, p); }

// first_bad = min(first_bad, idx).  The word only ever decreases, so a stale
// (larger) read can only cause an unneeded atomic, never skip a needed one;
// reading first keeps a batch of mostly corrupt pages from serialising on
// one address.
__device__ __forceinline__ void note_bad(unsigned long long* first_bad, uint64_t idx) {
    if ((unsigned long long)idx < __hip_atomic_load(first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMin(first_bad, (unsigned long long)idx);
}

__device__ __forceinline__ void emit(int mode, uint64_t idx, uint64_t h, uint64_t stored, uint8_t* page_w,
                                     uint64_t* out, uint8_t* ok, unsigned long long* first_bad) {
    if (mode == kStamp) {
        st_nt(reinterpret_cast<uint64_t*>(page_w), h);
        if (out) st_nt(out + idx, h);
    } else if (mode == kValidate) {
        const bool good = (h == stored);
        st_nt(ok + idx, (uint8_t)(good ? 1 : 0));
        if (out) st_nt(out + idx, h);
        if (!good && first_bad) note_bad(first_bad, idx);
    } else {
        st_nt(out + idx, h);
    }
}

// ---------------------------------------------------------------------------
// XXH3 long-input page hash, one 16-lane group per page
// ---------------------------------------------------------------------------
//
// Index bookkeeping.  Page word w (u64) is input word j = w - 1 (the digest
// occupies page word 0).  Within a 1 KiB input block, input word jb sits in
// stripe s = jb >> 3, accumulator lane l = jb & 7, and is keyed with secret
// word k = s + l.  Lane g, chunk c, half e holds page word 128b + 32c + 2g + e,
// i.e. jb = 32c + 2g + e - 1:
//   e = 0 -> l odd  (pair (g-1) & 3): multiply term to the odd slot, raw add
//            to the even slot ("U" sums);
//   e = 1 -> l even (pair g & 3):     multiply term to the even slot, raw add
//            to the odd slot ("V" sums).
// The one word with jb = -1 (lane 0, chunk 0, e = 0) is page word 128b: it
// belongs to the PREVIOUS block (or is the stored digest for b = 0).  Lane 0
// instead takes page word 128(b+1) ("carry"), the block's own last input word
// (stripe 15, lane 7, key 22) — the low half of lane 0's chunk 0 of block b+1,
// which lane 0 loads for that block anyway.
struct Xxh3Lane {
    uint64_t k[4][2];     // accumulate keys, chunk c, half e
    uint64_t kl0, kl1;    // last-stripe keys (used by lanes 12..15)
    uint64_t ks_e, ks_o;  // scramble keys for pair p
    uint64_t km_e, km_o;  // merge keys for pair p
    uint64_t init_e, init_o;
    int g;
};

__device__ __forceinline__ Xxh3Lane make_xxh3_lane(int g) {
    Xxh3Lane L;
    L.g = g;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            int jb = 32 * c + 2 * g + e - 1;
            if (jb < 0) jb = 127;  // lane 0's carry word
            L.k[c][e] = c_keys.acc[(jb >> 3) + (jb & 7)];
        }
    const int gl = g & 3;
    L.kl0 = c_keys.last[2 * gl];
    L.kl1 = c_keys.last[2 * gl + 1];
    L.ks_e = c_keys.scr[2 * gl];
    L.ks_o = c_keys.scr[2 * gl + 1];
    L.km_e = c_keys.merge[2 * gl];
    L.km_o = c_keys.merge[2 * gl + 1];
    L.init_e = c_init_acc[2 * gl];
    L.init_o = c_init_acc[2 * gl + 1];
    return L;
}

// Fold one 1 KiB block (chunks 0..nchunks-1 present) into the sums (Te, To)
// of accumulator pair g & 3.  FINAL marks the last, partial block: no carry
// word, the last stripe (page words P/8-8 .. P/8-1, held by lanes 12..15 of
// the final chunk) keyed with secret + 121, and page words P/8-7 .. P/8-1
// excluded from the ordinary stripes (xxhash.h:6005-6016).
// NOCARRY leaves out the block's last input word (the carry, page word
// 128(b+1)); the caller adds its two terms later (split-page kernel).
template <bool FINAL, bool NOCARRY = false>
__device__ __forceinline__ void xxh3_block_terms(const Xxh3Lane& L, const u32x4 (&d)[4], uint64_t carry,
                                                 int nchunks, uint64_t& Te, uint64_t& To) {
    uint64_t Ue = 0, Uo = 0, Ve = 0, Vo = 0;
    const int g = L.g;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (FINAL && c >= nchunks) break;
        uint64_t w0 = lo64(d[c]);
        const uint64_t w1 = hi64(d[c]);
        bool use0 = true, use1 = true;
        if (c == 0) {
            if (FINAL || NOCARRY) use0 = (g != 0);
            else w0 = (g == 0) ? carry : w0;
        }
        if (FINAL && c == nchunks - 1 && g >= 12) {
            use1 = false;
            use0 = use0 && (g == 12);
            // last-stripe lane l' = 2(g-12) + e: both halves land on pair g & 3
            Ve += mul32x32(w0 ^ L.kl0) + w1;
            Vo += mul32x32(w1 ^ L.kl1) + w0;
        }
        const uint64_t m0 = mul32x32(w0 ^ L.k[c][0]);
        const uint64_t m1 = mul32x32(w1 ^ L.k[c][1]);
        Uo += use0 ? m0 : 0;
        Ue += use0 ? w0 : 0;
        Ve += use1 ? m1 : 0;
        Vo += use1 ? w1 : 0;
    }
    // pair p = g & 3 collects V of lanes g = p (mod 4) and U of lanes g = p + 1
    Te = Ve + dpp64<kRowRor15>(Ue);
    To = Vo + dpp64<kRowRor15>(Uo);
    Te += dpp64<kRowRor4>(Te);
    To += dpp64<kRowRor4>(To);
    Te += dpp64<kRowRor8>(Te);
    To += dpp64<kRowRor8>(To);
}

__device__ __forceinline__ uint64_t xxh3_merge(const Xxh3Lane& L, uint64_t Ae, uint64_t Ao, uint64_t len) {
    uint64_t m = mul_fold64(Ae ^ L.km_e, Ao ^ L.km_o);
    m += dpp64<kRowRor1>(m);
    m += dpp64<kRowRor2>(m);
    return xxh3_avalanche(len * kP64_1 + m);
}

// Whole page, compile-time page size P (P % 256 == 0, P >= 256).  Blocks are
// loaded in batches of up to 4 (4 KiB per page, 16 KiB per wave in flight)
// before any of them is folded, so a 4 KiB page is one batch.  The carry word
// of block b (page word 128(b+1)) is lane 0's low half of chunk 0 of block
// b+1, which lane 0 loads anyway: each batch also fetches chunk 0 of the
// following block and hands it on, so no byte is loaded twice.
template <int P, bool NT>
__device__ __forceinline__ uint64_t xxh3_page_fixed(const uint8_t* __restrict__ page, const Xxh3Lane& L,
                                                    uint64_t& stored, u32x4& first) {
    constexpr int NB = (P - 9) / 1024;   // full blocks (xxhash.h:5996)
    constexpr int R = P / 256 - 4 * NB;  // chunks in the final block, 1..4
    constexpr int TB = NB + 1;
    const u32x4* base = reinterpret_cast<const u32x4*>(page) + L.g;
    uint64_t Ae = L.init_e, Ao = L.init_o;
    u32x4 head = ld16<NT>(base);  // chunk 0 of the next block to fold
    stored = lo64(head);
    first = head;
#pragma unroll
    for (int b0 = 0; b0 < TB; b0 += 4) {
        constexpr int kMaxBatch = 4;
        u32x4 d[kMaxBatch + 1][4];
        d[0][0] = head;
#pragma unroll
        for (int i = 0; i <= kMaxBatch; ++i) {
            const int b = b0 + i;
            if (b >= TB) break;
            const int nc = (i == kMaxBatch) ? 1 : (b == NB) ? R : 4;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c < nc && !(i == 0 && c == 0)) d[i][c] = ld16<NT>(base + b * 64 + c * 16);
        }
#pragma unroll
        for (int i = 0; i < kMaxBatch; ++i) {
            const int b = b0 + i;
            if (b >= TB) break;
            uint64_t Te, To;
            if (b < NB) {
                xxh3_block_terms<false>(L, d[i], lo64(d[i + 1][0]), 4, Te, To);
                Ae = xxh3_scramble(Ae + Te, L.ks_e);
                Ao = xxh3_scramble(Ao + To, L.ks_o);
            } else {
                xxh3_block_terms<true>(L, d[i], 0, R, Te, To);
                Ae += Te;
                Ao += To;
            }
        }
        if (b0 + kMaxBatch < TB) head = d[kMaxBatch][0];
    }
    return xxh3_merge(L, Ae, Ao, (uint64_t)(P - 8));
}

// Run-time page size (P % 256 == 0, P >= 256): one block per step, chunk 0 of
// the next block prefetched with the current one (it supplies the carry).
template <bool NT>
__device__ __forceinline__ uint64_t xxh3_page_rt(const uint8_t* __restrict__ page, uint32_t P, const Xxh3Lane& L,
                                                 uint64_t& stored) {
    const int NB = (int)((P - 9) / 1024);
    const int R = (int)(P / 256) - 4 * NB;
    const u32x4* base = reinterpret_cast<const u32x4*>(page) + L.g;
    uint64_t Ae = L.init_e, Ao = L.init_o;
    u32x4 d[4];
    d[0] = ld16<NT>(base);
    stored = lo64(d[0]);
    for (int b = 0; b < NB; ++b) {
#pragma unroll
        for (int c = 1; c < 4; ++c) d[c] = ld16<NT>(base + b * 64 + c * 16);
        const u32x4 next0 = ld16<NT>(base + (b + 1) * 64);
        uint64_t Te, To;
        xxh3_block_terms<false>(L, d, lo64(next0), 4, Te, To);
        Ae = xxh3_scramble(Ae + Te, L.ks_e);
        Ao = xxh3_scramble(Ao + To, L.ks_o);
        d[0] = next0;
    }
#pragma unroll
    for (int c = 1; c < 4; ++c)
        if (c < R) d[c] = ld16<NT>(base + NB * 64 + c * 16);
    uint64_t Te, To;
    xxh3_block_terms<true>(L, d, 0, R, Te, To);
    return xxh3_merge(L, Ae + Te, Ao + To, (uint64_t)(P - 8));
}

// Run-time page size with the fixed kernel's batching: up to 4 blocks (4 KiB
// per group, 16 KiB per wave) are loaded before any is folded, so mixed-size
// batches keep as many bytes in flight as the fixed-size kernel.  Groups of a
// wave may have different page sizes; the loop then runs to the largest with
// the others masked.
template <bool NT>
__device__ __forceinline__ uint64_t xxh3_page_rt4(const uint8_t* __restrict__ page, uint32_t P, const Xxh3Lane& L,
                                                  uint64_t& stored) {
    const int NB = (int)((P - 9) / 1024);
    const int R = (int)(P / 256) - 4 * NB;
    const int TB = NB + 1;
    const u32x4* base = reinterpret_cast<const u32x4*>(page) + L.g;
    uint64_t Ae = L.init_e, Ao = L.init_o;
    u32x4 head = ld16<NT>(base);
    stored = lo64(head);
    for (int b0 = 0; b0 < TB; b0 += 4) {
        u32x4 d[5][4];
        d[0][0] = head;
#pragma unroll
        for (int i = 0; i <= 4; ++i) {
            const int b = b0 + i;
            const int nc = (b >= TB) ? 0 : (i == 4) ? 1 : (b == NB) ? R : 4;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c < nc && !(i == 0 && c == 0)) d[i][c] = ld16<NT>(base + b * 64 + c * 16);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int b = b0 + i;
            if (b < NB) {
                uint64_t Te, To;
                xxh3_block_terms<false>(L, d[i], lo64(d[i + 1][0]), 4, Te, To);
                Ae = xxh3_scramble(Ae + Te, L.ks_e);
                Ao = xxh3_scramble(Ao + To, L.ks_o);
            } else if (b == NB) {
                uint64_t Te, To;
                xxh3_block_terms<true>(L, d[i], 0, R, Te, To);
                Ae += Te;
                Ao += To;
            }
        }
        head = d[4][0];
    }
    return xxh3_merge(L, Ae, Ao, (uint64_t)(P - 8));
}

__device__ __forceinline__ bool xxh3_fast_ok(uint64_t off, uint32_t P) {
    return (P % 256u) == 0 && P >= 256u && (off % 16u) == 0;
}

// 8-byte load at any alignment (global_load_dwordx2; the part reads unaligned
// addresses in hardware)
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

// The final (partial) block for any page size P >= 249 (xxhash.h:6005-6016).
// Input word j of the block (page word 128 NB + 1 + j) is in an ordinary
// stripe iff j < 8 nbS, nbS = (P - 9 - 1024 NB) / 64; with the chunk layout
// of the full blocks (lane g, chunk c holds 16-byte piece k = 16c + g, words
// j = 2k - 1 and 2k), piece k < kmax = 4 nbS is used whole and piece kmax for
// its low word only (so it is loaded as 8 bytes: no load crosses the page
// end).  The last stripe (page bytes [P - 64, P), secret + 121) need not sit
// on the piece grid, so lanes 0-7 load its words separately (lastw): lane g
// holds last-stripe lane l = 2(g & 3) + (g >> 2), whose multiply term goes to
// acc[l] and raw word to acc[l ^ 1], both of pair g & 3, i.e. into this
// lane's V sums.  For P % 256 == 0 this is exactly xxh3_block_terms<true>.
__device__ __forceinline__ void xxh3_final_terms(const Xxh3Lane& L, const u32x4 (&d)[4], int kmax, uint64_t lastw,
                                                 uint64_t& Te, uint64_t& To) {
    uint64_t Ue = 0, Uo = 0, Ve = 0, Vo = 0;
    const int g = L.g;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int k = 16 * c + g;
        const uint64_t w0 = lo64(d[c]), w1 = hi64(d[c]);
        const bool use0 = k <= kmax && k != 0;  // piece 0's low word is the previous block's carry
        const bool use1 = k < kmax;
        const uint64_t m0 = mul32x32(w0 ^ L.k[c][0]);
        const uint64_t m1 = mul32x32(w1 ^ L.k[c][1]);
        Uo += use0 ? m0 : 0;
        Ue += use0 ? w0 : 0;
        Ve += use1 ? m1 : 0;
        Vo += use1 ? w1 : 0;
    }
    if (g < 8) {
        if (g < 4) {
            Ve += mul32x32(lastw ^ L.kl0);
            Vo += lastw;
        } else {
            Vo += mul32x32(lastw ^ L.kl1);
            Ve += lastw;
        }
    }
    Te = Ve + dpp64<kRowRor15>(Ue);
    To = Vo + dpp64<kRowRor15>(Uo);
    Te += dpp64<kRowRor4>(Te);
    To += dpp64<kRowRor4>(To);
    Te += dpp64<kRowRor8>(Te);
    To += dpp64<kRowRor8>(To);
}

// Any page size P >= 249 (hashed length > 240, the long path), any alignment:
// xxh3_page_rt4's batches of four 1 KiB blocks, the final block's pieces
// loaded in the same batch as the blocks before it (predicated per lane: only
// pieces holding ordinary-stripe words), its terms by xxh3_final_terms.
template <bool NT>
__device__ __forceinline__ uint64_t xxh3_page_any(const uint8_t* __restrict__ page, uint32_t P, const Xxh3Lane& L,
                                                  uint64_t& stored) {
    const int NB = (int)((P - 9) / 1024);
    const int kmax = 4 * (int)((P - 9 - 1024u * (uint32_t)NB) / 64u);  // 0..60
    const int TB = NB + 1;
    const int g = L.g;
    const u32x4* base = reinterpret_cast<const u32x4*>(page) + g;
    const uint64_t lastw = g < 8 ? ld64u(page + P - 64 + 8 * (2 * (g & 3) + (g >> 2))) : 0;
    stored = ld64u(page);
    uint64_t Ae = L.init_e, Ao = L.init_o;
    // piece c of the final block for this lane: whole, low word only, or none
    auto final_piece = [&](int c) -> u32x4 {
        const int k = 16 * c + g;
        const u32x4* q = base + NB * 64 + c * 16;
        if (k < kmax) return ld16<NT>(q);
        u32x4 v = {0, 0, 0, 0};
        if (k == kmax) {
            const uint64_t w = ld64u(reinterpret_cast<const uint8_t*>(q));
            v.x = (uint32_t)w;
            v.y = (uint32_t)(w >> 32);
        }
        return v;
    };
    u32x4 head = NB > 0 ? ld16<NT>(base) : final_piece(0);
    for (int b0 = 0; b0 < TB; b0 += 4) {
        u32x4 d[5][4];
        d[0][0] = head;
#pragma unroll
        for (int i = 0; i <= 4; ++i) {
            const int b = b0 + i;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (i == 0 && c == 0) continue;
                if (b < NB && (i < 4 || c == 0)) d[i][c] = ld16<NT>(base + b * 64 + c * 16);
                else if (b == NB && (i < 4 || c == 0)) d[i][c] = final_piece(c);
                else d[i][c] = u32x4{0, 0, 0, 0};
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int b = b0 + i;
            uint64_t Te, To;
            if (b < NB) {
                xxh3_block_terms<false>(L, d[i], lo64(d[i + 1][0]), 4, Te, To);
                Ae = xxh3_scramble(Ae + Te, L.ks_e);
                Ao = xxh3_scramble(Ao + To, L.ks_o);
            } else if (b == NB) {
                xxh3_final_terms(L, d[i], kmax, lastw, Te, To);
                Ae += Te;
                Ao += To;
            }
        }
        head = d[4][0];
    }
    return xxh3_merge(L, Ae, Ao, (uint64_t)(P - 8));
}

// pages the group kernels take at all: the XXH3 long path (hashed length > 240)
__device__ __forceinline__ bool xxh3_group_ok(uint32_t P) { return P >= 249u; }

// Block b of a grid that covers nb tiles once -> its tile.  Blocks are
// dispatched to the XCDs round-robin (XCD = b % 8); here each XCD takes
// chunks of C consecutive tiles (4 MiB of 4 KiB pages at C = 64 16-page
// tiles), and the chunks go to the XCDs round-robin, so at any moment the
// eight XCDs stream eight adjacent chunks.  Round 1 gave each XCD one
// contiguous eighth of the batch instead (cdna_hip_programming.md T1): on
// large or irregular batches that made the rate depend on where the buffer
// landed in physical memory (config 5: 0.815-0.924 over four allocations in
// one process, config 3: 0.844-0.896), while the chunked order holds
// 0.922-0.930 and 0.896-0.897 on the same allocations and is level or
// better on configs 2, 4 and 7 (profiles/r03/placement_*.txt).
// Tiles past the last whole round of chunks keep dispatch order (bijective).
// Round 1's order: the blocks of one XCD walk one contiguous eighth of the
// batch (cdna_hip_programming.md T1, bijective form).  Kept for the XXH64
// LDS kernel, where it beats the chunked order (config 2 0.863 against 0.800
// at 16-tile chunks, config 3 0.809 against 0.801, profiles/r03/
// x64_tile_order_ab.txt); chunks of 128-1024 of its 64-page tiles are no
// better either (config 2 -4.5..+0.2 %, config 3 -0.3..-1.0 %, config 4
// -12.8..+0.5 %, profiles/r03/lab_r03h/x64_order_c*.txt).
__device__ __forceinline__ uint64_t xcd_tile_eighths(uint64_t b, uint64_t nb) {
    const uint64_t q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

template <uint64_t C = 64>
__device__ __forceinline__ uint64_t xcd_tile(uint64_t b, uint64_t nb) {
    const uint64_t full = nb / (8 * C) * (8 * C);
    if (b >= full) return b;
    const uint64_t x = b % 8, k = b / 8;
    return ((k / C) * 8 + x) * C + k % C;
}

}  // namespace pcs
