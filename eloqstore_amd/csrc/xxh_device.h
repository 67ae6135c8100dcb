// xxh_device.h — CDNA4 device building blocks for the page-checksum kernels.
//
// Constants and scalar pieces of xxHash v0.8.3 as used on EloqStore's page
// path (reference: external/xxhash.h; page convention src/storage/page.cpp:18-31).
// The 192-byte default secret is only ever read at fixed offsets on the page
// path, so every secret word a kernel needs is folded into 64-bit constants at
// compile time (constexpr) and placed in __constant__ tables; no kernel indexes
// secret bytes at run time.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pcs {

// XXH_PRIME32_* (xxhash.h:2903-2907), XXH_PRIME64_* (:3454-3458), PRIME_MX* (:4380-4381)
constexpr uint32_t kP32_1 = 0x9E3779B1u;
constexpr uint32_t kP32_2 = 0x85EBCA77u;
constexpr uint32_t kP32_3 = 0xC2B2AE3Du;
constexpr uint64_t kP64_1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t kP64_2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t kP64_3 = 0x165667B19E3779F9ull;
constexpr uint64_t kP64_4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t kP64_5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t kMX1 = 0x165667919E3779F9ull;
constexpr uint64_t kMX2 = 0x9FB21C651E98DF25ull;

// XXH3_kSecret (xxhash.h:4365-4378).
constexpr uint8_t kSecretBytes[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

constexpr uint64_t secret64(int off) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | kSecretBytes[off + i];
    return v;
}
constexpr uint32_t secret32(int off) {
    uint32_t v = 0;
    for (int i = 3; i >= 0; --i) v = (v << 8) | kSecretBytes[off + i];
    return v;
}

// ---------------------------------------------------------------------------
// scalar pieces (one lane)
// ---------------------------------------------------------------------------

// XXH3_mul128_fold64 (xxhash.h:4566-4570)
__device__ __forceinline__ uint64_t mul_fold64(uint64_t a, uint64_t b) {
    return (a * b) ^ __umul64hi(a, b);
}

// lo32(x) * hi32(x) as a 64-bit product: the XXH3 accumulate multiply
// (XXH_mult32to64_add64, xxhash.h:5791) — one v_mad_u64_u32 with the add.
__device__ __forceinline__ uint64_t mul32x32(uint64_t x) {
    return (uint64_t)(uint32_t)x * (uint64_t)(uint32_t)(x >> 32);
}

// 64-bit rotate left by a compile-time 0 < r < 32: two v_alignbit_b32
// (the generic shift/or form costs ~5 VALU ops per rotate).
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
    if (__builtin_constant_p(r) && r > 0 && r < 32) {
        const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
        const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - r);
        const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - r);
        return ((uint64_t)nhi << 32) | nlo;
    }
    return (x << r) | (x >> (64 - r));
}

// XXH3_avalanche (xxhash.h:4583-4589)
__device__ __forceinline__ uint64_t xxh3_avalanche(uint64_t h) {
    h ^= h >> 37;
    h *= kMX1;
    return h ^ (h >> 32);
}

// XXH64_avalanche (xxhash.h:3503-3511)
__device__ __forceinline__ uint64_t xxh64_avalanche(uint64_t h) {
    h ^= h >> 33;
    h *= kP64_2;
    h ^= h >> 29;
    h *= kP64_3;
    return h ^ (h >> 32);
}

// XXH64_round (xxhash.h:3469-3491)
__device__ __forceinline__ uint64_t xxh64_round(uint64_t acc, uint64_t in) {
    acc += in * kP64_2;
    return rotl64(acc, 31) * kP64_1;
}

// XXH3 scramble of one accumulator lane (xxhash.h:5827-5856)
__device__ __forceinline__ uint64_t xxh3_scramble(uint64_t a, uint64_t key) {
    a ^= a >> 47;
    a ^= key;
    return a * (uint64_t)kP32_1;
}

// ---------------------------------------------------------------------------
// cross-lane moves inside a 16-lane DPP row
// ---------------------------------------------------------------------------
// DPP row_ror:n (ctrl 0x120 + n): lane i reads lane (i - n) mod 16 of its row.
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
constexpr int kRowRor1 = 0x121;
constexpr int kRowRor2 = 0x122;
constexpr int kRowRor4 = 0x124;
constexpr int kRowRor8 = 0x128;
constexpr int kRowRor15 = 0x12F;  // lane i reads lane i + 1
// quad_perm [s,s,s,s] broadcasts quad lane s to the quad
constexpr int quad_bcast(int s) { return s | (s << 2) | (s << 4) | (s << 6); }

}  // namespace pcs
