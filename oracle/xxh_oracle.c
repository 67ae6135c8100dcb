/*
 * xxh_oracle.c — TEST INFRASTRUCTURE ONLY (see xxh_oracle.h).
 *
 * A plain-C restatement of xxHash v0.8.3's XXH3_64bits (seed 0, default
 * secret) and XXH64, written from the algorithm as the vendored header
 * documents it.  Scalar, unvectorised, little-endian host assumed (x86-64 and
 * the GPU box are both LE).  Each function cites the reference lines it
 * follows; line numbers refer to /root/reference/external/xxhash.h.
 *
 * Never linked into the product library.  Used by tests/ (checker),
 * __graft_entry__.smoke() (checker) and bench.py (cpu_baseline, kind "port"
 * when oracle/_ref is absent).
 */
#include "xxh_oracle.h"

#include <string.h>

/* ---- constants ---------------------------------------------------------- */
/* XXH_PRIME32_1..3   xxhash.h:2903-2905 */
#define P32_1 0x9E3779B1u
#define P32_2 0x85EBCA77u
#define P32_3 0xC2B2AE3Du
/* XXH_PRIME64_1..5   xxhash.h:3454-3458 */
#define P64_1 0x9E3779B185EBCA87ull
#define P64_2 0xC2B2AE3D27D4EB4Full
#define P64_3 0x165667B19E3779F9ull
#define P64_4 0x85EBCA77C2B2AE63ull
#define P64_5 0x27D4EB2F165667C5ull
/* PRIME_MX1 / PRIME_MX2   xxhash.h:4380-4381 */
#define MX_1 0x165667919E3779F9ull
#define MX_2 0x9FB21C651E98DF25ull

/* XXH3_kSecret — the 192-byte default secret, xxhash.h:4365-4378. */
static const uint8_t kSecret[192] = {
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

/* ---- little-endian readers / small helpers ------------------------------ */
static uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

/* XXH3_mul128_fold64, xxhash.h:4566-4570: low64 ^ high64 of the 128-bit product. */
static uint64_t mul_fold(uint64_t a, uint64_t b)
{
    unsigned __int128 p = (unsigned __int128)a * b;
    return (uint64_t)p ^ (uint64_t)(p >> 64);
}

/* XXH3_avalanche, xxhash.h:4583-4589 */
static uint64_t xxh3_avalanche(uint64_t h)
{
    h ^= h >> 37;
    h *= MX_1;
    return h ^ (h >> 32);
}

/* XXH64_avalanche, xxhash.h:3503-3511 (also used by XXH3 len 0..3) */
static uint64_t xxh64_avalanche(uint64_t h)
{
    h ^= h >> 33; h *= P64_2;
    h ^= h >> 29; h *= P64_3;
    return h ^ (h >> 32);
}

/* XXH3_rrmxmx, xxhash.h:4595-4603 */
static uint64_t rrmxmx(uint64_t h, uint64_t len)
{
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= MX_2;
    h ^= (h >> 35) + len;
    h *= MX_2;
    return h ^ (h >> 28);
}

/* ---- XXH3 short inputs (seed 0) ----------------------------------------- */

/* XXH3_len_0to16_64b and its three helpers, xxhash.h:4641-4704. */
static uint64_t xxh3_0to16(const uint8_t *in, size_t len)
{
    if (len > 8) {                                  /* len_9to16, :4679 */
        uint64_t lo = rd64(in) ^ (rd64(kSecret + 24) ^ rd64(kSecret + 32));
        uint64_t hi = rd64(in + len - 8) ^ (rd64(kSecret + 40) ^ rd64(kSecret + 48));
        uint64_t acc = (uint64_t)len + bswap64(lo) + hi + mul_fold(lo, hi);
        return xxh3_avalanche(acc);
    }
    if (len >= 4) {                                 /* len_4to8, :4663; seed 0 */
        uint64_t in1 = rd32(in);
        uint64_t in2 = rd32(in + len - 4);
        uint64_t flip = rd64(kSecret + 8) ^ rd64(kSecret + 16);
        uint64_t keyed = (in2 + (in1 << 32)) ^ flip;
        return rrmxmx(keyed, len);
    }
    if (len > 0) {                                  /* len_1to3, :4641 */
        uint32_t combined = ((uint32_t)in[0] << 16) | ((uint32_t)in[len >> 1] << 24) |
                            (uint32_t)in[len - 1] | ((uint32_t)len << 8);
        uint64_t flip = (uint64_t)(rd32(kSecret) ^ rd32(kSecret + 4));
        return xxh64_avalanche((uint64_t)combined ^ flip);
    }
    return xxh64_avalanche(rd64(kSecret + 56) ^ rd64(kSecret + 64));
}

/* XXH3_mix16B with seed 0, xxhash.h:4740-4763 */
static uint64_t mix16(const uint8_t *in, const uint8_t *sec)
{
    return mul_fold(rd64(in) ^ rd64(sec), rd64(in + 8) ^ rd64(sec + 8));
}

/* XXH3_len_17to128_64b, xxhash.h:4766-4799 (non-size-opt branch). Pairs of
 * 16-byte lanes taken from the front and the back of the input. */
static uint64_t xxh3_17to128(const uint8_t *in, size_t len)
{
    uint64_t acc = (uint64_t)len * P64_1;
    size_t rounds = (len - 1) / 32;  /* 0..3 extra pairs */
    for (size_t i = 0; i <= rounds; ++i) {
        acc += mix16(in + 16 * i, kSecret + 32 * i);
        acc += mix16(in + len - 16 * (i + 1), kSecret + 32 * i + 16);
    }
    return xxh3_avalanche(acc);
}

/* XXH3_len_129to240_64b, xxhash.h:4802-4856 */
static uint64_t xxh3_129to240(const uint8_t *in, size_t len)
{
    uint64_t acc = (uint64_t)len * P64_1;
    size_t rounds = len / 16;
    for (size_t i = 0; i < 8; ++i) acc += mix16(in + 16 * i, kSecret + 16 * i);
    acc = xxh3_avalanche(acc);
    /* MIDSIZE_LASTOFFSET 17, SECRET_SIZE_MIN 136 -> secret + 119 */
    uint64_t tail = mix16(in + len - 16, kSecret + 136 - 17);
    for (size_t i = 8; i < rounds; ++i)  /* MIDSIZE_STARTOFFSET 3 */
        tail += mix16(in + 16 * i, kSecret + 16 * (i - 8) + 3);
    return xxh3_avalanche(acc + tail);
}

/* ---- XXH3 long inputs (> 240 bytes) ------------------------------------- */

/* One 64-byte stripe into acc[8]: XXH3_scalarRound x8, xxhash.h:5778-5817. */
static void stripe(uint64_t acc[8], const uint8_t *in, const uint8_t *sec)
{
    for (int l = 0; l < 8; ++l) {
        uint64_t v = rd64(in + 8 * l);
        uint64_t k = v ^ rd64(sec + 8 * l);
        acc[l ^ 1] += v;
        acc[l] += (uint64_t)(uint32_t)k * (k >> 32);
    }
}

/* XXH3_scalarScrambleRound x8, xxhash.h:5827-5856, secret + 192 - 64. */
static void scramble(uint64_t acc[8])
{
    for (int l = 0; l < 8; ++l) {
        uint64_t a = acc[l];
        a ^= a >> 47;
        a ^= rd64(kSecret + 128 + 8 * l);
        acc[l] = a * P32_1;
    }
}

/* XXH3_hashLong_64b_internal + internal_loop + finalizeLong,
 * xxhash.h:5988-6017, 6029-6081.  Block = 16 stripes (1024 bytes). */
static uint64_t xxh3_long(const uint8_t *in, size_t len)
{
    /* XXH3_INIT_ACC, :6064-6065 */
    uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    const size_t blocks = (len - 1) / 1024;
    for (size_t b = 0; b < blocks; ++b) {
        for (int s = 0; s < 16; ++s) stripe(acc, in + 1024 * b + 64 * s, kSecret + 8 * s);
        scramble(acc);
    }
    const size_t tail_stripes = ((len - 1) - 1024 * blocks) / 64;
    for (size_t s = 0; s < tail_stripes; ++s)
        stripe(acc, in + 1024 * blocks + 64 * s, kSecret + 8 * s);
    /* last stripe, secret + 192 - 64 - 7 (XXH_SECRET_LASTACC_START) */
    stripe(acc, in + len - 64, kSecret + 121);
    /* XXH3_mergeAccs with secret + 11 (XXH_SECRET_MERGEACCS_START) */
    uint64_t r = (uint64_t)len * P64_1;
    for (int i = 0; i < 4; ++i)
        r += mul_fold(acc[2 * i] ^ rd64(kSecret + 11 + 16 * i),
                      acc[2 * i + 1] ^ rd64(kSecret + 19 + 16 * i));
    return xxh3_avalanche(r);
}

/* XXH3_64bits_internal dispatch, xxhash.h:6160-6181 */
uint64_t oracle_xxh3_64(const void *input, size_t len)
{
    const uint8_t *in = (const uint8_t *)input;
    if (len <= 16) return xxh3_0to16(in, len);
    if (len <= 128) return xxh3_17to128(in, len);
    if (len <= 240) return xxh3_129to240(in, len);
    return xxh3_long(in, len);
}

/* ---- XXH64 -------------------------------------------------------------- */

/* XXH64_round, xxhash.h:3469-3491 */
static uint64_t r64(uint64_t acc, uint64_t v)
{
    acc += v * P64_2;
    return rotl64(acc, 31) * P64_1;
}

/* XXH64_endian_align + consumeLong + mergeAccs + finalize, xxhash.h:3521-3673 */
uint64_t oracle_xxh64(const void *input, size_t len, uint64_t seed)
{
    const uint8_t *p = (const uint8_t *)input;
    const uint8_t *end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v[4] = {seed + P64_1 + P64_2, seed + P64_2, seed, seed - P64_1};
        size_t stripes = len / 32;
        for (size_t s = 0; s < stripes; ++s, p += 32)
            for (int i = 0; i < 4; ++i) v[i] = r64(v[i], rd64(p + 8 * i));
        h = rotl64(v[0], 1) + rotl64(v[1], 7) + rotl64(v[2], 12) + rotl64(v[3], 18);
        for (int i = 0; i < 4; ++i) {  /* XXH64_mergeRound, :3494-3500 */
            h ^= r64(0, v[i]);
            h = h * P64_1 + P64_4;
        }
    } else {
        h = seed + P64_5;
    }
    h += (uint64_t)len;
    size_t rem = (size_t)(end - p);
    for (; rem >= 8; rem -= 8, p += 8) {
        h ^= r64(0, rd64(p));
        h = rotl64(h, 27) * P64_1 + P64_4;
    }
    if (rem >= 4) {
        h ^= (uint64_t)rd32(p) * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
        rem -= 4; p += 4;
    }
    for (; rem > 0; --rem, ++p) {
        h ^= (uint64_t)(*p) * P64_5;
        h = rotl64(h, 11) * P64_1;
    }
    return xxh64_avalanche(h);
}

/* ---- page convention (src/storage/page.cpp:18-31, include/coding.h) ----- */

uint64_t oracle_page_xxh3(const void *page, size_t page_size)
{
    return oracle_xxh3_64((const uint8_t *)page + 8, page_size - 8);
}

uint64_t oracle_page_xxh64(const void *page, size_t page_size)
{
    return oracle_xxh64((const uint8_t *)page + 8, page_size - 8, 0);
}

void oracle_set_checksum(void *page, size_t page_size)
{
    uint64_t h = oracle_page_xxh3(page, page_size);
    memcpy(page, &h, 8); /* EncodeFixed64: LE, coding.h:64-77 */
}

int oracle_validate_checksum(const void *page, size_t page_size)
{
    uint64_t stored = rd64((const uint8_t *)page); /* DecodeFixed64, coding.h:126-139 */
    return stored == oracle_page_xxh3(page, page_size);
}

uint64_t oracle_manifest_checksum(const void *content, size_t len)
{
    const uint8_t *c = (const uint8_t *)content;
    uint64_t agg = 0;
    for (size_t off = 0; off < len; off += (size_t)1 << 20) {
        size_t n = len - off < ((size_t)1 << 20) ? len - off : ((size_t)1 << 20);
        agg = rotl64(agg, 1) ^ oracle_xxh3_64(c + off, n);
        agg *= 0x9e3779b97f4a7c15ull;
    }
    return agg;
}

void oracle_pages_digest(const void *pages, size_t page_size, size_t n_pages, int algo,
                         uint64_t *out)
{
    const uint8_t *p = (const uint8_t *)pages;
    for (size_t i = 0; i < n_pages; ++i, p += page_size)
        out[i] = algo ? oracle_page_xxh64(p, page_size) : oracle_page_xxh3(p, page_size);
}

void oracle_desc_digest(const void *base, const uint64_t *off, const uint32_t *len, size_t n,
                        int algo, uint64_t *out)
{
    const uint8_t *b = (const uint8_t *)base;
    for (size_t i = 0; i < n; ++i)
        out[i] = algo ? oracle_page_xxh64(b + off[i], len[i]) : oracle_page_xxh3(b + off[i], len[i]);
}

void oracle_desc_raw_xxh3(const void *base, const uint64_t *off, const uint32_t *len, size_t n,
                          uint64_t *out)
{
    const uint8_t *b = (const uint8_t *)base;
    for (size_t i = 0; i < n; ++i) out[i] = oracle_xxh3_64(b + off[i], len[i]);
}

/* ---- synthetic page generator ------------------------------------------ */

uint64_t oracle_splitmix_word(uint64_t seed, uint64_t page_index, uint64_t word_index)
{
    uint64_t z = (seed ^ page_index) + (word_index + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_fill_pages(void *pages, size_t page_size, size_t n_pages, uint64_t seed,
                       uint64_t first_page_index)
{
    uint8_t *p = (uint8_t *)pages;
    const size_t words = page_size / 8;
    for (size_t i = 0; i < n_pages; ++i, p += page_size)
        for (size_t w = 0; w < words; ++w) {
            uint64_t v = oracle_splitmix_word(seed, first_page_index + i, w);
            memcpy(p + 8 * w, &v, 8);
        }
}
