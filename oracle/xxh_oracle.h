/*
 * xxh_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the arithmetic on EloqStore's page-checksum path, used
 * exclusively as the parity checker by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Nothing under eloqstore_amd/ links or calls
 * this code; the product path is the HIP kernels behind include/eloqstore_pcs.h.
 *
 * Parity pinning: this restatement is checked against
 *   (1) oracle/_ref/libxxhash_ref.so — the reference's own vendored
 *       external/xxhash.c (v0.8.3) compiled unmodified by oracle/Makefile, and
 *   (2) the committed golden vectors in tests/golden/ (generated from (1) and
 *       cross-checked against the system libxxhash 0.8.1 and python-xxhash
 *       3.8.1 / libxxhash 0.8.2 in the build container).
 *
 * Reference citations (paths relative to the reference tree):
 *   XXH3_64bits          external/xxhash.h:6185-6188
 *   XXH64                external/xxhash.h:3678-3693
 *   SetChecksum          src/storage/page.cpp:18-23
 *   ValidateChecksum     src/storage/page.cpp:25-31
 *   CalcChecksum (manifest) src/storage/root_meta.cpp:150-174
 */
#ifndef ELOQSTORE_XXH_ORACLE_H
#define ELOQSTORE_XXH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* XXH3_64bits(input, len) with seed 0 and the default 192-byte secret. */
uint64_t oracle_xxh3_64(const void *input, size_t len);

/* XXH64(input, len, seed). */
uint64_t oracle_xxh64(const void *input, size_t len, uint64_t seed);

/* Page convention: digest of bytes [8, page_size), stored LE in bytes [0, 8). */
uint64_t oracle_page_xxh3(const void *page, size_t page_size);
uint64_t oracle_page_xxh64(const void *page, size_t page_size);
void oracle_set_checksum(void *page, size_t page_size);           /* page.cpp:18-23 */
int oracle_validate_checksum(const void *page, size_t page_size); /* page.cpp:25-31 */

/* Manifest record aggregate (root_meta.cpp:150-174): XXH3 per <=1 MiB chunk,
 * agg = rotl(agg,1) ^ h; agg *= 0x9e3779b97f4a7c15.  Empty content -> 0. */
uint64_t oracle_manifest_checksum(const void *content, size_t len);

/* Batched helpers (pages contiguous, stride == page_size). algo 0 = XXH3, 1 = XXH64. */
void oracle_pages_digest(const void *pages, size_t page_size, size_t n_pages,
                         int algo, uint64_t *out);
/* Descriptor form: page i is [base + off[i], base + off[i] + len[i]). */
void oracle_desc_digest(const void *base, const uint64_t *off, const uint32_t *len,
                        size_t n, int algo, uint64_t *out);
/* Raw descriptor form: digest of the whole range (no 8-byte header skip). */
void oracle_desc_raw_xxh3(const void *base, const uint64_t *off, const uint32_t *len,
                          size_t n, uint64_t *out);

/* Synthetic page bytes shared with the device generator (pcs_fill_pages_dev):
 * word w of page p = splitmix64_mix((seed ^ p) + (w + 1) * 0x9E3779B97F4A7C15).
 * Writes n_pages * page_size bytes (page_size multiple of 8). */
void oracle_fill_pages(void *pages, size_t page_size, size_t n_pages,
                       uint64_t seed, uint64_t first_page_index);
uint64_t oracle_splitmix_word(uint64_t seed, uint64_t page_index, uint64_t word_index);

#ifdef __cplusplus
}
#endif
#endif
