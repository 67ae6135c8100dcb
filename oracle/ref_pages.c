/*
 * ref_pages.c — TEST INFRASTRUCTURE ONLY.  Compiled together with the
 * reference's external/xxhash.c (in place, see oracle/Makefile) into
 * oracle/_ref/libxxhash_ref.so: a plain loop calling the reference's
 * XXH3_64bits / XXH64 once per page, exactly like SetChecksum /
 * ValidateChecksum do (src/storage/page.cpp:18-31).  Used as the timed
 * "reference" CPU baseline and as a checker; never shipped.
 */
#include <stddef.h>
#include <stdint.h>

uint64_t XXH3_64bits(const void *input, size_t length);
uint64_t XXH64(const void *input, size_t length, uint64_t seed);

void ref_pages_digest(const void *pages, size_t page_size, size_t n_pages, int algo, uint64_t *out)
{
    const uint8_t *p = (const uint8_t *)pages;
    for (size_t i = 0; i < n_pages; ++i, p += page_size)
        out[i] = algo ? XXH64(p + 8, page_size - 8, 0) : XXH3_64bits(p + 8, page_size - 8);
}

/* Mixed-size pages (config 3): page i is len[i] bytes at base + off[i]. */
void ref_desc_digest(const void *base, const uint64_t *off, const uint32_t *len, size_t n, int algo, uint64_t *out)
{
    const uint8_t *b = (const uint8_t *)base;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t *p = b + off[i];
        out[i] = algo ? XXH64(p + 8, len[i] - 8, 0) : XXH3_64bits(p + 8, len[i] - 8);
    }
}
