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

/* Config 1 (BASELINE.json configs[0]): the reference tool's per-page work over
 * a file, on the calling thread — read one page (tools/page_checksum_tool.cpp:
 * 94-96 seeks and reads page_size bytes; pread here), then ValidateChecksum
 * (src/storage/page.cpp:25-31: DecodeFixed64(page) == XXH3_64bits(page+8,
 * P-8)).  Pages [first_page, first_page + n_pages) of the file; *bad_out =
 * pages that failed.  Returns the bytes read, or -1 on an open/read error.
 * Each call opens its own descriptor, so threads can scan disjoint ranges. */
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

long long ref_scan_file(const char *path, size_t page_size, uint64_t first_page, uint64_t n_pages,
                        uint64_t *bad_out)
{
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return -1;
    unsigned char *buf = (unsigned char *)malloc(page_size);
    uint64_t bad = 0;
    long long total = 0;
    for (uint64_t i = 0; i < n_pages; ++i) {
        const off_t off = (off_t)((first_page + i) * page_size);
        if (pread(fd, buf, page_size, off) != (ssize_t)page_size) {
            total = -1;
            break;
        }
        uint64_t stored;
        memcpy(&stored, buf, 8); /* DecodeFixed64, little-endian host */
        bad += stored != XXH3_64bits(buf + 8, page_size - 8);
        total += (long long)page_size;
    }
    free(buf);
    close(fd);
    if (bad_out) *bad_out = bad;
    return total;
}
