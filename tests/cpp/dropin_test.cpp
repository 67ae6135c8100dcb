// dropin_test.cpp — exercises the C++ drop-in surface the way EloqStore's call
// sites would (test infrastructure; links the CPU oracle as the checker).
//   * SetChecksum / ValidateChecksum on single pages  (page.cpp:18-31)
//   * ValidateChecksums over a scattered <=128-page read batch
//     (IouringMgr::ReadPages, async_io_manager.cpp:353-366)
//   * SetChecksums over a 256-page write batch (FlushBatchPages, write_task.cpp:155-167)
//   * ChecksumBatch submit + poll loop (shard work loop, shard.cpp:67-130)
//   * ManifestChecksum / ValidateManifestRecord (root_meta.cpp:138-174)
// Prints "dropin ok" and exits 0 on success.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "eloqstore/page_checksum.h"
#include "xxh_oracle.h"

#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::fprintf(stderr, "%s:%d CHECK(%s)\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                               \
        }                                                               \
    } while (0)

int main() {
    using namespace eloqstore;
    const size_t P = 4096;
    // a scattered "page pool": separate allocations, like PagesPool chunks
    std::vector<std::unique_ptr<char[]>> pool;
    std::vector<char*> pages;
    for (int i = 0; i < 300; ++i) {
        pool.emplace_back(new char[P]);
        oracle_fill_pages(pool.back().get(), P, 1, 0xD80F1, i);
        pages.push_back(pool.back().get());
    }
    // single page
    SetChecksum({pages[0], P});
    CHECK(ValidateChecksum({pages[0], P}));
    CHECK(oracle_validate_checksum(pages[0], P));
    pages[0][10] ^= 0x5A;
    CHECK(!ValidateChecksum({pages[0], P}));
    pages[0][10] ^= 0x5A;

    // write batch of 256 pages, then a read batch of 128 with one corrupted page
    SetChecksums(std::span<char* const>(pages.data(), 256), P);
    for (int i = 0; i < 256; ++i) CHECK(oracle_validate_checksum(pages[i], P));
    std::vector<const char*> rd(pages.begin() + 100, pages.begin() + 228);
    std::vector<uint8_t> ok(rd.size());
    CHECK(ValidateChecksums(rd, P, ok.data()) == rd.size());
    pages[150][P - 1] ^= 1;
    CHECK(ValidateChecksums(rd, P, ok.data()) == 50);
    CHECK(ok[50] == 0 && ok[49] == 1 && ok[51] == 1);
    CHECK(ValidateChecksums(rd, P, ok.data(), PageHash::XXH3_64, /*skip_verify=*/true) == rd.size());
    pages[150][P - 1] ^= 1;

    // async batches: two in flight, polled like the shard loop
    ChecksumBatch a, b;
    a.SubmitValidate(rd, P);
    std::vector<char*> wr(pages.begin() + 256, pages.end());
    b.SubmitStamp(wr, P);
    int spins = 0;
    bool da = false, db = false;
    while (!(da && db)) {
        da = da || a.Poll();
        db = db || b.Poll();
        ++spins;
    }
    CHECK(a.FirstBad() == rd.size());
    for (char* p : wr) CHECK(oracle_validate_checksum(p, P));

    // manifest record: checksum(8)|root(4)|ttl_root(4)|len(4)|payload
    for (size_t len : {0ul, 12ul, 300ul, 5000ul, (1ul << 20) + 77}) {
        std::vector<char> rec(20 + len);
        oracle_fill_pages(rec.data(), 8, rec.size() / 8, 77, len);
        const uint64_t h = ManifestChecksum({rec.data() + 8, rec.size() - 8});
        CHECK(h == oracle_manifest_checksum(rec.data() + 8, rec.size() - 8));
        std::memcpy(rec.data(), &h, 8);
        CHECK(ValidateManifestRecord({rec.data(), rec.size()}));
        rec[rec.size() / 2] ^= 0x10;
        CHECK(!ValidateManifestRecord({rec.data(), rec.size()}));
    }
    CHECK(!ValidateManifestRecord({pages[1], 19}));
    std::printf("dropin ok (%d polls)\n", spins);
    return 0;
}
