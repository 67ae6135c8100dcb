// host_logic_test.cpp — the library's pure host logic under the sanitizers
// (the reference builds with WITH_ASAN, CMakeLists.txt:19-44).
// Built three ways by eloqstore_amd/Makefile `sanitize` (ASAN+UBSan and TSan,
// g++, no HIP) and run by tests/test_sanitizers.py:
//   - RegionRegistry (eloqstore_amd/csrc/region_registry.h), the zero-copy
//     page-pool registry pcs_host_register / pcs_host_alloc_pinned /
//     pcs_host_unregister and the host batches share: overlap rules, kinds,
//     page translation at region edges, runs past a region's end, ranges that
//     would wrap the address space;
//   - the same registry hammered by registering / unregistering threads while
//     others translate batches (the shard threads of INTEGRATION.md §2 read it
//     under a shared lock): every translation must be all-or-nothing and land
//     inside the region it names.
#include "region_registry.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

using pcs::RegionRegistry;

static int g_fail = 0;
#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                       \
        }                                                                   \
    } while (0)

static const void* A(uintptr_t a) { return reinterpret_cast<const void*>(a); }

static void test_add_remove() {
    RegionRegistry r;
    CHECK(r.add(0x10000, 0x1000, 0xA0000, false) == RegionRegistry::kOk);
    // overlaps: same base, inside, covering, straddling either end
    CHECK(r.add(0x10000, 0x10, 0, false) == RegionRegistry::kOverlap);
    CHECK(r.add(0x10800, 0x10, 0, false) == RegionRegistry::kOverlap);
    CHECK(r.add(0xF000, 0x3000, 0, false) == RegionRegistry::kOverlap);
    CHECK(r.add(0xF000, 0x1001, 0, false) == RegionRegistry::kOverlap);
    CHECK(r.add(0x10FFF, 0x10, 0, false) == RegionRegistry::kOverlap);
    CHECK(r.overlaps(0x10FFF, 1));
    CHECK(!r.overlaps(0x11000, 1));
    CHECK(!r.overlaps(0xF000, 0x1000));
    // adjacent on both sides is fine
    CHECK(r.add(0xF000, 0x1000, 0xB0000, true) == RegionRegistry::kOk);
    CHECK(r.add(0x11000, 0x1000, 0xC0000, false) == RegionRegistry::kOk);
    CHECK(r.size() == 3);
    // empty and wrapping ranges
    CHECK(r.add(0x20000, 0, 0, false) == RegionRegistry::kBadRange);
    CHECK(r.add(UINTPTR_MAX - 0xF, 0x20, 0, false) == RegionRegistry::kBadRange);
    CHECK(r.add(UINTPTR_MAX - 0xF, 0x10, 0xD0000, false) == RegionRegistry::kOk);  // ends exactly at the top
    CHECK(r.overlaps(UINTPTR_MAX, 1));
    // kinds: an allocation is freed, a registration unregistered, never crosswise
    CHECK(r.remove(0xF000, false) == RegionRegistry::kWrongKind);
    CHECK(r.remove(0x10000, true) == RegionRegistry::kWrongKind);
    CHECK(r.remove(0x10001, false) == RegionRegistry::kNotFound);
    CHECK(r.remove(0xF000, true) == RegionRegistry::kOk);
    CHECK(r.remove(0xF000, true) == RegionRegistry::kNotFound);
    CHECK(r.remove(0x10000, false) == RegionRegistry::kOk);
    CHECK(r.remove(0x11000, false) == RegionRegistry::kOk);
    CHECK(r.remove(UINTPTR_MAX - 0xF, false) == RegionRegistry::kOk);
    CHECK(r.size() == 0);
}

static void test_translate() {
    RegionRegistry r;
    uint64_t dev[8] = {};
    const void* one[1] = {A(0x10000)};
    CHECK(!r.translate(one, 1, 4096, dev));  // nothing registered
    CHECK(r.add(0x10000, 4 * 4096, 0x900000, false) == RegionRegistry::kOk);
    CHECK(r.add(0x14000, 2 * 4096, 0x700000, false) == RegionRegistry::kOk);  // adjacent second region
    // pages in both regions, out of order
    const void* pages[4] = {A(0x13000), A(0x10000), A(0x15000), A(0x14000)};
    CHECK(r.translate(pages, 4, 4096, dev));
    CHECK(dev[0] == 0x903000 && dev[1] == 0x900000 && dev[2] == 0x701000 && dev[3] == 0x700000);
    // a page straddling the boundary between two regions is not inside one
    const void* strad[1] = {A(0x13800)};
    CHECK(!r.translate(strad, 1, 4096, dev));
    // last page of the second region exactly fits; one byte more does not
    const void* last[1] = {A(0x15000)};
    CHECK(r.translate(last, 1, 4096, dev));
    CHECK(!r.translate(last, 1, 4097, dev));
    // unaligned page pointer, page before any region, page size 0
    const void* unal[1] = {A(0x10008)};
    CHECK(!r.translate(unal, 1, 64, dev));
    const void* before[1] = {A(0x0F000)};
    CHECK(!r.translate(before, 1, 4096, dev));
    CHECK(!r.translate(one, 1, 0, dev));
    // a pointer whose page would wrap the address space
    const void* top[1] = {A(UINTPTR_MAX - 0xF)};
    CHECK(!r.translate(top, 1, 4096, dev));
    // run(): contiguous byte runs
    CHECK(r.run(0x10000, 0x13FFF) == RegionRegistry::kInside);
    CHECK(r.run(0x10000, 0x14000) == RegionRegistry::kPastEnd);  // spills into the adjacent region
    CHECK(r.run(0x0F000, 0x10FFF) == RegionRegistry::kNotRegistered);
    CHECK(r.run(0x16000, 0x16FFF) == RegionRegistry::kNotRegistered);
    CHECK(r.run(0x15FFF, 0x15FFF) == RegionRegistry::kInside);
}

// Writers register / unregister their own slot regions; readers translate
// batches that touch every slot.  A translation either fails or returns, for
// every page, the device address of the region it lies in.  Every fourth slot
// (an "anchor") stays registered throughout, so readers are guaranteed some
// successful translations however the threads are scheduled (a sanitizer
// build under load once saw the churned slots only while unregistered).
static void test_concurrent() {
    RegionRegistry r;
    constexpr int kSlots = 16, kPages = 64, kIters = 4000;
    constexpr uintptr_t kBase = 0x100000000ull, kSlotBytes = kPages * 4096ull;
    auto dev_of = [](int slot) { return (uintptr_t)0x7000000000ull + (uintptr_t)slot * 0x10000000ull; };
    std::atomic<bool> stop{false};
    std::atomic<uint64_t> ok{0}, miss{0}, bad{0};
    std::vector<std::thread> th;
    for (int s = 0; s < kSlots; s += 4) CHECK(r.add(kBase + s * kSlotBytes, kSlotBytes, dev_of(s), false) == RegionRegistry::kOk);
    for (int w = 0; w < 4; ++w)
        th.emplace_back([&, w] {
            for (int it = 0; it < kIters; ++it) {
                const int slot = (w * 4 + it) % kSlots;
                const uintptr_t b = kBase + slot * kSlotBytes;
                // a slot belongs to writer (slot / 4) only; register, then drop it
                if (slot / 4 != w || slot % 4 == 0) continue;  // anchors stay
                if (r.add(b, kSlotBytes, dev_of(slot), (it & 1) != 0) == RegionRegistry::kOk) {
                    for (int y = 0; y < 8; ++y) std::this_thread::yield();  // let readers see it
                    (void)r.remove(b, (it & 1) != 0);
                }
            }
        });
    for (int t = 0; t < 4; ++t)
        th.emplace_back([&, t] {
            std::vector<const void*> pages(16);
            std::vector<uint64_t> dev(pages.size());
            uint64_t x = 0x9E3779B97F4A7C15ull * (t + 1);
            // at least 2000 batches per reader even if the writers finish
            // before this thread is scheduled (a loaded sanitizer run)
            for (int iter = 0; iter < 2000 || !stop.load(std::memory_order_relaxed); ++iter) {
                // a batch from one pool chunk (the common case) or, every 4th, from two
                x ^= x << 13, x ^= x >> 7, x ^= x << 17;
                const int s0 = (int)(x % kSlots), s1 = (x & 3) ? s0 : (int)((x >> 20) % kSlots);
                for (size_t i = 0; i < pages.size(); ++i) {
                    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
                    const int slot = (i & 1) ? s1 : s0, pg = (int)((x >> 8) % kPages);
                    pages[i] = A(kBase + slot * kSlotBytes + pg * 4096ull);
                }
                if (r.translate(pages.data(), pages.size(), 4096, dev.data())) {
                    ++ok;
                    for (size_t i = 0; i < pages.size(); ++i) {
                        const uintptr_t a = reinterpret_cast<uintptr_t>(pages[i]);
                        const int slot = (int)((a - kBase) / kSlotBytes);
                        if (dev[i] != dev_of(slot) + (a - kBase - slot * kSlotBytes)) ++bad;
                    }
                } else {
                    ++miss;
                }
                (void)r.run(reinterpret_cast<uintptr_t>(pages[0]), reinterpret_cast<uintptr_t>(pages[0]) + 4095);
            }
        });
    for (int w = 0; w < 4; ++w) th[w].join();
    stop = true;
    for (size_t i = 4; i < th.size(); ++i) th[i].join();
    CHECK(bad.load() == 0);
    CHECK(ok.load() > 0);  // batches within an anchor slot always translate
    for (int s = 0; s < kSlots; s += 4) CHECK(r.remove(kBase + s * kSlotBytes, false) == RegionRegistry::kOk);
    CHECK(r.size() == 0);
    // with every slot registered, every batch must translate
    for (int s = 0; s < kSlots; ++s) CHECK(r.add(kBase + s * kSlotBytes, kSlotBytes, dev_of(s), false) == RegionRegistry::kOk);
    const void* p[2] = {A(kBase), A(kBase + kSlots * kSlotBytes - 4096)};
    uint64_t d[2];
    CHECK(r.translate(p, 2, 4096, d));
    CHECK(d[1] == dev_of(kSlots - 1) + kSlotBytes - 4096);
    std::printf("concurrent: %llu translated, %llu refused, %llu wrong\n", (unsigned long long)ok.load(),
                (unsigned long long)miss.load(), (unsigned long long)bad.load());
}

// Round 6 replaced the registry's std::map with a sorted array and a
// branchless binary search: random non-overlapping regions (sub-page to
// multi-MiB, some adjacent), random adds and removes, and random page
// queries (inside, straddling an end, in gaps, before the first and after the
// last region) must agree with a brute-force scan on every translate and run.
static void test_random_against_brute_force() {
    uint64_t s = 0x5EED;
    auto rnd = [&s] {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    struct R {
        uintptr_t base;
        uint64_t bytes;
        uintptr_t dev;
    };
    for (int round = 0; round < 40; ++round) {
        RegionRegistry r;
        std::vector<R> live;
        uintptr_t at = 0x100000 + (rnd() % 64) * 16;
        for (int i = 0; i < 300; ++i) {
            const uint64_t bytes = 16 * (1 + rnd() % (rnd() % 4 ? 64 : 65536));
            if (rnd() % 3) at += 16 * (rnd() % 4096);  // a gap, or adjacent
            const uintptr_t dev = 0x7000000000ull + rnd() % (1ull << 32) * 16;
            CHECK(r.add(at, bytes, dev, false) == RegionRegistry::kOk);
            live.push_back({at, bytes, dev});
            at += bytes;
        }
        for (int i = 0; i < 60; ++i) {  // remove some
            const size_t k = rnd() % live.size();
            CHECK(r.remove(live[k].base, false) == RegionRegistry::kOk);
            live.erase(live.begin() + k);
        }
        CHECK(r.size() == live.size());
        const uintptr_t lo = live.front().base - 4096, hi = at + 4096;
        for (int q = 0; q < 3000; ++q) {
            const uintptr_t a = (lo + rnd() % (hi - lo)) & ~uintptr_t(15);
            const uint64_t P = 16 * (1 + rnd() % 16);
            const R* hit = nullptr;
            for (const R& x : live)
                if (a >= x.base && a - x.base < x.bytes) hit = &x;
            const bool want = hit && P <= hit->bytes - (a - hit->base);
            const void* page[1] = {reinterpret_cast<const void*>(a)};
            uint64_t dev = 0;
            CHECK(r.translate(page, 1, P, &dev) == want);
            if (want) CHECK(dev == hit->dev + (a - hit->base));
            const RegionRegistry::Run run = r.run(a, a + P - 1);
            CHECK(run == (!hit ? RegionRegistry::kNotRegistered : want ? RegionRegistry::kInside : RegionRegistry::kPastEnd));
        }
        // a batch across many regions, then one page outside fails the batch
        std::vector<const void*> batch;
        std::vector<uint64_t> want;
        for (int i = 0; i < 128; ++i) {
            const R& x = live[rnd() % live.size()];
            const uintptr_t a = x.base + 16 * (rnd() % (x.bytes / 16));
            batch.push_back(reinterpret_cast<const void*>(a));
            want.push_back(x.dev + (a - x.base));
        }
        std::vector<uint64_t> got(batch.size());
        CHECK(r.translate(batch.data(), batch.size(), 16, got.data()) && got == want);
        batch[77] = reinterpret_cast<const void*>(hi + 4096);
        CHECK(!r.translate(batch.data(), batch.size(), 16, got.data()));
    }
}

int main() {
    test_add_remove();
    test_translate();
    test_concurrent();
    test_random_against_brute_force();
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("host_logic_test: all checks passed\n");
    return 0;
}
