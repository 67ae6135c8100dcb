// region_registry.h — registered host page pools (zero-copy path), pure host
// logic with no HIP dependency so that it is unit-tested under ASAN/UBSan and
// TSan on the CPU (tests/cpp/host_logic_test.cpp).
//
// A region is a page-locked, device-mapped host range: either one this library
// allocated (pcs_host_alloc_pinned) or one the caller registered
// (pcs_host_register / eloqstore::RegisterPagePool, the PagesPool chunks of
// src/storage/page.cpp:95-120).  The registry maps a host page pointer to the
// device-visible address the zero-copy kernels read through.
#pragma once

#include <cstdint>
#include <cstddef>
#include <vector>
#include <mutex>
#include <shared_mutex>

namespace pcs {

class RegionRegistry {
public:
    struct Region {
        uint64_t bytes;
        uintptr_t dev;   // device-visible address of the region base
        bool allocated;  // pcs_host_alloc_pinned (freed there, not unregistered)
    };
    enum Status : int { kOk = 0, kOverlap = 1, kBadRange = 2, kNotFound = 3, kWrongKind = 4 };
    enum Run : int { kNotRegistered = -1, kPastEnd = 0, kInside = 1 };

    // [base, base + bytes) must be non-empty and must not wrap the address space.
    static bool valid_range(uintptr_t base, uint64_t bytes) { return bytes != 0 && bytes - 1 <= UINTPTR_MAX - base; }

    // Would [base, base + bytes) overlap a registered region?  (Checked before
    // the caller pins anything; add() re-checks under the exclusive lock.)
    bool overlaps(uintptr_t base, uint64_t bytes) const {
        std::shared_lock lk(mu_);
        return overlaps_locked(base, bytes);
    }

    Status add(uintptr_t base, uint64_t bytes, uintptr_t dev, bool allocated) {
        if (!valid_range(base, bytes)) return kBadRange;
        std::unique_lock lk(mu_);
        if (overlaps_locked(base, bytes)) return kOverlap;
        const size_t k = count_le(base);  // insertion point: bases stay sorted
        bases_.insert(bases_.begin() + k, base);
        regions_.insert(regions_.begin() + k, Region{bytes, dev, allocated});
        return kOk;
    }

    // Removes the region that starts exactly at base, if it is of the given kind.
    Status remove(uintptr_t base, bool allocated) {
        std::unique_lock lk(mu_);
        const size_t k = count_le(base);
        if (k == 0 || bases_[k - 1] != base) return kNotFound;
        if (regions_[k - 1].allocated != allocated) return kWrongKind;
        bases_.erase(bases_.begin() + (k - 1));
        regions_.erase(regions_.begin() + (k - 1));
        return kOk;
    }

    // Device-visible addresses of pages[0..n) when every page [p, p + P) lies
    // inside one registered region and is 16-byte aligned; false otherwise.
    // One shared lock per batch; per page, the previous page's region first,
    // then a branchless binary search over the sorted bases (round 6: the
    // std::map walk this replaces cost ~76 ns per page, ~9.7 us of a 128-page
    // batch's host time, on random pages of 256 pool chunks).
    bool translate(const void* const* pages, uint64_t n, uint64_t P, uint64_t* dev_out) const {
        std::shared_lock lk(mu_);
        if (bases_.empty() || P == 0) return false;
        size_t hint = SIZE_MAX;
        for (uint64_t i = 0; i < n; ++i) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(pages[i]);
            if (a % 16 || P - 1 > UINTPTR_MAX - a) return false;
            if (hint == SIZE_MAX || !inside(hint, a, P)) {
                const size_t k = count_le(a);
                if (k == 0) return false;
                hint = k - 1;
                if (!inside(hint, a, P)) return false;
            }
            dev_out[i] = regions_[hint].dev + (a - bases_[hint]);
        }
        return true;
    }

    // Where does the contiguous byte run [first, last] sit?  kInside: within
    // one region; kPastEnd: it starts in a region and runs past its end;
    // kNotRegistered: it does not start in any region.
    Run run(uintptr_t first, uintptr_t last) const {
        std::shared_lock lk(mu_);
        const size_t k = count_le(first);
        if (k == 0) return kNotRegistered;
        const uintptr_t rb = bases_[k - 1];
        const Region& r = regions_[k - 1];
        if (first - rb >= r.bytes) return kNotRegistered;
        return (last >= first && last - rb < r.bytes) ? kInside : kPastEnd;
    }

    size_t size() const {
        std::shared_lock lk(mu_);
        return bases_.size();
    }

private:
    // Number of region bases <= a (the index after the region that may hold
    // a): a branchless binary search, ~log2(regions) dependent loads from a
    // contiguous array with no mispredicted branches.
    size_t count_le(uintptr_t a) const {
        const uintptr_t* b = bases_.data();
        size_t n = bases_.size(), lo = 0;
        while (n > 1) {
            const size_t half = n / 2;
            lo = (b[lo + half - 1] <= a) ? lo + half : lo;
            n -= half;
        }
        return n == 1 && lo < bases_.size() && b[lo] <= a ? lo + 1 : lo;
    }

    // a >= the region's base is guaranteed by count_le
    bool inside(size_t k, uintptr_t a, uint64_t P) const {
        const uintptr_t rb = bases_[k];
        return a >= rb && a - rb < regions_[k].bytes && P <= regions_[k].bytes - (a - rb);
    }

    bool overlaps_locked(uintptr_t base, uint64_t bytes) const {
        const size_t k = count_le(base);  // regions [0, k) start at or before base
        if (k < bases_.size() && bases_[k] - base < bytes) return true;  // a later region starts inside
        if (k > 0 && base - bases_[k - 1] < regions_[k - 1].bytes) return true;  // base falls inside the previous one
        return false;
    }

    mutable std::shared_mutex mu_;
    std::vector<uintptr_t> bases_;  // sorted host base addresses
    std::vector<Region> regions_;   // regions_[k] starts at bases_[k]
};

}  // namespace pcs
