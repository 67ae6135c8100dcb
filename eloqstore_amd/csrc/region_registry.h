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
#include <iterator>
#include <map>
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
        regions_.emplace(base, Region{bytes, dev, allocated});
        return kOk;
    }

    // Removes the region that starts exactly at base, if it is of the given kind.
    Status remove(uintptr_t base, bool allocated) {
        std::unique_lock lk(mu_);
        auto it = regions_.find(base);
        if (it == regions_.end()) return kNotFound;
        if (it->second.allocated != allocated) return kWrongKind;
        regions_.erase(it);
        return kOk;
    }

    // Device-visible addresses of pages[0..n) when every page [p, p + P) lies
    // inside one registered region and is 16-byte aligned; false otherwise.
    bool translate(const void* const* pages, uint64_t n, uint64_t P, uint64_t* dev_out) const {
        std::shared_lock lk(mu_);
        if (regions_.empty() || P == 0) return false;
        auto hint = regions_.end();
        for (uint64_t i = 0; i < n; ++i) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(pages[i]);
            if (a % 16 || P - 1 > UINTPTR_MAX - a) return false;
            if (hint == regions_.end() || !inside(*hint, a, P)) {
                auto it = regions_.upper_bound(a);
                if (it == regions_.begin()) return false;
                hint = std::prev(it);
                if (!inside(*hint, a, P)) return false;
            }
            dev_out[i] = hint->second.dev + (a - hint->first);
        }
        return true;
    }

    // Where does the contiguous byte run [first, last] sit?  kInside: within
    // one region; kPastEnd: it starts in a region and runs past its end;
    // kNotRegistered: it does not start in any region.
    Run run(uintptr_t first, uintptr_t last) const {
        std::shared_lock lk(mu_);
        auto it = regions_.upper_bound(first);
        if (it == regions_.begin()) return kNotRegistered;
        const auto& [rb, r] = *std::prev(it);
        if (first - rb >= r.bytes) return kNotRegistered;
        return (last >= first && last - rb < r.bytes) ? kInside : kPastEnd;
    }

    size_t size() const {
        std::shared_lock lk(mu_);
        return regions_.size();
    }

private:
    using Map = std::map<uintptr_t, Region>;

    // a >= region base is guaranteed by the upper_bound lookups
    static bool inside(const Map::value_type& r, uintptr_t a, uint64_t P) {
        return a >= r.first && a - r.first < r.second.bytes && P <= r.second.bytes - (a - r.first);
    }

    bool overlaps_locked(uintptr_t base, uint64_t bytes) const {
        auto it = regions_.upper_bound(base);
        if (it != regions_.end() && it->first - base < bytes) return true;  // a later region starts inside
        if (it != regions_.begin()) {
            const auto& [pb, pr] = *std::prev(it);
            if (base - pb < pr.bytes) return true;  // base falls inside the previous region
        }
        return false;
    }

    mutable std::shared_mutex mu_;
    Map regions_;  // keyed by host base address
};

}  // namespace pcs
