// pcs_capi.cpp — extern "C" boundary of libeloqstore_pcs.so (include/eloqstore_pcs.h).
//
// Argument checking, error reporting and the host-memory batch pipeline
// (gather scattered pool pages into pinned staging -> H2D -> kernel -> D2H of
// 8-byte digests / 1-byte verdicts), double-buffered over two HIP streams.
// All compute is on the GPU; there is no CPU hashing in this library.
#include "eloqstore_pcs.h"
#include "eloqstore_pcs_internal.h"
#include "region_registry.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

thread_local std::string t_last_error;

int fail(int code, const std::string& msg) {
    t_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(PCS_ERR_HIP, std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")");
}

// A compute entry point must see a usable device; otherwise fail loudly
// (there is no CPU fallback by design).
int require_device() {
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        return fail(PCS_ERR_NO_DEVICE, std::string("no usable HIP device: ") +
                                           (e != hipSuccess ? hipGetErrorString(e) : "device count is 0"));
    return PCS_OK;
}

bool valid_algo(int algo) { return algo == PCS_XXH3_64 || algo == PCS_XXH64; }

// PCS_TUNE_FAIL_INJECT (test only): the next k host-batch calls fail as a
// HIP error would, so call sites can prove their fallback.
bool injected_failure() { return pcs::take_tuning(PCS_TUNE_FAIL_INJECT); }

int finish(hipError_t e, const char* what) { return e == hipSuccess ? PCS_OK : hip_fail(e, what); }

// Fixed-stride pages: fast kernels when the shape allows, else descriptor
// path over a device-side descriptor array built on the fly.
int pages_common(int mode, const void* d_pages, uint64_t P, uint64_t n, int algo, uint64_t* d_out, uint8_t* d_ok,
                 uint64_t* d_first_bad, pcs_stream_t stream) {
    if (int rc = require_device()) return rc;
    if (!valid_algo(algo)) return fail(PCS_ERR_INVALID, "algo must be PCS_XXH3_64 or PCS_XXH64");
    if (P < 8) return fail(PCS_ERR_INVALID, "page_size must be >= 8 (8-byte digest header)");
    if (P > 0xFFFFFFFFull) return fail(PCS_ERR_INVALID, "page_size must fit in 32 bits");
    if (n && !d_pages) return fail(PCS_ERR_INVALID, "d_pages is null");
    if (mode == 0 && n && !d_out) return fail(PCS_ERR_INVALID, "d_digests is null");
    if (mode == 1 && n && !d_ok) return fail(PCS_ERR_INVALID, "d_ok is null");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (d_first_bad) {
        hipError_t e = hipMemsetAsync(d_first_bad, 0xFF, sizeof(uint64_t), s);
        if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(first_bad)");
    }
    if (n == 0) return PCS_OK;
    auto* fb = reinterpret_cast<unsigned long long*>(d_first_bad);
    return finish(pcs::run_pages(mode, algo, static_cast<const uint8_t*>(d_pages), P, n, d_out, d_ok, fb, s),
                  "page kernel launch");
}

int desc_common(int mode, const void* d_base, const uint64_t* d_off, const uint32_t* d_len, uint64_t n, int algo,
                int skip, uint64_t seed, uint64_t* d_out, uint8_t* d_ok, uint64_t* d_first_bad, pcs_stream_t stream) {
    if (int rc = require_device()) return rc;
    if (!valid_algo(algo)) return fail(PCS_ERR_INVALID, "algo must be PCS_XXH3_64 or PCS_XXH64");
    if (n && (!d_base || !d_off || !d_len)) return fail(PCS_ERR_INVALID, "null descriptor pointer");
    if (mode == 0 && n && !d_out) return fail(PCS_ERR_INVALID, "d_digests is null");
    if (mode == 1 && n && !d_ok) return fail(PCS_ERR_INVALID, "d_ok is null");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (d_first_bad) {
        hipError_t e = hipMemsetAsync(d_first_bad, 0xFF, sizeof(uint64_t), s);
        if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(first_bad)");
    }
    if (n == 0) return PCS_OK;
    return finish(pcs::run_desc(mode, algo, static_cast<const uint8_t*>(d_base), d_off, d_len, n, skip, seed, d_out,
                                d_ok, reinterpret_cast<unsigned long long*>(d_first_bad), s),
                  "descriptor kernel launch");
}

// ---------------------------------------------------------------------------
// registered host regions (zero-copy page pools)
// ---------------------------------------------------------------------------
pcs::RegionRegistry g_regions;

int add_region(void* p, uint64_t bytes, bool allocated) {
    void* dev = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&dev, p, 0);
    if (e != hipSuccess) return hip_fail(e, "hipHostGetDevicePointer");
    switch (g_regions.add(reinterpret_cast<uintptr_t>(p), bytes, reinterpret_cast<uintptr_t>(dev), allocated)) {
        case pcs::RegionRegistry::kOk: return PCS_OK;
        case pcs::RegionRegistry::kOverlap: return fail(PCS_ERR_INVALID, "region overlaps a registered one");
        default: return fail(PCS_ERR_INVALID, "region wraps the address space");
    }
}

// Device-visible addresses of pages[0..n) when every page [p, p + P) lies in a
// registered region and is 16-byte aligned; false otherwise.
bool translate_registered(const void* const* pages, uint64_t n, uint64_t P, uint64_t* dev_out) {
    return g_regions.translate(pages, n, P, dev_out);
}

template <typename T>
T* dev_alias(T* host_pinned) {
    void* d = nullptr;
    return hipHostGetDevicePointer(&d, host_pinned, 0) == hipSuccess ? static_cast<T*>(d) : nullptr;
}

// Pinned, device-mapped result buffers of one zero-copy launch.
struct ZcBufs {
    uint64_t* h_ptrs = nullptr;
    uint64_t* h_dig = nullptr;
    uint8_t* h_ok = nullptr;
    uint64_t* d_ptrs = nullptr;  // device aliases of the above
    uint64_t* d_dig = nullptr;
    uint8_t* d_ok = nullptr;
    size_t cap = 0;
    void release() {
        (void)hipHostFree(h_ptrs);
        (void)hipHostFree(h_dig);
        (void)hipHostFree(h_ok);
        *this = ZcBufs{};
    }
    // At least a service-sized batch (256 pages): a batch the service gives
    // back re-runs here from a poll, and growing would free pinned memory,
    // which synchronises the device (the poll would wait for every kernel).
    int ensure(size_t n) {
        if (n <= cap) return PCS_OK;
        n = std::max<size_t>(n, pcs::kServiceMaxPages);
        release();
        if (hipHostMalloc(reinterpret_cast<void**>(&h_ptrs), n * 8, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&h_dig), n * 8, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&h_ok), n, hipHostMallocDefault) != hipSuccess) {
            release();
            return fail(PCS_ERR_NOMEM, "zero-copy buffer allocation failed");
        }
        d_ptrs = dev_alias(h_ptrs);
        d_dig = dev_alias(h_dig);
        d_ok = dev_alias(h_ok);
        if (!d_ptrs || !d_dig || !d_ok) {
            release();
            return fail(PCS_ERR_HIP, "hipHostGetDevicePointer failed for zero-copy buffers");
        }
        cap = n;
        return PCS_OK;
    }
};

std::atomic<uint64_t> g_counters[4];
void count(int which) { g_counters[which].fetch_add(1, std::memory_order_relaxed); }

int64_t zero_copy_policy() { return pcs::get_tuning(PCS_TUNE_ZERO_COPY); }

// Validate batches from host memory: the verdicts (0 or 1) land in pinned
// host memory, written by the kernel itself (zero-copy) or by the D2H copy
// behind it (staged), and every page read of the batch precedes the verdict
// it produces.  So once no byte of the verdict array holds the sentinel the
// host wrote before the batch, its results are complete, and the host can
// stop waiting without the stream's completion signal (PCS_TUNE_ZC_POLL = 1;
// 5-6 us less per call).  The stream still orders the next
// batch behind this one.  Zero-copy XXH3 stamps of up to PCS_TUNE_ZC_STAMP_POLL_PAGES
// wait the same way on a done byte per page, which the list kernel stores
// after a system-scope release that follows the page's header.
constexpr uint8_t kVerdictPending = 0xA5;
bool zc_poll() { return pcs::get_tuning(PCS_TUNE_ZC_POLL) != 0; }
void arm_verdicts(uint8_t* h_ok, uint64_t n) { std::memset(h_ok, kVerdictPending, n); }
// First index from `from` whose verdict has not landed yet (n when all have).
uint64_t verdicts_landed(const uint8_t* h_ok, uint64_t from, uint64_t n) {
    const volatile uint8_t* v = h_ok;
    while (from < n && v[from] != kVerdictPending) ++from;
    return from;
}
// A synchronous caller's wait between checks: spin (pause) for the first
// PCS_TUNE_SYNC_SPIN_US microseconds of the call, then sleep ~10 µs per
// check (0, the default: spin throughout).  A spinning caller costs its core
// for the whole wait; once several shard threads share the GPU's PCIe link
// the sync calls cost as much CPU as the loop they replace,
// and sleeping gives that time to other threads at some latency.
class SyncWaiter {
public:
    SyncWaiter() : spin_us_(pcs::get_tuning(PCS_TUNE_SYNC_SPIN_US)) {
        if (spin_us_ > 0) t0_ = std::chrono::steady_clock::now();
    }
    // one wait between two checks; true once the caller sleeps
    bool pause() {
        if (spin_us_ <= 0 || (!sleeping_ && (++n_ & 63) != 0)) {
            __builtin_ia32_pause();  // spin politely: the sibling hyperthread may be a shard thread
            return false;
        }
        if (!sleeping_ && std::chrono::steady_clock::now() - t0_ < std::chrono::microseconds(spin_us_)) {
            __builtin_ia32_pause();
            return false;
        }
        sleeping_ = true;
        std::this_thread::sleep_for(std::chrono::microseconds(10));
        return true;
    }

private:
    int64_t spin_us_;
    std::chrono::steady_clock::time_point t0_{};
    uint32_t n_ = 0;
    bool sleeping_ = false;
};

// Wait until every verdict has landed; the stream is queried every 4096
// spins (every 16 sleeps) so a failed or finished launch that wrote no
// verdict cannot hang the caller (then the stream's own status decides).
hipError_t wait_verdicts(const uint8_t* h_ok, uint64_t n, hipStream_t s) {
    uint64_t at = 0;
    SyncWaiter w;
    for (uint32_t spin = 0, naps = 0;; ++spin) {
        at = verdicts_landed(h_ok, at, n);
        if (at == n) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return hipSuccess;
        }
        const bool slept = w.pause();
        if ((spin & 4095) == 4095 || (slept && (++naps & 15) == 0)) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) {  // finished: every verdict must be there now
                at = verdicts_landed(h_ok, at, n);
                return at == n ? hipSuccess : hipErrorUnknown;
            }
            if (q != hipErrorNotReady) return q;
        }
    }
}

// Zero-copy eligibility for a host batch: fast shape, policy, and every page
// registered (fills zc.h_ptrs with device-visible page addresses).
bool zero_copy_eligible(ZcBufs& zc, const void* const* pages, uint64_t n, uint64_t P, int algo) {
    const int64_t pol = zero_copy_policy();
    if (pol == 0 || n == 0 || !pcs::list_shape_ok(algo, P)) return false;
    if (zc.ensure(n) != PCS_OK) {
        (void)hipGetLastError();
        return false;  // staging path still works
    }
    return translate_registered(pages, n, P, zc.h_ptrs);
}

// ---------------------------------------------------------------------------
// host-memory pipeline
// ---------------------------------------------------------------------------
constexpr size_t kStageBytes = 32u << 20;  // per slot

struct Slot {
    hipStream_t stream = nullptr;
    uint8_t* h_pages = nullptr;  // pinned
    uint8_t* d_pages = nullptr;
    uint64_t* h_dig = nullptr;   // pinned
    uint64_t* d_dig = nullptr;
    uint8_t* h_ok = nullptr;     // pinned
    uint8_t* d_ok = nullptr;
    size_t cap_pages_bytes = 0, cap_dev_bytes = 0, cap_n = 0;
    uint64_t first = 0, count = 0;  // chunk currently in flight
    bool busy = false;
};

constexpr int kSlots = 3;  // H2D of chunk k+1 || kernel k || D2H k-1

struct HostCtx {
    Slot slot[kSlots];
    ZcBufs zc;
    ~HostCtx() {
        if (slot[0].stream) (void)hipStreamSynchronize(slot[0].stream);
        zc.release();
        for (auto& s : slot) {
            if (s.stream) (void)hipStreamSynchronize(s.stream);
            (void)hipHostFree(s.h_pages);
            (void)hipFree(s.d_pages);
            (void)hipHostFree(s.h_dig);
            (void)hipFree(s.d_dig);
            (void)hipHostFree(s.h_ok);
            (void)hipFree(s.d_ok);
            if (s.stream) (void)hipStreamDestroy(s.stream);
        }
    }
};

thread_local std::unordered_map<int, HostCtx> t_ctx;

// True when pages[0..n) are one contiguous run inside ONE pinned host
// allocation: a run starting in a registered region must end inside it;
// otherwise both the first and the last byte must be pinned host memory of
// the same allocation (hipMemGetAddressRange).  A run that starts in a pinned
// buffer and runs past its end, or spans two adjacent allocations, is
// gathered instead.
bool contiguous_pinned(const void* const* pages, uint64_t n, uint64_t P) {
    if (n == 0) return false;
    const uint8_t* base = static_cast<const uint8_t*>(pages[0]);
    for (uint64_t i = 1; i < n; ++i)
        if (pages[i] != base + i * P) return false;
    const uint8_t* last = base + n * P - 1;
    // Regions this library registered or allocated have known extents
    // (hipMemGetAddressRange does not resolve hipHostRegister'ed memory).
    switch (g_regions.run(reinterpret_cast<uintptr_t>(base), reinterpret_cast<uintptr_t>(last))) {
        case pcs::RegionRegistry::kInside: return true;
        case pcs::RegionRegistry::kPastEnd: return false;
        case pcs::RegionRegistry::kNotRegistered: break;
    }
    auto pinned_alloc = [](const uint8_t* p, uintptr_t* alloc_base, size_t* alloc_size) {
        hipPointerAttribute_t attr{};
        if (hipPointerGetAttributes(&attr, p) != hipSuccess || attr.type != hipMemoryTypeHost) return false;
        hipDeviceptr_t b = nullptr;
        size_t sz = 0;
        if (hipMemGetAddressRange(&b, &sz, const_cast<uint8_t*>(p)) != hipSuccess || !b || !sz) return false;
        *alloc_base = reinterpret_cast<uintptr_t>(b);
        *alloc_size = sz;
        return true;
    };
    uintptr_t b0 = 0, b1 = 0;
    size_t s0 = 0, s1 = 0;
    const bool ok = pinned_alloc(base, &b0, &s0) && pinned_alloc(last, &b1, &s1) && b0 == b1 && s0 == s1;
    (void)hipGetLastError();
    return ok;
}

// Gather scattered host pages into pinned staging.  Large chunks are split
// over several threads: one thread's memcpy from pageable memory (~14 GiB/s
// measured) is well below PCIe Gen5, so the host-fed path was gather-bound.
// PCS_GATHER_THREADS overrides the thread count (1 = serial).
unsigned gather_threads() {
    static const unsigned k = [] {
        if (const char* e = std::getenv("PCS_GATHER_THREADS")) {
            const long v = std::strtol(e, nullptr, 10);
            if (v >= 1 && v <= 64) return (unsigned)v;
        }
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        return std::min(8u, std::max(1u, hw / 2));
    }();
    return k;
}

void gather(uint8_t* dst, const void* const* pages, uint64_t first, uint64_t cnt, uint64_t P) {
    const uint64_t bytes = cnt * P;
    const unsigned T = bytes >= (8u << 20) ? gather_threads() : 1;
    auto run = [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; ++i) std::memcpy(dst + i * P, pages[first + i], P);
    };
    if (T <= 1) {
        run(0, cnt);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(T - 1);
    for (unsigned k = 1; k < T; ++k) th.emplace_back(run, cnt * k / T, cnt * (k + 1) / T);
    run(0, cnt / T);
    for (auto& x : th) x.join();
}

int ensure_slot(Slot& s, size_t page_bytes, size_t n) {
    hipError_t e;
    if (!s.stream && (e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess)
        return hip_fail(e, "hipStreamCreate");
    if (page_bytes > s.cap_pages_bytes) {
        (void)hipHostFree(s.h_pages);
        s.h_pages = nullptr;
        s.cap_pages_bytes = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&s.h_pages), page_bytes, hipHostMallocDefault) != hipSuccess)
            return fail(PCS_ERR_NOMEM, "staging allocation failed");
        s.cap_pages_bytes = page_bytes;
    }
    if (page_bytes > s.cap_dev_bytes) {
        (void)hipFree(s.d_pages);
        s.d_pages = nullptr;
        s.cap_dev_bytes = 0;
        if (hipMalloc(reinterpret_cast<void**>(&s.d_pages), page_bytes) != hipSuccess)
            return fail(PCS_ERR_NOMEM, "staging allocation failed");
        s.cap_dev_bytes = page_bytes;
    }
    if (n > s.cap_n) {
        (void)hipHostFree(s.h_dig);
        (void)hipFree(s.d_dig);
        (void)hipHostFree(s.h_ok);
        (void)hipFree(s.d_ok);
        s.h_dig = nullptr; s.d_dig = nullptr; s.h_ok = nullptr; s.d_ok = nullptr;
        s.cap_n = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&s.h_dig), n * 8, hipHostMallocDefault) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&s.d_dig), n * 8) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&s.h_ok), n, hipHostMallocDefault) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&s.d_ok), n) != hipSuccess)
            return fail(PCS_ERR_NOMEM, "result staging allocation failed");
        s.cap_n = n;
    }
    return PCS_OK;
}

int check_flags(uint32_t flags) {
    return (flags & ~uint32_t(PCS_FLAG_SKIP_VERIFY)) ? fail(PCS_ERR_INVALID, "unknown flag bits") : PCS_OK;
}

// Argument checks shared by the synchronous and asynchronous host batches.
int check_host_batch_args(const void* const* pages, uint64_t P, uint64_t n, int algo) {
    if (!valid_algo(algo)) return fail(PCS_ERR_INVALID, "algo must be PCS_XXH3_64 or PCS_XXH64");
    if (P < 8 || P > 0xFFFFFFFFull) return fail(PCS_ERR_INVALID, "page_size must be in [8, 2^32)");
    if (n && !pages) return fail(PCS_ERR_INVALID, "pages is null");
    if (n > UINT64_MAX / P) return fail(PCS_ERR_INVALID, "n_pages * page_size overflows 64 bits");
    for (uint64_t i = 0; i < n; ++i)
        if (!pages[i]) return fail(PCS_ERR_INVALID, "null page pointer in batch");
    return PCS_OK;
}

// Zero-copy XXH3 stamps of up to PCS_TUNE_ZC_STAMP_POLL_PAGES pages complete
// from per-page done bytes (each released after its header) rather than the
// stream's signal (PCS_TUNE_ZC_POLL on).  The default (256, a full
// FlushBatchPages batch) comes from integration_snippets --crossover with the
// columns in a fresh random order every repetition: done bytes beat the
// signal at every size to 256 (15.2 vs 20.3 us for one page, 33.5 vs 35.0 for
// 256; profiles/r05/crossover_r05e.txt).  Round 4's fixed-order columns had
// put the limit at 128 on a 16 % order bias.
bool zc_stamp_poll(uint64_t n) { return n <= (uint64_t)pcs::get_tuning(PCS_TUNE_ZC_STAMP_POLL_PAGES); }

// mode 0: digests -> out_dig;  mode 1: verdicts -> out_ok (+ first_bad);
// mode 2: digests stamped into the caller's pages.
int host_batch(int mode, const void* const* pages, uint64_t P, uint64_t n, int algo, uint8_t* out_ok,
               uint64_t* first_bad, uint64_t* out_dig) {
    if (int rc = require_device()) return rc;
    if (int rc = check_host_batch_args(pages, P, n, algo)) return rc;
    if (first_bad) *first_bad = UINT64_MAX;
    if (n == 0) return PCS_OK;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    HostCtx& ctx = t_ctx[dev];
    const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(n, kStageBytes / P));
    // Pages that are one contiguous, pinned (hipHostMalloc'd / hipHostRegister'ed)
    // run are DMA'd straight from the caller's memory: no gather copy.
    if (zero_copy_eligible(ctx.zc, pages, n, P, algo)) {
        // Registered pages: one launch reads them in place and writes the
        // verdicts / digests / page headers straight to host memory.
        if (int rc = ensure_slot(ctx.slot[0], 0, 1)) return rc;
        hipStream_t zs = ctx.slot[0].stream;
        // validate: completion from the landed verdicts; small XXH3 stamps:
        // from a done byte per page the kernel writes after each header
        const bool poll_stamp = mode == 2 && algo == PCS_XXH3_64 && zc_stamp_poll(n);
        const bool poll = (mode == 1 || poll_stamp) && zc_poll();
        if (poll) arm_verdicts(ctx.zc.h_ok, n);
        e = pcs::run_list(mode, algo, ctx.zc.d_ptrs, ctx.zc.h_ptrs, P, n, mode == 0 ? ctx.zc.d_dig : nullptr,
                          poll || mode == 1 ? ctx.zc.d_ok : nullptr, zs);
        if (e == hipSuccess) e = poll ? wait_verdicts(ctx.zc.h_ok, n, zs) : hipStreamSynchronize(zs);
        if (e != hipSuccess) return hip_fail(e, "zero-copy page list");
        count(PCS_COUNTER_ZERO_COPY_LAUNCHES);
        if (mode == 1) {
            std::memcpy(out_ok, ctx.zc.h_ok, n);
            if (first_bad)
                for (uint64_t i = 0; i < n; ++i)
                    if (!out_ok[i]) {
                        *first_bad = i;
                        break;
                    }
        } else if (mode == 0) {
            std::memcpy(out_dig, ctx.zc.h_dig, n * 8);
        }
        return PCS_OK;
    }
    const uint8_t* base = static_cast<const uint8_t*>(pages[0]);
    const bool direct = contiguous_pinned(pages, n, P);
    for (auto& s : ctx.slot)
        if (int rc = ensure_slot(s, direct ? 0 : chunk * P, chunk)) return rc;
    if (direct)  // device page buffers are still needed per slot
        for (auto& s : ctx.slot)
            if (chunk * P > s.cap_dev_bytes) {
                (void)hipFree(s.d_pages);
                s.d_pages = nullptr;
                s.cap_dev_bytes = 0;
                if (hipMalloc(reinterpret_cast<void**>(&s.d_pages), chunk * P) != hipSuccess)
                    return fail(PCS_ERR_NOMEM, "staging allocation failed");
                s.cap_dev_bytes = chunk * P;
            }

    uint64_t bad = UINT64_MAX;
    const bool poll = mode == 1 && zc_poll();
    auto drain = [&](Slot& s) -> int {
        if (!s.busy) return PCS_OK;
        hipError_t err = poll ? wait_verdicts(s.h_ok, s.count, s.stream) : hipStreamSynchronize(s.stream);
        s.busy = false;
        if (err != hipSuccess) return hip_fail(err, "hipStreamSynchronize");
        for (uint64_t i = 0; i < s.count; ++i) {
            const uint64_t gi = s.first + i;
            if (mode == 1) {
                out_ok[gi] = s.h_ok[i];
                if (!s.h_ok[i] && gi < bad) bad = gi;
            } else if (mode == 2) {
                std::memcpy(const_cast<void*>(pages[gi]), &s.h_dig[i], 8);  // EncodeFixed64 (LE)
            } else {
                out_dig[gi] = s.h_dig[i];
            }
        }
        return PCS_OK;
    };

    int rc = PCS_OK;
    uint64_t k = 0;
    for (uint64_t first = 0; first < n && rc == PCS_OK; first += chunk, ++k) {
        Slot& s = ctx.slot[k % kSlots];
        if ((rc = drain(s))) break;
        const uint64_t cnt = std::min(chunk, n - first);
        if (!direct) gather(s.h_pages, pages, first, cnt, P);
        count(direct ? PCS_COUNTER_DIRECT_DMA_CHUNKS : PCS_COUNTER_GATHER_CHUNKS);
        s.first = first;
        s.count = cnt;
        if (poll) arm_verdicts(s.h_ok, cnt);
        e = hipMemcpyAsync(s.d_pages, direct ? base + first * P : s.h_pages, cnt * P, hipMemcpyHostToDevice,
                           s.stream);
        if (e == hipSuccess)
            e = pcs::run_pages(mode == 1 ? 1 : 0, algo, s.d_pages, P, cnt, s.d_dig, s.d_ok, nullptr, s.stream);
        if (e == hipSuccess) {
            if (mode == 1) e = hipMemcpyAsync(s.h_ok, s.d_ok, cnt, hipMemcpyDeviceToHost, s.stream);
            else e = hipMemcpyAsync(s.h_dig, s.d_dig, cnt * 8, hipMemcpyDeviceToHost, s.stream);
        }
        if (e != hipSuccess) {
            rc = hip_fail(e, "host batch enqueue");
            break;
        }
        s.busy = true;
    }
    for (auto& s : ctx.slot) {
        const int r2 = drain(s);
        if (!rc) rc = r2;
    }
    if (first_bad) *first_bad = bad;
    return rc;
}

// ---------------------------------------------------------------------------
// pre-armed validate service (pcs_service_*)
// ---------------------------------------------------------------------------
// One service per device, started and stopped on the calling thread's current
// device, with `lines` request lines (pcs_service_start_ex; 1 by default).  A
// request (a synchronous validate / stamp call, or an asynchronous
// pcs_batch) claims a free line with an atomic flag, writes the request
// words, posts seq, and is answered through the line's verdict words; the
// flag is released when the owner has read its results.  A call that finds
// every line owned takes the launch path instead of queueing, so threads
// never starve on a line.  Requests are served by a resident kernel
// (pcs_kernels.hip k_service) with `wpl` workgroups per line; a workgroup
// leaves after idle_us without a request on its line or, between requests,
// after 2 * idle_us of life.  The host tracks those clocks from its side
// (conservatively: the kernel starts after its launch call and restarts a
// line's idle clock before the host sees the verdicts); while it is sure, by
// a margin of idle_us / 4, that the line's workgroups still wait, a request
// is one mailbox write and a wait on the verdicts.  Otherwise it starts the
// next generation: the box names it first, so every workgroup of the old
// kernel leaves at its next poll, and the new kernel, queued behind the old
// one, starts once they have.
//
// A request is only ever served by the workgroups of its own generation, and
// it is re-posted under a newer generation only once the kernel of the
// generation it was posted to has left (an event recorded behind each
// service kernel says so).  A re-post re-arms every verdict word first: the
// old generation may have answered some pages (with wpl > 1, some of a
// line's workgroups can leave before picking the request up while others
// answer it), and the new generation's workgroups hash all of them again.
// The host then waits for every verdict of the new generation, and a
// workgroup writes a page's verdict after its last read of the request, so
// no workgroup can still be reading a request's words or writing its
// verdicts after its owner has read them and released the line.
//
// The mailbox is allocated at a device's first start and kept for the life
// of the process, so an asynchronous request still in flight when the
// service stops can never read freed memory: it finds the service off and
// re-runs its pages on the launch path.
//
// Nothing waits on the GPU while holding the service's lock (VERDICT r05 #1:
// a poll on a shard thread must never stall behind another thread's stop).
// Stopping or giving up on the kernels *retires* them: the box names a
// generation no kernel serves, so every queued workgroup leaves at its next
// poll, and an event recorded behind them says when they have.  pcs_service_stop
// waits on that event after releasing the lock; a request that gives up on a
// kernel that has not left (no answer in 5 s) quarantines its line until that
// kernel's event completes, so no late verdict store can land in a later
// request's words.  The poll path takes the lock with try_lock only.
constexpr int kServiceEvents = 16;  // ring of events, one per generation (gen % 16)
struct Service {
    using clock = std::chrono::steady_clock;
    struct Line {
        std::atomic<int> owner{0};  // 0 free, 1 owned by a request, 2 quarantined (service_release)
        uint32_t count = 0;         // requests posted on it (low half of seq)
        // when its last request was answered (>= its workgroups' idle clock), steady-clock ticks
        std::atomic<clock::rep> answered{0};
        std::atomic<uint32_t> fence{0};  // quarantined: the generation whose kernel must leave first
    };
    std::mutex mu;                 // everything below except the atomics; never held while waiting
    std::atomic<int> callers{0};   // eligible calls in progress on this device, on either path
    std::atomic<int> load{0};      // decaying average of `callers` seen at entry, x256
    std::atomic<bool> gate_closed{false};  // the contention gate's state (with hysteresis)
    std::atomic<int> device{-1};   // -1: off (read without the lock by the entry points)
    std::atomic<int> lines{0};     // request lines (read without the lock when claiming one)
    int wpl = 0;                   // workgroups per line
    uint32_t idle_us = 0;
    hipStream_t stream = nullptr;  // kept across restarts; recreated only when its kind changes
    int64_t stream_kind = -1;      // PCS_TUNE_SERVICE_STREAM it was created with
    hipEvent_t done[kServiceEvents] = {};  // done[g % 16]: recorded behind generation g's kernel
    uint64_t slot_gen[kServiceEvents] = {};  // g << 1 | 1 queued a kernel of g, | 0 retired g (none)
    pcs::ServiceBox* h = nullptr;  // pinned, coherent, device-mapped; never freed
    pcs::ServiceBox* d = nullptr;  // its device alias
    std::atomic<uint32_t> gen{0};  // generation of the newest queued kernel (never reset; read unlocked)
    bool live = false;             // it has been queued (it may have left since)
    clock::time_point launched;
    Line line[pcs::kServiceMaxLines];
};
constexpr int kServiceDevices = 64;
Service g_services[kServiceDevices];
std::atomic<int> g_services_on{0};  // devices with a service: the validate / stamp paths look only when > 0

// The service's stream.  HIP multiplexes a process's streams onto a few
// hardware queues (GPU_MAX_HW_QUEUES, 4 here), in order within each queue, so
// a kernel of another stream that shares the resident kernel's queue can wait
// behind it until it leaves.  PCS_TUNE_SERVICE_STREAM = 1 (default) creates
// the service's stream at the highest priority (HIP pools its hardware queues
// by priority); under 4-16 threads of small batches that kept every thread
// served (tools/lab/service_load.cpp, profiles/r03/service_load_*.txt).
// 0: a plain stream.  A CU-masked stream is not offered: a resident kernel on
// one blocks the creation of other threads' streams.
hipError_t service_stream(hipStream_t* s) {
    if (pcs::get_tuning(PCS_TUNE_SERVICE_STREAM) == 1) {
        int lo = 0, hi = 0;
        const hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
        if (e != hipSuccess) return e;
        return hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

// Queue generation gen + 1: the box names it first, so the old kernel's
// workgroups leave at their next poll; the new kernel is queued behind them.
int service_launch_locked(Service& sv) {
    const uint32_t g = sv.gen.load(std::memory_order_relaxed) + 1;
    __atomic_store_n(&sv.h->gen, (uint64_t)g, __ATOMIC_RELEASE);
    sv.gen.store(g, std::memory_order_release);
    sv.live = true;
    sv.launched = Service::clock::now();
    for (int k = 0; k < sv.lines; ++k)
        sv.line[k].answered.store(sv.launched.time_since_epoch().count(), std::memory_order_relaxed);
    const uint64_t exit_ticks = (uint64_t)std::max<int64_t>(0, pcs::get_tuning(PCS_TUNE_SERVICE_SLOW_EXIT_TEST)) * 100;
    hipError_t e = pcs::run_service(sv.d, sv.lines, sv.wpl, g, (uint64_t)sv.idle_us * 100,
                                    (uint64_t)sv.idle_us * 200, exit_ticks, sv.stream);
    if (e == hipSuccess) e = hipEventRecord(sv.done[g % kServiceEvents], sv.stream);
    sv.slot_gen[g % kServiceEvents] = (uint64_t)g << 1 | 1;
    return finish(e, "service kernel launch");
}

// Have line k's workgroups of generation `gen` (wpl per line) all left?
// Each stores its generation into its departure word after its last verdict
// or header store is visible (k_service); a later generation's word in the
// same slot says so too, since kernels on the service's one stream run in
// order.  PCS_TUNE_SERVICE_DEPARTURE = 0: never consulted.
bool departure_words() { return pcs::get_tuning(PCS_TUNE_SERVICE_DEPARTURE) != 0; }
bool line_departed(const Service& sv, int k, int wpl, uint32_t gen) {
    const volatile uint32_t* d = sv.h->departed + k * wpl;
    for (int w = 0; w < wpl; ++w)
        if ((int32_t)(d[w] - gen) < 0) return false;
    return true;
}

// Line k's workgroups certainly still wait: launched less than life - margin
// ago and the line last answered less than idle - margin ago (host time
// bounds the kernel's clocks), and none of them has said it left.
bool service_waiting(const Service& sv, int k, Service::clock::time_point now) {
    const auto margin = std::chrono::microseconds(sv.idle_us / 4);
    const Service::clock::time_point answered{
        Service::clock::duration(sv.line[k].answered.load(std::memory_order_relaxed))};
    return sv.live && now - sv.launched < std::chrono::microseconds(2 * (uint64_t)sv.idle_us) - margin &&
           now - answered < std::chrono::microseconds(sv.idle_us) - margin &&
           !(departure_words() && line_departed(sv, k, sv.wpl, sv.gen.load(std::memory_order_relaxed)));
}

// The check word of line `ln`'s request words as they now stand, with `seq`
// in word 0 (service_word_mix, eloqstore_pcs_internal.h).
uint64_t service_check(const pcs::ServiceLine* ln, uint64_t seq) {
    const uint64_t* w = &ln->seq;
    uint64_t c = pcs::service_word_mix(seq, 0);
    for (int i = 1; i < pcs::kServiceLineWords; ++i)
        if (i != pcs::kServiceCheckWord) c += pcs::service_word_mix(w[i], (uint64_t)i);
    return c;
}

// Post the request words already on line k under generation `gen` (the
// current one but for the re-post drill): the check word, then seq last.
uint64_t service_post_locked(Service& sv, int k, uint32_t gen) {
    pcs::ServiceLine* ln = &sv.h->line[k];
    const uint64_t seq = (uint64_t)gen << 32 | ++sv.line[k].count;
    ln->check = service_check(ln, seq);
    std::atomic_thread_fence(std::memory_order_release);
    __atomic_store_n(&ln->seq, seq, __ATOMIC_RELEASE);
    return seq;
}

// Wait (bounded, outside every lock) until `ev` has completed.
hipError_t event_wait_bounded(hipEvent_t ev, std::chrono::milliseconds limit) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q != hipErrorNotReady) return q;
        if (std::chrono::steady_clock::now() - t0 > limit) return hipErrorNotReady;
        // gently: other threads' polls query the runtime too
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// Retire every queued kernel without waiting for it: the box names
// generation g + 1, which no kernel serves, so each workgroup leaves at its
// next poll, and done[(g + 1) % 16], recorded behind them all, completes once
// every one has.  The next request starts generation g + 2.  Returns that
// event's generation.
uint32_t service_retire_locked(Service& sv, hipError_t* err) {
    const uint32_t g = sv.gen.load(std::memory_order_relaxed) + 1;
    __atomic_store_n(&sv.h->gen, (uint64_t)g, __ATOMIC_RELEASE);
    sv.gen.store(g, std::memory_order_release);
    sv.live = false;
    const hipError_t e = hipEventRecord(sv.done[g % kServiceEvents], sv.stream);
    sv.slot_gen[g % kServiceEvents] = (uint64_t)g << 1;
    if (err) *err = e;
    return g;
}

// Turn the service off and retire its kernels under the lock, then wait for
// them to leave (bounded) after releasing it.
int service_stop(Service& sv) {
    std::unique_lock<std::mutex> lk(sv.mu);
    if (sv.device < 0) return PCS_OK;
    g_services_on.fetch_sub(1, std::memory_order_relaxed);
    int cur = -1;
    const bool other = hipGetDevice(&cur) == hipSuccess && cur != sv.device;
    if (other) (void)hipSetDevice(sv.device);
    sv.device = -1;  // a request in flight now re-runs on the launch path
    hipError_t e = hipSuccess;
    const uint32_t g = service_retire_locked(sv, &e);
    hipEvent_t ev = sv.done[g % kServiceEvents];
    if (other) (void)hipSetDevice(cur);
    lk.unlock();
    if (e != hipSuccess) return hip_fail(e, "service stop");
    // A later generation re-recording this ring slot meanwhile only makes the
    // wait longer: it completes after ours.
    e = event_wait_bounded(ev, std::chrono::milliseconds(2000));
    if (e == hipErrorNotReady) return fail(PCS_ERR_HIP, "service stop: kernels did not leave within 2 s");
    return finish(e, "service stop");
}

// Process exit with the service on: end the queued kernels before the HIP
// runtime tears down (handlers registered after the runtime's first use run
// before its own destructors).
void service_at_exit() {
    for (Service& sv : g_services) (void)service_stop(sv);
}

// A quarantined line may be claimed again once the kernel of its fence
// generation has left (its event; a newer generation's record in the same
// ring slot completes later still, so this never clears a line too early).
bool line_fence_passed(const Service& sv, int k) {
    hipEvent_t ev = sv.done[sv.line[k].fence.load(std::memory_order_acquire) % kServiceEvents];
    return ev && hipEventQuery(ev) == hipSuccess;
}

// The calling thread's device's service slot, or null.
Service* current_service() {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kServiceDevices) return nullptr;
    return &g_services[dev];
}

constexpr int kNotServed = 1;  // not eligible or declined: the caller takes the launch path
constexpr int kFallback = 2;   // the service could not answer (stopped, no answer in time): launch path
constexpr int kBusy = 3;       // the service's lock stayed held past kSubmitLockWait: launch path
// A submit waits this long at most for the service's lock (held for a launch
// of a new generation by another thread, which now and then takes
// milliseconds inside the runtime: the soak's 1.2-6.1 ms submits, round 6),
// then takes the launch path instead.
constexpr auto kSubmitLockWait = std::chrono::microseconds(20);

// PCS_TUNE_SERVICE_TEAR_TEST (test only): microseconds between posting seq
// and writing the request words, so the kernel's polls see a new seq beside
// the previous request's words; they must fail the check word and be ignored.
constexpr int kTuneServiceTearTest = PCS_TUNE_SERVICE_TEAR_TEST;
// PCS_TUNE_SERVICE_MAX_CALLERS: the contention gate (below).
constexpr int kTuneServiceMaxCallers = PCS_TUNE_SERVICE_MAX_CALLERS;

// Contention gate.  With more threads than request lines on a GPU the lines
// are mostly owned by other threads, the calls that find them busy launch
// anyway, and the resident kernel only widens the tail.
// Every eligible call counts itself in `callers` for its whole duration, on
// either path, and folds the count it saw at entry into a decaying average
// (1/16 per call); once the average exceeds PCS_TUNE_SERVICE_MAX_CALLERS +
// lines - 1 + 0.5 the service declines and the calls launch, until it drops
// below that limit - 0.5.  Counting calls
// on both paths keeps the signal alive while the gate is closed, so it
// reopens only when the callers thin out; the kernel idles out meanwhile and
// frees its CUs.
void caller_enter(Service& sv) {
    const int c = sv.callers.fetch_add(1, std::memory_order_relaxed) + 1;
    const int a = sv.load.load(std::memory_order_relaxed);
    sv.load.store(a + (((c << 8) - a) >> 4), std::memory_order_relaxed);  // racy by design: an estimate
}
void caller_leave(Service& sv) { sv.callers.fetch_sub(1, std::memory_order_relaxed); }

// The shape the service takes (service_submit): XXH3, 1..256 pages, a page
// size on the 256-byte grid.  Only such calls count as callers, so XXH64,
// large or odd-size traffic on the launch path cannot close the gate for the
// small XXH3 batches it exists for.  Whether the pages lie in
// registered memory is found out later, under the service's lock; such calls
// are counted.
bool service_shape_ok(uint64_t P, uint64_t n, int algo) {
    return algo == PCS_XXH3_64 && n >= 1 && n <= (uint64_t)pcs::kServiceMaxPages && pcs::list_shape_ok(0, P);
}

// The calling thread's device's service when it is on and the call has the
// service's shape (else null), counted as a caller for the guard's lifetime.
class CallerGuard {
public:
    CallerGuard(Service* sv, uint64_t P, uint64_t n, int algo)
        : sv_(sv && sv->device >= 0 && service_shape_ok(P, n, algo) ? sv : nullptr) {
        if (sv_) caller_enter(*sv_);
    }
    ~CallerGuard() {
        if (sv_) caller_leave(*sv_);
    }
    Service* service() const { return sv_; }
    CallerGuard(const CallerGuard&) = delete;
    CallerGuard& operator=(const CallerGuard&) = delete;

private:
    Service* sv_;
};

// With hysteresis: the gate closes above limit + 0.5 and reopens only below
// limit - 0.5, so a caller count near the limit does not flap between the
// paths (a flapping gate relaunches the idled-out kernel again and again:
// p99 54.7 µs at 4 threads on 2 lines, profiles/r04/service_load_wpl.txt).
bool service_gate_open(Service& sv) {
    const int64_t m = std::min<int64_t>(pcs::get_tuning(kTuneServiceMaxCallers), 1 << 20);  // (m + 8) << 8 fits
    if (m <= 0) return true;
    const int limit = (int)((m + sv.lines - 1) << 8);
    const int a = sv.load.load(std::memory_order_relaxed);
    bool closed = sv.gate_closed.load(std::memory_order_relaxed);
    if (!closed && a > limit + 128) sv.gate_closed.store(closed = true, std::memory_order_relaxed);
    else if (closed && a < limit - 128) sv.gate_closed.store(closed = false, std::memory_order_relaxed);
    return !closed;
}

// One request through the service, from claim to release.
struct ServiceReq {
    Service* sv = nullptr;  // set while the request owns a line
    int k = 0;              // its line
    uint64_t n = 0, landed = 0, seq = 0;
    uint32_t gen = 0;       // the generation it is posted to
    int wpl = 0;            // that generation's workgroups per line
    bool stamp = false;
    int relaunched = 0;
    uint32_t checked_gen = 0;  // the service's generation at the last check
    int path = 0;           // PCS_PATH_* bits gathered so far
    bool quarantine = false;  // given up while its generation's kernel may still run
    Service::clock::time_point posted, checked;
};

// Release the request's line: free, or quarantined until the kernel of the
// request's generation has left when the request gave up on it before then
// (a workgroup of it may still store a verdict into the line).
void service_release(ServiceReq& r) {
    if (!r.sv) return;
    Service::Line& l = r.sv->line[r.k];
    if (r.quarantine) {
        l.fence.store(r.gen, std::memory_order_relaxed);
        l.owner.store(2, std::memory_order_release);
    } else {
        l.owner.store(0, std::memory_order_release);
    }
    r.sv = nullptr;
}

std::atomic<uint64_t> g_torn_requests{0};
std::atomic<uint64_t> g_reposts{0};  // PCS_COUNTER_SERVICE_REPOSTS
thread_local int t_line_hint = -1;  // the line this thread used last: its first try

// PCS_TUNE_SERVICE_REPOST_TEST (test only): post a request as an earlier
// generation would have left it, partly answered, so the re-post path must
// re-arm it.  seq names generation gen - 1, which no waiting kernel serves
// (its kernel was queued before the current one and has left or leaves at
// its next poll); the verdict words of pages 16 and up hold a stale answer
// (validate: 0, a verdict no good page deserves; stamp: 1, a done word for a
// header never written).  A host that re-posted without re-arming would
// collect those as answers.  Needs gen >= 2 (generation gen - 1 then had a
// kernel and its event); otherwise the request is posted normally and the
// knob is not consumed.  So is a generation gen - 1 that queued no kernel
// (the one a stop or give-up retired): no workgroup of it could have
// answered part of a request.
constexpr int kTuneServiceRepostTest = PCS_TUNE_SERVICE_REPOST_TEST;
uint32_t repost_drill(const Service& sv, pcs::ServiceLine* ln, uint64_t n, bool stamp, uint32_t gen) {
    if (gen < 2 || sv.slot_gen[(gen - 1) % kServiceEvents] != ((uint64_t)(gen - 1) << 1 | 1) ||
        pcs::get_tuning(kTuneServiceRepostTest) <= 0 || !pcs::take_tuning(kTuneServiceRepostTest))
        return gen;
    for (uint64_t i = 16; i < n; ++i) ln->ok[i] = stamp ? 1u : 0u;
    return gen - 1;
}

// Claim a free line and post a validate (stamp = false) or stamp request:
// XXH3, registered 16-byte-aligned pages with page_size % 256 == 0, 1..256
// pages, on the calling thread's device with its service on and the gate
// open.  PCS_OK: posted, r owns the line.  kNotServed: nothing done.  < 0:
// error.
int service_submit(ServiceReq& r, Service* svp, const void* const* pages, uint64_t P, uint64_t n, int algo,
                   bool stamp) {
    if (!svp || !service_shape_ok(P, n, algo)) return kNotServed;
    Service& sv = *svp;
    if (!service_gate_open(sv)) return kNotServed;
    const int nl = std::max(1, std::min(sv.lines.load(std::memory_order_relaxed), pcs::kServiceMaxLines));
    int k = -1;
    const int h0 = t_line_hint >= 0 ? t_line_hint : 0;
    for (int i = 0; i < nl && k < 0; ++i) {
        const int c = (h0 + i) % nl;
        const int o = sv.line[c].owner.load(std::memory_order_relaxed);
        int expect = o;
        if ((o == 0 || (o == 2 && line_fence_passed(sv, c))) &&
            sv.line[c].owner.compare_exchange_strong(expect, 1, std::memory_order_acquire))
            k = c;
    }
    if (k < 0) return kNotServed;
    // The line is ours: translate the page addresses into it and arm its
    // verdict words before taking the lock (round 6: 256-page requests
    // spent 0.4-0.6 ms in submit with both under the lock while other threads
    // posted theirs).  No workgroup reads or writes a free line's words for
    // a request: its last request was answered or given up (its kernel
    // gone), and a waiting kernel only looks past them at a new seq, which
    // is posted under the lock below.
    pcs::ServiceLine* ln = sv.h ? &sv.h->line[k] : nullptr;
    const int64_t tear_us = pcs::get_tuning(kTuneServiceTearTest);
    uint64_t local[pcs::kServiceMaxPages];
    if (!ln || !g_regions.translate(pages, n, P, tear_us > 0 ? local : ln->ptrs)) {
        sv.line[k].owner.store(0, std::memory_order_release);
        return kNotServed;
    }
    for (uint64_t i = 0; i < n; ++i) ln->ok[i] = pcs::kServicePending;
    std::unique_lock<std::mutex> lk(sv.mu, std::defer_lock);
    for (const auto t0 = Service::clock::now(); !lk.try_lock();) {
        if (Service::clock::now() - t0 > kSubmitLockWait) {
            sv.line[k].owner.store(0, std::memory_order_release);
            return kBusy;
        }
        __builtin_ia32_pause();
    }
    if (sv.device < 0 || k >= sv.lines) {
        sv.line[k].owner.store(0, std::memory_order_release);
        return kNotServed;
    }
    t_line_hint = k;
    r = ServiceReq{};
    r.sv = &sv;
    r.k = k;
    r.n = n;
    r.stamp = stamp;
    if (!service_waiting(sv, k, Service::clock::now())) {
        if (int rc = service_launch_locked(sv)) {
            (void)service_retire_locked(sv, nullptr);  // nothing was posted: the line is free again
            service_release(r);
            return rc;
        }
        r.path |= PCS_PATH_NEW_GENERATION;
    }
    const uint64_t page_word = P | (stamp ? pcs::kServiceStamp : 0);
    if (tear_us > 0) {
        // seq first, the request words after it, the check word last: until
        // then every poll sees the new seq beside the previous request's words
        const uint64_t seq = (uint64_t)sv.gen.load(std::memory_order_relaxed) << 32 | ++sv.line[k].count;
        std::atomic_thread_fence(std::memory_order_release);
        __atomic_store_n(&ln->seq, seq, __ATOMIC_RELEASE);
        std::this_thread::sleep_for(std::chrono::microseconds(tear_us));
        std::memcpy(ln->ptrs, local, n * 8);
        ln->n = n;
        ln->page_size = page_word;
        const uint64_t c = service_check(ln, seq);
        std::atomic_thread_fence(std::memory_order_release);
        __atomic_store_n(&ln->check, c, __ATOMIC_RELEASE);
        r.seq = seq;
        r.gen = sv.gen.load(std::memory_order_relaxed);
    } else {
        ln->n = n;
        ln->page_size = page_word;
        r.gen = repost_drill(sv, ln, n, stamp, sv.gen.load(std::memory_order_relaxed));
        r.seq = service_post_locked(sv, k, r.gen);
    }
    r.wpl = sv.wpl;
    r.posted = r.checked = Service::clock::now();
    r.checked_gen = r.gen;
    return PCS_OK;
}

// Progress of a posted request (the line stays owned): 1 answered (results in
// the mailbox), 0 pending, kFallback (the service cannot answer it: stopped,
// or no answer in time; the caller re-runs it on the launch path and releases
// the line), < 0 error.
int service_progress(ServiceReq& r) {
    Service& sv = *r.sv;
    const volatile uint32_t* v = sv.h->line[r.k].ok;
    while (r.landed < r.n && v[r.landed] != pcs::kServicePending) ++r.landed;
    if (r.landed == r.n) {
        std::atomic_thread_fence(std::memory_order_acquire);
        return 1;
    }
    // Has the request's generation left its line?  With departure words the
    // line's own words say so (re-post at once), and the runtime is asked
    // about the kernel every 1 ms, for a failed kernel and the 5 s give-up.
    // Without them the runtime is asked every 50 µs, and at once when a
    // newer generation has been started since the last check (this request
    // must then be re-posted as soon as its own generation's kernel has left).
    const auto now = Service::clock::now();
    const uint32_t g_now = sv.gen.load(std::memory_order_acquire);
    const bool departure = departure_words();
    const bool gone = departure && line_departed(sv, r.k, r.wpl, r.gen);
    if (!gone && (departure ? now - r.checked < std::chrono::milliseconds(1)
                            : now - r.checked < std::chrono::microseconds(50) && g_now == r.checked_gen))
        return 0;
    r.checked = now;
    r.checked_gen = g_now;
    // Never wait for the lock: its holder (another thread's submit, start,
    // stop or re-post) holds it for a launch at most, and this request is
    // looked at again on the next call.
    std::unique_lock<std::mutex> lk(sv.mu, std::try_to_lock);
    if (!lk.owns_lock()) {
        r.path |= PCS_PATH_LOCK_SKIPPED;
        return 0;
    }
    // Has the kernel of the generation this request was posted to left?  (Its
    // event; a newer generation's event in the same ring slot is later on
    // the stream, so its completion implies this one's.)
    const hipError_t q = hipEventQuery(sv.done[r.gen % kServiceEvents]);
    if (q == hipErrorNotReady && !gone) {
        if (now - r.posted < std::chrono::seconds(5)) return 0;
        // no answer in 5 s (a latency problem, not a failure): retire the
        // kernels and give the line up only once this one has left
        (void)service_retire_locked(sv, nullptr);
        r.quarantine = true;
        return kFallback;
    }
    if (q != hipSuccess && q != hipErrorNotReady) {
        (void)service_retire_locked(sv, nullptr);
        r.quarantine = true;
        return hip_fail(q, "service stream");
    }
    std::atomic_thread_fence(std::memory_order_acquire);  // after the departure words
    // That kernel has left (or its workgroups on this line have, which is
    // all that can write the line) and this request is not fully answered (its
    // workgroups reached a limit just before the post, a newer generation
    // replaced it, or the service was stopped): no workgroup can write this
    // line any more, and verdicts are idempotent, so the request is posted
    // again to the current generation (started now if none is waiting).
    while (r.landed < r.n && v[r.landed] != pcs::kServicePending) ++r.landed;
    if (r.landed == r.n) {
        std::atomic_thread_fence(std::memory_order_acquire);
        return 1;
    }
    // (a restart with fewer lines serves no workgroup on this one)
    if (sv.device < 0 || r.k >= sv.lines || ++r.relaunched > 3) return kFallback;
    if (r.gen == sv.gen.load(std::memory_order_relaxed) || !service_waiting(sv, r.k, now)) {
        if (int rc = service_launch_locked(sv)) {
            (void)service_retire_locked(sv, nullptr);  // this request's own kernel has left: no quarantine
            return rc;
        }
        r.path |= PCS_PATH_NEW_GENERATION;
    }
    // Re-arm the whole request: verdicts the old generation left must not
    // count as answers of the new one, whose workgroups re-hash those pages
    // (and would otherwise still be doing so once the host had released the
    // line).  No workgroup writes this line now: its kernel has left and the
    // newer ones serve only the seq posted below.
    uint32_t* ok = sv.h->line[r.k].ok;
    for (uint64_t i = 0; i < r.n; ++i) ok[i] = pcs::kServicePending;
    r.landed = 0;
    g_reposts.fetch_add(1, std::memory_order_relaxed);
    r.path |= PCS_PATH_REPOSTED;
    r.gen = sv.gen.load(std::memory_order_relaxed);
    r.wpl = sv.wpl;
    r.seq = service_post_locked(sv, r.k, r.gen);
    r.posted = Service::clock::now();
    return 0;
}

// After progress returned 1: verdicts (validate) or the done words (stamp).
int service_collect(ServiceReq& r, uint8_t* ok, uint64_t* first_bad) {
    Service& sv = *r.sv;
    const pcs::ServiceLine* ln = &sv.h->line[r.k];
    sv.line[r.k].answered.store(Service::clock::now().time_since_epoch().count(), std::memory_order_relaxed);
    r.path |= PCS_PATH_SERVED;
    if (__atomic_load_n(&ln->torn_seq, __ATOMIC_RELAXED) == r.seq)
        g_torn_requests.fetch_add(1, std::memory_order_relaxed);
    if (!r.stamp) {
        uint64_t bad = UINT64_MAX;
        for (uint64_t i = 0; i < r.n; ++i) {
            ok[i] = (uint8_t)ln->ok[i];
            if (!ok[i] && bad == UINT64_MAX) bad = i;
        }
        if (first_bad) *first_bad = bad;
    } else {
        for (uint64_t i = 0; i < r.n; ++i)
            if (ln->ok[i] != 1u) return fail(PCS_ERR_HIP, "validate service: stamp not confirmed");
    }
    count(PCS_COUNTER_SERVICE_BATCHES);
    return PCS_OK;
}

// A synchronous host validate (ok != null) or stamp (ok == null) batch
// through the service: PCS_OK, kNotServed (take the launch path) or < 0.
thread_local int t_path = 0;  // pcs_last_path

int service_run(Service* svp, const void* const* pages, uint64_t P, uint64_t n, int algo, uint8_t* ok,
                uint64_t* first_bad) {
    ServiceReq r;
    const int s = service_submit(r, svp, pages, P, n, algo, ok == nullptr);
    if (s == kBusy) t_path |= PCS_PATH_LOCK_SKIPPED;
    if (s != PCS_OK) return s == kBusy ? kNotServed : s;
    int p;
    SyncWaiter w;
    while ((p = service_progress(r)) == 0) w.pause();
    int rc = p == 1 ? service_collect(r, ok, first_bad) : p == kFallback ? kNotServed : p;
    if (p == kFallback) r.path |= PCS_PATH_FALLBACK;
    t_path = r.path;
    service_release(r);
    return rc;
}

// Device copy of one host buffer + a result word, for the manifest host API.
int manifest_host(const void* content, uint64_t len, uint64_t* out) {
    if (injected_failure()) return fail(PCS_ERR_HIP, "injected failure (PCS_TUNE_FAIL_INJECT)");
    if (int rc = require_device()) return rc;
    if (!out || (len && !content)) return fail(PCS_ERR_INVALID, "null pointer");
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    Slot& slot = t_ctx[dev].slot[0];  // the calling thread's stream on this device
    if (int rc = ensure_slot(slot, 0, 1)) return rc;
    hipStream_t s = slot.stream;
    // [content | pad to 16 | digest word]: the content starts at the
    // buffer's base (hipMalloc alignment), so the 16-byte-load block-sum
    // kernel (k_manifest_sums16) serves the host API too.
    const uint64_t dig_off = (len + 15) & ~uint64_t(15);
    void* buf = nullptr;
    int id = -1;
    e = pcs::scratch_acquire(dig_off + 8, &buf, &id);
    uint8_t* d = static_cast<uint8_t*>(buf);
    uint64_t* d_out = reinterpret_cast<uint64_t*>(d + dig_off);
    if (e == hipSuccess && len) e = hipMemcpyAsync(d, content, len, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = pcs::run_manifest(d, len, d_out, s);
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (id >= 0) (void)pcs::scratch_release(id, s);
    if (e != hipSuccess) (void)hipStreamSynchronize(s);  // nothing of this call left in flight
    return finish(e, "manifest checksum");
}

}  // namespace

// ---------------------------------------------------------------------------
// asynchronous batches
// ---------------------------------------------------------------------------
struct pcs_batch {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint8_t* h_pages = nullptr;
    uint8_t* d_pages = nullptr;
    uint64_t* h_dig = nullptr;
    uint64_t* d_dig = nullptr;
    uint8_t* h_ok = nullptr;
    uint8_t* d_ok = nullptr;
    size_t cap_bytes = 0, cap_n = 0;
    std::vector<void*> stamp_pages;
    ZcBufs zc;
    bool zero_copy = false;  // in-flight batch reads registered pages in place
    bool zc_polled = false;  // completion seen from the landed verdicts / done bytes (zc_poll)
    uint64_t zc_landed = 0;  // verdicts seen so far
    uint32_t zc_polls = 0;   // polls since submit (the stream is queried every kZcEventQueryPolls-th)
    uint64_t n = 0, P = 0, first_bad = UINT64_MAX;
    int mode = 0, state = 0;  // 0 idle, 1 in flight, 2 done, -1 failed
    int algo = 0;
    bool all_ok = false;      // completed at submit with nothing hashed (skip_verify / empty)
    // A batch the validate service took: the request owns the device's line
    // until completion; its pages are kept to re-run them on the launch path
    // if the service cannot answer (stopped meanwhile, or no answer in time).
    ServiceReq svc;
    bool via_service = false;          // in flight through the service
    bool svc_results = false;          // the completed batch's results are svc_ok / svc_dig
    Service* caller = nullptr;         // counted in this service's callers until completion
    std::vector<const void*> svc_pages;
    std::vector<uint8_t> svc_ok;
    std::vector<uint64_t> svc_dig;
    int path = 0;                      // PCS_PATH_* bits of the last submission (pcs_batch_path)
    bool has_event = true;             // `done` was recorded behind the in-flight launch
};

namespace {
void batch_uncount(pcs_batch* b) {
    if (b->caller) caller_leave(*b->caller);
    b->caller = nullptr;
}

int batch_finalize(pcs_batch* b) {
    b->first_bad = UINT64_MAX;
    if (b->zero_copy) {  // results already in host memory, pages stamped in place
        if (b->n) std::memcpy(b->mode == PCS_BATCH_VALIDATE ? static_cast<void*>(b->h_ok) : b->h_dig,
                              b->mode == PCS_BATCH_VALIDATE ? static_cast<void*>(b->zc.h_ok) : b->zc.h_dig,
                              b->mode == PCS_BATCH_VALIDATE ? b->n : b->n * 8);
        if (b->mode == PCS_BATCH_VALIDATE)
            for (uint64_t i = 0; i < b->n; ++i)
                if (!b->h_ok[i]) {
                    b->first_bad = i;
                    break;
                }
    } else if (b->mode == PCS_BATCH_VALIDATE) {
        for (uint64_t i = 0; i < b->n; ++i)
            if (!b->h_ok[i]) {
                b->first_bad = i;
                break;
            }
    } else if (b->mode == PCS_BATCH_STAMP) {
        for (uint64_t i = 0; i < b->n; ++i) std::memcpy(b->stamp_pages[i], &b->h_dig[i], 8);  // EncodeFixed64
    }
    b->state = 2;
    batch_uncount(b);
    return 1;
}

int batch_failed(pcs_batch* b, int rc) {
    b->state = -1;
    batch_uncount(b);
    return rc;
}

// Result buffers of a batch: at least a service-sized batch (256 pages), so a
// batch the service gives back never grows them from a poll (freeing device
// or pinned memory synchronises the device: the poll would wait for every
// kernel, the service's included).  pcs_batch_create sizes them at once.
int batch_results(pcs_batch* b, uint64_t n) {
    if (n <= b->cap_n) return PCS_OK;
    n = std::max<uint64_t>(n, pcs::kServiceMaxPages);
    (void)hipHostFree(b->h_dig);
    (void)hipFree(b->d_dig);
    (void)hipHostFree(b->h_ok);
    (void)hipFree(b->d_ok);
    b->h_dig = nullptr; b->d_dig = nullptr; b->h_ok = nullptr; b->d_ok = nullptr;
    b->cap_n = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&b->h_dig), n * 8, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&b->d_dig), n * 8) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&b->h_ok), n, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&b->d_ok), n) != hipSuccess)
        return fail(PCS_ERR_NOMEM, "batch result allocation failed");
    b->cap_n = n;
    return PCS_OK;
}

// Launch path of an asynchronous batch (arguments checked, n > 0): zero-copy
// over registered pages, else staged (gather or direct DMA), on the batch's
// own stream; completion is seen by poll / wait.
int batch_launch(pcs_batch* b, int mode, const void* const* pages, uint64_t P, uint64_t n, int algo) {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != b->device) (void)hipSetDevice(b->device);
    hipError_t e = hipSuccess;
    if (int rc = batch_results(b, n)) return rc;
    b->zero_copy = false;
    b->path |= PCS_PATH_LAUNCHED;
    b->stamp_pages.assign(n, nullptr);
    if (mode == PCS_BATCH_STAMP)
        for (uint64_t i = 0; i < n; ++i) b->stamp_pages[i] = const_cast<void*>(pages[i]);
    hipStream_t s = b->stream;
    b->zero_copy = zero_copy_eligible(b->zc, pages, n, P, algo);
    // page staging only off the zero-copy path
    if (!b->zero_copy && n * P > b->cap_bytes) {
        (void)hipHostFree(b->h_pages);
        (void)hipFree(b->d_pages);
        b->h_pages = nullptr;
        b->d_pages = nullptr;
        b->cap_bytes = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&b->h_pages), n * P, hipHostMallocDefault) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&b->d_pages), n * P) != hipSuccess)
            return fail(PCS_ERR_NOMEM, "batch staging allocation failed");
        b->cap_bytes = n * P;
    }
    // validate: completion from the landed verdicts; small zero-copy XXH3
    // stamps: from the per-page done bytes (each released after the header
    // and the digest word)
    const bool poll_stamp = mode == PCS_BATCH_STAMP && b->zero_copy && algo == PCS_XXH3_64 && zc_stamp_poll(n);
    b->zc_polled = (mode == PCS_BATCH_VALIDATE || poll_stamp) && zc_poll();
    b->zc_landed = 0;
    b->zc_polls = 0;
    if (b->zc_polled) arm_verdicts(b->zero_copy ? b->zc.h_ok : b->h_ok, n);
    if (b->zero_copy) {
        // stamp writes digests into the pages and into zc.h_dig (the digest
        // result of a stamp batch)
        e = pcs::run_list(mode, algo, b->zc.d_ptrs, b->zc.h_ptrs, P, n, mode == PCS_BATCH_VALIDATE ? nullptr : b->zc.d_dig,
                          mode == PCS_BATCH_VALIDATE || b->zc_polled ? b->zc.d_ok : nullptr, s);
        // A batch that completes from its landed verdicts / done bytes needs
        // no event behind its kernel: its own stream answers the occasional
        // "did the launch fail?" query (PCS_TUNE_ZC_BATCH_EVENT = 0, the
        // default; one runtime call less per batch).
        b->has_event = !b->zc_polled || pcs::get_tuning(PCS_TUNE_ZC_BATCH_EVENT) != 0;
        if (e == hipSuccess && b->has_event) e = hipEventRecord(b->done, s);
        if (e != hipSuccess) return hip_fail(e, "pcs_batch_submit (zero-copy)");
        count(PCS_COUNTER_ZERO_COPY_LAUNCHES);
        b->state = 1;
        return PCS_OK;
    }
    const bool direct = contiguous_pinned(pages, n, P);
    if (!direct) gather(b->h_pages, pages, 0, n, P);
    count(direct ? PCS_COUNTER_DIRECT_DMA_CHUNKS : PCS_COUNTER_GATHER_CHUNKS);
    e = hipMemcpyAsync(b->d_pages, direct ? pages[0] : b->h_pages, n * P, hipMemcpyHostToDevice, s);
    const int kmode = mode == PCS_BATCH_VALIDATE ? 1 : 0;
    if (e == hipSuccess) e = pcs::run_pages(kmode, algo, b->d_pages, P, n, b->d_dig, b->d_ok, nullptr, s);
    if (e == hipSuccess)
        e = kmode ? hipMemcpyAsync(b->h_ok, b->d_ok, n, hipMemcpyDeviceToHost, s)
                  : hipMemcpyAsync(b->h_dig, b->d_dig, n * 8, hipMemcpyDeviceToHost, s);
    b->has_event = true;
    if (e == hipSuccess) e = hipEventRecord(b->done, s);
    if (e != hipSuccess) return hip_fail(e, "pcs_batch_submit");
    b->state = 1;
    return PCS_OK;
}

constexpr uint32_t kZcEventQueryPolls = 256;

// Progress of a batch the service took: 1 done, 0 in flight (also after it
// was moved to the launch path), < 0 failed.
int batch_service_poll(pcs_batch* b) {
    const int p = service_progress(b->svc);
    b->path |= b->svc.path;
    if (p == 0) return 0;
    if (p == 1) {
        uint64_t fb = UINT64_MAX;
        if (b->mode == PCS_BATCH_VALIDATE) b->svc_ok.resize(b->n);
        const int rc = service_collect(b->svc, b->mode == PCS_BATCH_VALIDATE ? b->svc_ok.data() : nullptr, &fb);
        b->path |= b->svc.path;  // + PCS_PATH_SERVED
        service_release(b->svc);
        b->via_service = false;
        if (rc) return batch_failed(b, rc);
        if (b->mode == PCS_BATCH_STAMP) {  // the digests are the headers just landed
            b->svc_dig.resize(b->n);
            for (uint64_t i = 0; i < b->n; ++i) std::memcpy(&b->svc_dig[i], b->svc_pages[i], 8);  // DecodeFixed64
        }
        b->first_bad = fb;
        b->svc_results = true;
        b->state = 2;
        batch_uncount(b);
        return 1;
    }
    service_release(b->svc);
    b->via_service = false;
    if (p < 0) return batch_failed(b, p);
    // kFallback: the same pages on the launch path
    b->path |= PCS_PATH_FALLBACK;
    if (int rc = batch_launch(b, b->mode, b->svc_pages.data(), b->P, b->n, b->algo)) return batch_failed(b, rc);
    return 0;
}
}  // namespace

extern "C" {

const char* pcs_version(void) { return "eloqstore-pcs 0.4.0 (gfx950; xxHash v0.8.3 page path)"; }

int pcs_abi_version(void) { return PCS_ABI_VERSION; }

const char* pcs_last_error(void) { return t_last_error.c_str(); }

int pcs_device_count(int* count) {
    if (!count) return fail(PCS_ERR_INVALID, "count is null");
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    *count = (e == hipSuccess) ? n : 0;
    return e == hipSuccess ? PCS_OK : fail(PCS_ERR_NO_DEVICE, hipGetErrorString(e));
}

int pcs_set_device(int device) {
    if (int rc = require_device()) return rc;
    return finish(hipSetDevice(device), "hipSetDevice");
}

int pcs_synchronize(pcs_stream_t stream) {
    if (int rc = require_device()) return rc;
    return finish(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)), "hipStreamSynchronize");
}

int pcs_pages_digest_dev(const void* d_pages, uint64_t page_size, uint64_t n_pages, int algo, uint64_t* d_digests,
                         pcs_stream_t stream) {
    return pages_common(0, d_pages, page_size, n_pages, algo, d_digests, nullptr, nullptr, stream);
}

int pcs_pages_validate_dev(const void* d_pages, uint64_t page_size, uint64_t n_pages, int algo, uint8_t* d_ok,
                           uint64_t* d_first_bad, pcs_stream_t stream) {
    return pages_common(1, d_pages, page_size, n_pages, algo, nullptr, d_ok, d_first_bad, stream);
}

int pcs_pages_stamp_dev(void* d_pages, uint64_t page_size, uint64_t n_pages, int algo, pcs_stream_t stream) {
    return pages_common(2, d_pages, page_size, n_pages, algo, nullptr, nullptr, nullptr, stream);
}

int pcs_desc_digest_dev(const void* d_base, const uint64_t* d_off, const uint32_t* d_len, uint64_t n, int algo,
                        uint64_t* d_digests, pcs_stream_t stream) {
    return desc_common(0, d_base, d_off, d_len, n, algo, 8, 0, d_digests, nullptr, nullptr, stream);
}

int pcs_desc_validate_dev(const void* d_base, const uint64_t* d_off, const uint32_t* d_len, uint64_t n, int algo,
                          uint8_t* d_ok, uint64_t* d_first_bad, pcs_stream_t stream) {
    return desc_common(1, d_base, d_off, d_len, n, algo, 8, 0, nullptr, d_ok, d_first_bad, stream);
}

int pcs_desc_stamp_dev(void* d_base, const uint64_t* d_off, const uint32_t* d_len, uint64_t n, int algo,
                       pcs_stream_t stream) {
    return desc_common(2, d_base, d_off, d_len, n, algo, 8, 0, nullptr, nullptr, nullptr, stream);
}

int pcs_xxh3_64_ranges_dev(const void* d_base, const uint64_t* d_off, const uint32_t* d_len, uint64_t n,
                           uint64_t* d_out, pcs_stream_t stream) {
    return desc_common(0, d_base, d_off, d_len, n, PCS_XXH3_64, 0, 0, d_out, nullptr, nullptr, stream);
}

int pcs_xxh64_ranges_dev(const void* d_base, const uint64_t* d_off, const uint32_t* d_len, uint64_t n, uint64_t seed,
                         uint64_t* d_out, pcs_stream_t stream) {
    return desc_common(0, d_base, d_off, d_len, n, PCS_XXH64, 0, seed, d_out, nullptr, nullptr, stream);
}

int pcs_pages_validate_host(const void* const* pages, uint64_t page_size, uint64_t n_pages, int algo, uint8_t* ok,
                            uint64_t* first_bad) {
    return pcs_pages_validate_host_ex(pages, page_size, n_pages, algo, ok, first_bad, PCS_FLAG_NONE);
}

int pcs_pages_validate_host_ex(const void* const* pages, uint64_t page_size, uint64_t n_pages, int algo, uint8_t* ok,
                               uint64_t* first_bad, uint32_t flags) {
    if (n_pages && !ok) return fail(PCS_ERR_INVALID, "ok is null");
    if (int rc = check_flags(flags)) return rc;
    if (flags & PCS_FLAG_SKIP_VERIFY) {  // kv_options.h:41: the validate loop is not run
        if (int rc = check_host_batch_args(pages, page_size, n_pages, algo)) return rc;
        if (n_pages) std::memset(ok, 1, n_pages);
        if (first_bad) *first_bad = UINT64_MAX;
        return PCS_OK;
    }
    if (injected_failure()) return fail(PCS_ERR_HIP, "injected failure (PCS_TUNE_FAIL_INJECT)");
    t_path = 0;
    if (g_services_on.load(std::memory_order_relaxed) > 0) {
        if (int rc = check_host_batch_args(pages, page_size, n_pages, algo)) return rc;
        CallerGuard g(current_service(), page_size, n_pages, algo);
        const int r = service_run(g.service(), pages, page_size, n_pages, algo, ok, first_bad);
        if (r != kNotServed) return r;
        t_path |= PCS_PATH_LAUNCHED;
        return host_batch(1, pages, page_size, n_pages, algo, ok, first_bad, nullptr);  // still counted as a caller (the guard): the gate sees both paths
    }
    t_path |= PCS_PATH_LAUNCHED;
    return host_batch(1, pages, page_size, n_pages, algo, ok, first_bad, nullptr);
}

int pcs_service_start(int workgroups, uint32_t idle_us) { return pcs_service_start_ex(1, workgroups, idle_us); }

int pcs_service_start_ex(int lines, int workgroups_per_line, uint32_t idle_us) {
    if (lines < 1 || lines > pcs::kServiceMaxLines)
        return fail(PCS_ERR_INVALID, "lines must be in [1, " + std::to_string(pcs::kServiceMaxLines) + "]");
    if (workgroups_per_line < 1 || lines * workgroups_per_line > 256)
        return fail(PCS_ERR_INVALID, "workgroups must be in [1, 256] (lines x workgroups per line)");
    if (idle_us && (idle_us < 200 || idle_us > 1000000))
        return fail(PCS_ERR_INVALID, "idle_us must be 0 (1000) or in [200, 1000000]");
    if (int rc = require_device()) return rc;
    Service* svp = current_service();
    if (!svp) return fail(PCS_ERR_INVALID, "no service slot for the current device");
    Service& sv = *svp;
    std::lock_guard<std::mutex> lk(sv.mu);
    if (sv.device >= 0) return fail(PCS_ERR_INVALID, "the validate service is already running on this device");
    int dev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "service start");
    // The stream is kept across restarts: destroying and creating streams
    // stalls other threads' HIP calls for ~2 ms (the soak's launch-path calls
    // at a restart, profiles/r06/soak_*.txt).  It is recreated only when
    // PCS_TUNE_SERVICE_STREAM (read here) asks for another kind, and then
    // only if no asynchronous request of the previous run still owns a line
    // (or a line is quarantined behind one) and the previous run's kernels
    // have left (a stop waits for them outside the lock; destroying the
    // stream here would wait under it); the mailbox and the events are made
    // once.
    bool owned = false;
    for (int k = 0; k < pcs::kServiceMaxLines; ++k) {
        Service::Line& l = sv.line[k];
        int q = 2;
        if (l.owner.load(std::memory_order_acquire) == 2 && line_fence_passed(sv, k))
            l.owner.compare_exchange_strong(q, 0, std::memory_order_acq_rel);
        owned |= l.owner.load(std::memory_order_acquire) != 0;
    }
    const hipEvent_t last = sv.done[sv.gen.load(std::memory_order_relaxed) % kServiceEvents];
    const bool left = !last || hipEventQuery(last) == hipSuccess;
    const int64_t kind = pcs::get_tuning(PCS_TUNE_SERVICE_STREAM);
    if (sv.stream && kind != sv.stream_kind && !owned && left) {
        (void)hipStreamDestroy(sv.stream);
        sv.stream = nullptr;
    }
    if (!sv.stream) {
        if ((e = service_stream(&sv.stream)) != hipSuccess) {
            sv.stream = nullptr;
            return hip_fail(e, "service start");
        }
        sv.stream_kind = kind;
    }
    for (auto& ev : sv.done)
        if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) {
            ev = nullptr;
            return hip_fail(e, "service start (events)");
        }
    if (!sv.h) {
        pcs::ServiceBox* h = nullptr;
        if (hipHostMalloc(reinterpret_cast<void**>(&h), sizeof(pcs::ServiceBox),
                          hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
            return fail(PCS_ERR_NOMEM, "service mailbox allocation failed");
        std::memset(static_cast<void*>(h), 0, sizeof(pcs::ServiceBox));
        pcs::ServiceBox* d = dev_alias(h);
        if (!d) {
            (void)hipHostFree(h);
            return fail(PCS_ERR_HIP, "service mailbox has no device alias");
        }
        sv.h = h;
        sv.d = d;
    }
    // a line still owned by a request of the previous run stays out of use
    // until that request is released (its owner re-runs it on the launch path)
    sv.lines = lines;
    sv.wpl = workgroups_per_line;
    sv.idle_us = idle_us ? idle_us : 1000;
    sv.live = false;
    sv.load.store(0, std::memory_order_relaxed);
    sv.gate_closed.store(false, std::memory_order_relaxed);
    sv.device = dev;
    g_services_on.fetch_add(1, std::memory_order_relaxed);
    static std::once_flag hook;
    std::call_once(hook, [] { std::atexit(service_at_exit); });
    return PCS_OK;
}

int pcs_service_stop(void) {
    Service* svp = current_service();
    if (!svp) return PCS_OK;
    return service_stop(*svp);
}

int pcs_service_running(void) {
    Service* svp = current_service();
    return svp && svp->device.load(std::memory_order_acquire) >= 0 ? 1 : 0;
}

int pcs_last_path(void) { return t_path; }

int pcs_pages_stamp_host(void* const* pages, uint64_t page_size, uint64_t n_pages, int algo) {
    const void* const* cp = const_cast<const void* const*>(pages);
    if (injected_failure()) return fail(PCS_ERR_HIP, "injected failure (PCS_TUNE_FAIL_INJECT)");
    t_path = 0;
    if (g_services_on.load(std::memory_order_relaxed) > 0) {
        if (int rc = check_host_batch_args(cp, page_size, n_pages, algo)) return rc;
        CallerGuard g(current_service(), page_size, n_pages, algo);
        const int r = service_run(g.service(), cp, page_size, n_pages, algo, nullptr, nullptr);
        if (r != kNotServed) return r;
        t_path |= PCS_PATH_LAUNCHED;
        return host_batch(2, cp, page_size, n_pages, algo, nullptr, nullptr, nullptr);  // still counted as a caller (the guard): the gate sees both paths
    }
    t_path |= PCS_PATH_LAUNCHED;
    return host_batch(2, cp, page_size, n_pages, algo, nullptr, nullptr, nullptr);
}

int pcs_pages_digest_host(const void* const* pages, uint64_t page_size, uint64_t n_pages, int algo,
                          uint64_t* digests) {
    if (n_pages && !digests) return fail(PCS_ERR_INVALID, "digests is null");
    if (injected_failure()) return fail(PCS_ERR_HIP, "injected failure (PCS_TUNE_FAIL_INJECT)");
    return host_batch(0, pages, page_size, n_pages, algo, nullptr, nullptr, digests);
}

int pcs_host_alloc_pinned(uint64_t bytes, void** out) {
    if (!out) return fail(PCS_ERR_INVALID, "out is null");
    *out = nullptr;
    if (int rc = require_device()) return rc;
    if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return fail(PCS_ERR_NOMEM, "hipHostMalloc failed");
    }
    if (int rc = add_region(*out, bytes ? bytes : 1, true)) {
        (void)hipHostFree(*out);
        *out = nullptr;
        return rc;
    }
    return PCS_OK;
}

int pcs_host_free_pinned(void* p) {
    if (!p) return PCS_OK;
    if (g_regions.remove(reinterpret_cast<uintptr_t>(p), true) != pcs::RegionRegistry::kOk)
        return fail(PCS_ERR_INVALID, "not a pcs_host_alloc_pinned allocation");
    return finish(hipHostFree(p), "hipHostFree");
}

int pcs_host_register(void* p, uint64_t bytes) {
    if (!p || bytes == 0) return fail(PCS_ERR_INVALID, "null pointer or zero size");
    if (int rc = require_device()) return rc;
    const uintptr_t b = reinterpret_cast<uintptr_t>(p);
    if (!pcs::RegionRegistry::valid_range(b, bytes)) return fail(PCS_ERR_INVALID, "region wraps the address space");
    if (g_regions.overlaps(b, bytes))  // reject overlaps before pinning anything
        return fail(PCS_ERR_INVALID, "region overlaps a registered one");
    hipError_t e = hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) return hip_fail(e, "hipHostRegister");
    if (int rc = add_region(p, bytes, false)) {
        (void)hipHostUnregister(p);
        return rc;
    }
    return PCS_OK;
}

int pcs_thread_prepare(void) {
    if (int rc = require_device()) return rc;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    if (dev < 0 || dev >= kServiceDevices) return fail(PCS_ERR_INVALID, "device index out of range");
    HostCtx& ctx = t_ctx[dev];
    if (int rc = ensure_slot(ctx.slot[0], 0, pcs::kServiceMaxPages)) return rc;
    if (int rc = ctx.zc.ensure(pcs::kServiceMaxPages)) return rc;
    // one process-wide pinned, mapped 4 KiB page per device to validate, kept
    // for the life of the process (freeing pinned memory synchronises the device)
    static std::mutex mu;
    static void* warm[kServiceDevices] = {};
    void* page = nullptr;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!warm[dev]) {
            void* p = nullptr;
            if (hipHostMalloc(&p, 4096, hipHostMallocMapped) != hipSuccess) return fail(PCS_ERR_NOMEM, "warm page");
            std::memset(p, 0, 4096);
            warm[dev] = p;
        }
        page = warm[dev];
    }
    void* d_page = nullptr;
    if ((e = hipHostGetDevicePointer(&d_page, page, 0)) != hipSuccess) return hip_fail(e, "hipHostGetDevicePointer");
    ctx.zc.h_ptrs[0] = reinterpret_cast<uint64_t>(d_page);
    hipStream_t s = ctx.slot[0].stream;
    e = pcs::run_list(1, PCS_XXH3_64, ctx.zc.d_ptrs, ctx.zc.h_ptrs, 4096, 1, nullptr, ctx.zc.d_ok, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return finish(e, "pcs_thread_prepare");
}

int pcs_host_unregister(void* p) {
    if (!p) return fail(PCS_ERR_INVALID, "null pointer");
    if (g_regions.remove(reinterpret_cast<uintptr_t>(p), false) != pcs::RegionRegistry::kOk)
        return fail(PCS_ERR_INVALID, "not the base of a pcs_host_register region");
    return finish(hipHostUnregister(p), "hipHostUnregister");
}

int pcs_batch_create(pcs_batch** out) {
    if (!out) return fail(PCS_ERR_INVALID, "out is null");
    *out = nullptr;
    if (int rc = require_device()) return rc;
    auto* b = new pcs_batch();
    hipError_t e = hipGetDevice(&b->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&b->done, hipEventDisableTiming);
    if (e != hipSuccess) {
        pcs_batch_destroy(b);
        return hip_fail(e, "pcs_batch_create");
    }
    // result and zero-copy buffers for a service-sized batch up front: no
    // poll of a batch of up to 256 pages ever allocates or frees
    if (int rc = batch_results(b, pcs::kServiceMaxPages)) {
        pcs_batch_destroy(b);
        return rc;
    }
    if (int rc = b->zc.ensure(pcs::kServiceMaxPages)) {
        pcs_batch_destroy(b);
        return rc;
    }
    *out = b;
    return PCS_OK;
}

int pcs_batch_submit(pcs_batch* b, int mode, const void* const* pages, uint64_t P, uint64_t n, int algo) {
    return pcs_batch_submit_ex(b, mode, pages, P, n, algo, PCS_FLAG_NONE);
}

int pcs_batch_submit_ex(pcs_batch* b, int mode, const void* const* pages, uint64_t P, uint64_t n, int algo,
                        uint32_t flags) {
    if (!b) return fail(PCS_ERR_INVALID, "batch is null");
    if (b->state == 1) return fail(PCS_ERR_INVALID, "batch already in flight");
    // From here on the previous batch's results are gone: a submit that fails
    // below leaves the batch idle, so poll/wait/result refuse instead of
    // reporting the last batch's verdicts.
    b->state = 0;
    b->n = 0;
    b->first_bad = UINT64_MAX;
    b->all_ok = false;
    b->svc_results = false;
    b->path = 0;
    if (mode < 0 || mode > 2) return fail(PCS_ERR_INVALID, "bad batch mode");
    if (int rc = check_flags(flags)) return rc;
    if ((flags & PCS_FLAG_SKIP_VERIFY) && mode != PCS_BATCH_VALIDATE)
        return fail(PCS_ERR_INVALID, "PCS_FLAG_SKIP_VERIFY applies to validate batches only");
    if (int rc = check_host_batch_args(pages, P, n, algo)) return rc;
    b->mode = mode;
    b->P = P;
    b->algo = algo;
    b->zero_copy = false;
    if (n == 0 || (flags & PCS_FLAG_SKIP_VERIFY)) {
        // nothing to hash: complete at submit, before any staging is sized
        // (a skipped batch allocates and pins nothing; result() reports 1s)
        b->n = n;
        b->stamp_pages.clear();
        b->all_ok = true;
        b->state = 2;
        return PCS_OK;
    }
    if (injected_failure()) return fail(PCS_ERR_HIP, "injected failure (PCS_TUNE_FAIL_INJECT)");
    b->n = n;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != b->device) (void)hipSetDevice(b->device);
    if (mode != PCS_BATCH_DIGEST && g_services_on.load(std::memory_order_relaxed) > 0) {
        Service* svp = current_service();
        if (svp && svp->device >= 0 && service_shape_ok(P, n, algo)) {
            b->caller = svp;  // counted until the batch completes, on either path
            caller_enter(*svp);
            const int r = service_submit(b->svc, svp, pages, P, n, algo, mode == PCS_BATCH_STAMP);
            if (r == PCS_OK) {
                b->path |= b->svc.path;
                b->svc_pages.assign(pages, pages + n);
                b->via_service = true;
                b->state = 1;
                return PCS_OK;
            }
            if (r < 0) return batch_failed(b, r);
            if (r == kBusy) b->path |= PCS_PATH_LOCK_SKIPPED;
        }
    }
    if (int rc = batch_launch(b, mode, pages, P, n, algo)) return batch_failed(b, rc);
    return PCS_OK;
}

int pcs_batch_poll(pcs_batch* b) {
    if (!b) return fail(PCS_ERR_INVALID, "batch is null");
    if (b->state == 2) return 1;
    if (b->state != 1) return fail(PCS_ERR_INVALID, "no batch submitted");
    if (b->via_service) {
        const int r = batch_service_poll(b);
        if (r != 0 || b->via_service || b->state != 1) return r;
        // moved to the launch path: fall through to its completion check
    }
    if (injected_failure()) {
        (void)hipStreamSynchronize(b->stream);  // nothing of this batch left in flight
        return batch_failed(b, fail(PCS_ERR_HIP, "injected failure (PCS_TUNE_FAIL_INJECT)"));
    }
    if (b->zc_polled) {
        b->zc_landed = verdicts_landed(b->zero_copy ? b->zc.h_ok : b->h_ok, b->zc_landed, b->n);
        if (b->zc_landed == b->n) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return batch_finalize(b);
        }
        // Completion comes from the verdicts; the stream is asked only every
        // kZcEventQueryPolls-th poll, for a launch that failed (the runtime
        // call costs more than a scan of the verdict bytes).
        if (++b->zc_polls % kZcEventQueryPolls != 0) return 0;
    }
    const hipError_t e = b->has_event ? hipEventQuery(b->done) : hipStreamQuery(b->stream);
    if (e == hipErrorNotReady) return 0;
    if (e != hipSuccess) return batch_failed(b, hip_fail(e, "pcs_batch_poll"));
    if (b->zc_polled) {  // the launch has finished: every verdict / done byte must be there now
        b->zc_landed = verdicts_landed(b->zero_copy ? b->zc.h_ok : b->h_ok, b->zc_landed, b->n);
        if (b->zc_landed != b->n)
            return batch_failed(b, fail(PCS_ERR_HIP, "pcs_batch_poll: the launch finished without its results"));
        std::atomic_thread_fence(std::memory_order_acquire);
    }
    return batch_finalize(b);
}

int pcs_batch_wait(pcs_batch* b) {
    if (!b) return fail(PCS_ERR_INVALID, "batch is null");
    if (b->state == 2) return PCS_OK;
    if (b->state != 1) return fail(PCS_ERR_INVALID, "no batch submitted");
    while (b->via_service) {
        const int r = batch_service_poll(b);
        if (r < 0) return r;
        if (r == 1) return PCS_OK;
        if (b->via_service) __builtin_ia32_pause();
    }
    if (injected_failure()) {
        (void)hipStreamSynchronize(b->stream);
        return batch_failed(b, fail(PCS_ERR_HIP, "injected failure (PCS_TUNE_FAIL_INJECT)"));
    }
    const hipError_t e = b->zc_polled ? wait_verdicts(b->zero_copy ? b->zc.h_ok : b->h_ok, b->n, b->stream)
                                      : hipEventSynchronize(b->done);
    if (e != hipSuccess) return batch_failed(b, hip_fail(e, "pcs_batch_wait"));
    batch_finalize(b);
    return PCS_OK;
}

int pcs_batch_result(pcs_batch* b, uint8_t* ok, uint64_t* digests, uint64_t* first_bad) {
    if (!b) return fail(PCS_ERR_INVALID, "batch is null");
    if (b->state != 2) return fail(PCS_ERR_INVALID, "batch not complete");
    if (ok) {
        if (b->mode != PCS_BATCH_VALIDATE) return fail(PCS_ERR_INVALID, "verdicts exist only in validate mode");
        if (b->all_ok)
            std::memset(ok, 1, b->n);
        else if (b->n)
            std::memcpy(ok, b->svc_results ? b->svc_ok.data() : b->h_ok, b->n);
    }
    if (digests) {
        if (b->mode == PCS_BATCH_VALIDATE) return fail(PCS_ERR_INVALID, "digests exist in digest/stamp mode");
        if (b->n) std::memcpy(digests, b->svc_results ? b->svc_dig.data() : b->h_dig, b->n * 8);
    }
    if (first_bad) *first_bad = b->first_bad;
    return PCS_OK;
}

int pcs_batch_path(const pcs_batch* b) { return b ? b->path : 0; }

int pcs_batch_destroy(pcs_batch* b) {
    if (!b) return PCS_OK;
    if (b->via_service) {  // the request owns the device's line: see it answered (or given up) first
        while (service_progress(b->svc) == 0) __builtin_ia32_pause();
        service_release(b->svc);
        b->via_service = false;
    }
    batch_uncount(b);
    if (b->stream) (void)hipStreamSynchronize(b->stream);
    (void)hipHostFree(b->h_pages);
    (void)hipFree(b->d_pages);
    (void)hipHostFree(b->h_dig);
    (void)hipFree(b->d_dig);
    (void)hipHostFree(b->h_ok);
    (void)hipFree(b->d_ok);
    b->zc.release();
    if (b->done) (void)hipEventDestroy(b->done);
    if (b->stream) (void)hipStreamDestroy(b->stream);
    delete b;
    return PCS_OK;
}

int pcs_manifest_checksum_dev(const void* d_content, uint64_t len, uint64_t* d_out, pcs_stream_t stream) {
    if (int rc = require_device()) return rc;
    if (!d_out || (len && !d_content)) return fail(PCS_ERR_INVALID, "null pointer");
    return finish(pcs::run_manifest(static_cast<const uint8_t*>(d_content), len, d_out,
                                    reinterpret_cast<hipStream_t>(stream)),
                  "manifest checksum");
}

int pcs_manifest_checksum_host(const void* content, uint64_t len, uint64_t* out) {
    return manifest_host(content, len, out);
}

int pcs_manifest_validate_host(const void* record, uint64_t size, int* valid) {
    if (!valid || (size && !record)) return fail(PCS_ERR_INVALID, "null pointer");
    constexpr uint64_t kHeaderBytes = 8 + 4 + 4 + 4;  // root_meta.h:61-63
    if (size < kHeaderBytes) {
        *valid = 0;
        return PCS_OK;
    }
    uint64_t h = 0;
    if (int rc = manifest_host(static_cast<const uint8_t*>(record) + 8, size - 8, &h)) return rc;
    uint64_t stored;
    std::memcpy(&stored, record, 8);  // DecodeFixed64
    *valid = stored == h ? 1 : 0;
    return PCS_OK;
}

int pcs_shard_range(uint64_t n, int world, int rank, uint64_t* begin, uint64_t* end) {
    if (!begin || !end) return fail(PCS_ERR_INVALID, "begin/end is null");
    if (world <= 0 || rank < 0 || rank >= world) return fail(PCS_ERR_INVALID, "rank must be in [0, world)");
    const unsigned __int128 N = n;
    *begin = (uint64_t)(N * (unsigned)rank / (unsigned)world);
    *end = (uint64_t)(N * (unsigned)(rank + 1) / (unsigned)world);
    return PCS_OK;
}

int pcs_set_tuning(int key, int64_t value) {
    if (pcs::set_tuning(key, value)) return fail(PCS_ERR_INVALID, "unknown tuning key or negative value");
    return PCS_OK;
}

int64_t pcs_get_tuning(int key) { return pcs::get_tuning(key); }

uint64_t pcs_counter(int which) {
    if (which == PCS_COUNTER_SERVICE_TORN_REQUESTS) return g_torn_requests.load(std::memory_order_relaxed);
    if (which == PCS_COUNTER_SERVICE_REPOSTS) return g_reposts.load(std::memory_order_relaxed);
    return (which < 0 || which > 3) ? 0 : g_counters[which].load(std::memory_order_relaxed);
}

int pcs_gen_pages_dev(void* d_pages, uint64_t page_size, uint64_t n_pages, uint64_t seed, uint64_t first_page_index,
                      pcs_stream_t stream) {
    if (int rc = require_device()) return rc;
    if (page_size == 0 || page_size % 8) return fail(PCS_ERR_INVALID, "page_size must be a positive multiple of 8");
    if (n_pages && !d_pages) return fail(PCS_ERR_INVALID, "d_pages is null");
    return finish(pcs::run_gen_pages(static_cast<uint8_t*>(d_pages), page_size, n_pages, seed, first_page_index,
                                     reinterpret_cast<hipStream_t>(stream)),
                  "gen kernel launch");
}

int pcs_gen_desc_dev(void* d_base, const uint64_t* d_off, const uint32_t* d_len, uint64_t n, uint64_t seed,
                     uint64_t first_page_index, pcs_stream_t stream) {
    if (int rc = require_device()) return rc;
    if (n && (!d_base || !d_off || !d_len)) return fail(PCS_ERR_INVALID, "null descriptor pointer");
    return finish(pcs::run_gen_desc(static_cast<uint8_t*>(d_base), d_off, d_len, n, seed, first_page_index,
                                    reinterpret_cast<hipStream_t>(stream)),
                  "gen kernel launch");
}

int pcs_flip_byte_dev(void* d_pages, uint64_t page_size, uint64_t n_pages, uint64_t every, uint64_t byte_offset,
                      pcs_stream_t stream) {
    if (int rc = require_device()) return rc;
    if (every == 0 || byte_offset >= page_size) return fail(PCS_ERR_INVALID, "every must be > 0, byte_offset < page_size");
    if (n_pages && !d_pages) return fail(PCS_ERR_INVALID, "d_pages is null");
    return finish(pcs::run_flip(static_cast<uint8_t*>(d_pages), page_size, n_pages, every, byte_offset,
                                reinterpret_cast<hipStream_t>(stream)),
                  "flip kernel launch");
}

int pcs_stream_read_dev(const void* d_buf, uint64_t bytes, uint64_t* d_out, pcs_stream_t stream) {
    if (int rc = require_device()) return rc;
    if (bytes && (!d_buf || !d_out)) return fail(PCS_ERR_INVALID, "null pointer");
    if (reinterpret_cast<uintptr_t>(d_buf) % 16) return fail(PCS_ERR_INVALID, "d_buf must be 16-byte aligned");
    const hipError_t e = pcs::run_stream_read(static_cast<const uint8_t*>(d_buf), bytes, d_out,
                                              reinterpret_cast<hipStream_t>(stream));
    if (e == hipErrorNotSupported) return fail(PCS_ERR_INVALID, "bytes too large (more than 2^31 windows)");
    return finish(e, "stream-read kernel launch");
}

}  // extern "C"
