// tail_lab.hip — launch ramp / tail of the config-2 XXH3 page kernel.
// Not part of the product.
//
// The product kernel (k_xxh3_fixed<4096, kDigest>) runs one 256-thread block
// per 16-page tile: 65,536 blocks for config 2.  Config 5 (8x the pages) runs
// at 93 % of spec against config 2's 90-91 %, i.e. about 14 us of fixed cost
// per launch.  This harness (1) instruments the product body with per-block
// wall-clock stamps and the XCC id to show where that time goes (dispatch
// ramp, per-XCD finish spread), and (2) times persistent-grid alternatives:
//   static      product schedule (block per tile, XCD-contiguous tiles)
//   pstatic     persistent grid, each XCD's blocks stride over its eighth
//   pdyn        persistent grid, per-XCD atomic tile queue (ticket for the
//               next tile taken while the current one loads), steal from
//               the other XCDs' queues when the own one runs dry
// All variants produce the product's digests (checked against each other).
//
//   make -C tools/lab tail_lab && ./tools/lab/tail_lab [rounds]
#include <hip/hip_runtime.h>

#include "xxh3_page.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

using namespace pcs;

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xF;
}
__device__ __forceinline__ uint32_t hw_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(x));
    return x;
}

// one tile = 16 pages of P bytes, digests staged in LDS, one coalesced store
template <int P>
__device__ __forceinline__ void do_tile(const uint8_t* __restrict__ pages, uint64_t n, uint64_t t, const Xxh3Lane& L,
                                        uint64_t* __restrict__ out, uint64_t* tile_h) {
    const int grp = threadIdx.x >> 4;
    const uint64_t pg = t * 16 + grp;
    if (pg < n) {
        uint64_t stored;
        u32x4 first;
        const uint64_t h = xxh3_page_fixed<P, true>(pages + pg * (uint64_t)P, L, stored, first);
        if (L.g == 0) tile_h[grp] = h;
    }
    __syncthreads();
    const uint64_t i = t * 16 + threadIdx.x;
    if (threadIdx.x < 16 && i < n) st_nt(out + i, tile_h[threadIdx.x]);
    __syncthreads();
}

struct Stamp {
    uint64_t t0, t1;
    uint32_t xcc, hw;
};

template <int P, bool INSTR>
__global__ __launch_bounds__(256) void k_static(const uint8_t* __restrict__ pages, uint64_t n,
                                               uint64_t* __restrict__ out, Stamp* st) {
    __shared__ uint64_t tile_h[16];
    uint64_t t0 = 0;
    if (INSTR) t0 = (uint64_t)wall_clock64();
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    do_tile<P>(pages, n, xcd_tile(blockIdx.x, ntiles), L, out, tile_h);
    if (INSTR && threadIdx.x == 0) {
        Stamp s{t0, (uint64_t)wall_clock64(), xcc_id(), hw_id()};
        st[blockIdx.x] = s;
    }
}

// persistent, static: XCD x = blockIdx % 8 (round-robin dispatch) owns tiles
// [x*nt/8, (x+1)*nt/8); its blocks stride over them.
template <int P>
__global__ __launch_bounds__(256) void k_pstatic(const uint8_t* __restrict__ pages, uint64_t n,
                                                uint64_t* __restrict__ out) {
    __shared__ uint64_t tile_h[16];
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    const uint32_t x = blockIdx.x % 8, per = gridDim.x / 8, k = blockIdx.x / 8;
    const uint64_t lo = x * ntiles / 8, hi = (x + 1) * ntiles / 8;
    for (uint64_t t = lo + k; t < hi; t += per) do_tile<P>(pages, n, t, L, out, tile_h);
}

// persistent, dynamic: per-XCD queue heads q[8] (zeroed before the launch),
// each 128 B apart.  Queue x hands out tiles lo_x + ticket.  A block takes
// the ticket for its next tile before processing the current one.
template <int P, bool HWXCC>
__global__ __launch_bounds__(256) void k_pdyn(const uint8_t* __restrict__ pages, uint64_t n,
                                             uint64_t* __restrict__ out, unsigned long long* q) {
    __shared__ uint64_t tile_h[16];
    __shared__ long long s_next;
    const Xxh3Lane L = make_xxh3_lane(threadIdx.x & 15);
    const uint64_t ntiles = (n + 15) / 16;
    const uint32_t home = HWXCC ? xcc_id() : blockIdx.x % 8;
    auto grab = [&](uint32_t& xq) -> long long {  // thread 0 only
        for (int probe = 0; probe < 8; ++probe) {
            const uint32_t x = (xq + probe) % 8;
            const uint64_t lo = x * ntiles / 8, hi = (x + 1) * ntiles / 8;
            unsigned long long* h = q + 16 * x;
            if (__hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= hi - lo) continue;
            const unsigned long long tk = atomicAdd(h, 1ull);
            if (tk < hi - lo) {
                xq = x;
                return (long long)(lo + tk);
            }
        }
        return -1;
    };
    uint32_t xq = home;
    if (threadIdx.x == 0) s_next = grab(xq);
    __syncthreads();
    long long cur = s_next;
    while (cur >= 0) {
        __syncthreads();  // everyone has read s_next
        if (threadIdx.x == 0) s_next = grab(xq);
        do_tile<P>(pages, n, (uint64_t)cur, L, out, tile_h);  // ends with a barrier: s_next visible
        cur = s_next;
    }
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 9;
    constexpr int P = 4096;
    const uint64_t n = 1ull << 20, ntiles = n / 16, bytes = n * P;
    uint8_t* pages;
    uint64_t *out, *ref;
    unsigned long long* q;
    Stamp* st;
    CK(hipMalloc(&pages, bytes));
    CK(hipMalloc(&out, n * 8));
    CK(hipMalloc(&ref, n * 8));
    CK(hipMalloc(&q, 8 * 128));
    CK(hipMalloc(&st, ntiles * sizeof(Stamp)));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(pages), bytes / 8);
    int cus = 0, wclk = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0));  // kHz
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_static<P, false>, 256, 0));
    std::printf("CUs %d, wall clock %d kHz, static occupancy %d blocks/CU\n", cus, wclk, occ);

    // ---- (1) instrumented product schedule
    hipLaunchKernelGGL((k_static<P, false>), dim3(ntiles), dim3(256), 0, 0, pages, n, ref, st);
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL((k_static<P, true>), dim3(ntiles), dim3(256), 0, 0, pages, n, out, st);
        CK(hipDeviceSynchronize());
        std::vector<Stamp> h(ntiles);
        CK(hipMemcpy(h.data(), st, ntiles * sizeof(Stamp), hipMemcpyDeviceToHost));
        uint64_t t0 = ~0ull, t1 = 0;
        for (auto& s : h) t0 = std::min(t0, s.t0), t1 = std::max(t1, s.t1);
        const double us = 1e3 / wclk;  // ticks -> us
        std::printf("instrumented run %d: span %.1f us\n", rep, (t1 - t0) * us);
        std::vector<double> xs0(8, 1e30), xs1(8, 0), xdur(8, 0);
        std::vector<long> xn(8, 0);
        std::vector<double> ends, starts, durs;
        for (auto& s : h) {
            const int x = s.xcc;
            xs0[x] = std::min(xs0[x], (s.t0 - t0) * us);
            xs1[x] = std::max(xs1[x], (s.t1 - t0) * us);
            xdur[x] += (s.t1 - s.t0) * us;
            xn[x]++;
            ends.push_back((s.t1 - t0) * us);
            starts.push_back((s.t0 - t0) * us);
            durs.push_back((s.t1 - s.t0) * us);
        }
        for (int x = 0; x < 8; ++x)
            std::printf("  xcc %d: blocks %6ld  first start %6.2f  last end %7.1f  mean block %.2f us\n", x, xn[x],
                        xs0[x], xs1[x], xn[x] ? xdur[x] / xn[x] : 0.0);
        std::sort(ends.begin(), ends.end());
        std::sort(starts.begin(), starts.end());
        std::sort(durs.begin(), durs.end());
        const size_t N = ends.size();
        std::printf("  start of block #%d (chip full): %.2f us; block #%zu start %.2f\n", cus * occ,
                    starts[std::min(N - 1, (size_t)cus * occ)], N / 2, starts[N / 2]);
        std::printf("  ends: 90%% %.1f  99%% %.1f  99.9%% %.1f  last %.1f us\n", ends[N * 90 / 100], ends[N * 99 / 100],
                    ends[N * 999 / 1000], ends[N - 1]);
        std::printf("  block duration: p10 %.2f  median %.2f  p90 %.2f  p99 %.2f  max %.2f us\n", durs[N / 10],
                    durs[N / 2], durs[N * 9 / 10], durs[N * 99 / 100], durs[N - 1]);
        // active blocks in the last 20 us of the span
        const double span = (t1 - t0) * us;
        for (double w : {40.0, 20.0, 10.0, 5.0}) {
            long act = 0;
            for (size_t i = 0; i < N; ++i)
                if (ends[i] > span - w) ++act;
            std::printf("  blocks still running in the last %.0f us: %ld\n", w, act);
        }
    }

    // ---- (2) timed variants, interleaved
    struct V {
        std::string name;
        int kind;  // 0 static, 1 pstatic, 2 pdyn(blockIdx), 3 pdyn(hw xcc)
        int per_cu;
    };
    std::vector<V> vs = {{"static (product)", 0, 0}};
    for (int pc : {4, 8})
        vs.push_back({"pstatic x" + std::to_string(pc), 1, pc}), vs.push_back({"pdyn x" + std::to_string(pc), 2, pc}),
            vs.push_back({"pdyn-hwxcc x" + std::to_string(pc), 3, pc});
    auto launch = [&](const V& v) {
        if (v.kind == 0) {
            hipLaunchKernelGGL((k_static<P, false>), dim3(ntiles), dim3(256), 0, 0, pages, n, out, st);
        } else if (v.kind == 1) {
            hipLaunchKernelGGL((k_pstatic<P>), dim3(cus * v.per_cu), dim3(256), 0, 0, pages, n, out);
        } else {
            CK(hipMemsetAsync(q, 0, 8 * 128, 0));
            if (v.kind == 2)
                hipLaunchKernelGGL((k_pdyn<P, false>), dim3(cus * v.per_cu), dim3(256), 0, 0, pages, n, out, q);
            else
                hipLaunchKernelGGL((k_pdyn<P, true>), dim3(cus * v.per_cu), dim3(256), 0, 0, pages, n, out, q);
        }
    };
    for (auto& v : vs) {
        CK(hipMemset(out, 0, n * 8));
        launch(v);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> a(n), b(n);
        CK(hipMemcpy(a.data(), out, n * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), ref, n * 8, hipMemcpyDeviceToHost));
        if (a != b) {
            std::printf("PARITY FAIL: %s\n", v.name.c_str());
            return 1;
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ts(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            CK(hipEventRecord(e0, 0));
            launch(vs[i]);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts[i].push_back(ms);
        }
    for (size_t i = 0; i < vs.size(); ++i) {
        auto t = ts[i];
        std::sort(t.begin(), t.end());
        const float med = t[t.size() / 2];
        std::printf("  %-20s med %7.1f us  %7.1f GB/s  best %7.1f GB/s\n", vs[i].name.c_str(), med * 1e3,
                    (bytes + n * 8) / (med * 1e-3) / 1e9, (bytes + n * 8) / (t[0] * 1e-3) / 1e9);
    }

    // ---- (3) K back-to-back launches: per-launch events vs two events
    for (int K : {20, 50}) {
        for (int mode = 0; mode < 2; ++mode) {
            std::vector<hipEvent_t> ev(2 * K);
            for (auto& e : ev) CK(hipEventCreate(&e));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int k = 0; k < K; ++k) {
                if (mode) CK(hipEventRecord(ev[2 * k], 0));
                launch(vs[0]);
                if (mode) CK(hipEventRecord(ev[2 * k + 1], 0));
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            double sum = 0;
            if (mode)
                for (int k = 0; k < K; ++k) {
                    float m;
                    CK(hipEventElapsedTime(&m, ev[2 * k], ev[2 * k + 1]));
                    sum += m;
                }
            std::printf("  K=%d %-22s %.1f us/step%s\n", K, mode ? "per-launch events" : "two events", ms * 1e3 / K,
                        mode ? (" (launch avg " + std::to_string(sum * 1e3 / K) + " us)").c_str() : "");
            for (auto& e : ev) CK(hipEventDestroy(e));
        }
    }
    return 0;
}
