// stamp_readback_lab.cpp — LAB (not part of the library): what reading back
// the headers of a just-stamped batch costs the shard thread.
//
// An asynchronous stamp the validate service answered returns its digests by
// reading every page's header once the done words have landed
// (pcs_capi.cpp, batch_service_poll: DecodeFixed64 of each header).  Those
// headers were just written by the GPU over PCIe, so each read is a miss to
// DRAM on a line the device wrote.  This lab stamps batches of 1-256 random
// pages of a registered 1 GiB pool through the service (SetChecksums, which
// does not read the headers back), then times one read of those headers, the
// same loop the library runs, against:
//   - the same loop over headers the CPU itself just wrote (page.cpp's
//     SetChecksum; the lines are in this core's cache);
//   - the same loop over headers nobody touched for a while (cold lines);
//   - a contiguous copy of n 8-byte words (what a digest array would cost).
// Prints per-batch microseconds (median of R repetitions) and, for 256-page
// batches, the shard CPU that read costs per GiB stamped.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <span>
#include <vector>

#include "eloqstore/page_checksum.h"
#include "eloqstore_pcs.h"
#include "xxh_oracle.h"  // the CPU stamp (page.cpp's SetChecksum, restated)

namespace {
using Clock = std::chrono::steady_clock;
constexpr size_t P = 4096;
constexpr size_t kPages = 262144;  // 1 GiB

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// the library's loop: one 8-byte load per page header
__attribute__((noinline)) uint64_t read_headers(char* const* pages, size_t n, uint64_t* out) {
    uint64_t x = 0;
    for (size_t i = 0; i < n; ++i) {
        std::memcpy(&out[i], pages[i], 8);
        x ^= out[i];
    }
    return x;
}

double us_since(Clock::time_point t0) { return std::chrono::duration<double, std::micro>(Clock::now() - t0).count(); }

double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}
}  // namespace

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 400;
    char* pool = static_cast<char*>(std::aligned_alloc(4096, kPages * P));
    if (!pool) return 1;
    uint64_t seed = 7;
    for (size_t i = 0; i < kPages * P / 8; ++i) reinterpret_cast<uint64_t*>(pool)[i] = splitmix(seed);
    eloqstore::RegisterPagePool(pool, kPages * P);
    if (pcs_thread_prepare() != PCS_OK) return 1;
    eloqstore::StartChecksumService(2, 1000, 1);
    std::vector<uint64_t> out(256), sink(256);
    uint64_t guard = 0;
    std::printf("pages  device_written_us  cpu_written_us  cold_us  contiguous_copy_us  served\n");
    for (size_t n : {1, 8, 32, 64, 128, 256}) {
        std::vector<double> dev, cpu, cold, copy;
        uint64_t served0 = pcs_counter(PCS_COUNTER_SERVICE_BATCHES), calls = 0;
        for (int r = 0; r < reps; ++r) {
            std::vector<char*> pages(n);
            for (auto& p : pages) p = pool + (splitmix(seed) % kPages) * P;
            std::sort(pages.begin(), pages.end());
            pages.erase(std::unique(pages.begin(), pages.end()), pages.end());
            const size_t m = pages.size();
            // device-written: a stamp through the service, then the read-back
            eloqstore::SetChecksums(std::span<char* const>(pages.data(), m), P);
            ++calls;
            auto t0 = Clock::now();
            guard ^= read_headers(pages.data(), m, out.data());
            dev.push_back(us_since(t0));
            // CPU-written: the same pages' headers stamped here, then read
            for (char* p : pages) oracle_set_checksum(p, P);
            t0 = Clock::now();
            guard ^= read_headers(pages.data(), m, out.data());
            cpu.push_back(us_since(t0));
            // cold: another random set nobody wrote recently
            std::vector<char*> other(m);
            for (auto& p : other) p = pool + (splitmix(seed) % kPages) * P;
            t0 = Clock::now();
            guard ^= read_headers(other.data(), m, out.data());
            cold.push_back(us_since(t0));
            // a contiguous array of m digests
            t0 = Clock::now();
            std::memcpy(sink.data(), out.data(), m * 8);
            guard ^= sink[m - 1];
            copy.push_back(us_since(t0));
        }
        const double served = (double)(pcs_counter(PCS_COUNTER_SERVICE_BATCHES) - served0) / (double)calls;
        std::printf("%5zu  %17.2f  %14.2f  %7.2f  %18.3f  %6.3f\n", n, median(dev), median(cpu), median(cold), median(copy),
                    served);
        if (n == 256)
            std::printf("256-page stamps: reading back the device-written headers costs %.4f shard-CPU s per GiB "
                        "stamped (%.4f for headers in this core's cache)\n",
                        median(dev) * 1e-6 * (1024.0 * 1024 * 1024 / (256.0 * P)),
                        median(cpu) * 1e-6 * (1024.0 * 1024 * 1024 / (256.0 * P)));
    }
    eloqstore::StopChecksumService();
    eloqstore::UnregisterPagePool(pool);
    std::free(pool);
    std::printf("stamp readback lab ok (%llx)\n", (unsigned long long)(guard & 1));
    return 0;
}
