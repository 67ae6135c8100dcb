// page_checksum_tool — GPU-backed, contract-compatible replacement for the
// reference CLI (tools/page_checksum_tool.cpp:47-123).
//
//   page_checksum_tool <file_path> <offset_bytes> [page_size_bytes]
//       Reference contract: numbers parsed like std::stoull(s, &idx, 0) with the
//       whole string consumed (decimal, 0x hex, leading-0 octal); page size 0
//       rejected; default page size 4096 (KvOptions::data_page_size,
//       include/kv_options.h:184); [offset, offset+P) must lie inside the file.
//       Prints "Checksum OK|FAILED for page at offset <dec>", then
//       "Page bytes (offset:value)" and a hex dump (16 bytes per row,
//       "%06x: " + "%02x " each).  Exit 0 = OK, 2 = FAILED, 1 = usage / IO error.
//
// Added modes (not in the reference):
//   page_checksum_tool --scan  <file_path> [page_size]   validate every page
//   page_checksum_tool --stamp <file_path> [page_size]   SetChecksum on every page
//   page_checksum_tool --gen   <file_path> <n_pages> [page_size] [seed]
//       write n synthetic pages (splitmix64 words, see include/eloqstore_pcs.h)
//       and stamp them.
//   --scan/--stamp print a summary line with the GiB/s of the call; exit codes
//   as above (--scan: 2 if any page is corrupted).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "eloqstore/page_checksum.h"
#include "eloqstore_pcs.h"

namespace {

bool parse_u64(const char* s, uint64_t& out) {
    try {
        size_t idx = 0;
        const std::string str(s);
        const unsigned long long v = std::stoull(str, &idx, 0);
        if (idx != str.size()) return false;
        out = v;
        return true;
    } catch (...) {
        return false;
    }
}

void usage(const char* prog) {
    std::fprintf(stderr,
                 "Usage: %s <file_path> <offset_bytes> [page_size_bytes]\n"
                 "Offset and page size accept decimal or 0x-prefixed hex values.\n"
                 "       %s --scan|--stamp <file_path> [page_size_bytes]\n"
                 "       %s --gen <file_path> <n_pages> [page_size_bytes] [seed]\n",
                 prog, prog, prog);
}

constexpr uint64_t kDefaultPageSize = 4096;  // KvOptions{}.data_page_size

int single_page(const char* path, const char* off_s, const char* size_s) {
    uint64_t offset = 0, P = kDefaultPageSize;
    if (!parse_u64(off_s, offset)) {
        std::fprintf(stderr, "Invalid offset: %s\n", off_s);
        return 1;
    }
    if (size_s && (!parse_u64(size_s, P) || P == 0)) {
        std::fprintf(stderr, "Invalid page size: %s\n", size_s);
        return 1;
    }
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        std::fprintf(stderr, "Failed to open %s: %s\n", path, std::strerror(errno));
        return 1;
    }
    std::fseek(f, 0, SEEK_END);
    const uint64_t fsize = (uint64_t)std::ftell(f);
    if (offset + P > fsize) {
        std::fprintf(stderr, "Requested range [%llu, %llu) exceeds file size %llu\n", (unsigned long long)offset,
                     (unsigned long long)(offset + P), (unsigned long long)fsize);
        std::fclose(f);
        return 1;
    }
    std::vector<char> page(P);
    std::fseek(f, (long)offset, SEEK_SET);
    const size_t got = std::fread(page.data(), 1, P, f);
    std::fclose(f);
    if (got != P) {
        std::fprintf(stderr, "Unable to read %llu bytes at offset %llu\n", (unsigned long long)P,
                     (unsigned long long)offset);
        return 1;
    }
    const bool ok = eloqstore::ValidateChecksum(std::string_view(page.data(), P));
    std::printf("%s for page at offset %llu\n", ok ? "Checksum OK" : "Checksum FAILED", (unsigned long long)offset);
    std::printf("Page bytes (offset:value)\n");
    for (uint64_t i = 0; i < P; i += 16) {
        std::printf("%06llx: ", (unsigned long long)i);
        for (uint64_t j = 0; j < 16 && i + j < P; ++j) std::printf("%02x ", (unsigned)(uint8_t)page[i + j]);
        std::printf("\n");
    }
    return ok ? 0 : 2;
}

// Whole-file scrub / stamp: the file is read with pread into two pinned
// 64 MiB buffers and each chunk goes to the GPU as an asynchronous batch
// (pcs_batch_*); a contiguous pinned run is DMA'd in place, so the host does
// no gather copy.  Reading chunk k+1 overlaps checking chunk k.
struct Fd {
    int fd = -1;
    ~Fd() {
        if (fd >= 0) close(fd);
    }
};

bool pread_full(int fd, char* buf, uint64_t len, uint64_t off) {
    while (len) {
        const ssize_t r = pread(fd, buf, len, (off_t)off);
        if (r <= 0) return false;
        buf += r;
        len -= (uint64_t)r;
        off += (uint64_t)r;
    }
    return true;
}

bool pwrite_full(int fd, const char* buf, uint64_t len, uint64_t off) {
    while (len) {
        const ssize_t r = pwrite(fd, buf, len, (off_t)off);
        if (r <= 0) return false;
        buf += r;
        len -= (uint64_t)r;
        off += (uint64_t)r;
    }
    return true;
}

// pread of one chunk split over a few threads: a single thread's copy out of
// the page cache (~6 GiB/s) would otherwise bound the scrub.
// PCS_SCAN_THREADS / PCS_SCAN_PIECE_MIB / PCS_SCAN_CHUNK_MIB override the
// reader threads (16, at most the host's), the read piece (4 MiB) and the
// chunk per batch (64 MiB); tools/lab/scan_lab.sh sweeps them: 16 x 4 MiB
// against 8 x 8 MiB: 19.2-19.8 vs 13.5-14.9 GiB/s on a 1 GiB file, 25-31 vs
// 27.5 on 4 GiB; 128 MiB chunks slower (profiles/r02/scan_lab.txt).
uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* v = std::getenv(name);
    uint64_t x;
    return v && parse_u64(v, x) && x > 0 ? x : dflt;
}

bool pread_parallel(int fd, char* buf, uint64_t len, uint64_t off) {
    static const uint64_t kThreads =
        env_u64("PCS_SCAN_THREADS", std::min<uint64_t>(16, std::max(1u, std::thread::hardware_concurrency())));
    static const uint64_t kPiece = env_u64("PCS_SCAN_PIECE_MIB", 4) << 20;
    const unsigned T = (unsigned)std::min<uint64_t>(kThreads, (len + kPiece - 1) / kPiece);
    if (T <= 1) return pread_full(fd, buf, len, off);
    std::vector<std::thread> th;
    std::vector<char> ok(T, 1);
    for (unsigned k = 0; k < T; ++k) {
        const uint64_t b = len * k / T, e = len * (k + 1) / T;
        th.emplace_back([&, k, b, e] { ok[k] = pread_full(fd, buf + b, e - b, off + b); });
    }
    for (auto& x : th) x.join();
    return std::all_of(ok.begin(), ok.end(), [](char c) { return c != 0; });
}

int bulk(bool stamp, const char* path, const char* size_s) {
    uint64_t P = kDefaultPageSize;
    if (size_s && (!parse_u64(size_s, P) || P < 8)) {
        std::fprintf(stderr, "Invalid page size: %s\n", size_s);
        return 1;
    }
    Fd f;
    f.fd = open(path, stamp ? O_RDWR : O_RDONLY);
    struct stat st;
    if (f.fd < 0 || fstat(f.fd, &st) != 0) {
        std::fprintf(stderr, "Failed to open %s: %s\n", path, std::strerror(errno));
        return 1;
    }
    const uint64_t n = (uint64_t)st.st_size / P;
    if (n == 0) {
        std::fprintf(stderr, "File %s holds no whole page of %llu bytes\n", path, (unsigned long long)P);
        return 1;
    }
    const uint64_t chunk = std::max<uint64_t>(1, (env_u64("PCS_SCAN_CHUNK_MIB", 64) << 20) / P);
    void* buf[2] = {nullptr, nullptr};
    pcs_batch* batch[2] = {nullptr, nullptr};
    int rc = 0;
    for (int k = 0; k < 2 && !rc; ++k) {
        rc = pcs_host_alloc_pinned(chunk * P, &buf[k]);
        if (!rc) rc = pcs_batch_create(&batch[k]);
    }
    if (rc) {
        std::fprintf(stderr, "GPU setup failed (%d): %s\n", rc, pcs_last_error());
        return 1;
    }
    std::vector<const void*> ptrs[2];
    std::vector<uint8_t> ok(chunk);
    uint64_t first[2] = {0, 0}, count[2] = {0, 0}, bad = 0, first_bad = n;
    bool busy[2] = {false, false};
    auto collect = [&](int k) -> bool {
        if (!busy[k]) return true;
        busy[k] = false;
        if (pcs_batch_wait(batch[k])) return false;
        if (stamp) return pwrite_full(f.fd, static_cast<char*>(buf[k]), count[k] * P, first[k] * P);
        uint64_t fb = UINT64_MAX;
        if (pcs_batch_result(batch[k], ok.data(), nullptr, &fb)) return false;
        for (uint64_t i = 0; i < count[k]; ++i) bad += ok[i] == 0;
        if (fb != UINT64_MAX) first_bad = std::min(first_bad, first[k] + fb);
        return true;
    };
    {
        // warm the GPU path (code-object load, first launch) before the clock
        // starts: ~30 ms that would otherwise land on the first chunk of a
        // scrub (a long-running service pays it once)
        std::memset(buf[0], 0, (size_t)P);
        const void* one = buf[0];
        if (pcs_batch_submit(batch[0], stamp ? PCS_BATCH_DIGEST : PCS_BATCH_VALIDATE, &one, P, 1,
                             PCS_XXH3_64) == PCS_OK)
            (void)pcs_batch_wait(batch[0]);
    }
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t k = 0;
    for (uint64_t p0 = 0; p0 < n; p0 += chunk, ++k) {
        const int s = (int)(k & 1);
        if (!collect(s)) {
            rc = 1;
            break;
        }
        const uint64_t cnt = std::min(chunk, n - p0);
        char* b = static_cast<char*>(buf[s]);
        if (!pread_parallel(f.fd, b, cnt * P, p0 * P)) {
            std::fprintf(stderr, "read failed at offset %llu: %s\n", (unsigned long long)(p0 * P), std::strerror(errno));
            rc = 1;
            break;
        }
        ptrs[s].resize(cnt);
        for (uint64_t i = 0; i < cnt; ++i) ptrs[s][i] = b + i * P;
        if (pcs_batch_submit(batch[s], stamp ? PCS_BATCH_STAMP : PCS_BATCH_VALIDATE, ptrs[s].data(), P, cnt,
                             PCS_XXH3_64)) {
            rc = 1;
            break;
        }
        first[s] = p0;
        count[s] = cnt;
        busy[s] = true;
    }
    for (int s = 0; s < 2; ++s)
        if (!collect(s)) rc = 1;
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int s = 0; s < 2; ++s) {
        pcs_batch_destroy(batch[s]);
        pcs_host_free_pinned(buf[s]);
    }
    if (rc) {
        std::fprintf(stderr, "%s failed: %s\n", stamp ? "stamp" : "scan", pcs_last_error());
        return 1;
    }
    const double gib = (double)(n * P) / (1024.0 * 1024.0 * 1024.0);
    if (stamp) {
        std::printf("Stamped %llu pages of %llu bytes in %.3f s (%.2f GiB/s incl. file I/O)\n", (unsigned long long)n,
                    (unsigned long long)P, secs, gib / secs);
        return 0;
    }
    std::printf("Scanned %llu pages of %llu bytes: %llu corrupted", (unsigned long long)n, (unsigned long long)P,
                (unsigned long long)bad);
    if (bad) std::printf(", first at offset %llu", (unsigned long long)(first_bad * P));
    std::printf(" (%.3f s, %.2f GiB/s incl. file I/O)\n", secs, gib / secs);
    return bad ? 2 : 0;
}

int gen(const char* path, const char* n_s, const char* size_s, const char* seed_s) {
    uint64_t n = 0, P = kDefaultPageSize, seed = 0x5EED0001;
    if (!parse_u64(n_s, n) || n == 0 || (size_s && (!parse_u64(size_s, P) || P < 8 || P % 8)) ||
        (seed_s && !parse_u64(seed_s, seed))) {
        std::fprintf(stderr, "Invalid --gen arguments\n");
        return 1;
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        std::fprintf(stderr, "Failed to open %s: %s\n", path, std::strerror(errno));
        return 1;
    }
    std::vector<uint64_t> page(P / 8);
    for (uint64_t p = 0; p < n; ++p) {
        for (uint64_t w = 0; w < P / 8; ++w) {
            uint64_t z = (seed ^ p) + (w + 1) * 0x9E3779B97F4A7C15ull;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            page[w] = z ^ (z >> 31);
        }
        if (std::fwrite(page.data(), 1, P, f) != P) {
            std::fprintf(stderr, "write failed: %s\n", std::strerror(errno));
            std::fclose(f);
            return 1;
        }
    }
    std::fclose(f);
    return bulk(true, path, size_s);  // stamp the pages just written
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 2 && (!std::strcmp(argv[1], "--scan") || !std::strcmp(argv[1], "--stamp"))) {
        if (argc < 3 || argc > 4) {
            usage(argv[0]);
            return 1;
        }
        return bulk(argv[1][2] == 's' && argv[1][3] == 't', argv[2], argc == 4 ? argv[3] : nullptr);
    }
    if (argc >= 2 && !std::strcmp(argv[1], "--gen")) {
        if (argc < 4 || argc > 6) {
            usage(argv[0]);
            return 1;
        }
        return gen(argv[2], argv[3], argc > 4 ? argv[4] : nullptr, argc > 5 ? argv[5] : nullptr);
    }
    if (argc < 3 || argc > 4) {
        usage(argv[0]);
        return 1;
    }
    return single_page(argv[1], argv[2], argc == 4 ? argv[3] : nullptr);
}
