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
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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

struct Mapped {
    void* p = MAP_FAILED;
    size_t n = 0;
    int fd = -1;
    ~Mapped() {
        if (p != MAP_FAILED) munmap(p, n);
        if (fd >= 0) close(fd);
    }
};

int bulk(bool stamp, const char* path, const char* size_s) {
    uint64_t P = kDefaultPageSize;
    if (size_s && (!parse_u64(size_s, P) || P < 8)) {
        std::fprintf(stderr, "Invalid page size: %s\n", size_s);
        return 1;
    }
    Mapped m;
    m.fd = open(path, stamp ? O_RDWR : O_RDONLY);
    struct stat st;
    if (m.fd < 0 || fstat(m.fd, &st) != 0) {
        std::fprintf(stderr, "Failed to open %s: %s\n", path, std::strerror(errno));
        return 1;
    }
    m.n = (size_t)st.st_size;
    const uint64_t n = m.n / P;
    if (n == 0) {
        std::fprintf(stderr, "File %s holds no whole page of %llu bytes\n", path, (unsigned long long)P);
        return 1;
    }
    m.p = mmap(nullptr, m.n, stamp ? PROT_READ | PROT_WRITE : PROT_READ, MAP_SHARED, m.fd, 0);
    if (m.p == MAP_FAILED) {
        std::fprintf(stderr, "mmap %s: %s\n", path, std::strerror(errno));
        return 1;
    }
    std::vector<char*> pages(n);
    for (uint64_t i = 0; i < n; ++i) pages[i] = static_cast<char*>(m.p) + i * P;
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t bad = 0, first_bad = n;
    if (stamp) {
        eloqstore::SetChecksums(pages, P);
    } else {
        std::vector<uint8_t> ok(n);
        first_bad = eloqstore::ValidateChecksums(std::span<const char* const>(pages.data(), n), P, ok.data());
        for (uint64_t i = 0; i < n; ++i) bad += ok[i] == 0;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double gib = (double)(n * P) / (1024.0 * 1024.0 * 1024.0);
    if (stamp) {
        std::printf("Stamped %llu pages of %llu bytes in %.3f s (%.2f GiB/s incl. host staging)\n",
                    (unsigned long long)n, (unsigned long long)P, s, gib / s);
        return 0;
    }
    std::printf("Scanned %llu pages of %llu bytes: %llu corrupted", (unsigned long long)n, (unsigned long long)P,
                (unsigned long long)bad);
    if (bad) std::printf(", first at offset %llu", (unsigned long long)(first_bad * P));
    std::printf(" (%.3f s, %.2f GiB/s incl. host staging)\n", s, gib / s);
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
    return bulk(true, path, size_s);
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
