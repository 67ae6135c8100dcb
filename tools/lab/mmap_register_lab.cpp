// mmap_register_lab.cpp — can a whole-file scrub read the page cache in place?
// Not part of the product.
//
// Maps a file of 4 KiB pages, tries hipHostRegister on the mapping with the
// flag sets a read-only scrub could use, and, where one succeeds, validates
// every page with pcs_pages_validate_dev on the mapped device pointer (the
// GPU reading the page cache over PCIe, no CPU copy).  Prints registration
// time, validate time and the rate; the pread pipeline of
// page_checksum_tool --scan is the comparison (tools/lab/scan_lab.sh).
//
//   ./tools/lab/mmap_register_lab <file>
#include <hip/hip_runtime.h>

#include "eloqstore_pcs.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

static void attempt(const char* name, const char* path, int oflags, int prot, unsigned hflags) {
    const int fd = open(path, oflags);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) {
        std::printf("%-40s open failed\n", name);
        return;
    }
    const size_t len = (size_t)st.st_size;
    void* p = mmap(nullptr, len, prot, MAP_SHARED | MAP_POPULATE, fd, 0);
    if (p == MAP_FAILED) {
        std::printf("%-40s mmap failed\n", name);
        close(fd);
        return;
    }
    const auto t0 = clk::now();
    const hipError_t e = hipHostRegister(p, len, hflags);
    const auto t1 = clk::now();
    if (e != hipSuccess) {
        std::printf("%-40s hipHostRegister: %s (%.1f ms)\n", name, hipGetErrorString(e), ms(t0, t1));
        (void)hipGetLastError();
        munmap(p, len);
        close(fd);
        return;
    }
    void* d = nullptr;
    (void)hipHostGetDevicePointer(&d, p, 0);
    const uint64_t n = len / 4096;
    uint8_t* ok = nullptr;
    unsigned long long* fb = nullptr;
    (void)hipMalloc(&ok, n);
    (void)hipMalloc(&fb, 8);
    double best = 1e30;
    int rc = 0;
    for (int r = 0; r < 4; ++r) {
        const auto a = clk::now();
        rc |= pcs_pages_validate_dev(d, 4096, n, PCS_XXH3_64, ok, reinterpret_cast<uint64_t*>(fb), nullptr);
        rc |= pcs_synchronize(nullptr);
        const auto b = clk::now();
        if (ms(a, b) < best) best = ms(a, b);
    }
    unsigned long long h_fb = 0;
    (void)hipMemcpy(&h_fb, fb, 8, hipMemcpyDeviceToHost);
    std::printf("%-40s registered in %.1f ms; validate %.2f ms = %.2f GiB/s (rc %d, first_bad %llu)\n", name, ms(t0, t1),
                best, (double)len / (1 << 30) / (best / 1e3), rc, h_fb);
    (void)hipFree(ok);
    (void)hipFree(fb);
    const auto u0 = clk::now();
    (void)hipHostUnregister(p);
    std::printf("%-40s unregistered in %.1f ms\n", name, ms(u0, clk::now()));
    munmap(p, len);
    close(fd);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <file>\n", argv[0]);
        return 1;
    }
    (void)hipSetDevice(0);
    attempt("ro mapping, Mapped|ReadOnly", argv[1], O_RDONLY, PROT_READ, hipHostRegisterMapped | hipHostRegisterReadOnly);
    attempt("ro mapping, Mapped", argv[1], O_RDONLY, PROT_READ, hipHostRegisterMapped);
    attempt("rw shared mapping, Mapped", argv[1], O_RDWR, PROT_READ | PROT_WRITE, hipHostRegisterMapped);
    return 0;
}
