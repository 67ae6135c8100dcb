// x64_ab_lab.cpp — config 3 XXH64 (1 M mixed 4/8/16 KiB descriptors,
// digest) through whichever libeloqstore_pcs.so is named on the command
// line (dlopen), so two builds can be A/B'd in alternating processes on one
// box: round 4's two-launch form (k_xxh64_lds + the flag-gated generic pass)
// against round 5's one launch.  Not part of the product.  Prints the median
// of 7 rounds x 20 launches bracketed by HIP events, and the frac.
//
//   ./x64_ab_lab path/to/libeloqstore_pcs.so
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HIPCHECK(x)                                                                     \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                               \
        }                                                                               \
    } while (0)

static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    if (argc < 2) return 1;
    void* so = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!so) {
        std::fprintf(stderr, "dlopen: %s\n", dlerror());
        return 1;
    }
    using gen_fn = int (*)(void*, const uint64_t*, const uint32_t*, uint64_t, uint64_t, uint64_t, void*);
    using dig_fn = int (*)(const void*, const uint64_t*, const uint32_t*, uint64_t, int, uint64_t*, void*);
    auto gen = reinterpret_cast<gen_fn>(dlsym(so, "pcs_gen_desc_dev"));
    auto dig = reinterpret_cast<dig_fn>(dlsym(so, "pcs_desc_digest_dev"));
    if (!gen || !dig) return 1;
    // config 3's layout (tests/workload.py mixed_layout, seed 0x5EED0003)
    const uint64_t n = 1ull << 20, seed = 0x5EED0003ull;
    const uint32_t cls[3] = {4096, 8192, 16384};
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t p = i ^ seed;
        len[i] = cls[mix(p + (0x5A5A5A5Aull + 1) * 0x9E3779B97F4A7C15ull) % 3];
        off[i] = pos;
        pos += len[i];
    }
    uint8_t* d_base;
    uint64_t *d_off, *d_out;
    uint32_t* d_len;
    HIPCHECK(hipMalloc(&d_base, pos));
    HIPCHECK(hipMalloc(&d_off, n * 8));
    HIPCHECK(hipMalloc(&d_len, n * 4));
    HIPCHECK(hipMalloc(&d_out, n * 8));
    HIPCHECK(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_len, len.data(), n * 4, hipMemcpyHostToDevice));
    if (gen(d_base, d_off, d_len, n, seed, 0, nullptr)) return 1;
    HIPCHECK(hipDeviceSynchronize());
    for (int i = 0; i < 5; ++i)
        if (dig(d_base, d_off, d_len, n, 1, d_out, nullptr)) return 1;
    HIPCHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    HIPCHECK(hipEventCreate(&e0));
    HIPCHECK(hipEventCreate(&e1));
    std::vector<double> t;
    for (int r = 0; r < 7; ++r) {
        HIPCHECK(hipEventRecord(e0, nullptr));
        for (int i = 0; i < 20; ++i) dig(d_base, d_off, d_len, n, 1, d_out, nullptr);
        HIPCHECK(hipEventRecord(e1, nullptr));
        HIPCHECK(hipEventSynchronize(e1));
        float ms = 0;
        HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3 / 20);
    }
    std::sort(t.begin(), t.end());
    const double us = t[t.size() / 2];
    const double alg = (double)pos + 8.0 * n;
    std::printf("%s: config 3 XXH64 digest %.1f us per launch (min %.1f max %.1f), frac %.4f\n", argv[1], us, t.front(),
                t.back(), alg / (us * 1e-6) / 8e12);
    return 0;
}
