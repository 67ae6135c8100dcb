// mailbox_lab.hip — where should the validate service's request line live?
// Not part of the product.  A resident one-workgroup kernel polls a request
// word; the host posts seq and spins on an ack word the kernel stores
// (system scope) into pinned host memory as soon as it sees the post.  The
// round trip is the service's request detection plus its answer path
// without any page read or hash.
//   host   request word in pinned host memory (hipHostMalloc coherent|mapped,
//          the product's mailbox): the kernel polls over PCIe
//   device request word in device memory the host writes through the BAR
//          (hipExtMallocWithFlags fine-grained; the host pointer is the
//          device pointer if the runtime maps it for the CPU): the kernel
//          polls its own HBM / L2, the host's write crosses PCIe once
// Median / p99 of 20,000 round trips after 2,000 warm-up.
//
//   ./mailbox_lab host|device
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HIPCHECK(x)                                                                     \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                               \
        }                                                                               \
    } while (0)

__global__ void k_pingpong(const uint64_t* req, uint64_t* ack, uint64_t n, uint64_t limit_ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t born = __builtin_amdgcn_s_memrealtime();
    uint64_t last = 0;
    while (last < n) {
        const uint64_t v = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v != last) {
            last = v;
            __hip_atomic_store(ack, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (__builtin_amdgcn_s_memrealtime() - born > limit_ticks) break;  // never outlive the run
    }
}

int main(int argc, char** argv) {
    const bool device = argc > 1 && std::strcmp(argv[1], "device") == 0;
    uint64_t* ack = nullptr;
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&ack), 64, hipHostMallocCoherent | hipHostMallocMapped));
    uint64_t* d_ack = nullptr;
    HIPCHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_ack), ack, 0));
    uint64_t* req_host = nullptr;  // what the host writes
    uint64_t* req_dev = nullptr;   // what the kernel reads
    if (device) {
        HIPCHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&req_dev), 64, hipDeviceMallocFinegrained));
        hipPointerAttribute_t at{};
        HIPCHECK(hipPointerGetAttributes(&at, req_dev));
        std::printf("device mailbox: type %d, device ptr %p, host ptr %p\n", (int)at.type, at.devicePointer,
                    at.hostPointer);
        if (!at.hostPointer) {
            std::printf("no host mapping of fine-grained device memory: device mailbox not possible here\n");
            return 0;
        }
        req_host = static_cast<uint64_t*>(at.hostPointer);
    } else {
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&req_host), 64, hipHostMallocCoherent | hipHostMallocMapped));
        HIPCHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&req_dev), req_host, 0));
    }
    __atomic_store_n(req_host, 0, __ATOMIC_SEQ_CST);
    __atomic_store_n(ack, 0, __ATOMIC_SEQ_CST);
    const uint64_t warm = 2000, reps = 20000, n = warm + reps;
    hipStream_t s;
    HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_pingpong, dim3(1), dim3(64), 0, s, req_dev, d_ack, n, (uint64_t)100 * 1000 * 1000 * 20);
    HIPCHECK(hipGetLastError());
    std::vector<double> us;
    us.reserve(reps);
    const auto t_limit = std::chrono::steady_clock::now() + std::chrono::seconds(15);
    for (uint64_t i = 1; i <= n; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(req_host, i, __ATOMIC_RELEASE);
        if (device) __builtin_ia32_sfence();  // WC / uncached mapping: push the store out
        while (__atomic_load_n(ack, __ATOMIC_ACQUIRE) != i) {
            if (std::chrono::steady_clock::now() > t_limit) {
                std::fprintf(stderr, "no ack for %llu after 15 s\n", (unsigned long long)i);
                __atomic_store_n(req_host, n, __ATOMIC_RELEASE);
                HIPCHECK(hipStreamSynchronize(s));
                return 1;
            }
        }
        if (i > warm) us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    HIPCHECK(hipStreamSynchronize(s));
    std::sort(us.begin(), us.end());
    std::printf("%s mailbox: round trip p50 %.2f us  p90 %.2f  p99 %.2f  min %.2f  (%zu trips)\n",
                device ? "device" : "host", us[us.size() / 2], us[us.size() * 9 / 10], us[us.size() * 99 / 100],
                us.front(), us.size());
    return 0;
}
