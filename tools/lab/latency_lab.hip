// latency_lab.hip — where does a small host batch's wall time go?
//   empty kernel launch + hipStreamSynchronize / + event spin
//   zero-copy validate of 1 / 16 / 128 / 256 registered 4 KiB pages
//   staged (gather) validate of the same pages, unregistered
// Experiment harness, not part of the product.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "eloqstore_pcs.h"

__global__ void k_empty() {}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename F>
static double median_us(F&& f, int reps = 300) {
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
        const double t0 = now_us();
        f();
        t.push_back(now_us() - t0);
    }
    std::sort(t.begin() + 0, t.end());
    return t[t.size() / 2];
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    printf("empty launch + hipStreamSynchronize : %6.1f us\n", median_us([&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
               hipStreamSynchronize(s);
           }));
    printf("empty launch + event query spin     : %6.1f us\n", median_us([&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
               hipEventRecord(ev, s);
               while (hipEventQuery(ev) == hipErrorNotReady) {
               }
           }));
    printf("hipStreamSynchronize (idle)         : %6.1f us\n", median_us([&] { hipStreamSynchronize(s); }));

    const size_t P = 4096, N = 1024;
    void* pool = std::aligned_alloc(4096, N * P);
    void* loose = std::aligned_alloc(4096, N * P);
    std::mt19937_64 rng(1);
    for (size_t i = 0; i < N * P / 8; ++i) static_cast<uint64_t*>(pool)[i] = rng();
    std::memcpy(loose, pool, N * P);
    if (pcs_host_register(pool, N * P)) {
        printf("register failed: %s\n", pcs_last_error());
        return 1;
    }
    std::vector<size_t> perm(N);
    for (size_t i = 0; i < N; ++i) perm[i] = i;
    std::shuffle(perm.begin(), perm.end(), rng);
    std::vector<uint8_t> ok(N);
    uint64_t fb;
    for (int inl : {1, 0})
    for (size_t nb : {1, 16, 128, 256}) {
        pcs_set_tuning(PCS_TUNE_INLINE_LIST, inl);
        std::vector<const void*> zp(nb), gp(nb);
        for (size_t i = 0; i < nb; ++i) {
            zp[i] = static_cast<uint8_t*>(pool) + perm[i] * P;
            gp[i] = static_cast<uint8_t*>(loose) + perm[i] * P;
        }
        const double z = median_us([&] { pcs_pages_validate_host(zp.data(), P, nb, PCS_XXH3_64, ok.data(), &fb); });
        const double g = median_us([&] { pcs_pages_validate_host(gp.data(), P, nb, PCS_XXH3_64, ok.data(), &fb); });
        pcs_batch* b;
        pcs_batch_create(&b);
        const double a = median_us([&] {
            pcs_batch_submit(b, PCS_BATCH_VALIDATE, zp.data(), P, nb, PCS_XXH3_64);
            while (pcs_batch_poll(b) == 0) {
            }
        });
        const double sub = median_us([&] {
            pcs_batch_submit(b, PCS_BATCH_VALIDATE, zp.data(), P, nb, PCS_XXH3_64);
            pcs_batch_wait(b);
        });
        pcs_batch_destroy(b);
        printf("inline=%d %4zu pages: zero-copy sync %6.1f us | async poll %6.1f | async wait %6.1f | staged %6.1f us\n", inl, nb, z, a,
               sub, g);
    }
    pcs_host_unregister(pool);
    return 0;
}
