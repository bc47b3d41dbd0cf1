// rocPRIM onesweep radix sort of the TD update stream's shape -- 32.2M
// (uint64 key < 2^54, double) pairs -- at the default gfx950 config (8 bits a
// pass: 7 passes) against wider digits (fewer passes).  Prints ms per sort.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

template <class Config>
float run(const uint64_t* k, const double* v, uint64_t* ko, double* vo, size_t n, const char* name) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs<Config>(nullptr, bytes, k, ko, v, vo, n, 0, 54);
    void* tmp;
    if (hipMalloc(&tmp, bytes) != hipSuccess) return -1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 2; w++) (void)rocprim::radix_sort_pairs<Config>(tmp, bytes, k, ko, v, vo, n, 0, 54);
    (void)hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; r++) (void)rocprim::radix_sort_pairs<Config>(tmp, bytes, k, ko, v, vo, n, 0, 54);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // check sortedness
    std::vector<uint64_t> h(n);
    (void)hipMemcpy(h.data(), ko, n * 8, hipMemcpyDeviceToHost);
    bool ok = true;
    for (size_t i = 1; i < n; i++) ok &= h[i - 1] <= h[i];
    printf("%-28s %7.3f ms  sorted=%d  temp=%zu MB\n", name, ms / reps, (int)ok, bytes >> 20);
    (void)hipFree(tmp);
    return ms / reps;
}

template <class O>
using C = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, O>;

int main() {
    const size_t n = 32199510;
    std::vector<uint64_t> hk(n);
    std::mt19937_64 g(7);
    // a skewed key distribution like the TD stream: many repeats of few keys
    for (size_t i = 0; i < n; i++) {
        const uint64_t r = g();
        hk[i] = (r & 7) == 0 ? (r >> 20) % 4096 : (r >> 10) & ((1ull << 54) - 1);
    }
    std::vector<double> hv(n, 1.0);
    uint64_t *k, *ko;
    double *v, *vo;
    (void)hipMalloc(&k, n * 8);
    (void)hipMalloc(&ko, n * 8);
    (void)hipMalloc(&v, n * 8);
    (void)hipMalloc(&vo, n * 8);
    (void)hipMemcpy(k, hk.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(v, hv.data(), n * 8, hipMemcpyHostToDevice);
    using namespace rocprim;
    run<default_config>(k, v, ko, vo, n, "default (8 bits)");
    using M = block_radix_rank_algorithm;
    run<C<radix_sort_onesweep_config<kernel_config<1024, 8>, kernel_config<1024, 8>, 8, M::match>>>(k, v, ko, vo, n, "1024x8, 8 bits");
    run<C<radix_sort_onesweep_config<kernel_config<1024, 8>, kernel_config<1024, 8>, 9, M::match>>>(k, v, ko, vo, n, "1024x8, 9 bits (6 passes)");
    run<C<radix_sort_onesweep_config<kernel_config<1024, 8>, kernel_config<1024, 12>, 9, M::match>>>(k, v, ko, vo, n, "1024x12, 9 bits");
    run<C<radix_sort_onesweep_config<kernel_config<512, 8>, kernel_config<512, 8>, 10, M::match>>>(k, v, ko, vo, n, "512x8, 10 bits (6 passes)");
    run<default_config>(k, v, ko, vo, n, "default again");
    return 0;
}
