// Memory-ceiling probe for the step kernel: the same per-board byte mix as
// oth_step (read boards 16 B + turn 1 B + move 1 B; write boards 16 B + turn
// 1 B + flips 8 B + legal 8 B + ret 1 B = 52 B/board) with trivial compute, so
// the achieved rate is the layout's HBM ceiling.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -o tools/diag/step_bw tools/diag/step_bw.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void copy16(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ b, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) b[i] = a[i];
}

// one board per thread, exactly oth_step's access pattern
__global__ __launch_bounds__(256) void mix1(const ulonglong2* __restrict__ bi, const uint8_t* __restrict__ ti,
                                            const uint8_t* __restrict__ mi, ulonglong2* __restrict__ bo,
                                            uint8_t* __restrict__ to, u64* __restrict__ fo, u64* __restrict__ lo,
                                            int8_t* __restrict__ ro, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 b = bi[i];
    const unsigned t = ti[i], m = mi[i];
    bo[i] = make_ulonglong2(b.x ^ m, b.y + t);
    to[i] = (uint8_t)(t ^ 3);
    fo[i] = b.x & b.y;
    lo[i] = ~(b.x | b.y);
    ro[i] = (int8_t)(m + t);
}

// boards 16 B moved as two 8-B streams per lane (black/white planes are still
// interleaved in memory; this only changes the instruction width)
__global__ __launch_bounds__(256) void mix1_nt(const ulonglong2* __restrict__ bi, const uint8_t* __restrict__ ti,
                                               const uint8_t* __restrict__ mi, ulonglong2* __restrict__ bo,
                                               uint8_t* __restrict__ to, u64* __restrict__ fo, u64* __restrict__ lo,
                                               int8_t* __restrict__ ro, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    typedef u64 v2 __attribute__((ext_vector_type(2)));
    const v2 bv = __builtin_nontemporal_load(reinterpret_cast<const v2*>(bi) + i);
    const ulonglong2 b = make_ulonglong2(bv.x, bv.y);
    const unsigned t = __builtin_nontemporal_load(&ti[i]), m = __builtin_nontemporal_load(&mi[i]);
    v2 ov;
    ov.x = b.x ^ m;
    ov.y = b.y + t;
    __builtin_nontemporal_store(ov, reinterpret_cast<v2*>(bo) + i);
    __builtin_nontemporal_store((uint8_t)(t ^ 3), &to[i]);
    __builtin_nontemporal_store(b.x & b.y, &fo[i]);
    __builtin_nontemporal_store(~(b.x | b.y), &lo[i]);
    __builtin_nontemporal_store((int8_t)(m + t), &ro[i]);
}

// reads only / writes only, to split the two directions
__global__ __launch_bounds__(256) void rd_only(const ulonglong2* __restrict__ bi, const uint8_t* __restrict__ ti,
                                               const uint8_t* __restrict__ mi, u64* __restrict__ sink, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 b = bi[i];
    const u64 v = b.x ^ b.y ^ ti[i] ^ ((u64)mi[i] << 8);
    if (v == 0x123456789ull) sink[0] = v;
}
__global__ __launch_bounds__(256) void wr_only(ulonglong2* __restrict__ bo, uint8_t* __restrict__ to,
                                               u64* __restrict__ fo, u64* __restrict__ lo, int8_t* __restrict__ ro,
                                               int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    bo[i] = make_ulonglong2(i, i);
    to[i] = (uint8_t)i;
    fo[i] = i;
    lo[i] = i;
    ro[i] = (int8_t)i;
}

template <class F>
static float timeit(F f, int reps = 20) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) f();
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / reps;  // us
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : (1ll << 24);
    ulonglong2 *bi, *bo;
    uint8_t *ti, *mi, *to;
    int8_t* ro;
    u64 *fo, *lo, *sink;
    CK(hipMalloc(&bi, n * 16));
    CK(hipMalloc(&bo, n * 16));
    CK(hipMalloc(&ti, n));
    CK(hipMalloc(&mi, n));
    CK(hipMalloc(&to, n));
    CK(hipMalloc(&ro, n));
    CK(hipMalloc(&fo, n * 8));
    CK(hipMalloc(&lo, n * 8));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(bi, 1, n * 16));
    CK(hipMemset(ti, 1, n));
    CK(hipMemset(mi, 19, n));
    const unsigned g = (unsigned)((n + 255) / 256);
    float us;
    us = timeit([&] { copy16<<<g, 256>>>(bi, bo, n); });
    printf("copy16   %8.1f us  %.2f TB/s (32 B/board)\n", us, n * 32.0 / us / 1e6);
    us = timeit([&] { mix1<<<g, 256>>>(bi, ti, mi, bo, to, fo, lo, ro, n); });
    printf("mix1     %8.1f us  %.2f TB/s (52 B/board)\n", us, n * 52.0 / us / 1e6);
    us = timeit([&] { mix1_nt<<<g, 256>>>(bi, ti, mi, bo, to, fo, lo, ro, n); });
    printf("mix1_nt  %8.1f us  %.2f TB/s (52 B/board)\n", us, n * 52.0 / us / 1e6);
    us = timeit([&] { rd_only<<<g, 256>>>(bi, ti, mi, sink, n); });
    printf("rd_only  %8.1f us  %.2f TB/s (18 B/board)\n", us, n * 18.0 / us / 1e6);
    us = timeit([&] { wr_only<<<g, 256>>>(bo, to, fo, lo, ro, n); });
    printf("wr_only  %8.1f us  %.2f TB/s (34 B/board)\n", us, n * 34.0 / us / 1e6);
    CK(hipDeviceSynchronize());
    return 0;
}
