// Microbenchmark: cost of one Kogge-Stone step (4 independent directions interleaved)
// in three encodings, at 1..4 waves/SIMD (NOT product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 2048
typedef unsigned long long u64;
template <int V>
__global__ __launch_bounds__(256) void k(u64* out, u64 seed) {
    u64 g0 = seed + threadIdx.x, g1 = g0 * 3, g2 = g0 * 5, g3 = g0 * 7;
    u64 p0 = g0 ^ 0x5555, p1 = g1 ^ 0x3333, p2 = g2 ^ 0x0F0F, p3 = g3 ^ 0x7777;
    for (int i = 0; i < ITERS; i++) {
#define STEP_BFI(g, p, S) { u64 t; asm volatile("v_lshlrev_b64 %0, " #S ", %1" : "=v"(t) : "v"(g)); \
        unsigned lo, hi; asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(lo) : "v"((unsigned)p), "v"((unsigned)t), "v"((unsigned)g)); \
        asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(hi) : "v"((unsigned)(p>>32)), "v"((unsigned)(t>>32)), "v"((unsigned)(g>>32))); g = ((u64)hi << 32) | lo; }
#define STEP_ANDOR(g, p, S) { u64 t; asm volatile("v_lshlrev_b64 %0, " #S ", %1" : "=v"(t) : "v"(g)); \
        unsigned lo, hi; asm volatile("v_and_or_b32 %0, %1, %2, %3" : "=v"(lo) : "v"((unsigned)p), "v"((unsigned)t), "v"((unsigned)g)); \
        asm volatile("v_and_or_b32 %0, %1, %2, %3" : "=v"(hi) : "v"((unsigned)(p>>32)), "v"((unsigned)(t>>32)), "v"((unsigned)(g>>32))); g = ((u64)hi << 32) | lo; }
#define STEP_VOP2(g, p, S) { u64 t; asm volatile("v_lshlrev_b64 %0, " #S ", %1" : "=v"(t) : "v"(g)); \
        unsigned a, b; asm volatile("v_and_b32_e32 %0, %1, %2" : "=v"(a) : "v"((unsigned)p), "v"((unsigned)t)); \
        asm volatile("v_and_b32_e32 %0, %1, %2" : "=v"(b) : "v"((unsigned)(p>>32)), "v"((unsigned)(t>>32))); \
        asm volatile("v_or_b32_e32 %0, %1, %2" : "=v"(a) : "v"(a), "v"((unsigned)g)); \
        asm volatile("v_or_b32_e32 %0, %1, %2" : "=v"(b) : "v"(b), "v"((unsigned)(g>>32))); g = ((u64)b << 32) | a; }
        if (V == 0) { STEP_BFI(g0, p0, 1) STEP_BFI(g1, p1, 8) STEP_BFI(g2, p2, 9) STEP_BFI(g3, p3, 7) }
        if (V == 1) { STEP_ANDOR(g0, p0, 1) STEP_ANDOR(g1, p1, 8) STEP_ANDOR(g2, p2, 9) STEP_ANDOR(g3, p3, 7) }
        if (V == 2) { STEP_VOP2(g0, p0, 1) STEP_VOP2(g1, p1, 8) STEP_VOP2(g2, p2, 9) STEP_VOP2(g3, p3, 7) }
    }
    out[blockIdx.x * 256 + threadIdx.x] = g0 ^ g1 ^ g2 ^ g3;
}
template <int V> float run(u64* out, int blocks) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    k<V><<<blocks, 256>>>(out, 1);
    hipEventRecord(e0);
    for (int r = 0; r < 3; r++) k<V><<<blocks, 256>>>(out, 1);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / 3;
}
int main() {
    u64* out; hipMalloc(&out, (size_t)8192 * 256 * 8);
    const char* names[] = {"shift+2 bfi", "shift+2 and_or", "shift+2 and+2 or (VOP2)"};
    const int ninstr[] = {3, 3, 5};
    for (int blocks : {256, 512, 768, 1024}) {
        float t[3] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks)};
        for (int v = 0; v < 3; v++) {
            double steps = (double)blocks * 4 * ITERS * 4;  // wave-level KS steps
            double ns_per_step_simd = t[v] * 1e6 / (steps / 1024);
            printf("%d waves/SIMD  %-26s %.3f ms  %.2f cyc/KS-step/SIMD  %.2f cyc/instr @2.4GHz\n", blocks / 256, names[v], t[v],
                   ns_per_step_simd * 2.4, ns_per_step_simd * 2.4 / ninstr[v]);
        }
    }
    return 0;
}
