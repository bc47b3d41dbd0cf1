// Microbenchmark 2: which VALU encodings issue at the full wave64 rate on gfx950 (NOT product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 4096
#define B8(s) s "\n" s "\n" s "\n" s "\n" s "\n" s "\n" s "\n" s "\n"
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed, int wave_mul) {
    unsigned x = seed + threadIdx.x, y = x * 3, z = x * 5, w = x * 7, s0 = seed * 11;
    unsigned long long a = x, b = y;
    for (int i = 0; i < ITERS; i++) {
        if (OP == 0) asm volatile(B8("v_and_b32_e32 %0, %1, %0\n v_and_b32_e32 %1, %2, %1\n v_and_b32_e32 %2, %3, %2\n v_and_b32_e32 %3, %0, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 1) asm volatile(B8("v_and_b32_e64 %0, %1, %0\n v_and_b32_e64 %1, %2, %1\n v_and_b32_e64 %2, %3, %2\n v_and_b32_e64 %3, %0, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 2) asm volatile(B8("v_and_b32_e32 %0, 0x7e7e7e7e, %0\n v_and_b32_e32 %1, 0x7e7e7e7e, %1\n v_and_b32_e32 %2, 0x7e7e7e7e, %2\n v_and_b32_e32 %3, 0x7e7e7e7e, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 3) asm volatile(B8("v_and_b32_e32 %0, %4, %0\n v_and_b32_e32 %1, %4, %1\n v_and_b32_e32 %2, %4, %2\n v_and_b32_e32 %3, %4, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "s"(s0));
        if (OP == 4) asm volatile(B8("v_lshlrev_b32_e32 %0, 7, %0\n v_lshrrev_b32_e32 %1, 9, %1\n v_lshlrev_b32_e32 %2, 1, %2\n v_lshrrev_b32_e32 %3, 8, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 5) asm volatile(B8("v_cndmask_b32_e32 %0, %1, %0, vcc\n v_cndmask_b32_e32 %1, %2, %1, vcc\n v_cndmask_b32_e32 %2, %3, %2, vcc\n v_cndmask_b32_e32 %3, %0, %3, vcc") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 6) asm volatile(B8("v_add_u32_e32 %0, %1, %0\n v_add_u32_e32 %1, %2, %1\n v_add_u32_e32 %2, %3, %2\n v_add_u32_e32 %3, %0, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 7) asm volatile(B8("v_not_b32_e32 %0, %1\n v_not_b32_e32 %1, %2\n v_not_b32_e32 %2, %3\n v_not_b32_e32 %3, %0") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 8) asm volatile(B8("v_or3_b32 %0, %1, %2, %0\n v_or3_b32 %1, %2, %3, %1\n v_or3_b32 %2, %3, %0, %2\n v_or3_b32 %3, %0, %1, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 9) asm volatile(B8("v_lshlrev_b64 %0, 7, %0\n v_lshrrev_b64 %1, 9, %1\n v_lshlrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 8, %1") : "+v"(a), "+v"(b));
        if (OP == 10) asm volatile(B8("v_pk_mov_b32 %0, %1, %0 op_sel:[0,1]\n v_pk_mov_b32 %1, %0, %1 op_sel:[0,1]\n v_pk_mov_b32 %0, %1, %0 op_sel:[0,1]\n v_pk_mov_b32 %1, %0, %1 op_sel:[0,1]") : "+v"(a), "+v"(b));
        if (OP == 11) asm volatile(B8("v_xor_b32_e32 %0, %1, %0\n v_or_b32_e32 %1, %2, %1\n v_and_b32_e32 %2, %3, %2\n v_xor_b32_e32 %3, %0, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
    }
    out[blockIdx.x * 256 + threadIdx.x] = x ^ y ^ z ^ w ^ (unsigned)a ^ (unsigned)b;
}

template <int OP> float run(unsigned* out, int blocks) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    k<OP><<<blocks, 256>>>(out, 1, 1);
    hipEventRecord(e0);
    k<OP><<<blocks, 256>>>(out, 1, 1);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    unsigned* out; hipMalloc(&out, (size_t)8192 * 256 * 4);
    const char* names[] = {"and_e32 (VOP2)", "and_e64 (VOP3)", "and_e32 literal", "and_e32 sgpr", "lshl/lshr_b32 e32", "cndmask_e32", "add_u32_e32", "not_b32 (VOP1)", "or3_b32 (VOP3)", "lshl/lshr_b64", "pk_mov_b32", "xor/or/and mix e32"};
    for (int blocks : {256, 512, 1024, 2048}) {  // 1,2,4,8 waves per SIMD
        printf("-- %d blocks of 256 (%d waves/SIMD)\n", blocks, blocks / 256);
        float t[12];
        t[0] = run<0>(out, blocks); t[1] = run<1>(out, blocks); t[2] = run<2>(out, blocks); t[3] = run<3>(out, blocks);
        t[4] = run<4>(out, blocks); t[5] = run<5>(out, blocks); t[6] = run<6>(out, blocks); t[7] = run<7>(out, blocks);
        t[8] = run<8>(out, blocks); t[9] = run<9>(out, blocks); t[10] = run<10>(out, blocks); t[11] = run<11>(out, blocks);
        for (int op = 0; op < 12; op++) {
            double winstr = (double)blocks * 4 * ITERS * 32;
            printf("  %-20s %.3f ms  %.3e wave-instr/s = %.2f cyc/instr/SIMD @2.4GHz\n", names[op], t[op], winstr / (t[op] * 1e-3),
                   1024 * 2.4e9 / (winstr / (t[op] * 1e-3)));
        }
    }
    return 0;
}
