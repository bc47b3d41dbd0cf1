// Microbenchmark 3: selects, compares, 64-bit helpers on gfx950 (NOT product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 2048
#define B8(s) s "\n" s "\n" s "\n" s "\n" s "\n" s "\n" s "\n" s "\n"
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed) {
    unsigned x = seed + threadIdx.x, y = x * 3, z = x * 5, w = x * 7, m = x * 13;
    unsigned long long a = x, b = y;
    for (int i = 0; i < ITERS; i++) {
        // each asm body = 32 instructions
        if (OP == 0) asm volatile(B8("v_cndmask_b32_e32 %0, %1, %0, vcc\n v_cndmask_b32_e32 %1, %2, %1, vcc\n v_cndmask_b32_e32 %2, %3, %2, vcc\n v_cndmask_b32_e32 %3, %0, %3, vcc") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) :: "vcc");
        if (OP == 1) asm volatile("s_mov_b64 s[40:41], exec\n" B8("v_cndmask_b32_e64 %0, %1, %0, s[40:41]\n v_cndmask_b32_e64 %1, %2, %1, s[40:41]\n v_cndmask_b32_e64 %2, %3, %2, s[40:41]\n v_cndmask_b32_e64 %3, %0, %3, s[40:41]") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) :: "s40", "s41");
        if (OP == 2) asm volatile(B8("v_cmp_gt_u32_e32 vcc, %0, %1\n v_cndmask_b32_e32 %2, %3, %2, vcc\n v_cmp_gt_u32_e32 vcc, %1, %2\n v_cndmask_b32_e32 %3, %0, %3, vcc") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) :: "vcc");
        if (OP == 3) asm volatile(B8("v_cmp_gt_u32_e64 s[40:41], %0, %1\n v_cndmask_b32_e64 %2, %3, %2, s[40:41]\n v_cmp_gt_u32_e64 s[42:43], %1, %2\n v_cndmask_b32_e64 %3, %0, %3, s[42:43]") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) :: "s40", "s41", "s42", "s43");
        if (OP == 4) asm volatile(B8("v_bfi_b32 %0, %4, %1, %0\n v_bfi_b32 %1, %4, %2, %1\n v_bfi_b32 %2, %4, %3, %2\n v_bfi_b32 %3, %4, %0, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(m));
        if (OP == 5) asm volatile(B8("v_bcnt_u32_b32 %0, %1, 0\n v_bcnt_u32_b32 %1, %2, 0\n v_bcnt_u32_b32 %2, %3, 0\n v_bcnt_u32_b32 %3, %0, 0") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 6) asm volatile(B8("v_ffbh_u32_e32 %0, %1\n v_ffbh_u32_e32 %1, %2\n v_ffbl_b32_e32 %2, %3\n v_ffbl_b32_e32 %3, %0") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 7) asm volatile(B8("v_sub_co_u32_e32 %0, vcc, 0, %0\n v_subb_co_u32_e32 %1, vcc, 0, %1, vcc\n v_sub_co_u32_e32 %2, vcc, 0, %2\n v_subb_co_u32_e32 %3, vcc, 0, %3, vcc") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) :: "vcc");
        if (OP == 8) asm volatile(B8("v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %1, %1, 0, %0\n v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %1, %1, 0, %0") : "+v"(a), "+v"(b));
        if (OP == 9) asm volatile(B8("v_mul_lo_u32 %0, %1, %0\n v_mul_lo_u32 %1, %2, %1\n v_mul_lo_u32 %2, %3, %2\n v_mul_lo_u32 %3, %0, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 10) asm volatile(B8("v_cmp_ne_u64_e32 vcc, 0, %0\n v_cmp_ne_u64_e32 vcc, 0, %1\n v_cmp_ne_u64_e32 vcc, 0, %0\n v_cmp_ne_u64_e32 vcc, 0, %1") : "+v"(a), "+v"(b) :: "vcc");
        if (OP == 11) asm volatile(B8("v_mov_b32_e32 %0, %1\n v_mov_b32_e32 %1, %2\n v_mov_b32_e32 %2, %3\n v_mov_b32_e32 %3, %0") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 12) asm volatile(B8("v_and_b32_e32 %0, %1, %0\n v_lshlrev_b64 %4, 8, %4\n v_or_b32_e32 %2, %3, %2\n v_and_b32_e32 %3, %0, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w), "+v"(a));
        if (OP == 13) asm volatile(B8("v_and_b32_e32 %0, %1, %0\n v_and_b32_e32 %1, %2, %1\n v_and_b32_e32 %2, %3, %2\n v_lshlrev_b64 %4, 8, %4") : "+v"(x), "+v"(y), "+v"(z), "+v"(w), "+v"(a));
        if (OP == 14) asm volatile(B8("v_and_b32_e32 %0, %1, %0\n v_and_b32_e32 %1, %2, %1\n v_and_b32_e32 %2, %3, %2\n v_and_b32_e32 %3, %0, %3\n") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 15) asm volatile(B8("v_and_b32_e32 %0, %1, %0\n v_and_b32_e32 %1, %0, %1\n v_and_b32_e32 %0, %1, %0\n v_and_b32_e32 %1, %0, %1\n") : "+v"(x), "+v"(y));
    }
    out[blockIdx.x * 256 + threadIdx.x] = x ^ y ^ z ^ w ^ (unsigned)a ^ (unsigned)b;
}

template <int OP> float run(unsigned* out, int blocks) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    k<OP><<<blocks, 256>>>(out, 1);
    hipEventRecord(e0);
    k<OP><<<blocks, 256>>>(out, 1);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    unsigned* out; hipMalloc(&out, (size_t)8192 * 256 * 4);
    const char* names[] = {"cndmask_e32 vcc", "cndmask_e64 s-pair", "cmp+cndmask vcc", "cmp_e64+cndmask_e64 s", "bfi_b32 vgpr mask", "bcnt_u32", "ffbh/ffbl", "sub_co/subb_co", "lshl_add_u64", "mul_lo_u32", "cmp_ne_u64", "mov_b32", "3 vop2 + 1 shl_b64 (mix)", "3 vop2 + 1 shl_b64 (dep)", "and only (4 chains)", "and only (2 chains, dependent)"};
    for (int blocks : {512, 1024, 2048}) {
        printf("-- %d waves/SIMD\n", blocks / 256);
        float t[16];
        t[0] = run<0>(out, blocks); t[1] = run<1>(out, blocks); t[2] = run<2>(out, blocks); t[3] = run<3>(out, blocks);
        t[4] = run<4>(out, blocks); t[5] = run<5>(out, blocks); t[6] = run<6>(out, blocks); t[7] = run<7>(out, blocks);
        t[8] = run<8>(out, blocks); t[9] = run<9>(out, blocks); t[10] = run<10>(out, blocks); t[11] = run<11>(out, blocks);
        t[12] = run<12>(out, blocks); t[13] = run<13>(out, blocks); t[14] = run<14>(out, blocks); t[15] = run<15>(out, blocks);
        for (int op = 0; op < 16; op++) {
            double winstr = (double)blocks * 4 * ITERS * 32;
            printf("  %-28s %.3f ms  %.2f cyc/instr/SIMD @2.4GHz\n", names[op], t[op], 1024 * 2.4e9 / (winstr / (t[op] * 1e-3)));
        }
    }
    return 0;
}
