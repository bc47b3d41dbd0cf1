// Microbenchmark 4: 64-bit shifts and their 32-bit substitutes on gfx950 (NOT
// product code).  Each asm body is 32 instructions over 4 independent chains.
//   hipcc --offload-arch=gfx950 -O3 -o tools/diag/valu_rate4 tools/diag/valu_rate4.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 2048
#define B8(s) s "\n" s "\n" s "\n" s "\n" s "\n" s "\n" s "\n" s "\n"
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed) {
    unsigned x = seed + threadIdx.x, y = x * 3, z = x * 5, w = x * 7, m = x * 13;
    unsigned long long a = x, b = y, c = z, d = w;
    for (int i = 0; i < ITERS; i++) {
        if (OP == 0) asm volatile(B8("v_lshlrev_b64 %0, 8, %0\n v_lshlrev_b64 %1, 8, %1\n v_lshlrev_b64 %2, 8, %2\n v_lshlrev_b64 %3, 8, %3") : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        if (OP == 1) asm volatile(B8("v_lshrrev_b64 %0, 9, %0\n v_lshrrev_b64 %1, 9, %1\n v_lshrrev_b64 %2, 9, %2\n v_lshrrev_b64 %3, 9, %3") : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        if (OP == 2) asm volatile(B8("v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %1, %1, 0, %2\n v_lshl_add_u64 %2, %2, 0, %3\n v_lshl_add_u64 %3, %3, 0, %0") : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        if (OP == 3) asm volatile(B8("v_alignbit_b32 %0, %0, %1, 24\n v_alignbit_b32 %1, %1, %2, 24\n v_alignbit_b32 %2, %2, %3, 24\n v_alignbit_b32 %3, %3, %0, 24") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 4) asm volatile(B8("v_perm_b32 %0, %0, %1, %4\n v_perm_b32 %1, %1, %2, %4\n v_perm_b32 %2, %2, %3, %4\n v_perm_b32 %3, %3, %0, %4") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(m));
        if (OP == 5) asm volatile(B8("v_lshlrev_b32_e32 %0, 8, %0\n v_lshlrev_b32_e32 %1, 8, %1\n v_lshlrev_b32_e32 %2, 8, %2\n v_lshlrev_b32_e32 %3, 8, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 6) asm volatile(B8("v_bfi_b32 %0, %4, %1, %0\n v_bfi_b32 %1, %4, %2, %1\n v_bfi_b32 %2, %4, %3, %2\n v_bfi_b32 %3, %4, %0, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(m));
        if (OP == 7) asm volatile(B8("v_and_b32_e32 %0, %1, %0\n v_and_b32_e32 %1, %2, %1\n v_and_b32_e32 %2, %3, %2\n v_and_b32_e32 %3, %0, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 8) asm volatile(B8("v_lshlrev_b64 %0, %4, %0\n v_lshlrev_b64 %1, %4, %1\n v_lshlrev_b64 %2, %4, %2\n v_lshlrev_b64 %3, %4, %3") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(m));
        if (OP == 9) asm volatile(B8("v_lshlrev_b64 %0, 8, %0\n v_bfi_b32 %4, %5, %6, %4\n v_bfi_b32 %5, %6, %4, %5\n v_bfi_b32 %6, %4, %5, %6") : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(x), "+v"(y), "+v"(z));
        if (OP == 10) asm volatile(B8("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x80\n v_bitop3_b32 %1, %2, %3, %1 bitop3:0x80\n v_bitop3_b32 %2, %3, %0, %2 bitop3:0x80\n v_bitop3_b32 %3, %0, %1, %3 bitop3:0x80") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 11) asm volatile(B8("v_bfrev_b32_e32 %0, %0\n v_bfrev_b32_e32 %1, %1\n v_bfrev_b32_e32 %2, %2\n v_bfrev_b32_e32 %3, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        // operand patterns swapped between bfi and bitop3 (a bfi is bitop3 0xCA)
        if (OP == 12) asm volatile(B8("v_bitop3_b32 %0, %4, %1, %0 bitop3:0xca\n v_bitop3_b32 %1, %4, %2, %1 bitop3:0xca\n v_bitop3_b32 %2, %4, %3, %2 bitop3:0xca\n v_bitop3_b32 %3, %4, %0, %3 bitop3:0xca") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(m));
        if (OP == 13) asm volatile(B8("v_bfi_b32 %0, %1, %2, %0\n v_bfi_b32 %1, %2, %3, %1\n v_bfi_b32 %2, %3, %0, %2\n v_bfi_b32 %3, %0, %1, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 14) asm volatile(B8("v_or3_b32 %0, %1, %2, %0\n v_or3_b32 %1, %2, %3, %1\n v_or3_b32 %2, %3, %0, %2\n v_or3_b32 %3, %0, %1, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 16) asm volatile(B8("v_add_co_u32_e32 %0, vcc, %2, %0\n v_addc_co_u32_e32 %1, vcc, %3, %1, vcc\n v_add_co_u32_e32 %2, vcc, %0, %2\n v_addc_co_u32_e32 %3, vcc, %1, %3, vcc") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) :: "vcc");
        if (OP == 17) asm volatile(B8("v_bcnt_u32_b32 %0, %1, 0\n v_bcnt_u32_b32 %1, %2, 0\n v_bcnt_u32_b32 %2, %3, 0\n v_bcnt_u32_b32 %3, %0, 0") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 18) asm volatile(B8("v_cndmask_b32_e32 %0, %1, %0, vcc\n v_cndmask_b32_e32 %1, %2, %1, vcc\n v_cndmask_b32_e32 %2, %3, %2, vcc\n v_cndmask_b32_e32 %3, %0, %3, vcc") : "+v"(x), "+v"(y), "+v"(z), "+v"(w) :: "vcc");
        if (OP == 19) asm volatile(B8("v_and_or_b32 %0, %1, %2, %0\n v_and_or_b32 %1, %2, %3, %1\n v_and_or_b32 %2, %3, %0, %2\n v_and_or_b32 %3, %0, %1, %3") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        if (OP == 15) asm volatile(B8("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xca\n v_bitop3_b32 %1, %2, %3, %1 bitop3:0xca\n v_bitop3_b32 %2, %3, %0, %2 bitop3:0xca\n v_bitop3_b32 %3, %0, %1, %3 bitop3:0xca") : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
    }
    out[blockIdx.x * 256 + threadIdx.x] = x ^ y ^ z ^ w ^ (unsigned)a ^ (unsigned)b ^ (unsigned)c ^ (unsigned)d;
}

template <int OP> float run(unsigned* out, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k<OP><<<blocks, 256>>>(out, 1);
    (void)hipEventRecord(e0);
    k<OP><<<blocks, 256>>>(out, 1);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    unsigned* out;
    (void)hipMalloc(&out, (size_t)8192 * 256 * 4);
    const char* names[] = {"lshlrev_b64 imm", "lshrrev_b64 imm", "lshl_add_u64", "alignbit_b32", "perm_b32",
                           "lshlrev_b32", "bfi_b32", "and_b32", "lshlrev_b64 vgpr amt", "1 shl_b64 + 3 bfi",
                           "bitop3_b32 (and3)", "bfrev_b32", "bitop3 0xca, bfi's operands", "bfi, bitop3's operands",
                           "or3_b32", "bitop3 0xca, own operands", "add_co/addc_co e32 (2/64-bit add)",
                           "bcnt_u32", "cndmask_e32 vcc", "and_or_b32"};
    for (int i = 0; i < 3; i++) run<0>(out, 2048);  // clock ramp
    for (int blocks : {2048}) {
        printf("-- %d waves/SIMD\n", blocks / 256);
        float t[20];
        t[0] = run<0>(out, blocks); t[1] = run<1>(out, blocks); t[2] = run<2>(out, blocks); t[3] = run<3>(out, blocks);
        t[4] = run<4>(out, blocks); t[5] = run<5>(out, blocks); t[6] = run<6>(out, blocks); t[7] = run<7>(out, blocks);
        t[8] = run<8>(out, blocks); t[9] = run<9>(out, blocks); t[10] = run<10>(out, blocks); t[11] = run<11>(out, blocks);
        t[12] = run<12>(out, blocks); t[13] = run<13>(out, blocks); t[14] = run<14>(out, blocks); t[15] = run<15>(out, blocks);
        t[16] = run<16>(out, blocks); t[17] = run<17>(out, blocks); t[18] = run<18>(out, blocks); t[19] = run<19>(out, blocks);
        for (int op = 0; op < 20; op++) {
            const double winstr = (double)blocks * 4 * ITERS * 32;
            printf("  %-24s %.3f ms  %.2f cyc/instr/SIMD @2.4GHz\n", names[op], t[op],
                   1024 * 2.4e9 / (winstr / (t[op] * 1e-3)));
        }
    }
    return 0;
}
