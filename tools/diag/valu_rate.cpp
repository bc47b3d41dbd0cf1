// Microbenchmark: issue rate of the VALU ops the bitboard kernels use (NOT product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 4096
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned long long* out, unsigned long long seed) {
    unsigned long long a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7;
    unsigned x = (unsigned)a, y = (unsigned)b, z = (unsigned)c, w = (unsigned)d;
    for (int i = 0; i < ITERS; i++) {
        if (OP == 0) {  // 8 x v_lshlrev_b64
            asm volatile("v_lshlrev_b64 %0, 1, %0\n v_lshlrev_b64 %1, 7, %1\n v_lshlrev_b64 %2, 8, %2\n v_lshlrev_b64 %3, 9, %3\n"
                         "v_lshlrev_b64 %0, 1, %0\n v_lshlrev_b64 %1, 7, %1\n v_lshlrev_b64 %2, 8, %2\n v_lshlrev_b64 %3, 9, %3\n"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        } else if (OP == 1) {  // 8 x v_and_b32
            asm volatile("v_and_b32 %0, %1, %0\n v_and_b32 %1, %2, %1\n v_and_b32 %2, %3, %2\n v_and_b32 %3, %0, %3\n"
                         "v_and_b32 %0, %1, %0\n v_and_b32 %1, %2, %1\n v_and_b32 %2, %3, %2\n v_and_b32 %3, %0, %3\n"
                         : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        } else if (OP == 2) {  // 8 x v_lshrrev_b64
            asm volatile("v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 7, %1\n v_lshrrev_b64 %2, 8, %2\n v_lshrrev_b64 %3, 9, %3\n"
                         "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 7, %1\n v_lshrrev_b64 %2, 8, %2\n v_lshrrev_b64 %3, 9, %3\n"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        } else if (OP == 3) {  // 8 x v_bcnt_u32_b32
            asm volatile("v_bcnt_u32_b32 %0, %1, %0\n v_bcnt_u32_b32 %1, %2, %1\n v_bcnt_u32_b32 %2, %3, %2\n v_bcnt_u32_b32 %3, %0, %3\n"
                         "v_bcnt_u32_b32 %0, %1, %0\n v_bcnt_u32_b32 %1, %2, %1\n v_bcnt_u32_b32 %2, %3, %2\n v_bcnt_u32_b32 %3, %0, %3\n"
                         : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        } else if (OP == 4) {  // 8 x v_or3_b32
            asm volatile("v_or3_b32 %0, %1, %2, %0\n v_or3_b32 %1, %2, %3, %1\n v_or3_b32 %2, %3, %0, %2\n v_or3_b32 %3, %0, %1, %3\n"
                         "v_or3_b32 %0, %1, %2, %0\n v_or3_b32 %1, %2, %3, %1\n v_or3_b32 %2, %3, %0, %2\n v_or3_b32 %3, %0, %1, %3\n"
                         : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        } else if (OP == 5) {  // 8 x v_alignbit_b32 (32-bit funnel shift)
            asm volatile("v_alignbit_b32 %0, %1, %0, 7\n v_alignbit_b32 %1, %2, %1, 9\n v_alignbit_b32 %2, %3, %2, 1\n v_alignbit_b32 %3, %0, %3, 8\n"
                         "v_alignbit_b32 %0, %1, %0, 7\n v_alignbit_b32 %1, %2, %1, 9\n v_alignbit_b32 %2, %3, %2, 1\n v_alignbit_b32 %3, %0, %3, 8\n"
                         : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        } else if (OP == 6) {  // 8 x v_and_b32 with a 2-wide dependency-free pattern + v_bfi
            asm volatile("v_bfi_b32 %0, %1, %2, %0\n v_bfi_b32 %1, %2, %3, %1\n v_bfi_b32 %2, %3, %0, %2\n v_bfi_b32 %3, %0, %1, %3\n"
                         "v_bfi_b32 %0, %1, %2, %0\n v_bfi_b32 %1, %2, %3, %1\n v_bfi_b32 %2, %3, %0, %2\n v_bfi_b32 %3, %0, %1, %3\n"
                         : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d ^ x ^ y ^ z ^ w;
}

int main() {
    const int blocks = 256 * 16;  // 16 waves... 4 waves/block -> 64 waves/CU requested; capped by residency
    unsigned long long* out; hipMalloc(&out, (size_t)blocks * 256 * 8);
    const char* names[] = {"v_lshlrev_b64", "v_and_b32", "v_lshrrev_b64", "v_bcnt_u32_b32", "v_or3_b32", "v_alignbit_b32", "v_bfi_b32"};
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++)
    for (int op = 0; op < 7; op++) {
        hipEventRecord(e0);
        switch (op) {
            case 0: k<0><<<blocks, 256>>>(out, 1); break;
            case 1: k<1><<<blocks, 256>>>(out, 1); break;
            case 2: k<2><<<blocks, 256>>>(out, 1); break;
            case 3: k<3><<<blocks, 256>>>(out, 1); break;
            case 4: k<4><<<blocks, 256>>>(out, 1); break;
            case 5: k<5><<<blocks, 256>>>(out, 1); break;
            case 6: k<6><<<blocks, 256>>>(out, 1); break;
        }
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double winstr = (double)blocks * 4 * ITERS * 8;
        printf("%-16s %.3f ms  %.3e wave-instr/s  (peak 1.229e12 @2.4GHz, 2 cyc/wave-instr/SIMD)\n", names[op], ms, winstr / (ms * 1e-3));
    }
    return 0;
}
