// Microbenchmark 6 (NOT product code): does the order of slow (~4-cycle) and
// fast (~2.2-cycle) VALU instructions change their cost?  Each body has 8
// 64-bit shifts (slow) and 24 v_and_b32 (fast), independent, on fixed
// registers, in different orders; 8 waves/SIMD.  Additive cost would be
// 8 x 4.25 + 24 x 2.25 = 88 cycles per 32 instructions (2.75 each).
//   hipcc --offload-arch=gfx950 -O3 -o tools/diag/valu_rate6 tools/diag/valu_rate6.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 2048
#define S "v_lshlrev_b64 v[56:57], 8, v[42:43]\n"
#define F1 "v_and_b32 v60, v45, v46\n"
#define F2 "v_and_b32 v61, v49, v50\n"
#define F3 "v_and_b32 v62, v53, v54\n"
#define B1 "v_bitop3_b32 v60, v45, v46, v47 bitop3:0xca\n"
#define B2 "v_bitop3_b32 v61, v49, v50, v51 bitop3:0xca\n"
#define B3 "v_bitop3_b32 v62, v53, v54, v55 bitop3:0xca\n"
#define SF3 S F1 F2 F3
#define FFF F1 F2 F3
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
             "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed) {
    asm volatile(
        "v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n"
        "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, %0\n"
        "v_mov_b32 v48, %0\n v_mov_b32 v49, %0\n v_mov_b32 v50, %0\n v_mov_b32 v51, %0\n"
        "v_mov_b32 v52, %0\n v_mov_b32 v53, %0\n v_mov_b32 v54, %0\n v_mov_b32 v55, %0\n" ::"v"(seed + threadIdx.x)
        : CLOB);
    for (int i = 0; i < ITERS; i++) {
        if (OP == 0) asm volatile(SF3 SF3 SF3 SF3 SF3 SF3 SF3 SF3 ::: CLOB);                       // S FFF x8
        if (OP == 1) asm volatile(S S FFF FFF SF3 SF3 S S FFF FFF SF3 SF3 ::: CLOB);                // pairs
        if (OP == 2) asm volatile(S S S S FFF FFF FFF FFF S S S S FFF FFF FFF FFF ::: CLOB);         // groups of 4
        if (OP == 3) asm volatile(S S S S S S S S FFF FFF FFF FFF FFF FFF FFF FFF ::: CLOB);         // all slow first
        if (OP == 4) asm volatile(S B1 B2 B3 S B1 B2 B3 S B1 B2 B3 S B1 B2 B3 S B1 B2 B3 S B1 B2 B3 S B1 B2 B3 S B1 B2 B3 ::: CLOB);
        if (OP == 5) asm volatile(S S S S S S S S B1 B2 B3 B1 B2 B3 B1 B2 B3 B1 B2 B3 B1 B2 B3 B1 B2 B3 B1 B2 B3 B1 B2 B3 ::: CLOB);
        if (OP == 6) asm volatile(FFF FFF FFF FFF FFF FFF FFF FFF FFF FFF F1 F2 ::: CLOB);             // 32 fast
        if (OP == 7) asm volatile(S S S S S S S S S S S S S S S S S S S S S S S S S S S S S S S S ::: CLOB);  // 32 slow
    }
    unsigned r;
    asm volatile("v_mov_b32 %0, v56" : "=v"(r)::CLOB);
    out[blockIdx.x * 256 + threadIdx.x] = r;
}
template <int OP>
float run(unsigned* out, int blocks) {
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
template <int OP>
void report(unsigned* out, const char* name, int blocks) {
    const float t = run<OP>(out, blocks);
    const double winstr = (double)blocks * 4 * ITERS * 32;
    printf("  %-52s %.3f ms  %.2f cyc/instr  %.1f cyc per 32\n", name, t, 1024 * 2.4e9 / (winstr / (t * 1e-3)),
           32 * 1024 * 2.4e9 / (winstr / (t * 1e-3)));
}
int main() {
    unsigned* out;
    (void)hipMalloc(&out, (size_t)8192 * 256 * 4);
    for (int i = 0; i < 3; i++) run<0>(out, 2048);
    for (int b : {1024, 2048}) {
        printf("-- %d waves/SIMD\n", b / 256);
        report<0>(out, "8 x (shl64, and, and, and)", b);
        report<1>(out, "shl pairs, 6 ands between", b);
        report<2>(out, "4 shl, 12 and, x2", b);
        report<3>(out, "8 shl then 24 and", b);
        report<4>(out, "8 x (shl64, bitop3 x3)", b);
        report<5>(out, "8 shl then 24 bitop3", b);
        report<6>(out, "32 and", b);
        report<7>(out, "32 shl64", b);
    }
    return 0;
}
