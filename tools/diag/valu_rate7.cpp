// Microbenchmark 7 (NOT product code): is the cost of fast ops issued among
// 64-bit shifts a matter of their encoding?  8 shifts + 24 others per body
// (independent, fixed registers), e32 (VOP1/VOP2) against e64 (VOP3) forms.
//   hipcc --offload-arch=gfx950 -O3 -o tools/diag/valu_rate7 tools/diag/valu_rate7.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 2048
#define S "v_lshlrev_b64 v[56:57], 8, v[42:43]\n"
#define A32 "v_and_b32_e32 v60, v45, v46\n v_and_b32_e32 v61, v49, v50\n v_and_b32_e32 v62, v53, v54\n"
#define A64 "v_and_b32_e64 v60, v45, v46\n v_and_b32_e64 v61, v49, v50\n v_and_b32_e64 v62, v53, v54\n"
#define R32 "v_bfrev_b32_e32 v60, v45\n v_bfrev_b32_e32 v61, v49\n v_bfrev_b32_e32 v62, v53\n"
#define R64 "v_bfrev_b32_e64 v60, v45\n v_bfrev_b32_e64 v61, v49\n v_bfrev_b32_e64 v62, v53\n"
#define M32 "v_mov_b32_e32 v60, v45\n v_mov_b32_e32 v61, v49\n v_mov_b32_e32 v62, v53\n"
#define M64 "v_mov_b32_e64 v60, v45\n v_mov_b32_e64 v61, v49\n v_mov_b32_e64 v62, v53\n"
#define B3 "v_bitop3_b32 v60, v45, v46, v47 bitop3:0xca\n v_bitop3_b32 v61, v49, v50, v51 bitop3:0xca\n v_bitop3_b32 v62, v53, v54, v55 bitop3:0xca\n"
#define X8(x) x x x x x x x x
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
        if (OP == 0) asm volatile(X8(S A32) ::: CLOB);
        if (OP == 1) asm volatile(X8(S A64) ::: CLOB);
        if (OP == 2) asm volatile(X8(S R32) ::: CLOB);
        if (OP == 3) asm volatile(X8(S R64) ::: CLOB);
        if (OP == 4) asm volatile(X8(S M32) ::: CLOB);
        if (OP == 5) asm volatile(X8(S M64) ::: CLOB);
        if (OP == 6) asm volatile(X8(S B3) ::: CLOB);
        if (OP == 7) asm volatile(X8(A32 A32 "v_and_b32_e32 v63, v41, v42\n v_and_b32_e32 v59, v44, v43\n") ::: CLOB);
        if (OP == 8) asm volatile(X8(A64 A64 "v_and_b32_e64 v63, v41, v42\n v_and_b32_e64 v59, v44, v43\n") ::: CLOB);
        if (OP == 9) asm volatile(X8(B3 A32 "v_and_b32_e32 v63, v41, v42\n v_bitop3_b32 v59, v44, v43, v42 bitop3:0xca\n") ::: CLOB);
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
    printf("  %-40s %.3f ms  %.2f cyc/instr  %.1f cyc per 32\n", name, t, 1024 * 2.4e9 / (winstr / (t * 1e-3)),
           32 * 1024 * 2.4e9 / (winstr / (t * 1e-3)));
}
int main() {
    unsigned* out;
    (void)hipMalloc(&out, (size_t)8192 * 256 * 4);
    for (int i = 0; i < 3; i++) run<0>(out, 2048);
    for (int b : {1280, 2048}) {
        printf("-- %d waves/SIMD\n", b / 256);
        report<0>(out, "8 x (shl64, 3 and_e32)", b);
        report<1>(out, "8 x (shl64, 3 and_e64)", b);
        report<2>(out, "8 x (shl64, 3 bfrev_e32)", b);
        report<3>(out, "8 x (shl64, 3 bfrev_e64)", b);
        report<4>(out, "8 x (shl64, 3 mov_e32)", b);
        report<5>(out, "8 x (shl64, 3 mov_e64)", b);
        report<6>(out, "8 x (shl64, 3 bitop3)", b);
        report<7>(out, "32 and_e32", b);
        report<8>(out, "32 and_e64", b);
        report<9>(out, "8 x (3 bitop3, 3 and_e32, and, bitop3)", b);
    }
    return 0;
}
