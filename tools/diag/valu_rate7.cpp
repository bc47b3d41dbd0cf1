// Microbenchmark 7 (NOT product code): which fast instructions keep their
// rate next to slow ones?  valu_rate6 found a v_and_b32_e32 after a 64-bit
// shift costs ~3.6 cycles where a v_bitop3_b32 costs ~3.0 (each ~2.2 / 2.5
// alone).  Here: the VOP2 and VOP3 (e64) encodings of and/or, bitop3, and
// other slow partners (bfrev, bcnt, lshl_add_u64), 32 independent
// instructions on fixed registers per body; 4 and 8 waves/SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/diag/valu_rate7 tools/diag/valu_rate7.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 2048
#define S "v_lshlrev_b64 v[56:57], 8, v[42:43]\n"
#define SA "v_lshl_add_u64 v[56:57], v[42:43], 1, v[40:41]\n"
#define SR "v_bfrev_b32_e32 v58, v44\n"
#define SC "v_bcnt_u32_b32 v58, v44, 0\n"
#define SR6 "v_bfrev_b32_e64 v58, v44\n"
#define SL32 "v_lshrrev_b32_e64 v58, 4, v44\n"
#define SCN "v_cndmask_b32_e64 v58, v44, v45, s[0:1]\n"
#define SMN "v_min_u32_e64 v58, v44, v45\n"
#define D1 "v_add_u32_e64 v60, v45, v46\n"
#define SL2 "v_lshrrev_b32_e64 v59, 4, v47\n"
#define SL32E "v_lshrrev_b32_e32 v58, 4, v44\n"
#define SCNE "v_cndmask_b32_e32 v58, v44, v45, vcc\n"
#define SCNT "v_bcnt_u32_b32 v58, v44, 0\n"
#define SAB "v_alignbit_b32 v58, v44, v45, 4\n"
#define SMAD "v_mul_hi_u32 v58, v44, v45\n"
#define A1 "v_and_b32_e32 v60, v45, v46\n"
#define A2 "v_and_b32_e32 v61, v49, v50\n"
#define A3 "v_and_b32_e32 v62, v53, v54\n"
#define E1 "v_and_b32_e64 v60, v45, v46\n"
#define E2 "v_and_b32_e64 v61, v49, v50\n"
#define E3 "v_and_b32_e64 v62, v53, v54\n"
#define O1 "v_or_b32_e32 v60, v45, v46\n"
#define O2 "v_or_b32_e32 v61, v49, v50\n"
#define O3 "v_or_b32_e32 v62, v53, v54\n"
#define B1 "v_bitop3_b32 v60, v45, v46, v47 bitop3:0xca\n"
#define B2 "v_bitop3_b32 v61, v49, v50, v51 bitop3:0xca\n"
#define B3 "v_bitop3_b32 v62, v53, v54, v55 bitop3:0xca\n"
#define C1 "v_bitop3_b32 v60, v45, v46, v46 bitop3:0xc0\n"
#define C2 "v_bitop3_b32 v61, v49, v50, v50 bitop3:0xc0\n"
#define C3 "v_bitop3_b32 v62, v53, v54, v54 bitop3:0xc0\n"
#define X8(a) a a a a a a a a
#define X4(a) a a a a
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
             "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "s0", "s1"
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed) {
    asm volatile(
        "v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n"
        "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, %0\n"
        "v_mov_b32 v48, %0\n v_mov_b32 v49, %0\n v_mov_b32 v50, %0\n v_mov_b32 v51, %0\n"
        "v_mov_b32 v52, %0\n v_mov_b32 v53, %0\n v_mov_b32 v54, %0\n v_mov_b32 v55, %0\n" ::"v"(seed + threadIdx.x)
        : CLOB);
    for (int i = 0; i < ITERS; i++) {
        if (OP == 0) asm volatile(X8(S A1 A2 A3) ::: CLOB);
        if (OP == 1) asm volatile(X8(S E1 E2 E3) ::: CLOB);
        if (OP == 2) asm volatile(X8(S B1 B2 B3) ::: CLOB);
        if (OP == 3) asm volatile(X8(S C1 C2 C3) ::: CLOB);
        if (OP == 4) asm volatile(X8(S O1 O2 O3) ::: CLOB);
        if (OP == 5) asm volatile(X8(SR A1 A2 A3) ::: CLOB);
        if (OP == 6) asm volatile(X8(SR C1 C2 C3) ::: CLOB);
        if (OP == 7) asm volatile(X8(SC A1 A2 A3) ::: CLOB);
        if (OP == 8) asm volatile(X8(SC C1 C2 C3) ::: CLOB);
        if (OP == 9) asm volatile(X8(SA A1 A2 A3) ::: CLOB);
        if (OP == 10) asm volatile(X8(SA C1 C2 C3) ::: CLOB);
        if (OP == 11) asm volatile(X8(A1 B1 A2 B2) ::: CLOB);
        if (OP == 12) asm volatile(X8(E1 B1 E2 B2) ::: CLOB);
        if (OP == 13) asm volatile(X8(E1 E2 E3 E1) ::: CLOB);
        if (OP == 14) asm volatile(X8(C1 C2 C3 C1) ::: CLOB);
        if (OP == 15) asm volatile(X8(S S A1 A2) ::: CLOB);
        if (OP == 16) asm volatile(X8(S S C1 C2) ::: CLOB);
        if (OP == 17) asm volatile(X8(SR6 C1 C2 C3) ::: CLOB);
        if (OP == 18) asm volatile(X8(SL32 C1 C2 C3) ::: CLOB);
        if (OP == 19) asm volatile(X8(SCN C1 C2 C3) ::: CLOB);
        if (OP == 20) asm volatile(X8(SMN C1 C2 C3) ::: CLOB);
        if (OP == 21) asm volatile(X8(S D1 C2 C3) ::: CLOB);
        if (OP == 22) asm volatile(X8(S C1 S C2) ::: CLOB);
        if (OP == 23) asm volatile(X4(S C1 C2 C3 C1 C2 C3 C1) ::: CLOB);
        if (OP == 24) asm volatile(X8(S SR6 C1 C2) ::: CLOB);
        if (OP == 25) asm volatile(X8(SR6 SR6 C1 C2) ::: CLOB);
        if (OP == 26) asm volatile(X8(SR6 SR6 SR6 SR6) ::: CLOB);
        if (OP == 27) asm volatile(X8(SL32 SL2 SL32 SL2) ::: CLOB);
        if (OP == 28) asm volatile(X8(SL32E SL32E SL32E SL32E) ::: CLOB);
        if (OP == 29) asm volatile(X8(SCN SCN SCN SCN) ::: CLOB);
        if (OP == 30) asm volatile(X8(SCNE SCNE SCNE SCNE) ::: CLOB);
        if (OP == 31) asm volatile(X8(SL32 C1 SL2 C2) ::: CLOB);
        if (OP == 32) asm volatile(X8(S SL32 SL2 C1) ::: CLOB);
        if (OP == 33) asm volatile(X8(S SL32 S SL2) ::: CLOB);
        if (OP == 34) asm volatile(X8(SL32E C1 C2 C3) ::: CLOB);
        if (OP == 35) asm volatile(X8(SAB C1 C2 C3) ::: CLOB);
        if (OP == 36) asm volatile(X8(SMAD C1 C2 C3) ::: CLOB);
        if (OP == 37) asm volatile(X8(SCNT SCNT SCNT SCNT) ::: CLOB);
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
    printf("  %-44s %.3f ms  %.2f cyc/instr  %.1f cyc per 32\n", name, t, 1024 * 2.4e9 / (winstr / (t * 1e-3)),
           32 * 1024 * 2.4e9 / (winstr / (t * 1e-3)));
}
int main() {
    unsigned* out;
    (void)hipMalloc(&out, (size_t)8192 * 256 * 4);
    for (int i = 0; i < 3; i++) run<0>(out, 2048);
    for (int b : {2048}) {
        printf("-- %d waves/SIMD\n", b / 256);
        report<0>(out, "8 x (shl64, and_e32 x3)", b);
        report<1>(out, "8 x (shl64, and_e64 x3)", b);
        report<2>(out, "8 x (shl64, bitop3 bfi x3)", b);
        report<3>(out, "8 x (shl64, bitop3 and x3)", b);
        report<4>(out, "8 x (shl64, or_e32 x3)", b);
        report<5>(out, "8 x (bfrev, and_e32 x3)", b);
        report<6>(out, "8 x (bfrev, bitop3 and x3)", b);
        report<7>(out, "8 x (bcnt, and_e32 x3)", b);
        report<8>(out, "8 x (bcnt, bitop3 and x3)", b);
        report<9>(out, "8 x (lshl_add_u64, and_e32 x3)", b);
        report<10>(out, "8 x (lshl_add_u64, bitop3 and x3)", b);
        report<11>(out, "16 x (and_e32, bitop3)", b);
        report<12>(out, "16 x (and_e64, bitop3)", b);
        report<13>(out, "32 and_e64", b);
        report<14>(out, "32 bitop3 and", b);
        report<15>(out, "8 x (shl64 x2, and_e32 x2)", b);
        report<16>(out, "8 x (shl64 x2, bitop3 and x2)", b);
        report<17>(out, "8 x (bfrev_e64, bitop3 and x3)", b);
        report<18>(out, "8 x (lshrrev_b32_e64, bitop3 and x3)", b);
        report<19>(out, "8 x (cndmask_e64, bitop3 and x3)", b);
        report<20>(out, "8 x (min_u32_e64, bitop3 and x3)", b);
        report<21>(out, "8 x (shl64, add_u32_e64, bitop3 x2)", b);
        report<22>(out, "16 x (shl64, bitop3)", b);
        report<23>(out, "4 x (shl64, bitop3 x7)", b);
        report<24>(out, "8 x (shl64, bfrev_e64, bitop3 x2)", b);
        report<25>(out, "8 x (bfrev_e64 x2, bitop3 x2)", b);
        report<26>(out, "32 bfrev_e64", b);
        report<27>(out, "32 lshrrev_b32_e64", b);
        report<28>(out, "32 lshrrev_b32_e32", b);
        report<29>(out, "32 cndmask_e64 (sgpr mask)", b);
        report<30>(out, "32 cndmask_e32 (vcc)", b);
        report<31>(out, "16 x (lshrrev_b32_e64, bitop3)", b);
        report<32>(out, "8 x (shl64, lshrrev_e64 x2, bitop3)", b);
        report<33>(out, "16 x (shl64, lshrrev_e64)", b);
        report<34>(out, "8 x (lshrrev_b32_e32, bitop3 x3)", b);
        report<35>(out, "8 x (alignbit, bitop3 x3)", b);
        report<36>(out, "8 x (mul_hi_u32, bitop3 x3)", b);
        report<37>(out, "32 bcnt", b);
    }
    return 0;
}
