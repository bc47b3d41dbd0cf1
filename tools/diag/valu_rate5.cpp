// Microbenchmark 5 (NOT product code): VALU issue cost by operand register
// banks, and the remaining instructions of the rollout loop.  Each asm body
// is 32 independent instructions on fixed registers (v40..v63, declared
// clobbered), 8 waves/SIMD; the cost printed is cycles per wave-instruction
// per SIMD at 2.4 GHz.  VGPR bank = register number mod 4.
//   hipcc --offload-arch=gfx950 -O3 -o tools/diag/valu_rate5 tools/diag/valu_rate5.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 2048
#define R4(a, b, c, d) a "\n" b "\n" c "\n" d "\n"
#define X8(s) s s s s s s s s
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
             "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "vcc", "s20", "s21"

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed) {
    asm volatile(
        "v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n"
        "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, %0\n"
        "v_mov_b32 v48, %0\n v_mov_b32 v49, %0\n v_mov_b32 v50, %0\n v_mov_b32 v51, %0\n"
        "v_mov_b32 v52, %0\n v_mov_b32 v53, %0\n v_mov_b32 v54, %0\n v_mov_b32 v55, %0\n"
        "s_mov_b64 s[20:21], -1\n s_mov_b64 vcc, -1\n" ::"v"(seed + threadIdx.x)
        : CLOB);
    for (int i = 0; i < ITERS; i++) {
        // bitop3, sources in three different banks (1, 2, 3), dst bank 0
        if (OP == 0) asm volatile(X8(R4("v_bitop3_b32 v56, v41, v42, v43 bitop3:0xca", "v_bitop3_b32 v60, v45, v46, v47 bitop3:0xca",
                                        "v_bitop3_b32 v56, v49, v50, v51 bitop3:0xca", "v_bitop3_b32 v60, v53, v54, v55 bitop3:0xca")) ::: CLOB);
        // bitop3, all three sources in one bank (1)
        if (OP == 1) asm volatile(X8(R4("v_bitop3_b32 v56, v41, v45, v49 bitop3:0xca", "v_bitop3_b32 v60, v45, v49, v53 bitop3:0xca",
                                        "v_bitop3_b32 v56, v49, v53, v41 bitop3:0xca", "v_bitop3_b32 v60, v53, v41, v45 bitop3:0xca")) ::: CLOB);
        // bitop3, two sources in one bank
        if (OP == 2) asm volatile(X8(R4("v_bitop3_b32 v56, v41, v45, v42 bitop3:0xca", "v_bitop3_b32 v60, v45, v49, v46 bitop3:0xca",
                                        "v_bitop3_b32 v56, v49, v53, v50 bitop3:0xca", "v_bitop3_b32 v60, v53, v41, v54 bitop3:0xca")) ::: CLOB);
        // bitop3, one register read twice (andn form a & ~b as bitop3(a, b, b))
        if (OP == 3) asm volatile(X8(R4("v_bitop3_b32 v56, v41, v42, v42 bitop3:0x30", "v_bitop3_b32 v60, v45, v46, v46 bitop3:0x30",
                                        "v_bitop3_b32 v56, v49, v50, v50 bitop3:0x30", "v_bitop3_b32 v60, v53, v54, v54 bitop3:0x30")) ::: CLOB);
        // v_and_b32, two sources in different banks / in the same bank
        if (OP == 4) asm volatile(X8(R4("v_and_b32 v56, v41, v42", "v_and_b32 v60, v45, v46", "v_and_b32 v56, v49, v50", "v_and_b32 v60, v53, v54")) ::: CLOB);
        if (OP == 5) asm volatile(X8(R4("v_and_b32 v56, v41, v45", "v_and_b32 v60, v45, v49", "v_and_b32 v56, v49, v53", "v_and_b32 v60, v53, v41")) ::: CLOB);
        // 64-bit shift, independent
        if (OP == 6) asm volatile(X8(R4("v_lshlrev_b64 v[56:57], 8, v[42:43]", "v_lshlrev_b64 v[58:59], 8, v[46:47]",
                                        "v_lshlrev_b64 v[60:61], 8, v[50:51]", "v_lshlrev_b64 v[62:63], 8, v[54:55]")) ::: CLOB);
        // 32-bit shift, independent
        if (OP == 7) asm volatile(X8(R4("v_lshlrev_b32 v56, 8, v42", "v_lshlrev_b32 v58, 8, v46", "v_lshlrev_b32 v60, 8, v50", "v_lshlrev_b32 v62, 8, v54")) ::: CLOB);
        if (OP == 8) asm volatile(X8(R4("v_bfrev_b32 v56, v42", "v_bfrev_b32 v58, v46", "v_bfrev_b32 v60, v50", "v_bfrev_b32 v62, v54")) ::: CLOB);
        if (OP == 9) asm volatile(X8(R4("v_mul_hi_u32 v56, v41, v42", "v_mul_hi_u32 v58, v45, v46", "v_mul_hi_u32 v60, v49, v50", "v_mul_hi_u32 v62, v53, v54")) ::: CLOB);
        if (OP == 10) asm volatile(X8(R4("v_mad_u64_u32 v[56:57], s[20:21], v41, v42, v[44:45]", "v_mad_u64_u32 v[58:59], s[20:21], v45, v46, v[48:49]",
                                         "v_mad_u64_u32 v[60:61], s[20:21], v49, v50, v[52:53]", "v_mad_u64_u32 v[62:63], s[20:21], v53, v54, v[40:41]")) ::: CLOB);
        if (OP == 11) asm volatile(X8(R4("v_lshl_add_u64 v[56:57], v[42:43], 0, -1", "v_lshl_add_u64 v[58:59], v[46:47], 0, -1",
                                         "v_lshl_add_u64 v[60:61], v[50:51], 0, -1", "v_lshl_add_u64 v[62:63], v[54:55], 0, -1")) ::: CLOB);
        if (OP == 12) asm volatile(X8(R4("v_bcnt_u32_b32 v56, v42, 0", "v_bcnt_u32_b32 v58, v46, 0", "v_bcnt_u32_b32 v60, v50, 0", "v_bcnt_u32_b32 v62, v54, 0")) ::: CLOB);
        if (OP == 13) asm volatile(X8(R4("v_cndmask_b32_e64 v56, v41, v42, s[20:21]", "v_cndmask_b32_e64 v58, v45, v46, s[20:21]",
                                         "v_cndmask_b32_e64 v60, v49, v50, s[20:21]", "v_cndmask_b32_e64 v62, v53, v54, s[20:21]")) ::: CLOB);
        if (OP == 14) asm volatile(X8(R4("v_cndmask_b32_e32 v56, v41, v42, vcc", "v_cndmask_b32_e32 v58, v45, v46, vcc",
                                         "v_cndmask_b32_e32 v60, v49, v50, vcc", "v_cndmask_b32_e32 v62, v53, v54, vcc")) ::: CLOB);
        if (OP == 15) asm volatile(X8(R4("v_cmp_gt_u32_e64 s[20:21], v41, v42", "v_cmp_gt_u32_e64 s[20:21], v45, v46",
                                         "v_cmp_gt_u32_e64 s[20:21], v49, v50", "v_cmp_gt_u32_e64 s[20:21], v53, v54")) ::: CLOB);
        if (OP == 16) asm volatile(X8(R4("v_sub_co_u32_e32 v56, vcc, v41, v42", "v_subb_co_u32_e32 v57, vcc, v43, v44, vcc",
                                         "v_sub_co_u32_e32 v60, vcc, v49, v50", "v_subb_co_u32_e32 v61, vcc, v51, v52, vcc")) ::: CLOB);
        if (OP == 17) asm volatile(X8(R4("v_bfe_u32 v56, v41, v42, 8", "v_bfe_u32 v58, v45, v46, 8", "v_bfe_u32 v60, v49, v50, 8", "v_bfe_u32 v62, v53, v54, 8")) ::: CLOB);
        if (OP == 18) asm volatile(X8(R4("v_min_u32 v56, v41, v42", "v_sub_u32 v58, v45, v46", "v_min_u32 v60, v49, v50", "v_sub_u32 v62, v53, v54")) ::: CLOB);
        if (OP == 19) asm volatile(X8(R4("v_lshrrev_b64 v[56:57], 40, v[42:43]", "v_lshrrev_b64 v[58:59], 40, v[46:47]",
                                         "v_lshrrev_b64 v[60:61], 40, v[50:51]", "v_lshrrev_b64 v[62:63], 40, v[54:55]")) ::: CLOB);
        // mixed: one 64-bit shift and three bitop3 (distinct banks): do they overlap?
        if (OP == 20) asm volatile(X8(R4("v_lshlrev_b64 v[56:57], 8, v[42:43]", "v_bitop3_b32 v60, v45, v46, v47 bitop3:0xca",
                                         "v_bitop3_b32 v61, v49, v50, v51 bitop3:0xca", "v_bitop3_b32 v62, v53, v54, v55 bitop3:0xca")) ::: CLOB);
        // mixed: one 64-bit shift and three v_and_b32
        if (OP == 21) asm volatile(X8(R4("v_lshlrev_b64 v[56:57], 8, v[42:43]", "v_and_b32 v60, v45, v46",
                                         "v_and_b32 v61, v49, v50", "v_and_b32 v62, v53, v54")) ::: CLOB);
        if (OP == 22) asm volatile(X8(R4("v_mov_b32 v56, v41", "v_mov_b32 v58, v45", "v_mov_b32 v60, v49", "v_mov_b32 v62, v53")) ::: CLOB);
        if (OP == 23) asm volatile(X8(R4("v_or_b32 v56, v41, v42", "v_xor_b32 v58, v45, v46", "v_or_b32 v60, v49, v50", "v_xor_b32 v62, v53, v54")) ::: CLOB);
        // round 3: other candidate classes (sub-dword selects, funnel/byte shifts, 24-bit multiplies, fused 3-op)
        if (OP == 24) asm volatile(X8(R4("v_mov_b32_sdwa v56, v41 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0", "v_mov_b32_sdwa v58, v45 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0",
                                         "v_mov_b32_sdwa v60, v49 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0", "v_mov_b32_sdwa v62, v53 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0")) ::: CLOB);
        if (OP == 25) asm volatile(X8(R4("v_and_b32_sdwa v56, v41, v42 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD", "v_and_b32_sdwa v58, v45, v46 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD",
                                         "v_and_b32_sdwa v60, v49, v50 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD", "v_and_b32_sdwa v62, v53, v54 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD")) ::: CLOB);
        if (OP == 26) asm volatile(X8(R4("v_alignbit_b32 v56, v41, v42, 8", "v_alignbit_b32 v58, v45, v46, 8", "v_alignbit_b32 v60, v49, v50, 8", "v_alignbit_b32 v62, v53, v54, 8")) ::: CLOB);
        if (OP == 27) asm volatile(X8(R4("v_alignbyte_b32 v56, v41, v42, 1", "v_alignbyte_b32 v58, v45, v46, 1", "v_alignbyte_b32 v60, v49, v50, 1", "v_alignbyte_b32 v62, v53, v54, 1")) ::: CLOB);
        if (OP == 28) asm volatile(X8(R4("v_perm_b32 v56, v41, v42, v43", "v_perm_b32 v58, v45, v46, v47", "v_perm_b32 v60, v49, v50, v51", "v_perm_b32 v62, v53, v54, v55")) ::: CLOB);
        if (OP == 29) asm volatile(X8(R4("v_mul_u32_u24 v56, v41, v42", "v_mul_u32_u24 v58, v45, v46", "v_mul_u32_u24 v60, v49, v50", "v_mul_u32_u24 v62, v53, v54")) ::: CLOB);
        if (OP == 30) asm volatile(X8(R4("v_mad_u32_u24 v56, v41, v42, v43", "v_mad_u32_u24 v58, v45, v46, v47", "v_mad_u32_u24 v60, v49, v50, v51", "v_mad_u32_u24 v62, v53, v54, v55")) ::: CLOB);
        if (OP == 31) asm volatile(X8(R4("v_lshl_or_b32 v56, v41, 8, v42", "v_lshl_or_b32 v58, v45, 8, v46", "v_lshl_or_b32 v60, v49, 8, v50", "v_lshl_or_b32 v62, v53, 8, v54")) ::: CLOB);
        if (OP == 32) asm volatile(X8(R4("v_add_u32 v56, v41, v42", "v_add_u32 v58, v45, v46", "v_add_u32 v60, v49, v50", "v_add_u32 v62, v53, v54")) ::: CLOB);
        if (OP == 33) asm volatile(X8(R4("v_pk_mov_b32 v[56:57], v[42:43], v[42:43] op_sel:[0,1]", "v_pk_mov_b32 v[58:59], v[46:47], v[46:47] op_sel:[0,1]",
                                         "v_pk_mov_b32 v[60:61], v[50:51], v[50:51] op_sel:[0,1]", "v_pk_mov_b32 v[62:63], v[54:55], v[54:55] op_sel:[0,1]")) ::: CLOB);
        if (OP == 34) asm volatile(X8(R4("v_pk_lshlrev_b16 v56, 8, v42", "v_pk_lshlrev_b16 v58, 8, v46", "v_pk_lshlrev_b16 v60, 8, v50", "v_pk_lshlrev_b16 v62, 8, v54")) ::: CLOB);
        if (OP == 35) asm volatile(X8(R4("v_lshlrev_b16 v56, 8, v42", "v_lshlrev_b16 v58, 8, v46", "v_lshlrev_b16 v60, 8, v50", "v_lshlrev_b16 v62, 8, v54")) ::: CLOB);
        if (OP == 36) asm volatile(X8(R4("v_ffbh_u32 v56, v42", "v_ffbh_u32 v58, v46", "v_ffbh_u32 v60, v50", "v_ffbh_u32 v62, v54")) ::: CLOB);
        if (OP == 37) asm volatile(X8(R4("v_bitop3_b16 v56, v41, v42, v43 bitop3:0xca", "v_bitop3_b16 v60, v45, v46, v47 bitop3:0xca",
                                         "v_bitop3_b16 v56, v49, v50, v51 bitop3:0xca", "v_bitop3_b16 v60, v53, v54, v55 bitop3:0xca")) ::: CLOB);
        if (OP == 38) asm volatile(X8(R4("v_mov_b64 v[56:57], v[42:43]", "v_mov_b64 v[58:59], v[46:47]", "v_mov_b64 v[60:61], v[50:51]", "v_mov_b64 v[62:63], v[54:55]")) ::: CLOB);
        if (OP == 39) asm volatile(X8(R4("v_not_b32 v56, v42", "v_not_b32 v58, v46", "v_not_b32 v60, v50", "v_not_b32 v62, v54")) ::: CLOB);
        if (OP == 40) asm volatile(X8(R4("v_and_or_b32 v56, v41, v42, v43", "v_and_or_b32 v58, v45, v46, v47", "v_and_or_b32 v60, v49, v50, v51", "v_and_or_b32 v62, v53, v54, v55")) ::: CLOB);
        if (OP == 42) asm volatile(X8(R4("v_sub_u32 v56, v41, v42", "v_sub_u32 v58, v45, v46", "v_sub_u32 v60, v49, v50", "v_sub_u32 v62, v53, v54")) ::: CLOB);
        if (OP == 43) asm volatile(X8(R4("v_min_u32 v56, v41, v42", "v_min_u32 v58, v45, v46", "v_min_u32 v60, v49, v50", "v_min_u32 v62, v53, v54")) ::: CLOB);
        if (OP == 44) asm volatile(X8(R4("v_add_co_u32 v56, vcc, v41, v42", "v_add_co_u32 v58, vcc, v45, v46", "v_add_co_u32 v60, vcc, v49, v50", "v_add_co_u32 v62, vcc, v53, v54")) ::: CLOB);
        if (OP == 45) asm volatile(X8(R4("v_addc_co_u32 v56, vcc, v41, v42, vcc", "v_addc_co_u32 v58, vcc, v45, v46, vcc", "v_addc_co_u32 v60, vcc, v49, v50, vcc", "v_addc_co_u32 v62, vcc, v53, v54, vcc")) ::: CLOB);
        if (OP == 46) asm volatile(X8(R4("v_lshrrev_b16 v56, 8, v42", "v_lshrrev_b16 v58, 8, v46", "v_lshrrev_b16 v60, 8, v50", "v_lshrrev_b16 v62, 8, v54")) ::: CLOB);
        if (OP == 47) asm volatile(X8(R4("v_lshlrev_b16_sdwa v56, 8, v42 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:WORD_1", "v_lshlrev_b16_sdwa v58, 8, v46 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:WORD_1", "v_lshlrev_b16_sdwa v60, 8, v50 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:WORD_1", "v_lshlrev_b16_sdwa v62, 8, v54 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:WORD_1")) ::: CLOB);
        if (OP == 48) asm volatile(X8(R4("v_add_u16 v56, v41, v42", "v_add_u16 v58, v45, v46", "v_add_u16 v60, v49, v50", "v_add_u16 v62, v53, v54")) ::: CLOB);
        if (OP == 49) asm volatile(X8(R4("v_max_u32 v56, v41, v42", "v_max_u32 v58, v45, v46", "v_max_u32 v60, v49, v50", "v_max_u32 v62, v53, v54")) ::: CLOB);
        if (OP == 50) asm volatile(X8(R4("v_add3_u32 v56, v41, v42, v43", "v_add3_u32 v58, v45, v46, v47", "v_add3_u32 v60, v49, v50, v51", "v_add3_u32 v62, v53, v54, v55")) ::: CLOB);
        if (OP == 51) asm volatile(X8(R4("v_cmp_gt_u32_e32 vcc, v41, v42", "v_cmp_gt_u32_e32 vcc, v45, v46", "v_cmp_gt_u32_e32 vcc, v49, v50", "v_cmp_gt_u32_e32 vcc, v53, v54")) ::: CLOB);
        if (OP == 52) asm volatile(X8(R4("v_and_b32 v56, 0x7e7e7e7e, v42", "v_and_b32 v58, 0x7e7e7e7e, v46", "v_and_b32 v60, 0x7e7e7e7e, v50", "v_and_b32 v62, 0x7e7e7e7e, v54")) ::: CLOB);
        if (OP == 53) asm volatile(X8(R4("v_cmp_gt_u32_e32 vcc, v41, v42", "v_cndmask_b32_e32 v58, v45, v46, vcc", "v_cmp_gt_u32_e32 vcc, v49, v50", "v_cndmask_b32_e32 v62, v53, v54, vcc")) ::: CLOB);
        if (OP == 54) asm volatile(X8(R4("v_mul_lo_u16 v56, v41, v42", "v_mul_lo_u16 v58, v45, v46", "v_mul_lo_u16 v60, v49, v50", "v_mul_lo_u16 v62, v53, v54")) ::: CLOB);
        if (OP == 55) asm volatile(X8(R4("v_lshlrev_b32_e64 v56, v41, v42", "v_lshlrev_b32_e64 v58, v45, v46", "v_lshlrev_b32_e64 v60, v49, v50", "v_lshlrev_b32_e64 v62, v53, v54")) ::: CLOB);
        if (OP == 56) asm volatile(X8(R4("v_sub_u16 v56, v41, v42", "v_sub_u16 v58, v45, v46", "v_sub_u16 v60, v49, v50", "v_sub_u16 v62, v53, v54")) ::: CLOB);
        if (OP == 57) asm volatile(X8(R4("v_min_u16 v56, v41, v42", "v_min_u16 v58, v45, v46", "v_min_u16 v60, v49, v50", "v_min_u16 v62, v53, v54")) ::: CLOB);
        if (OP == 41) asm volatile(X8(R4("v_mbcnt_lo_u32_b32 v56, v42, 0", "v_mbcnt_lo_u32_b32 v58, v46, 0", "v_mbcnt_lo_u32_b32 v60, v50, 0", "v_mbcnt_lo_u32_b32 v62, v54, 0")) ::: CLOB);
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
    printf("  %-48s %.3f ms  %.2f cyc/instr/SIMD @2.4GHz\n", name, t, 1024 * 2.4e9 / (winstr / (t * 1e-3)));
}

int main() {
    unsigned* out;
    (void)hipMalloc(&out, (size_t)8192 * 256 * 4);
    for (int i = 0; i < 3; i++) run<0>(out, 2048);  // clock ramp
    const int b = 2048;                              // 8 waves / SIMD
    report<0>(out, "bitop3, srcs in 3 banks", b);
    report<1>(out, "bitop3, srcs in 1 bank", b);
    report<2>(out, "bitop3, 2 srcs in 1 bank", b);
    report<3>(out, "bitop3 andn (a, b, b)", b);
    report<4>(out, "and_b32, srcs in 2 banks", b);
    report<5>(out, "and_b32, srcs in 1 bank", b);
    report<6>(out, "lshlrev_b64 8", b);
    report<7>(out, "lshlrev_b32 8", b);
    report<8>(out, "bfrev_b32", b);
    report<9>(out, "mul_hi_u32", b);
    report<10>(out, "mad_u64_u32", b);
    report<11>(out, "lshl_add_u64 (x - 1)", b);
    report<12>(out, "bcnt_u32_b32", b);
    report<13>(out, "cndmask_b32_e64 (sgpr mask)", b);
    report<14>(out, "cndmask_b32_e32 (vcc)", b);
    report<15>(out, "cmp_gt_u32_e64", b);
    report<16>(out, "sub_co / subb_co pair (64-bit sub)", b);
    report<17>(out, "bfe_u32", b);
    report<18>(out, "min_u32 / sub_u32", b);
    report<19>(out, "lshrrev_b64 40", b);
    report<20>(out, "1 lshlrev_b64 + 3 bitop3 (per instr)", b);
    report<21>(out, "1 lshlrev_b64 + 3 and_b32 (per instr)", b);
    report<22>(out, "mov_b32", b);
    report<23>(out, "or / xor", b);
    report<24>(out, "mov_b32_sdwa (x << 16 as a word move)", b);
    report<25>(out, "and_b32_sdwa (byte 1 of src0)", b);
    report<26>(out, "alignbit_b32 (funnel shift 8)", b);
    report<27>(out, "alignbyte_b32 (funnel shift 1 byte)", b);
    report<28>(out, "perm_b32", b);
    report<29>(out, "mul_u32_u24", b);
    report<30>(out, "mad_u32_u24", b);
    report<31>(out, "lshl_or_b32", b);
    report<32>(out, "add_u32", b);
    report<33>(out, "pk_mov_b32 (64-bit swap halves)", b);
    report<34>(out, "pk_lshlrev_b16", b);
    report<35>(out, "lshlrev_b16", b);
    report<36>(out, "ffbh_u32", b);
    report<37>(out, "bitop3_b16", b);
    report<38>(out, "mov_b64", b);
    report<39>(out, "not_b32", b);
    report<40>(out, "and_or_b32", b);
    report<41>(out, "mbcnt_lo_u32_b32", b);
    report<42>(out, "sub_u32", b);
    report<43>(out, "min_u32", b);
    report<44>(out, "add_co_u32 (carry out)", b);
    report<45>(out, "addc_co_u32 (carry in and out)", b);
    report<46>(out, "lshrrev_b16", b);
    report<47>(out, "lshlrev_b16_sdwa (high word, preserve)", b);
    report<48>(out, "add_u16", b);
    report<49>(out, "max_u32", b);
    report<50>(out, "add3_u32", b);
    report<51>(out, "cmp_gt_u32_e32 (vcc)", b);
    report<52>(out, "and_b32 with a literal", b);
    report<53>(out, "cmp_e32 + cndmask_e32 pair (per instr)", b);
    report<54>(out, "mul_lo_u16", b);
    report<55>(out, "lshlrev_b32_e64 (variable)", b);
    report<56>(out, "sub_u16", b);
    report<57>(out, "min_u16", b);
    return 0;
}
