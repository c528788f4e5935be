// valu_ops.hpp -- the VALU opcode table shared by the issue-rate probe
// (valu_rate.hip) and the counter calibration (pmc_cal.hip): op<OP> issues ONE
// instruction of opcode OP (two for the marked pairs, insts_per_op) on chain a
// (q: 64-bit chain, b: a second operand, m: an SGPR-pair mask, sc: scalar sink).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
typedef short v2s __attribute__((ext_vector_type(2)));


// one opcode per OP; a[]: 32-bit chains, q[]: 64-bit chains.  `n` is the next
// chain's value (for the rotation forms).
template <int OP>
__device__ __forceinline__ void op(uint32_t& a, uint32_t n, uint64_t& q, uint32_t b, uint64_t m, int seed, uint64_t& sc) {
    if constexpr (OP == 0) a = (uint32_t)__builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, b), (v2s){83, -36}, (int)a, false);
    else if constexpr (OP == 1) asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(a) : "v"(b), "s"(seed + 83));
    else if constexpr (OP == 2) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 4) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a));
    else if constexpr (OP == 5) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(m));
    else if constexpr (OP == 6) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(0x05040100));
    else if constexpr (OP == 7) asm volatile("v_bfe_i32 %0, %0, 5, 11" : "+v"(a));
    else if constexpr (OP == 8) asm volatile("v_ashrrev_i32 %0, 5, %0" : "+v"(a));
    else if constexpr (OP == 9) asm volatile("v_pk_mad_u16 %0, %0, %1, %0" : "+v"(a) : "v"(b));
    else if constexpr (OP == 10) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 11) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 12) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 13) asm volatile("v_mov_b32 %0, %0" : "+v"(a));
    else if constexpr (OP == 14) asm volatile("v_pk_sub_i16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 15) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(q) : "v"(m));
    else if constexpr (OP == 16) asm volatile("v_cmp_gt_i32_e64 %0, %1, %2" : "=s"(sc) : "v"(a), "v"(b));
    else if constexpr (OP == 17) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 18) asm volatile("v_floor_f32 %0, %0" : "+v"(a));
    else if constexpr (OP == 19) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(a));
    else if constexpr (OP == 20) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(seed));
    else if constexpr (OP == 21) asm volatile("v_pk_lshrrev_b16 %0, 1, %0" : "+v"(a));
    else if constexpr (OP == 22) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(q), "=s"(sc) : "v"(a), "v"(b));
    else if constexpr (OP == 23) {
        uint32_t s;
        asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(s) : "v"(a));
        sc = s;
    } else if constexpr (OP == 24) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 25) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 26) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a));
    else if constexpr (OP == 27) asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a) : "v"(b), "s"(0x00530024));
    else if constexpr (OP == 28) asm volatile("v_lshl_or_b32 %0, %0, 2, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 29) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 30) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(a));
    else if constexpr (OP == 31) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 32) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 33) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 34) asm volatile("v_mul_i32_i24_sdwa %0, sext(%0), sext(%1) dst_sel:DWORD src0_sel:WORD_0 src1_sel:WORD_1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 35) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a) : "v"(b));
    // ---- round 4: siblings and the classes priced without a measurement before
    else if constexpr (OP == 36) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(n));            // rotation: a_i = a_{i+1}
    else if constexpr (OP == 37) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 38) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 39) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 40) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a) : "v"(b));   // VGPR amount
    else if constexpr (OP == 41) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a) : "v"(b));
    else if constexpr (OP == 42) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(a) : "v"(b));
    else if constexpr (OP == 43) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b));   // VOP2, VCC
    else if constexpr (OP == 44) asm volatile("v_not_b32 %0, %0" : "+v"(a));
    else if constexpr (OP == 45) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a) : "v"(b), "s"(seed));
    else if constexpr (OP == 46) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(q));
    else if constexpr (OP == 47) {
        uint32_t s;
        asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(s) : "v"(a));
        sc = s;
    } else if constexpr (OP == 48) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 49) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    else if constexpr (OP == 50) asm volatile("v_cvt_rpi_i32_f32 %0, %0" : "+v"(a));
    else if constexpr (OP == 51) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 52) asm volatile("v_lshlrev_b16 %0, 3, %0" : "+v"(a));
    else if constexpr (OP == 53) asm volatile("v_sub_i32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 54) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 55) asm volatile("v_accvgpr_write_b32 a0, %0\n v_accvgpr_read_b32 %0, a0" : "+v"(a) :: "a0");
    // ---- round 4, second pass: every remaining VALU opcode of the product kernels, and the VCC forms
    else if constexpr (OP == 56) asm volatile("v_accvgpr_read_b32 %0, a1" : "=v"(a) :: "a1");
    else if constexpr (OP == 57) asm volatile("v_accvgpr_write_b32 a1, %0" :: "v"(a) : "a1");
    else if constexpr (OP == 58) asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(q), "=s"(sc) : "v"(a), "v"(b));
    else if constexpr (OP == 59) asm volatile("v_writelane_b32 %0, %1, 5" : "+v"(a) : "s"(seed));
    else if constexpr (OP == 60) asm volatile("v_cmp_lt_i32_e64 %0, %1, %2" : "=s"(sc) : "v"(a), "v"(b));
    else if constexpr (OP == 61) asm volatile("v_cmp_eq_u32_e32 vcc, %0, %1" :: "v"(a), "v"(b) : "vcc");
    else if constexpr (OP == 62) asm volatile("v_pk_min_i16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 63) asm volatile("v_pk_sub_u16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 64) asm volatile("v_mov_b64 %0, %0" : "+v"(q));
    else if constexpr (OP == 65) asm volatile("v_bfe_u32 %0, %0, 5, 11" : "+v"(a));
    else if constexpr (OP == 66) asm volatile("v_mul_hi_i32_i24 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 67) asm volatile("v_add_lshl_u32 %0, %0, %1, 2" : "+v"(a) : "v"(b));
    else if constexpr (OP == 68) asm volatile("v_add_u16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 69) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 70) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a) : "v"(b));
    else if constexpr (OP == 71) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a));
    else if constexpr (OP == 72) asm volatile("v_rcp_iflag_f32 %0, %0" : "+v"(a));
    else if constexpr (OP == 73) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 74) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(a));
    else if constexpr (OP == 75) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 76) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 77) asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 78) asm volatile("v_max3_u32 %0, %0, %1, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 79) asm volatile("v_alignbit_b32 %0, %0, %1, 5" : "+v"(a) : "v"(b));
    else if constexpr (OP == 80) asm volatile("v_add_f64 %0, %0, %0" : "+v"(q));
    else if constexpr (OP == 81) asm volatile("v_cvt_pkrtz_f16_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 82) asm volatile("v_cvt_f16_i16 %0, %0" : "+v"(a));
    else if constexpr (OP == 83) asm volatile("v_med3_i16 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(seed));
    else if constexpr (OP == 84) asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %0" : "+v"(a) : "s"(seed));
    else if constexpr (OP == 85) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a) : "v"(b));
    else if constexpr (OP == 86) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 87) asm volatile("v_lshrrev_b16 %0, 3, %0" : "+v"(a));
    else if constexpr (OP == 88) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(q));
    else if constexpr (OP == 89) asm volatile("v_mul_lo_u16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 90) asm volatile("v_sub_u16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 91) asm volatile("v_cmp_eq_u64_e64 %0, %1, %2" : "=s"(sc) : "v"(q), "v"(m));
    else if constexpr (OP == 92) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b));
    else if constexpr (OP == 93) asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1\n s_nop 1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b) : "vcc");
    else if constexpr (OP == 94) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a) : "v"(b));
    else if constexpr (OP == 95) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(m));
    else if constexpr (OP == 96) asm volatile("v_max_f32 %0, %1, %0" : "+v"(a) : "v"(b));
    else if constexpr (OP == 97) asm volatile("v_lshlrev_b32_e64 %0, 3, %0" : "+v"(a));
    else if constexpr (OP == 98) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 99) asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(a) : "v"(b));
}
constexpr int NOPS = 100;
const char* const kNames[NOPS] = {
    "v_dot2c_i32_i16", "v_mad_i32_i24", "v_pk_add_u16", "v_add_u32", "v_lshlrev_b32", "v_cndmask_b32",
    "v_perm_b32", "v_bfe_i32", "v_ashrrev_i32", "v_pk_mad_u16", "v_mul_lo_u32", "v_mul_i32_i24",
    "v_add3_u32", "v_mov_b32", "v_pk_sub_i16", "v_lshl_add_u64", "v_cmp_gt_i32", "v_add_f32",
    "v_floor_f32", "v_cvt_i32_f32", "v_med3_i32", "v_pk_lshrrev_b16", "v_mad_u64_u32", "v_readlane_b32",
    "v_xor_b32", "v_sub_u32", "v_lshrrev_b32", "v_dot2_i32_i16", "v_lshl_or_b32", "v_and_b32",
    "v_cvt_f32_i32", "v_pk_max_i16", "v_max_i32", "v_mul_u32_u24", "v_mul_i32_i24_sdwa", "v_lshl_add_u32",
    "v_mov_b32_rot", "v_or_b32", "v_max_u32", "v_min_i32", "v_lshlrev_b32_vamt", "v_lshrrev_b32_vamt",
    "v_ashrrev_i32_vamt", "v_cndmask_b32_vcc", "v_not_b32", "v_bfi_b32", "v_lshlrev_b64", "v_readfirstlane_b32",
    "v_fma_f32", "v_permlane32_swap", "v_cvt_rpi_i32_f32", "v_add_co_u32", "v_lshlrev_b16", "v_sub_i32",
    "v_max_f32", "v_accvgpr_write_read_pair",
    "v_accvgpr_read_b32", "v_accvgpr_write_b32", "v_mad_i64_i32", "v_writelane_b32", "v_cmp_lt_i32", "v_cmp_eq_u32_e32", "v_pk_min_i16", "v_pk_sub_u16", "v_mov_b64", "v_bfe_u32", "v_mul_hi_i32_i24", "v_add_lshl_u32", "v_add_u16", "v_mul_hi_u32", "v_mad_u32_u24", "v_cvt_f32_u32", "v_rcp_iflag_f32", "v_mul_f32", "v_cvt_u32_f32", "v_bcnt_u32_b32", "v_or3_b32", "v_subrev_u32", "v_max3_u32", "v_alignbit_b32", "v_add_f64", "v_cvt_pkrtz_f16_f32", "v_cvt_f16_i16", "v_med3_i16", "v_mbcnt_lo_u32_b32", "v_bitop3_b32", "v_and_or_b32", "v_lshrrev_b16", "v_lshrrev_b64", "v_mul_lo_u16", "v_sub_u16", "v_cmp_eq_u64", "v_cndmask_b32_vcc_init", "v_cmp+v_cndmask_vcc", "v_cndmask_b32_e64_vcc", "v_cndmask_b32_e64_s", "v_max_f32_vv", "v_lshlrev_b32_e64", "v_add_u32_e64", "v_mul_u32_u24_vv"};
// instructions per counted op (the accvgpr pair issues two)
__host__ __device__ constexpr int insts_per_op(int opi) { return opi == 55 || opi == 93 ? 2 : 1; }

