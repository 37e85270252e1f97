// VALU issue cost per instruction on gfx950 (measurement tool, not shipped): each kernel runs 8
// independent chains of one instruction per lane, 8 waves per SIMD on every CU; the result is SIMD
// cycles per wave-instruction (s_memtime cycles x waves per SIMD / instructions per wave), and the
// wall-clock rate relative to v_add_u32.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096
#define CHAINS 8

#define BODY32(INS)                                                                                     \
    asm volatile(INS : "+v"(a0) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a1) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a2) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a3) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a4) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a5) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a6) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a7) : "v"(b));

#define KERN32(NAME, INS)                                                                               \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint64_t *cyc, uint32_t seed)            \
    {                                                                                                   \
        uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
                 a6 = a0 + 6, a7 = a0 + 7, b = seed * 3u + 1u;                                          \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                               \
        for (int i = 0; i < ITERS; ++i) { BODY32(INS) }                                                 \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                               \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                    \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;                 \
    }

#define BODY64(INS)                                                                                     \
    asm volatile(INS : "+v"(a0) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a1) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a2) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a3) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a4) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a5) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a6) : "v"(b));                                                             \
    asm volatile(INS : "+v"(a7) : "v"(b));

#define KERN64(NAME, T, INS)                                                                            \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint64_t *cyc, uint32_t seed)            \
    {                                                                                                   \
        T a0 = (T)(threadIdx.x ^ seed), a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,  \
          a6 = a0 + 6, a7 = a0 + 7, b = (T)(seed * 3u + 1u);                                           \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                               \
        for (int i = 0; i < ITERS; ++i) { BODY64(INS) }                                                 \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                               \
        T x = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                                    \
        uint64_t y;                                                                                     \
        __builtin_memcpy(&y, &x, 8);                                                                    \
        out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(y ^ (y >> 32));                               \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;                 \
    }

#define KERN64B(NAME, T, INS)                                                                           \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint64_t *cyc, uint32_t seed)            \
    {                                                                                                   \
        T a0 = (T)(threadIdx.x ^ seed), a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,  \
          a6 = a0 + 6, a7 = a0 + 7;                                                                     \
        uint32_t b = seed * 3u + 1u;                                                                    \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                               \
        for (int i = 0; i < ITERS; ++i) { BODY64(INS) }                                                 \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                               \
        T x = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                                    \
        uint64_t y;                                                                                     \
        __builtin_memcpy(&y, &x, 8);                                                                    \
        out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(y ^ (y >> 32));                                \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;                 \
    }

KERN32(k_add_u32, "v_add_u32 %0, %0, %1")
KERN32(k_xor3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
KERN32(k_alignbit, "v_alignbit_b32 %0, %0, %1, 15")
KERN32(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
KERN32(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
KERN32(k_ffbh, "v_ffbh_u32 %0, %1")
KERN32(k_bfe, "v_bfe_u32 %0, %0, 3, 7")
KERN32(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %1")
KERN32(k_fma_f32, "v_fma_f32 %0, %0, %1, %0")
KERN64(k_lshl_add_u64, uint64_t, "v_lshl_add_u64 %0, %0, 0, %1")
KERN64(k_lshlrev_b64, uint64_t, "v_lshlrev_b64 %0, 21, %0")
KERN64(k_lshrrev_b64, uint64_t, "v_lshrrev_b64 %0, 11, %0")
KERN64B(k_mad_u64_u32, uint64_t, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
KERN64(k_fma_f64, double, "v_fma_f64 %0, %0, %1, %0")
KERN64(k_add_f64, double, "v_add_f64 %0, %0, %1")
KERN64(k_mul_f64, double, "v_mul_f64 %0, %0, %1")
KERN64(k_fract_f64, double, "v_fract_f64 %0, %1")
KERN64B(k_cvt_f64_u32, double, "v_cvt_f64_u32 %0, %1")
KERN64(k_mov_b64, uint64_t, "v_mov_b64 %0, %1")

KERN32(k_xor, "v_xor_b32 %0, %0, %1")
KERN32(k_and, "v_and_b32 %0, %0, %1")
KERN32(k_lshlrev32, "v_lshlrev_b32 %0, 3, %0")
KERN32(k_lshrrev32, "v_lshrrev_b32 %0, 3, %0")
KERN32(k_add_co, "v_add_co_u32 %0, vcc, %0, %1")
KERN32(k_addc_co, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
KERN32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERN32(k_lshl_or, "v_lshl_or_b32 %0, %0, 5, %1")
KERN32(k_and_or, "v_and_or_b32 %0, %0, %1, %0")
KERN32(k_lshl_add32, "v_lshl_add_u32 %0, %0, 4, %1")
KERN32(k_add3, "v_add3_u32 %0, %0, %1, %0")
KERN32(k_or3, "v_or3_b32 %0, %0, %1, %0")
KERN32(k_perm, "v_perm_b32 %0, %0, %1, %1")
KERN32(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
KERN32(k_mul_hi_u24, "v_mul_hi_u32_u24 %0, %0, %1")
KERN32(k_cmp_gt, "v_cmp_gt_u32 vcc, %0, %1")
KERN32(k_sub, "v_sub_u32 %0, %1, %0")
KERN32(k_min, "v_min_u32 %0, %0, %1")
KERN32(k_mov, "v_mov_b32 %0, %1")
KERN32(k_bfi, "v_bfi_b32 %0, %0, %1, %0")
KERN32(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 2")
KERN32(k_log_f32, "v_log_f32 %0, %0")
KERN32(k_lshlrev16x2, "v_pk_lshlrev_b16 %0, 3, %0")
KERN32(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
KERN64(k_cmp_lt_u64, uint64_t, "v_cmp_lt_u64 vcc, %0, %1")
KERN64(k_pk_fma_f32, uint64_t, "v_pk_fma_f32 %0, %0, %1, %0")
KERN64(k_pk_add_f32, uint64_t, "v_pk_add_f32 %0, %0, %1")
KERN64B(k_cvt_f64_i32, double, "v_cvt_f64_i32 %0, %1")
KERN64(k_ldexp_f64, double, "v_ldexp_f64 %0, %0, 3")
KERN64(k_frexp_mant_f64, double, "v_frexp_mant_f64 %0, %1")
KERN64(k_rcp_f64, double, "v_rcp_f64 %0, %0")
KERN64(k_fma_f64_sgpr, double, "v_fma_f64 %0, %0, %1, 1.0")

typedef void (*kfn)(uint32_t *, uint64_t *, uint32_t);
struct K { const char *name; kfn f; };

int main()
{
    K ks[] = {{"v_add_u32", k_add_u32}, {"v_bitop3_b32", k_xor3}, {"v_alignbit_b32", k_alignbit},
              {"v_mul_hi_u32", k_mul_hi_u32}, {"v_mul_lo_u32", k_mul_lo_u32}, {"v_ffbh_u32", k_ffbh},
              {"v_bfe_u32", k_bfe}, {"v_cvt_f32_u32", k_cvt_f32_u32}, {"v_fma_f32", k_fma_f32},
              {"v_lshl_add_u64", k_lshl_add_u64}, {"v_lshlrev_b64", k_lshlrev_b64}, {"v_lshrrev_b64", k_lshrrev_b64},
              {"v_mad_u64_u32", k_mad_u64_u32}, {"v_fma_f64", k_fma_f64}, {"v_add_f64", k_add_f64},
              {"v_mul_f64", k_mul_f64}, {"v_fract_f64", k_fract_f64}, {"v_cvt_f64_u32", k_cvt_f64_u32},
              {"v_mov_b64", k_mov_b64}, {"v_xor_b32", k_xor}, {"v_and_b32", k_and}, {"v_lshlrev_b32", k_lshlrev32},
              {"v_lshrrev_b32", k_lshrrev32}, {"v_add_co_u32", k_add_co}, {"v_addc_co_u32", k_addc_co},
              {"v_cndmask_b32", k_cndmask}, {"v_lshl_or_b32", k_lshl_or}, {"v_and_or_b32", k_and_or},
              {"v_lshl_add_u32", k_lshl_add32}, {"v_add3_u32", k_add3}, {"v_or3_b32", k_or3}, {"v_perm_b32", k_perm},
              {"v_mul_u32_u24", k_mul_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u24}, {"v_cmp_gt_u32", k_cmp_gt},
              {"v_sub_u32", k_sub}, {"v_min_u32", k_min}, {"v_mov_b32", k_mov}, {"v_bfi_b32", k_bfi},
              {"v_alignbyte_b32", k_alignbyte}, {"v_log_f32", k_log_f32}, {"v_pk_lshlrev_b16", k_lshlrev16x2},
              {"v_pk_add_u16", k_pk_add_u16}, {"v_cmp_lt_u64", k_cmp_lt_u64}, {"v_pk_fma_f32", k_pk_fma_f32},
              {"v_pk_add_f32", k_pk_add_f32}, {"v_cvt_f64_i32", k_cvt_f64_i32}, {"v_ldexp_f64", k_ldexp_f64},
              {"v_frexp_mant_f64", k_frexp_mant_f64}, {"v_rcp_f64", k_rcp_f64}, {"v_fma_f64 (const)", k_fma_f64_sgpr}};
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 8 x 4 waves per CU = 8 waves per SIMD
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&cyc, (size_t)blocks * 4 * 8);
    uint64_t *h = new uint64_t[(size_t)blocks * 4];
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    double base_ms = 0;
    printf("%-16s %10s %12s %12s\n", "instruction", "wall_ms", "rel_wall", "cyc/winst");
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, cyc, 7u);  // warm
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, cyc, 7u + r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        hipMemcpy(h, cyc, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost);
        double mean = 0;
        for (int i = 0; i < blocks * 4; ++i) mean += (double)h[i];
        mean /= blocks * 4;
        // s_memtime ticks: per wave, ITERS*CHAINS instructions, 8 waves share the SIMD
        const double cpi = mean * 8.0 / (ITERS * CHAINS);
        if (base_ms == 0) base_ms = ms;
        printf("%-16s %10.4f %12.3f %12.3f\n", k.name, ms, ms / base_ms, cpi);
    }
    return 0;
}
