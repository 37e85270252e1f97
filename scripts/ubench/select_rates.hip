// Issue cost of selects and SGPR-operand VALU instructions on gfx950 (measurement tool, not shipped): the
// same harness as valu_rates.hip (8 independent chains per wave, 8 waves per SIMD on every CU); the SGPR
// operands are written once before the timed loop.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096

#define BODY(INS)                                                                                       \
    asm volatile(INS : "+v"(a0) : "v"(b), "s"(sm), "s"(s32));                                                    \
    asm volatile(INS : "+v"(a1) : "v"(b), "s"(sm), "s"(s32));                                                    \
    asm volatile(INS : "+v"(a2) : "v"(b), "s"(sm), "s"(s32));                                                    \
    asm volatile(INS : "+v"(a3) : "v"(b), "s"(sm), "s"(s32));                                                    \
    asm volatile(INS : "+v"(a4) : "v"(b), "s"(sm), "s"(s32));                                                    \
    asm volatile(INS : "+v"(a5) : "v"(b), "s"(sm), "s"(s32));                                                    \
    asm volatile(INS : "+v"(a6) : "v"(b), "s"(sm), "s"(s32));                                                    \
    asm volatile(INS : "+v"(a7) : "v"(b), "s"(sm), "s"(s32));

// sm: a 64-bit SGPR pair (select mask / scalar operand), uniform
#define KERN(NAME, INS)                                                                                 \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint64_t *cyc, uint32_t seed)            \
    {                                                                                                   \
        uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
                 a6 = a0 + 6, a7 = a0 + 7, b = seed * 3u + 1u;                                          \
        uint64_t sm = __builtin_amdgcn_readfirstlane(seed) * 0x9E3779B97F4A7C15ull;                      \
        const uint32_t s32 = (uint32_t)(sm >> 7);                                                      \
        asm volatile("s_mov_b64 vcc, %0" ::"s"(sm));                                                    \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                               \
        for (int i = 0; i < ITERS; ++i) { BODY(INS) }                                                   \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                               \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                    \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;                 \
    }

KERN(k_add, "v_add_u32 %0, %0, %1")
KERN(k_cnd_vcc, "v_cndmask_b32 %0, %0, %1, vcc")
KERN(k_cnd_e64_s, "v_cndmask_b32_e64 %0, %0, %1, %2")
KERN(k_add_s, "v_add_u32 %0, %0, %3")
KERN(k_xor_s, "v_xor_b32 %0, %3, %0")
KERN(k_bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0xCA")
KERN(k_bfi, "v_bfi_b32 %0, %1, %0, %1")
KERN(k_max, "v_max_u32 %0, %0, %1")

typedef void (*kfn)(uint32_t *, uint64_t *, uint32_t);
struct K {
    const char *name;
    kfn f;
};

int main()
{
    K ks[] = {{"v_add_u32", k_add},
              {"v_cndmask_b32 (vcc)", k_cnd_vcc},
              {"v_cndmask_b32_e64 (sgpr mask)", k_cnd_e64_s},
              {"v_add_u32 (sgpr src)", k_add_s},
              {"v_xor_b32 (sgpr src0)", k_xor_s},
              {"v_bitop3_b32 (select form)", k_bitop3},
              {"v_bfi_b32", k_bfi},
              {"v_max_u32", k_max}};
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&cyc, (size_t)blocks * 4 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    double base = 0;
    printf("%-32s %10s %10s\n", "instruction", "wall_ms", "rel_wall");
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, cyc, 7u);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, cyc, 7u + r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        if (base == 0) base = ms;
        printf("%-32s %10.4f %10.3f\n", k.name, ms, ms / base);
    }
    return 0;
}
