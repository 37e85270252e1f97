// msim_draws.h — bit-exact random draws of the reference, usable from host and gfx950 device code.
//
//   RNG (xoroshiro128++ + SplitMix64 seeding)   /root/reference/xoroshiro128++.h:4-40
//   NextBlockInterval                          /root/reference/simulation.h:205-210
//   PickFinder                                 /root/reference/simulation.h:213-221
//
// The exponential draw calls glibc's log1p in the reference (xoroshiro128++.h:19). glibc 2.35's
// log1p (sysdeps/ieee754/dbl-64/s_log1p.c) is fdlibm's algorithm with an Estrin-split polynomial; the
// op sequence below was read off the x86-64 libm.so.6 disassembly in this container and is checked
// bit-for-bit against glibc by tests/test_draws.py (CPU) and tests/test_gpu_parity.py (gfx950).
// Every a*b+c here must stay two rounded ops: this header is compiled with -ffp-contract=off and
// carries `#pragma clang fp contract(off)`.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define MSIM_HD __host__ __device__ __forceinline__
#else
#define MSIM_HD inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace msim {

// simulation.h:18 PERC_MULTIPLIER
constexpr uint64_t PERC_MULTIPLIER = 0xFFFFFFFFFFFFFFFFull / 100u;
// simulation.h:16 BLOCK_INTERVAL (600 s) as the nanosecond mean fed to exporand (simulation.h:207)
constexpr double BLOCK_INTERVAL_NS = 600000000000.0;

struct Rng {
    uint64_t s0, s1;
};

MSIM_HD uint64_t splitmix64(uint64_t &seedval)  // xoroshiro128++.h:9-15
{
    uint64_t z = (seedval += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

MSIM_HD Rng rng_seed(uint64_t seed)  // xoroshiro128++.h:23-24
{
    Rng r;
    r.s0 = splitmix64(seed);
    r.s1 = splitmix64(seed);
    return r;
}

// 64-bit rotate; on gfx950 two 32-bit funnel shifts (v_alignbit_b32) per rotate instead of a 64-bit
// shift pair (k is a compile-time constant at every call site).
MSIM_HD uint64_t rotl64(uint64_t x, int k)
{
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if (k >= 32) {
        const uint32_t t = lo;
        lo = hi;
        hi = t;
        k -= 32;
    }
    if (k == 0) return ((uint64_t)hi << 32) | lo;
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - k);
    const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - k);
    return ((uint64_t)nhi << 32) | nlo;
#else
    return (x << k) | (x >> (64 - k));
#endif
}

#if defined(__HIP_DEVICE_COMPILE__)
// One 64-bit add as ONE v_lshl_add_u64. Written as plain C++, LLVM reassociates `rot + s0` (rot built
// from two alignbit halves) into two 64-bit adds plus a move; gfx950 issues every 64-bit integer op at
// the rate of an alignbit (scripts/ubench/valu_rates.hip), so that costs a third of an RNG step.
__device__ __forceinline__ uint64_t add64(uint64_t a, uint64_t b)
{
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
#endif

MSIM_HD uint64_t rng_next(Rng &r)  // xoroshiro128++.h:26-34
{
    const uint64_t s0 = r.s0;
    uint64_t s1 = r.s1;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint64_t result = add64(rotl64(s0 + s1, 17), s0);
    s1 ^= s0;
    // s0' = rotl(s0, 49) ^ s1 ^ (s1 << 21): one three-input XOR per half (v_bitop3_b32, table 0x96)
    const uint64_t ro = rotl64(s0, 49), sh = s1 << 21;
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)ro, (uint32_t)s1, (uint32_t)sh, 0x96);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(ro >> 32), (uint32_t)(s1 >> 32), (uint32_t)(sh >> 32), 0x96);
    r.s0 = ((uint64_t)hi << 32) | lo;
#else
    const uint64_t result = rotl64(s0 + s1, 17) + s0;
    s1 ^= s0;
    r.s0 = rotl64(s0, 49) ^ s1 ^ (s1 << 21);
#endif
    r.s1 = rotl64(s1, 28);
    return result;
}

MSIM_HD int32_t hi_word(double x) { return (int32_t)(__builtin_bit_cast(uint64_t, x) >> 32); }
MSIM_HD double with_hi_word(double x, uint32_t hi)
{
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    return __builtin_bit_cast(double, (b & 0xFFFFFFFFull) | ((uint64_t)hi << 32));
}

// glibc 2.35 log1p, restricted to what the reference's domain can reach: x = -(u>>11)*2^-53, i.e.
// x in [-(1-2^-53), -0]. (NaN/Inf/x<=-1/x>=2^53 branches are unreachable from exporand.)
MSIM_HD double glibc_log1p(double x)
{
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    const double ln2_hi = 6.93147180369123816490e-01;  // 3fe62e42 fee00000
    const double ln2_lo = 1.90821492927058770002e-10;  // 3dea39ef 35793c76
    const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                 Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                 Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                 Lp7 = 1.479819860511658591e-01;
    const int32_t hx = hi_word(x);
    const int32_t ax = hx & 0x7fffffff;
    int32_t k = 1, hu = 0;
    double f = 0.0, c = 0.0;
    if (hx < 0x3FDA827A) {
        if (ax < 0x3e200000) {               // |x| < 2^-29
            if (ax < 0x3c900000) return x;   // |x| < 2^-54
            return x - x * x * 0.5;
        }
        if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {  // -0.2929 < x < 0.41422
            k = 0;
            f = x;
            hu = 1;
        }
    }
    if (k != 0) {
        double u = 1.0 + x;
        hu = hi_word(u);
        k = (hu >> 20) - 1023;
        c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
        c /= u;
        hu &= 0x000fffff;
        if (hu < 0x6a09e) {
            u = with_hi_word(u, (uint32_t)hu | 0x3ff00000u);
        } else {
            k += 1;
            u = with_hi_word(u, (uint32_t)hu | 0x3fe00000u);
            hu = (0x00100000 - hu) >> 2;
        }
        f = u - 1.0;
    }
    const double hfsq = 0.5 * f * f;
    if (hu == 0) {  // |f| < 2^-20
        if (f == 0.0) {
            if (k == 0) return 0.0;
            c += (double)k * ln2_lo;
            return (double)k * ln2_hi + c;
        }
        const double R = hfsq * (1.0 - 0.66666666666666666 * f);
        if (k == 0) return f - R;
        return (double)k * ln2_hi - ((R - ((double)k * ln2_lo + c)) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double R1 = z * Lp1, z2 = z * z;
    const double R2 = Lp2 + z * Lp3, z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5, z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return (double)k * ln2_hi - ((hfsq - (s * (hfsq + R) + ((double)k * ln2_lo + c))) - f);
}

// xoroshiro128++.h:17-20 MakeExponentiallyDistributed
MSIM_HD double exponential_of(uint64_t uniform) { return -glibc_log1p((double)(uniform >> 11) * -0x1.0p-53); }

// simulation.h:205-210: llround(6e11 * E) ns (half away from zero), then duration_cast to ms.
// 6e11*E < 2.3e13 < 2^45, so trunc and the fraction test are exact; the ms quotient is computed
// by a reciprocal estimate plus one exact integer correction (no 64-bit divide on the GPU).
MSIM_HD int64_t interval_ms_of(uint64_t uniform)
{
    const double ns_d = BLOCK_INTERVAL_NS * exponential_of(uniform);
    const double tr = __builtin_trunc(ns_d);
    const int64_t ns = (int64_t)tr + ((ns_d - tr) >= 0.5 ? 1 : 0);
    int64_t q = (int64_t)((double)ns * 1e-6);
    const int64_t r = ns - q * 1000000;
    q += (r >= 1000000 ? 1 : 0) - (r < 0 ? 1 : 0);
    return q;
}

MSIM_HD int64_t next_interval(Rng &r) { return interval_ms_of(rng_next(r)); }

}  // namespace msim
