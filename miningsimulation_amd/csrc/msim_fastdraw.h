// msim_fastdraw.h — the draw kernels' fast, exactly-checked forms of the reference's two draws.
//
// NextBlockInterval (/root/reference/simulation.h:205-210 + xoroshiro128++.h:17-20,36-39) is
//     ms = trunc(llround(6e11 * -log1p(-(u>>11) * 2^-53)) / 1e6)
// with glibc's log1p. Only the millisecond value matters, and it changes only where 6e11*E + 0.5
// crosses a multiple of 1e6. So the fast path evaluates E with a cheap table method (64-entry 1/c
// table, degree-5 log1p polynomial, FMAs allowed) whose total error against glibc's bits is < 0.05 ns
// in 6e11*E, and accepts its result only when 6e11*E + 0.5 lies at least
// MARGIN_NS = 1 ns away from every millisecond boundary; anything closer (2e-6 of draws) is recomputed
// by the bit-exact glibc sequence of msim_draws.h. The result is therefore identical to the
// reference's for every input, not just statistically.
//
// PickFinder (simulation.h:213-221) returns the first miner whose cumulative perc*PERC_MULTIPLIER
// exceeds u. With integer percentages that is lut[q], q = floor(u / PERC_MULTIPLIER), and q is
// p = floor(100 * u_hi / 2^32) (u_hi = u >> 32) unless the low word of 100 * u_hi is within 101 of
// 2^32 (then q = p or p + 1, decided exactly by u >= (p+1) * PM): one 32-bit high multiply, one
// 32-bit low multiply and one 4-byte table read replace the M-step scan; 3e-8 of draws take the
// exact two-multiply path.
//
// Table sizes are set by the LDS banking of gfx950 (MI355X_MICROARCH.md §LDS): a lane-random 16-byte
// read from a 512-entry table conflicted 3-way on average (round-3 K1 counters: 68 % of the LDS cycles
// were bank conflicts), whereas the 64-entry f64 arrays below span at most two entries per bank pair
// and the 101-word pick table at most four words per bank.
#pragma once
#include <math.h>
#include <stdint.h>

#include "msim_draws.h"

namespace msim {

constexpr int LOG_BITS = 6;
constexpr int LOG_TAB = 1 << LOG_BITS;
constexpr int PICK_TAB = 101;  // q = 0 .. 100 (q = 100: PickFinder falls through, simulation.h:220)
constexpr double MARGIN_NS = 1.0;
// Pick info word: finder k in bits 10..13 (so that info & 0x3C00 is the byte offset of owner k's row of a
// [16][256] u32 LDS counter array), fast threshold fthr in bits 14..31. FTHR_CAP bounds fthr: an honest
// network whose delays reach it does not run the pipeline (msim_api.hip); PickFinder's fall-through
// (k = 15) carries FTHR_CAP and is caught by its own counter (msim_pipeline.h combine_run).
constexpr uint32_t INFO_K_SHIFT = 10, INFO_T_SHIFT = 14;
constexpr uint32_t FTHR_NEVER = (1u << 27) - 1;  // large-network tables (msim_wide.h): > any interval
constexpr uint32_t FTHR_CAP = (1u << (32 - INFO_T_SHIFT)) - 1;  // 262 143 ms
MSIM_HD uint32_t info_finder(uint32_t info) { return (info >> INFO_K_SHIFT) & 15u; }
MSIM_HD uint32_t info_fthr(uint32_t info) { return info >> INFO_T_SHIFT; }
MSIM_HD uint32_t make_info(uint32_t k, uint32_t fthr) { return (k << INFO_K_SHIFT) | (fthr << INFO_T_SHIFT); }

// Log table, structure of arrays: entry j covers w in [1 + j/LOG_TAB, 1 + (j+1)/LOG_TAB); invc ~ 1/c_j,
// c_j = 1 + (j + 1/2)/LOG_TAB, and A = (0.5 - 6e11 * log(1/invc)) * 1e-6: the entry's share of
// z = (6e11*E + 0.5) / 1e6 in ms.
struct LogTab {
    double invc[LOG_TAB];
    double A[LOG_TAB];
};
// Pick table: info[q] = make_info(k, fthr) for q = floor(u / PERC_MULTIPLIER): k = finder (15 = fell
// through), fthr = the interval the NEXT draw must exceed for the block to be "fast" (honest finder, next
// find after its arrival).
struct PickTab {
    uint32_t info[128];
};

// Fast interval with exactness check; on `ok == false` the caller must use the exact path.
// v = 1 - (u>>11)*2^-53 is formed EXACTLY from the two 32-bit halves of u (both partial results are
// multiples of 2^-53 in (0, 1], so neither rounding loses a bit), v = 2^e * w with w in [1, 2) read off
// its bits, and z = (6e11 * E + 0.5) / 1e6 = A_j - 6e5 * (e*ln2 + log1p(r)), E = -log(v), r = w*invc_j - 1
// (|r| <= 2^-7: the degree-5 truncation r^6/6 is < 4e-14, i.e. <= 0.025 ns in 6e11*E).
// The reference's interval is floor(z) whenever frac(z) is at least MARGIN_NS/1e6 from 0 and 1.
constexpr double FD_C1 = -6e5, FD_C2 = 3e5, FD_C3 = -2e5, FD_C4 = 1.5e5, FD_C5 = -1.2e5;  // -6e5 * (-1)^(k+1) / k
constexpr double FD_CE = -6e5 * 6.93147180559945309417e-01;                              // -6e5 * ln 2
#if defined(__HIP_DEVICE_COMPILE__)
// u32 -> f64 as one v_cvt_f64_u32 (LLVM widens a converted `u >> 32` into a 64-bit conversion that adds
// a +0.0 it cannot fold away).
__device__ __forceinline__ double u32_to_f64(uint32_t x)
{
    double d;
    asm("v_cvt_f64_u32 %0, %1" : "=v"(d) : "v"(x));
    return d;
}
#else
MSIM_HD double u32_to_f64(uint32_t x) { return (double)x; }
#endif

// Polynomial constants as values the caller hoists into scalar registers once (fd_consts) and passes
// down: every Horner step is then ONE three-operand VOP3 FMA with the constant as its SGPR addend. With
// literal constants the compiler emits v_fmac, which overwrites its addend, and copies the constant into
// a fresh register pair before every draw.
// The leading coefficient (a multiplicand of the first step, beside the SGPR addend) lives in a VGPR:
// one VOP3 instruction reads at most one SGPR on gfx950.
#ifndef MSIM_FD_C5_VGPR
#define MSIM_FD_C5_VGPR 1
#endif
struct FdConsts {
    double c1, c2, c3, c4, c5;
};
MSIM_HD FdConsts fd_consts()
{
    FdConsts k{FD_C1, FD_C2, FD_C3, FD_C4, FD_C5};
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+s"(k.c1));
    asm("" : "+s"(k.c2));
    asm("" : "+s"(k.c3));
    asm("" : "+s"(k.c4));
#if MSIM_FD_C5_VGPR
    asm("" : "+v"(k.c5));
#endif
#endif
    return k;
}
#define MSIM_FD_DEFAULT FdConsts{FD_C1, FD_C2, FD_C3, FD_C4, FD_C5}

MSIM_HD double interval_fast_z(uint64_t u, const LogTab *__restrict__ tab, FdConsts kc = MSIM_FD_DEFAULT)
{
    const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    const double c = __builtin_fma(u32_to_f64(lo >> 11), -0x1.0p-53, 1.0);  // exact
    const double v = __builtin_fma(u32_to_f64(hi), -0x1.0p-32, c);           // exact: 1 - (u>>11) 2^-53
    const uint64_t vb = __builtin_bit_cast(uint64_t, v);
    const uint32_t vh = (uint32_t)(vb >> 32);
    const int e = (int)(vh >> 20) - 1023;                                    // v = 2^e w, e in [-53, 0]
    const uint32_t j = (vh >> (20 - LOG_BITS)) & (LOG_TAB - 1);              // top LOG_BITS mantissa bits
    const double w = __builtin_bit_cast(double, (vb & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
#if defined(__HIP_DEVICE_COMPILE__)
    // A_j through a base the compiler cannot relate to invc_j's: two ds_read_b64 (64-bank, at most two
    // entries per bank pair) instead of one merged ds_read2st64_b64 (32-bank, up to four)
    uint32_t aoff = j * 8u;
    asm("" : "+v"(aoff));
    const double Aj = *(const double *)((const char *)tab->A + aoff);
#else
    const double Aj = tab->A[j];
#endif
    const double r = __builtin_fma(w, tab->invc[j], -1.0);
    double p = __builtin_fma(r, kc.c5, kc.c4);
    p = __builtin_fma(r, p, kc.c3);
    p = __builtin_fma(r, p, kc.c2);
    p = __builtin_fma(r, p, kc.c1);
    const double z0 = __builtin_fma(r, p, Aj);                               // A_j - 6e5 log1p(r)
    return __builtin_fma((double)e, FD_CE, z0);
}

// Acceptance on the high word of frac(z) (a positive double below 1: integer order = value order):
// strictly inside (hi(MARGIN), hi(1 - MARGIN)) implies frac in (MARGIN, 1 - MARGIN); a high word equal
// to either bound falls back to the exact path (a 2^-20 relative sliver of that band).
constexpr uint32_t FD_OK_LO = 0x3EB0C6F7u + 1u;  // hi(1e-6) + 1
constexpr uint32_t FD_OK_HI = 0x3FEFFFFDu;       // hi(1 - 1e-6) (exclusive)
constexpr uint32_t FD_OK_RANGE = FD_OK_HI - FD_OK_LO;
// Fast interval and its acceptance key: the result is the reference's iff key < FD_OK_RANGE (keys of
// several draws combine with max).
MSIM_HD int32_t interval_ms_fast_key(uint64_t u, const LogTab *__restrict__ tab, uint32_t &key,
                                     FdConsts kc = MSIM_FD_DEFAULT)
{
    const double z = interval_fast_z(u, tab, kc);
    const int32_t q = (int32_t)z;                 // z >= 0.5e-6 > 0: truncation = floor
#if defined(__HIP_DEVICE_COMPILE__)
    const double f = __builtin_amdgcn_fract(z);
#else
    const double f = z - (double)q;
#endif
    key = (uint32_t)(__builtin_bit_cast(uint64_t, f) >> 32) - FD_OK_LO;
    return q;
}
MSIM_HD int32_t interval_ms_fast(uint64_t u, const LogTab *__restrict__ tab, bool &ok, FdConsts kc = MSIM_FD_DEFAULT)
{
    uint32_t key;
    const int32_t q = interval_ms_fast_key(u, tab, key, kc);
    ok = key < FD_OK_RANGE;
    return q;
}

// PickFinder's table index q = floor(u / PERC_MULTIPLIER), fast form: p = floor(100 u_hi / 2^32), exact
// unless `rare` (the low word of 100 u_hi is >= 2^32 - 128; q = p + 1 needs it >= 2^32 - 101).
constexpr uint32_t PICK_RARE_LO = 0xFFFFFF80u;  // low word of 100 u_hi at or above it: the exact path
MSIM_HD uint32_t pick_q_fast_key(uint64_t u, uint32_t &key)  // key = low word of 100 u_hi
{
    const uint32_t h = (uint32_t)(u >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t p = __umulhi(h, 100u);
#else
    const uint32_t p = (uint32_t)(((uint64_t)h * 100u) >> 32);
#endif
    key = h * 100u;
    return p;
}
MSIM_HD uint32_t pick_q_fast(uint64_t u, bool &rare)
{
    uint32_t key;
    const uint32_t p = pick_q_fast_key(u, key);
    rare = key >= PICK_RARE_LO;
    return p;
}
// Exact q for any u: p or p + 1, exactly when u >= (p+1) * PERC_MULTIPLIER.
MSIM_HD uint32_t pick_q_exact(uint64_t u)
{
    bool rare;
    const uint32_t p = pick_q_fast(u, rare);
    return p + (u >= (uint64_t)(p + 1) * PERC_MULTIPLIER ? 1u : 0u);
}
MSIM_HD uint32_t pick_info(uint64_t u, const PickTab *__restrict__ tab)
{
    bool rare;
    uint32_t q = pick_q_fast(u, rare);
    if (rare) q = pick_q_exact(u);
    return tab->info[q];
}

// ---------------------------------------------------------------- host table builders
inline void build_log_table(LogTab *out)
{
    for (int j = 0; j < LOG_TAB; ++j) {
        const double c = 1.0 + (j + 0.5) / LOG_TAB;
        const double invc = 1.0 / c;
        out->invc[j] = invc;
        const long double L = -logl((long double)invc);  // log(1/invc), 80-bit
        out->A[j] = (double)((0.5L - 6e11L * L) * 1e-6L);
    }
}

// perc: integer percentages summing to 100 (validated by the caller); prop: ms; selfish flags.
inline void build_pick_table(const uint64_t *perc, const int64_t *prop, const uint8_t *selfish, int m, PickTab *out)
{
    for (int q = 0; q < 128; ++q) {
        uint64_t cum = 0;
        int k = 15;
        for (int i = 0; i < m && q < PICK_TAB; ++i) {
            cum += perc[i];
            if (cum > (uint64_t)q) {
                k = i;
                break;
            }
        }
        uint32_t fthr = FTHR_CAP;
        if (k < 15 && !selfish[k]) fthr = prop[k] < (int64_t)FTHR_CAP ? (uint32_t)prop[k] : FTHR_CAP;
        out->info[q] = make_info((uint32_t)k, fthr);
    }
}

}  // namespace msim
