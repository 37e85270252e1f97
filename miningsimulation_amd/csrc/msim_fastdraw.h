// msim_fastdraw.h — the draw kernel's fast, exactly-checked forms of the reference's two draws.
//
// NextBlockInterval (/root/reference/simulation.h:205-210 + xoroshiro128++.h:17-20,36-39) is
//     ms = trunc(llround(6e11 * -log1p(-(u>>11) * 2^-53)) / 1e6)
// with glibc's log1p. Only the millisecond value matters, and it changes only where 6e11*E + 0.5
// crosses a multiple of 1e6. So the fast path evaluates E with a cheap table method (128-entry
// 1/c table, degree-4 log1p polynomial, FMAs allowed) whose total error against glibc's bits is
// < 0.2 ns in 6e11*E, and accepts its result only when 6e11*E + 0.5 lies at least
// MARGIN_NS = 1 ns away from every millisecond boundary; anything closer (2e-6 of draws) is recomputed
// by the bit-exact glibc sequence of msim_draws.h. The result is therefore identical to the
// reference's for every input, not just statistically.
//
// PickFinder (simulation.h:213-221) returns the first miner whose cumulative perc*PERC_MULTIPLIER
// exceeds u. With integer percentages that is lut[floor(u / PERC_MULTIPLIER)], and
// floor(u / PERC_MULTIPLIER) is p1 = floor(100u / 2^64) or p1 + 1 (exactly when u >= (p1+1)*PM), so
// one 64x64 high multiply, one 16-byte table read and one compare replace the M-step scan.
#pragma once
#include <math.h>
#include <stdint.h>

#include "msim_draws.h"

namespace msim {

constexpr int LOG_TAB = 128;
constexpr int PICK_TAB = 100;
constexpr double MARGIN_NS = 1.0;
constexpr uint32_t FTHR_NEVER = (1u << 27) - 1;  // > any interval (max 22 044 720 ms < 2^25)

// Table entry j (w in [1 + j/128, 1 + (j+1)/128)): invc ~ 1/c_j, c_j = 1 + (j + 1/2)/128, and
// A = (0.5 - 6e11 * log(1/invc)) * 1e-6: the entry's share of z = (6e11*E + 0.5) / 1e6 in ms.
struct LogEntry {
    double invc;
    double A;
};
// Pick table entry for p1 = floor(100u/2^64): info for p = p1 (lo) and p = p1 + 1 (hi).
// info = k | fthr << 4: k = finder (15 = fell through, simulation.h:220), fthr = the interval that
// the NEXT draw must exceed for the block to be "fast" (honest finder, next find after arrival).
struct PickEntry {
    uint64_t thr_next;  // (p1 + 1) * PERC_MULTIPLIER
    uint32_t lo, hi;
};

// Fast interval with exactness check; on `ok == false` the caller must use the exact path.
// z = (6e11 * E + 0.5) / 1e6 = A_j - 6e5 * (e*ln2 + log1p(r)), E = -log(v), v = 2^e * w, r = w*invc - 1;
// log1p(r) by a degree-4 polynomial (|r| <= 2^-8: truncation <= 2e-13, i.e. 0.11 ns in 6e11*E).
// The reference's interval is floor(z) whenever frac(z) is at least MARGIN_NS/1e6 from 0 and 1.
constexpr double FD_C1 = -6e5, FD_C2 = 3e5, FD_C3 = -2e5, FD_C4 = 1.5e5;  // -6e5 * (1, -1/2, 1/3, -1/4)
constexpr double FD_CE = -6e5 * 6.93147180559945309417e-01;              // -6e5 * ln 2
MSIM_HD double interval_fast_z(uint64_t u, const LogEntry *__restrict__ tab)
{
    const uint64_t n = (1ull << 53) - (u >> 11);  // 2^53 * (1 + x), exact, in [1, 2^53]
    const int lz = __builtin_clzll(n);
    const int e = 10 - lz;                        // log2(n) - 53
    const uint64_t nn = n << lz;                  // leading one at bit 63
    const int j = (int)((nn >> 56) & (LOG_TAB - 1));
    const double w = __builtin_bit_cast(double, (0x3FFull << 52) | ((nn >> 11) & 0xFFFFFFFFFFFFFull));
    const LogEntry t = tab[j];
    const double r = __builtin_fma(w, t.invc, -1.0);
    double p = __builtin_fma(r, FD_C4, FD_C3);
    p = __builtin_fma(r, p, FD_C2);
    p = __builtin_fma(r, p, FD_C1);
    p = r * p;                                    // -6e5 * log1p(r)
    return __builtin_fma((double)e, FD_CE, t.A + p);
}

MSIM_HD int32_t interval_ms_fast(uint64_t u, const LogEntry *__restrict__ tab, bool &ok)
{
    const double z = interval_fast_z(u, tab);
    const int32_t q = (int32_t)z;                 // z >= 0.5e-6 > 0: truncation = floor
#if defined(__HIP_DEVICE_COMPILE__)
    const double f = __builtin_amdgcn_fract(z);
#else
    const double f = z - (double)q;
#endif
    ok = (f >= MARGIN_NS * 1e-6) && (f <= 1.0 - MARGIN_NS * 1e-6);
    return q;
}

MSIM_HD uint32_t pick_info(uint64_t u, const PickEntry *__restrict__ tab)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t p1 = (uint32_t)__umul64hi(u, 100ull);
#else
    const uint32_t p1 = (uint32_t)(((unsigned __int128)u * 100u) >> 64);
#endif
    const PickEntry e = tab[p1];
    return u >= e.thr_next ? e.hi : e.lo;
}

// ---------------------------------------------------------------- host table builders
inline void build_log_table(LogEntry *out)
{
    for (int j = 0; j < LOG_TAB; ++j) {
        const double c = 1.0 + (j + 0.5) / LOG_TAB;
        const double invc = 1.0 / c;
        out[j].invc = invc;
        const long double L = -logl((long double)invc);  // log(1/invc), 80-bit
        out[j].A = (double)((0.5L - 6e11L * L) * 1e-6L);
    }
}

// perc: integer percentages summing to 100 (validated by the caller); prop: ms; selfish flags.
inline void build_pick_table(const uint64_t *perc, const int64_t *prop, const uint8_t *selfish, int m,
                             PickEntry *out)
{
    uint32_t info[PICK_TAB + 1];
    for (int p = 0; p <= PICK_TAB; ++p) {
        uint64_t cum = 0;
        int k = 15;
        for (int i = 0; i < m; ++i) {
            cum += perc[i];
            if (cum > (uint64_t)p) {
                k = i;
                break;
            }
        }
        uint32_t fthr = FTHR_NEVER;
        if (k < 15 && !selfish[k]) fthr = prop[k] < (int64_t)FTHR_NEVER ? (uint32_t)prop[k] : FTHR_NEVER;
        info[p] = (uint32_t)k | (fthr << 4);
    }
    for (int p1 = 0; p1 < PICK_TAB; ++p1) {
        out[p1].thr_next = (uint64_t)(p1 + 1) * PERC_MULTIPLIER;
        out[p1].lo = info[p1];
        out[p1].hi = info[p1 + 1];
    }
}

}  // namespace msim
