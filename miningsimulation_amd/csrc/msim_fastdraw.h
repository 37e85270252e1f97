// msim_fastdraw.h — the draw kernel's fast, exactly-checked forms of the reference's two draws.
//
// NextBlockInterval (/root/reference/simulation.h:205-210 + xoroshiro128++.h:17-20,36-39) is
//     ms = trunc(llround(6e11 * -log1p(-(u>>11) * 2^-53)) / 1e6)
// with glibc's log1p. Only the millisecond value matters, and it changes only where 6e11*E + 0.5
// crosses a multiple of 1e6. So the fast path evaluates E with a cheap table method (128-entry
// 1/c table, degree-5 log1p polynomial, FMAs allowed) whose total error against glibc's bits is
// < 0.02 ns in 6e11*E, and accepts its result only when 6e11*E + 0.5 lies at least
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

struct LogEntry {
    double invc;  // ~1/c_j, c_j = 1 + (j + 1/2)/128
    double L;     // -log(invc) = log(1/invc), correctly rounded from an 80-bit evaluation
};

// Pick table entry for p1 = floor(100u/2^64): info for p = p1 (lo) and p = p1 + 1 (hi).
// info = k | fthr << 4: k = finder (15 = fell through, simulation.h:220), fthr = the interval that
// the NEXT draw must exceed for the block to be "fast" (honest finder, next find after arrival).
struct PickEntry {
    uint64_t thr_next;  // (p1 + 1) * PERC_MULTIPLIER
    uint32_t lo, hi;
};

// Fast interval with exactness check; on `ok == false` the caller must use the exact path.
MSIM_HD int32_t interval_ms_fast(uint64_t u, const LogEntry *__restrict__ tab, bool &ok)
{
    const uint64_t n = (1ull << 53) - (u >> 11);  // 2^53 * (1 + x), exact, in [1, 2^53]
    const int lz = __builtin_clzll(n);
    const int e = 10 - lz;                        // log2(n) - 53
    const uint64_t nn = n << lz;                  // leading one at bit 63
    const int j = (int)((nn >> 56) & (LOG_TAB - 1));
    const double w = __builtin_bit_cast(double, (0x3FFull << 52) | ((nn >> 11) & 0xFFFFFFFFFFFFFull));
    const LogEntry t = tab[j];
    const double r = __builtin_fma(w, t.invc, -1.0);
    double p = __builtin_fma(r, 0.2, -0.25);
    p = __builtin_fma(r, p, 1.0 / 3.0);
    p = __builtin_fma(r, p, -0.5);
    p = __builtin_fma(r * r, p, r);
    const double ed = (double)e;
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double lo = __builtin_fma(ed, ln2_lo, t.L + p);
    const double logv = __builtin_fma(ed, ln2_hi, lo);
    const double z = __builtin_fma(-BLOCK_INTERVAL_NS, logv, 0.5);  // 6e11*E + 0.5
    const int32_t q = (int32_t)(z * 1e-6);
    const double rem = __builtin_fma(-(double)q, 1e6, z);
    ok = (rem >= MARGIN_NS) && (rem <= 1e6 - MARGIN_NS);
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
        out[j].L = (double)(-logl((long double)invc));
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
