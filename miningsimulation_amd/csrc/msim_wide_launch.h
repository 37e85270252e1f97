// msim_wide_launch.h — host-side interface of the large-network pipeline (msim_wide.h / msim_wide.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include <vector>

#include "msim_wide.h"

namespace msim {

struct WideArgs {
    // per-config device tables
    const uint64_t *cf;       // [m + 1] cumulative weight | fast threshold << 32 (msim_wide.h wide_pick)
    const uint16_t *bucket;   // [WB_N]
    const int64_t *prop;                   // [m] propagation (ms)
    const LogTab *logt;
    const uint32_t *jmain;  // [64][128] uint4: T^(lane * S0)
    const uint32_t *jtail;  // [64][128] uint4: T^(B0 + lane * ST)
    const uint32_t *jstep;  // [128] uint4: T^(63 * ST - 1) (next tail chunk)
    uint32_t m, W;
    uint64_t mult;
    int64_t D;
    uint64_t run_begin;  // absolute index of the slice's first run
    uint32_t n;          // runs in the slice
    uint32_t seed_base;
    uint32_t S0, ST, nch, rcap;
    uint64_t B0;
    // per-slice workspace
    uint32_t *hist;   // [nr][m]
    uint32_t *info;   // [nr][4]: n_end, finder of block n_end - 1, candidates, error bits
    int64_t *tlast;   // [nr] T_{n_end - 1}
    WideLane *lanes;  // [nr][1 + nch][64]
    WideCand *cand;   // [nr][rcap]
    uint32_t *recs;   // [nr][rcap][WREC_WORDS]
    uint32_t *work;   // [nr * rcap] dense list of candidate slots (r * rcap + c) for W2
    uint32_t *retry;  // [nr * rcap] slots the first W2 pass flagged WREC_RETRY
    uint32_t *counts; // [2]: work entries, retry entries (zeroed per slice)
};

struct WideOut {
    uint64_t *sums;     // [m][6] msim_sums layout, zeroed before the launch
    uint32_t *records;  // [n_total][m][2] or null
    uint32_t *best_h;   // [n_total] or null
    uint32_t *fail;     // failed-run counter (zeroed before the launch)
    uint64_t run_begin;
    uint64_t n_total;
    uint32_t rel_begin;  // set per slice
};

struct WideLayout {
    uint32_t nr, rcap;
    WideGeom g;
    size_t hist_off, info_off, tlast_off, lanes_off, cand_off, recs_off, work_off, retry_off, counts_off, total;
};

// rho = P(a block is not fast) = sum_k w_k/W * P(I <= prop_k).
inline WideLayout wide_layout_for(double rho, uint32_t m, int64_t duration_ms, uint64_t n_runs, double budget)
{
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    WideLayout L;
    L.g = wide_geom(duration_ms);
    const double blocks = (double)L.g.B0 + 64.0 * L.g.ST * L.g.nch + 64.0;
    const double lam = rho * blocks;
    double rc = ceil(lam + 8.0 * sqrt(lam) + 16.0);
    if (rc > 32000.0) rc = 32000.0;  // slot index fits 15 bits in the combine
    L.rcap = (uint32_t)rc;
    const double per_run = m * 4.0 + 16 + 8 + (1.0 + L.g.nch) * 64 * sizeof(WideLane) +
                           L.rcap * (sizeof(WideCand) + 4.0 * WREC_WORDS + 8.0) + 64;
    uint64_t cap = (uint64_t)(budget / per_run) / 256 * 256;
    if (cap < 256) cap = 256;
    const uint64_t want = (n_runs + 3) / 4 * 4;
    L.nr = (uint32_t)(want < cap ? want : cap);
    size_t o = 0;
    L.hist_off = o;
    o = al(o + (size_t)L.nr * m * 4);
    L.info_off = o;
    o = al(o + (size_t)L.nr * 16);
    L.tlast_off = o;
    o = al(o + (size_t)L.nr * 8);
    L.lanes_off = o;
    o = al(o + (size_t)L.nr * (1 + L.g.nch) * 64 * sizeof(WideLane));
    L.cand_off = o;
    o = al(o + (size_t)L.nr * L.rcap * sizeof(WideCand));
    L.recs_off = o;
    o = al(o + (size_t)L.nr * L.rcap * WREC_WORDS * 4);
    L.work_off = o;
    o = al(o + (size_t)L.nr * L.rcap * 4);
    L.retry_off = o;
    o = al(o + (size_t)L.nr * L.rcap * 4);
    L.counts_off = o;
    o = al(o + 16);
    L.total = o;
    return L;
}

constexpr uint32_t W1_MAX_RUNS = 8;  // runs (waves) per W1 workgroup: 1, 2, 4 or 8, chosen per network
size_t wide_w1_lds(uint32_t m, uint32_t runs);
uint32_t wide_w1_runs(uint32_t m);
size_t wide_w3_lds(uint32_t m, uint32_t rcap, uint32_t nch);
// Runs out.n_total runs slice by slice (L.nr) on stream s; proto carries the tables and geometry.
hipError_t launch_wide(const WideArgs &proto, const WideLayout &L, char *ws, const WideOut &out, hipStream_t s,
                       std::vector<hipEvent_t> *w1_events);
hipError_t launch_sample(int mode, const uint32_t *pow2_jumps, uint64_t seed, uint64_t n, uint32_t S, const uint64_t *cf,
                         const uint16_t *bucket, uint32_t m, uint32_t W, uint64_t mult, const LogTab *logt,
                         unsigned long long *out, hipStream_t s);
hipError_t launch_wide_picks(const WideArgs &a, const uint64_t *u, int32_t *out, uint64_t n, hipStream_t s);

}  // namespace msim
