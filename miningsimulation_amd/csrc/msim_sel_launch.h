// msim_sel_launch.h — host/device interface of the entity-engine path (msim_sel.h): networks with
// selfish miners (BASELINE configs[2], configs[3]).
//
//   D1 msim_word_draws_kernel   (run, segment) workers jump both xoroshiro128++ streams of a run to the
//                               segment start (msim_jump.h) and write one 32-bit word per block:
//                                 interval_ms << 7 | code,  code = floor(u / PERC_MULTIPLIER) in [0, 100]
//                               (simulation.h:205-221). The word does not depend on the network, so a sweep
//                               draws once per run and every point decodes code -> finder with its own
//                               table; weighted networks store the finder itself (code < 16).
//                               Layout: tiles of 32 words per run, [block / 32][run][32], so a worker's
//                               stores and an engine lane's loads both stay inside 128-byte lines.
//   E1 msim_sel_kernel          one lane per (point, run): the settled form + entity engine over the run's
//                               draws, made in-lane (a single network: no word stream) or read from D1's
//                               words (a multi-point sweep); per-run MinerStats terms reduced per workgroup
//                               (fixed-point integers).
//   E2 msim_sel_retry_kernel    one lane per flagged run: the engine with wide capacities and the draws
//                               recomputed in-lane from the seeds, atomically added to per-point sums.
//   G  msim_gen_kernel          the runs E2 could not finish (a chain outgrew the 16-height window: a
//                               selfish majority), on the general engine's explicit chains (msim_general.h).
//   F  msim_sel_finalize        one workgroup per (point, summed value).
#pragma once
#include <hip/hip_runtime.h>

#include "msim_dispatch.h"
#include "msim_fastdraw.h"
#include "msim_sel.h"

namespace msim {

constexpr uint32_t SEL_TILE = 32;  // words per (run, tile)

// Capacities of E1: one selfish miner (the mixed schedule): 1 hot active slot, 4 reveal groups, 1 in-flight
// block per hot slot; several selfish miners (the engine alone): 2 / 4 / 2. Both are backed by SEL_NC cold
// slots in global memory (msim_sel.h). A run that exceeds them anyway is recomputed by E2 (wide capacities,
// one lane per run), so E1 must practically never flag: no run of configs[2] / configs[3] does.
constexpr int SEL_NC = 4;

// One network of a launch (a sweep point).
struct SelParams {
    int64_t duration_ms;
    int64_t prop[MAXM];
    uint64_t cum[MAXM];  // cumulative integer weights (retry draws)
    uint64_t mult;       // UINT64_MAX / W
    uint32_t W;          // total weight (100: the reference's percentages)
    uint32_t m;
    uint32_t ns;         // selfish miners
    uint32_t sids[SEL_MAXS];
    uint32_t uniform_prop;  // 1: every miner has prop[0]
    // word code -> finder = #{k : ccum[k] <= code}: W = 100 words carry q = floor(u / PERC_MULTIPLIER)
    // and ccum = cumulative percentages (first k with cum_k > q, simulation.h:217-218); weighted words
    // carry the finder and ccum[k] = k + 1. Unused entries 0xFFFFFFFF; a result >= m falls through.
    uint32_t ccum[MAXM];
    uint32_t macro;      // 1: one selfish miner, every propagation >= 1 ms (the settled form applies, msim_selm.h)
    uint32_t xth;        // waiting lanes that start an engine phase (mixed schedule, msim_sel_kernels.hip)
    uint32_t pad3;
};

struct WordArgs {
    const LogTab *logt;
    const uint32_t *jump;  // nseg * 128 columns of 4 words
    uint64_t run_begin;    // absolute index of the slice's first run
    uint32_t seed_base;
    uint32_t nr, seg, nseg;
    uint32_t mode;         // 0: code = floor(u / PERC_MULTIPLIER); 1: code = finder (weighted network)
    uint32_t W, m;
    uint64_t mult;
    uint64_t cum[MAXM];
    uint32_t *words;       // [nb / 32][nr][32]
};

struct SelArgs {
    const SelParams *pts;   // all points of the launch (device)
    const uint32_t *plist;  // points of this kernel (device), grid-x = nlist * wps workgroups
    uint32_t nlist;
    uint32_t rpp;           // runs per point
    uint32_t wpp;           // workgroups per point over all slices = ceil(rpp / TPB)
    uint64_t run_begin;
    uint32_t seed_base;
    uint32_t s0, sn;        // slice: runs [s0, s0 + sn) of every point (s0 a multiple of TPB)
    uint32_t nr, nb;        // word geometry of the slice
    const uint32_t *words;  // null: E1 draws in-lane (SelFastDraw) and D1 does not run
    const LogTab *logt;     // interval table of the in-lane draws
    uint64_t *partials;     // [n_points][wpp][6M]
    uint64_t *retry_sums;   // [n_points][6M]
    uint32_t *records;      // [n_points * rpp][M][2] or null
    uint32_t *best_h;       // [n_points * rpp] or null
    uint32_t *counts;       // [0] runs flagged for retry, [1] runs failed on retry
    uint32_t *err_list;     // err_cap codes point * rpp + run
    uint32_t err_cap;
    uint32_t force_retry;   // test switch (MSIM_SEL_FORCE_RETRY): E1 flags every run, E2 computes all
    ColdAct *cold;          // cold slots: [SEL_NC][cold_lanes] (E1 lane = point-list slot * sn + run; E2 lane)
    size_t cold_lanes;
    uint32_t *gen_list;     // runs E2 could not finish, for G (msim_general_launch.h), or null: counted as failed
    uint32_t force_gen;     // test switch (MSIM_SEL_FORCE_GEN): E2 hands every run it gets to G
    uint32_t uni;           // every point of this E1 launch has one propagation delay for all miners
};

struct SelLayout {
    uint32_t nr;    // runs per slice (multiple of 256)
    uint32_t seg;   // blocks per draw worker (multiple of SEL_TILE)
    uint32_t nseg;  // draw workers per run
    uint32_t nb;    // pre-generated blocks per run
    size_t words_bytes;
};

// Slice geometry: nb >= mu + 8 sigma + 64 blocks (a run needing more is flagged and recomputed in E2);
// draw workers per run chosen to fill `slots` resident waves in whole rounds (as msim_pipeline.h).
inline SelLayout sel_layout_for(int64_t duration_ms, uint64_t n_runs, double budget, uint32_t slots)
{
    SelLayout L;
    const double D = (double)duration_ms;
    const double mu = D / 599999.5, sd = sqrt(mu > 1.0 ? mu : 1.0);
    const double need = mu + 8.0 * sd + 64.0;
    const uint64_t want = (n_runs + 255) / 256 * 256;
    uint64_t cap = (uint64_t)(budget / ((need + 2.0 * 512.0) * 4.0)) / 256 * 256;
    if (cap < 256) cap = 256;
    L.nr = (uint32_t)(want < cap ? want : cap);
    if (slots < 1) slots = 1;
    const double rows = L.nr / 64.0;
    uint32_t best_w = 1;
    double best_f = 1e300;
    for (uint32_t w = 1; w <= 256; ++w) {
        const uint32_t sg = (uint32_t)ceil(need / w / SEL_TILE) * SEL_TILE;
        if (sg < 512 && w > 1) break;
        const double f = ceil(rows * w / slots) * (sg + 25.0);
        if (f < best_f * 0.999) {
            best_f = f;
            best_w = w;
        }
    }
    L.nseg = best_w;
    L.seg = (uint32_t)ceil(need / best_w / SEL_TILE) * SEL_TILE;
    if (L.seg < 2 * SEL_TILE) L.seg = 2 * SEL_TILE;
    L.nb = L.nseg * L.seg;
    L.words_bytes = (size_t)L.nb * L.nr * 4;
    return L;
}

hipError_t launch_word_draws(const WordArgs &a, hipStream_t s);
hipError_t word_draws_blocks_per_cu(int *blocks);
// E1 / E2 for miner count m and selfish class (1, 2, 4); dispatch in msim_common.hip.
hipError_t launch_sel(const SelArgs &a, uint32_t m, uint32_t ns_class, hipStream_t s);
hipError_t launch_sel_retry(const SelArgs &a, uint32_t m, uint32_t ns_class, hipStream_t s);
#define MSIM_DECL_SEL(MM)                                                                               \
    hipError_t launch_sel_m##MM(const SelArgs &a, uint32_t ns_class, hipStream_t s);                    \
    hipError_t launch_sel_retry_m##MM(const SelArgs &a, uint32_t ns_class, hipStream_t s);
MSIM_FOR_EACH_M(MSIM_DECL_SEL)
#undef MSIM_DECL_SEL
// F: out[p][i] = sum over the point's workgroup partials + its retried runs; status from counts.
hipError_t launch_sel_finalize(const uint64_t *partials, uint32_t n_points, uint32_t wpp, uint32_t nvals,
                               const uint64_t *retry_sums, uint64_t *out, const uint32_t *counts, uint32_t *status,
                               hipStream_t s);

inline uint32_t sel_ns_class(uint32_t ns) { return ns <= 1 ? 1u : (ns == 2 ? 2u : 4u); }

}  // namespace msim
