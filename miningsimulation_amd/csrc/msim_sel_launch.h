// msim_sel_launch.h — host/device interface of the entity-engine path (msim_sel.h): networks with
// selfish miners (BASELINE configs[2], configs[3]).
//
//   E1 msim_sel_kernel          one lane per (point, run): the settled form (msim_selm.h) with the draws made
//                               in-lane, engine phases per wave for the finds it cannot take (the mixed
//                               schedule, msim_sel_kernels.hip); per-run MinerStats terms reduced per
//                               workgroup (fixed-point integers).
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
    uint32_t xth;        // waiting lanes that start an engine phase (per-wave mixed schedule, E2)
    uint32_t pad3;
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

// Segment-parallel form of E1 for one network with one selfish miner (msim_selseg.h): SW workers over (run,
// segment), then ST stitches each run; ST writes E1's outputs (partials, records, flagged runs for E2).
struct SegArgs {
    const uint32_t *jump;  // nseg jump matrices, 128 uint4 columns each (msim_jump.h build_jump_table, offsets j*seg)
    void *recs;            // [nr][nseg][cap] SegRec<M> (msim_selseg.h)
    uint32_t *cnt;         // [nseg][nr] subs per (segment, run); SEG_OVERFLOW: the worker ran out of room
    void *qrecs;           // [nr][nseg][qcap] SegQRec<M>: the workers' quiet checkpoints
    uint32_t *qcnt;        // [nseg][nr] checkpoints per (segment, run)
    uint32_t nr, nseg, seg, cap, qcap;
    uint32_t xth;          // ST: waiting lanes that start an engine phase
};
constexpr uint32_t SEG_OVERFLOW = 0xFFFFFFFFu;

// E1 / E2 for miner count m and selfish class (1, 2, 4); SW / ST for miner count m; dispatch in msim_common.hip.
hipError_t launch_sel(const SelArgs &a, uint32_t m, uint32_t ns_class, hipStream_t s);
hipError_t launch_sel_retry(const SelArgs &a, uint32_t m, uint32_t ns_class, hipStream_t s);
hipError_t launch_segwork(const SelArgs &a, const SegArgs &g, uint32_t m, hipStream_t s);
hipError_t launch_stitch(const SelArgs &a, const SegArgs &g, uint32_t m, hipStream_t s);
// bytes of one SegRec<m> / SegQRec<m>
size_t seg_rec_bytes(uint32_t m);
size_t seg_qrec_bytes(uint32_t m);
// checkpoint room per (run, segment) for the expected cuts of seg blocks (msim_selseg.h SEG_QWIN, SEG_QEVERY):
// 3/4 of a quiet window per sub + one per SEG_QEVERY blocks + 16; a worker that fills it stores no more
uint32_t seg_qcap(uint32_t cuts, uint32_t seg);
#define MSIM_DECL_SEL(MM)                                                                               \
    hipError_t launch_sel_m##MM(const SelArgs &a, uint32_t ns_class, hipStream_t s);                    \
    hipError_t launch_sel_retry_m##MM(const SelArgs &a, uint32_t ns_class, hipStream_t s);             \
    hipError_t launch_segwork_m##MM(const SelArgs &a, const SegArgs &g, hipStream_t s);                 \
    hipError_t launch_stitch_m##MM(const SelArgs &a, const SegArgs &g, hipStream_t s);
MSIM_FOR_EACH_M(MSIM_DECL_SEL)
#undef MSIM_DECL_SEL
// F: out[p][i] = sum over the point's workgroup partials + its retried runs; status from counts.
hipError_t launch_sel_finalize(const uint64_t *partials, uint32_t n_points, uint32_t wpp, uint32_t nvals,
                               const uint64_t *retry_sums, uint64_t *out, const uint32_t *counts, uint32_t *status,
                               hipStream_t s);

inline uint32_t sel_ns_class(uint32_t ns) { return ns <= 1 ? 1u : (ns == 2 ? 2u : 4u); }

}  // namespace msim
