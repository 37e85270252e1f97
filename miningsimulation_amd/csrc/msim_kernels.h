// msim_kernels.h — host-side interface between the C ABI (msim_api.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "msim_dispatch.h"
#include "msim_pipeline.h"

namespace msim {

struct LaunchArgs {
    SimParams p;
    uint64_t run_begin;
    uint32_t n;
    uint32_t seed_base;
    uint64_t *partials;   // partials_words() u64
    uint64_t *sums;       // 6*M u64 (msim_sums layout)
    uint32_t *records;    // n*M*2 u32 or null
    uint32_t *best_h;     // n u32 or null
    uint32_t *err_count;  // 1 u32, zeroed before the launch
    uint32_t *fail_count; // 1 u32, zeroed before the launch
    uint32_t *err_list;   // err_cap u32
    uint32_t err_cap;
    uint32_t *status;     // 2 u32 or null
    hipStream_t stream;
    const PipeLayout *pl; // event-skipping pipeline layout (honest networks) or null (per-lane kernel)
    char *pipe_ws;        // pipeline workspace (pl->total bytes)
    PipeTables tab;       // device tables of the config on this device
    std::vector<hipEvent_t> *k1_events;  // stage timing: (begin, end) pairs around every K1, or null
};

hipError_t launch_runs(const LaunchArgs &a);

// Parameter sweep (BASELINE configs[3]): every point of the sweep in ONE launch of the per-lane kernel.
// Point p owns workgroups [p * wpp, (p + 1) * wpp); run rel of every point uses the seeds of run
// run_begin + rel (the same runs msim_run(cfg_p, run_begin, rpp) simulates).
struct SweepArgs {
    const SimParams *pts;  // n_points parameter blocks in device memory
    uint32_t m;            // miner count (same for every point)
    bool self;             // some point has a selfish miner: use the selfish instantiation for all
    uint32_t n_points;
    uint32_t rpp;          // runs per point
    uint32_t wpp;          // workgroups per point = ceil(rpp / TPB)
    uint64_t run_begin;
    uint32_t seed_base;
    uint64_t *partials;    // [n_points * wpp][6M]
    uint64_t *retry_sums;  // [n_points][6M], zeroed before the launch (retried runs add atomically)
    uint64_t *sums;        // [n_points][6M] out
    uint32_t *records;     // [n_points * rpp][M][2] or null
    uint32_t *best_h;      // [n_points * rpp] or null
    uint32_t *err_count;   // 2 u32 zeroed before the launch: [0] flagged for retry, [1] failed on retry
    uint32_t *err_list;    // err_cap codes (point * wpp * TPB + rel)
    uint32_t err_cap;
    uint32_t *status;      // 2 u32 or null
    hipStream_t stream;
};
hipError_t launch_sweep(const SweepArgs &a);
#define MSIM_DECL_SWEEP(MM) hipError_t launch_sweep_m##MM(const SweepArgs &a);
MSIM_FOR_EACH_M(MSIM_DECL_SWEEP)
#undef MSIM_DECL_SWEEP
hipError_t launch_sweep_finalize(const SweepArgs &a);
#define MSIM_DECL_LAUNCH(MM) hipError_t launch_runs_m##MM(const LaunchArgs &a);
MSIM_FOR_EACH_M(MSIM_DECL_LAUNCH)
#undef MSIM_DECL_LAUNCH
// Launches msim_finalize (msim_common.hip): partial sums -> msim_sums, and the retry status words.
hipError_t launch_finalize(const uint64_t *partials, uint32_t nparts, uint32_t nvals, uint64_t *out,
                           const uint32_t *retry_count, const uint32_t *fail_count, uint32_t retry_cap,
                           uint32_t *status, hipStream_t stream);
hipError_t launch_draws(const DrawArgs &a, hipStream_t s);
hipError_t draws_blocks_per_cu(int *blocks);  // resident K1 workgroups per CU
hipError_t launch_log1p(const double *x, double *out, uint64_t n, hipStream_t s);
// Production draw paths of the pipeline (msim_fastdraw.h) over given uniforms (test/sampler surface).
hipError_t launch_intervals(const LogTab *lt, const uint64_t *u, int64_t *out, uint64_t n, hipStream_t s);
hipError_t launch_picks(const PickTab *pt, const uint64_t *u, int32_t *out, uint64_t n, hipStream_t s);
constexpr int TPB = 256;  // 4 waves of 64 lanes per workgroup
size_t partials_words(uint32_t m, uint32_t n, uint32_t err_cap);

}  // namespace msim
