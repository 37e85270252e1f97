/*
 * msim.h — C ABI of libmsim, the MI355X (gfx950) engine for darosior/miningsimulation's per-run
 * simulation loop. Plain pointers and sizes only; no C++ or torch types cross this boundary.
 *
 * What each entry point replaces in the reference (/root/reference):
 *   msim_miner            <- Miner(unsigned id, uint64_t perc, milliseconds prop, bool selfish)
 *                            simulation.h:57-59, as built by SetupMiners() main.cpp:44-65
 *   msim_config_create    <- SetupMiners() + SIM_DURATION (main.cpp:7, 44-65); validates what the
 *                            reference only asserts (simulation.h:220: percentages must sum to 100)
 *   msim_run              <- the std::async batch loop of main() (main.cpp:195-220): SIM_RUNS calls of
 *                            RunSimulation(SIM_DURATION, miners) (main.cpp:128-192, :209) and the
 *                            stats_total[j] += stats[j] aggregation (main.cpp:211-217)
 *   msim_stats            <- MinerStats {long blocks_found; double blocks_share; double stale_rate;}
 *                            (main.cpp:13-20), same field order and types
 *   msim_run_multi        <- the same loop over several GPUs: shards + one RCCL all-reduce of msim_sums
 *   msim_launch           <- device-resident form of msim_run for hosts that own streams and an
 *                            RCCL communicator (multi-GPU: shard runs, all-reduce msim_sums)
 * Seeds: RunSimulation draws two 32-bit std::random_device values (main.cpp:131-134); run r of a
 * launch uses (seed_base + 2r, seed_base + 2r + 1) mod 2^32 for (block_interval, miner_picker).
 */
#ifndef MSIM_H
#define MSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSIM_OK 0
#define MSIM_E_INVALID (-1)  /* bad argument (null pointer, n == 0, negative duration/propagation) */
#define MSIM_E_WEIGHTS (-2)  /* weights do not add up to 100 (or total_weight): the reference asserts */
#define MSIM_E_SELFISH (-3)  /* reserved (round 2 rejected selfish networks the entity engine cannot serve;
                                every network with selfish miners now runs, those on the general engine) */
#define MSIM_E_MINERS (-4)   /* network too large for the general engine: one run's explicit chains (miners x
                                blocks a run can have x 12 B) would exceed 96 GiB (msim_config_create), or the
                                launch's workspace exceeds the device's free memory (msim_run, msim_sweep_run) */
#define MSIM_E_HIP (-5)      /* HIP runtime error (no device, launch failure, out of memory) */
#define MSIM_E_CAPACITY (-6) /* a run outgrew every window of the general engine (its last window holds every
                                block a run of the config's duration can have: practically never) */
#define MSIM_E_PICK (-7)     /* PickFinder fell through (simulation.h:220 assert): percentages < 100 */

#define MSIM_MAX_MINERS 15        /* networks on the compact per-lane / entity-engine state */
#define MSIM_MAX_SELFISH 4        /* selfish miners per network on the entity engine (msim_sel.h); more run on
                                     the general engine (msim_general.h) */
#define MSIM_MAX_WIDE_MINERS 4096 /* honest networks on the large-network pipeline (BASELINE configs[4]); larger
                                     honest networks run on the general engine */

typedef struct msim_miner {
    uint32_t id;            /* Miner::id (simulation.h:43) */
    uint64_t perc;          /* Miner::perc, integer percent of network hashrate (simulation.h:45) */
    int64_t propagation_ms; /* Miner::propagation (simulation.h:47) */
    uint8_t is_selfish;     /* Miner::is_selfish (simulation.h:55) */
} msim_miner;

typedef struct msim_config msim_config;

/* Per-miner aggregate over runs, bit layout of MinerStats (main.cpp:13-20). */
typedef struct msim_stats {
    int64_t blocks_found;
    double blocks_share;
    double stale_rate;
} msim_stats;

/* Order-independent device sums per miner (integers, so 1/2/4/8-GPU all-reduces are bit-identical).
 * share and stale_rate are summed as Q32.32 fixed point split into 32-bit limbs:
 *   sum(share) = share_hi + share_lo * 2^-32 (exact integer sums of per-run round(share * 2^32)). */
typedef struct msim_sums {
    int64_t blocks_found;
    int64_t stale_blocks;
    uint64_t share_hi, share_lo;
    uint64_t rate_hi, rate_lo;
} msim_sums;

/* Per-run, per-miner integer counters (the bit-exact parity surface). */
typedef struct msim_run_record {
    uint32_t found; /* blocks of this miner in the final best chain (main.cpp:24-26) */
    uint32_t stale; /* Miner::stale_blocks at the end of the run (simulation.h:133) */
} msim_run_record;

int msim_config_create(const msim_miner *miners, uint32_t n, int64_t duration_ms, msim_config **out);
/* Weight generalisation (not expressible in the reference, whose perc are integer
 * percentages, simulation.h:45, main.cpp:43): `perc` holds integer weights that must add up to
 * total_weight W < 2^31, and PickFinder uses UINT64_MAX / W in place of PERC_MULTIPLIER
 * (simulation.h:18, 217). W = 100 is exactly msim_config_create. Honest networks of more than
 * MSIM_MAX_MINERS miners (up to MSIM_MAX_WIDE_MINERS), or with W != 100, run on the large-network
 * pipeline; networks with up to MSIM_MAX_SELFISH selfish miners and n <= MSIM_MAX_MINERS (any W) run
 * on the entity engine; every other network with selfish miners (more selfish miners, or more miners) runs
 * on the general engine (msim_general.h: the reference's explicit chains in bounded windows of device
 * memory, slower per block, exact), which also finishes the runs the entity engine cannot (a selfish
 * majority whose withheld chain outgrows its window). The general engine also serves honest networks of
 * more than MSIM_MAX_WIDE_MINERS miners and every network whose ids are not distinct or include UINT_MAX
 * (Genesis's id, simulation.h:31-33): the reference identifies blocks, stale blocks and found blocks by
 * Miner::id (simulation.h:35-38, 133; main.cpp:24-26), and so does that engine. */
int msim_config_create_weighted(const msim_miner *miners, uint32_t n, int64_t duration_ms, uint64_t total_weight,
                                msim_config **out);
/* 1 when the config runs on the large-network pipeline (set MSIM_FORCE_WIDE=1 in the environment before
 * msim_config_create to route small honest networks there too, e.g. for cross-path parity checks). */
int msim_config_is_wide(const msim_config *cfg);
/* How many launches of this config the caller keeps in flight at once (default 1; e.g. 2 when steps
 * alternate over two HIP streams). The event-skipping pipeline plans its draw kernel's grid for it: three
 * rounds of resident waves for one launch, one round each for two. A tuning hint with no effect on results;
 * it changes msim_workspace_bytes, so set it before sizing the workspace. MSIM_E_INVALID outside 1..64.
 * (No reference counterpart: the reference runs one std::async batch at a time, main.cpp:205-220.) */
int msim_config_set_concurrent_launches(msim_config *cfg, uint32_t n);
void msim_config_destroy(msim_config *cfg);
uint32_t msim_config_miner_count(const msim_config *cfg);

/* Run runs [run_begin, run_begin + n_runs) on HIP device `device`.
 * out_sums: M entries (like stats_total, main.cpp:199); with opt_per_run given, the share/stale_rate
 *           doubles are summed on the host in run order exactly as main.cpp:211-217 does; otherwise
 *           they come from the fixed-point device sums (relative error < 1e-9).
 * opt_per_run: n_runs * M records or NULL; opt_best_height: n_runs entries (|best chain| - 1) or NULL.
 * opt_sums: M fixed-point msim_sums or NULL. */
int msim_run(const msim_config *cfg, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base, int device,
             msim_stats *out_sums, msim_sums *opt_sums, msim_run_record *opt_per_run, uint32_t *opt_best_height);

/* Several GPUs of one node (the std::async loop of main.cpp:205-220 across devices): runs
 * [run_begin, run_begin + n_runs) cut into contiguous shards, one per device in `devices` (NULL = devices
 * 0 .. n_devices - 1), each through msim_launch on its own stream (all devices run concurrently), then ONE
 * ncclAllReduce (RCCL over xGMI, single-process communicator from ncclCommInitAll, created once per device
 * list and kept for the process, issued for every device inside one group; none for one device) of the
 * integer msim_sums. Every device's buffers are allocated before anything runs, so
 * an allocation failure returns MSIM_E_HIP without entering a collective. The result is bit-identical to
 * msim_run for every n_devices (out_sums from the fixed-point sums; opt_sums or NULL). */
int msim_run_multi(const msim_config *cfg, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base,
                   const int *devices, uint32_t n_devices, msim_stats *out_sums, msim_sums *opt_sums);
/* msim_run_multi plus per-device timing: opt_shard_ms (2 * n_devices doubles or NULL) receives, for device g,
 * [2g] the milliseconds of its shard's launches and [2g + 1] those of the all-reduce that follows them
 * (HIP events on the device's stream), so a host can see how evenly the shards ran. */
int msim_run_multi_timed(const msim_config *cfg, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base,
                         const int *devices, uint32_t n_devices, msim_stats *out_sums, msim_sums *opt_sums,
                         double *opt_shard_ms);
/* Lifetime of the cached communicators of msim_run_multi / msim_sweep_run_multi: one set per device list,
 * created on first use and kept for the process. msim_multi_release destroys every set no call is using and
 * returns how many it released (a host that cycles through many device lists, or that resets its devices,
 * calls it first). A set whose collectives fail is destroyed at once and re-created by the next call. */
int msim_multi_release(void);

/* Device-resident launch on the current HIP device and the given hipStream_t (NULL = default).
 * d_sums: M msim_sums in device memory (overwritten). d_per_run / d_best_height: device buffers or NULL.
 * d_status: 2 uint32_t in device memory (required): [0] = runs that needed the retry kernel, [1] = runs
 * that failed even there (each failed run contributes nothing to d_sums: check it before using d_sums).
 * d_workspace / workspace_bytes: scratch from msim_workspace_bytes(); the call does no allocation
 * and no synchronisation, so it can be captured into a hipGraph. */
size_t msim_workspace_bytes(const msim_config *cfg, uint64_t n_runs);
int msim_launch(const msim_config *cfg, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base, void *d_sums,
                void *d_per_run, void *d_best_height, void *d_status, void *d_workspace, size_t workspace_bytes,
                void *stream);

/* Device draw primitives (bit-exact with the reference's host libm; test and sampler surface):
 *   msim_device_log1p     glibc log1p on the reference's domain (xoroshiro128++.h:19)
 *   msim_device_intervals NextBlockInterval of given uniform u64 draws, in ms (simulation.h:205-210),
 *                         through the draw kernel's production path (msim_fastdraw.h + exact fallback)
 *   msim_device_picks     PickFinder index of given uniform u64 draws (simulation.h:213-221), through
 *                         the draw kernel's table lookup; -1 where the reference would assert
 * All pointers are device memory; launches go to `stream` (hipStream_t, NULL = default). */
int msim_device_log1p(const double *d_x, double *d_out, uint64_t n, void *stream);
int msim_device_intervals(const uint64_t *d_uniform, int64_t *d_out_ms, uint64_t n, void *stream);
int msim_device_picks(const msim_config *cfg, const uint64_t *d_uniform, int32_t *d_out_index, uint64_t n,
                      void *stream);

/* Parameter sweeps (BASELINE configs[3]: selfish share x propagation grid). The reference runs one
 * network per build (SetupMiners, main.cpp:44-65, edited by hand per README.md:21-27); a sweep runs
 * every point of a grid in ONE device launch, one lane per (point, run). Point p, run r gives exactly
 * the result of msim_run(cfgs[p], run_begin, ...) for run run_begin + r (same seeds for every point).
 * All points must have the same miner count. Sums / records are point-major:
 *   sums[p * M + k], per_run[(p * runs_per_point + r) * M + k], best_height[p * runs_per_point + r]. */
typedef struct msim_sweep msim_sweep;
int msim_sweep_create(const msim_config *const *cfgs, uint32_t n_points, msim_sweep **out);
void msim_sweep_destroy(msim_sweep *sweep);
size_t msim_sweep_workspace_bytes(const msim_sweep *sweep, uint64_t runs_per_point);
/* Device-resident, asynchronous on `stream`; d_sums: n_points * M msim_sums; d_status as msim_launch. */
int msim_sweep_launch(const msim_sweep *sweep, uint64_t run_begin, uint64_t runs_per_point, uint32_t seed_base,
                      void *d_sums, void *d_per_run, void *d_best_height, void *d_status, void *d_workspace,
                      size_t workspace_bytes, void *stream);
uint32_t msim_sweep_point_count(const msim_sweep *sweep);
uint32_t msim_sweep_miner_count(const msim_sweep *sweep);
/* Host convenience: out_stats n_points * M (fixed-point sums converted), optional sums / records. */
int msim_sweep_run(const msim_sweep *sweep, uint64_t run_begin, uint64_t runs_per_point, uint32_t seed_base,
                   int device, msim_stats *out_stats, msim_sums *opt_sums, msim_run_record *opt_per_run,
                   uint32_t *opt_best_height);
/* A sweep over several GPUs as msim_run_multi: every device runs every point on its shard of the runs,
 * one RCCL all-reduce of the n_points * M sums; bit-identical to msim_sweep_run. */
int msim_sweep_run_multi(const msim_sweep *sweep, uint64_t run_begin, uint64_t runs_per_point, uint32_t seed_base,
                         const int *devices, uint32_t n_devices, msim_stats *out_stats, msim_sums *opt_sums);

/* Stage timing for measurement (bench.py): while enabled, every msim_launch records HIP events on its
 * stream around the whole launch and around each draw kernel (K1, the dominant kernel of the
 * event-skipping pipeline). msim_timing_read synchronises on those events, returns the summed
 * elapsed milliseconds and the number of launches since the last enable/read, and clears them. */
int msim_timing_enable(int on);
int msim_timing_read(double *draws_ms, double *launch_ms, uint32_t *launches);
/* Same, plus the entity engine's stage (networks with selfish miners: the E1 kernels of every slice;
 * draws_ms is then the word-draw kernel D1). */
int msim_timing_read_stages(double *draws_ms, double *engine_ms, double *launch_ms, uint32_t *launches);
/* Same, plus BUSY time: the union of the stage's (begin, end) intervals over every stream, i.e. how long at
 * least one such kernel was running (two launches in flight on two streams count their overlap once). With
 * launches alternating over streams this is the stage's share of the wall clock, never more than it. */
typedef struct msim_timing {
    double draws_ms, engine_ms, launch_ms;                 /* summed per-launch intervals */
    double draws_busy_ms, engine_busy_ms, launch_busy_ms;  /* union of the intervals */
    uint32_t launches;
} msim_timing;
int msim_timing_read_all(msim_timing *out);

/* How msim_launch will execute n_runs of this config on the current device. */
typedef struct msim_pipeline_layout {
    uint32_t uses_pipeline;   /* 1: event-skipping pipeline (honest network); 2: large-network pipeline;
                                 3: entity engine (selfish miners); 4: general engine (slice_runs = its
                                 lanes, segment_blocks = its first window, segments = window tiers,
                                 blocks_per_run = its last window); 6: segment-parallel selfish runs
                                 (opt-in, environment MSIM_SELSEG=1; one selfish miner: settled-form workers
                                 per segment + per-run stitch, rho = the expected cuts per find); 0: per-lane
                                 kernel (5 was the removed selfish pipeline) */
    uint32_t slice_runs;      /* runs per pipeline slice */
    uint32_t segment_blocks;  /* blocks per draw-kernel worker */
    uint32_t segments;        /* workers per run */
    uint64_t blocks_per_run;  /* pre-generated blocks per run (segments * segment_blocks) */
    uint64_t workspace_bytes; /* pipeline part of msim_workspace_bytes */
    double rho;               /* probability that a block starts a fork episode */
} msim_pipeline_layout;
int msim_pipeline_info(const msim_config *cfg, uint64_t n_runs, msim_pipeline_layout *out);

/* GPU-scale forms of test.cpp's samplers. One RNG stream RNG{seed} (xoroshiro128++.h:23)
 * of n draws, exactly as the reference's single loops draw it (integer results identical for any n):
 *   msim_sample_picks      out_counts[k] = #{i < n : PickFinder(draw i) == k}, k < M; out_counts[M] = draws
 *                          where PickFinder would assert (simulation.h:220). test.cpp:15-63
 *                          MinerPickerSample (10^8 picks over 100 miners of 1 %) and the stream of
 *                          test.cpp:68-118 MinerPickerSmallBig. out_counts: M + 1 host entries.
 *   msim_sample_intervals  exact integer moments of n NextBlockInterval draws (simulation.h:205-210):
 *                          test.cpp:191-208 BlockIntervalSample (mean and std dev follow from them).
 * Synchronous, on HIP device `device`. */
typedef struct msim_interval_moments {
    uint64_t n;
    uint64_t sum;                /* sum of intervals (ms) */
    uint64_t sumsq_lo, sumsq_hi; /* sum of squared intervals, 128-bit */
    uint64_t max;                /* largest interval (ms) */
} msim_interval_moments;
int msim_sample_picks(const msim_config *cfg, uint64_t seed, uint64_t n, uint64_t *out_counts, int device);
int msim_sample_intervals(uint64_t seed, uint64_t n, msim_interval_moments *out, int device);

/* Convert fixed-point sums to MinerStats-style doubles. */
void msim_sums_to_stats(const msim_sums *sums, uint32_t n, msim_stats *out);

const char *msim_strerror(int code);
const char *msim_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MSIM_H */
