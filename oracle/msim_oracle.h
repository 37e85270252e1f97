/* msim_oracle.h — CPU oracle (TEST INFRASTRUCTURE ONLY; see msim_oracle.c header). */
#ifndef MSIM_ORACLE_H
#define MSIM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_EINVAL (-1)
#define ORACLE_EPICK (-2) /* PickFinder fell through: reference asserts (simulation.h:220) */

typedef struct {
    uint64_t s0, s1;
} oracle_rng;

typedef struct {
    uint32_t id;
    uint64_t perc;
    int64_t propagation_ms;
    int32_t is_selfish;
} oracle_miner;

/* Per-run, per-miner MinerStats (main.cpp:13-30) plus the raw stale counter. */
typedef struct {
    int64_t blocks_found;
    int64_t stale_blocks;
    double blocks_share;
    double stale_rate;
} oracle_run_stats;

typedef struct {
    int64_t blocks_found;
    double blocks_share;
    double stale_rate;
} oracle_stats_sum;

typedef struct {
    uint64_t events, finds, best_len;
} oracle_trace;

void oracle_rng_seed(oracle_rng *r, uint64_t seed);
uint64_t oracle_rng_rand64(oracle_rng *r);
double oracle_exporand(oracle_rng *r, double mean);
int64_t oracle_next_block_interval(oracle_rng *r);
int oracle_pick_finder(const uint64_t *perc, int n, oracle_rng *r);
int oracle_pick_finder_w(const uint64_t *perc, int n, uint64_t mult, oracle_rng *r);
int oracle_run_w(const oracle_miner *miners, int n, int64_t duration_ms, uint64_t total_weight,
                 uint32_t seed_interval, uint32_t seed_picker, oracle_run_stats *out, oracle_trace *trace);
int oracle_run_batch_w(const oracle_miner *miners, int n, int64_t duration_ms, uint64_t total_weight,
                       uint64_t run_begin, uint64_t n_runs, uint32_t seed_base, int nthreads,
                       oracle_run_stats *per_run, oracle_stats_sum *sums);

int oracle_run(const oracle_miner *miners, int n, int64_t duration_ms, uint32_t seed_interval,
               uint32_t seed_picker, oracle_run_stats *out, oracle_trace *trace);
int oracle_run_batch(const oracle_miner *miners, int n, int64_t duration_ms, uint64_t run_begin,
                     uint64_t n_runs, uint32_t seed_base, int nthreads, oracle_run_stats *per_run,
                     oracle_stats_sum *sums);

typedef struct oracle_miner_state oracle_miner_state;
oracle_miner_state *oracle_state_new(const oracle_miner *d);
void oracle_state_free(oracle_miner_state *s);
void oracle_state_set_chain(oracle_miner_state *s, const uint32_t *ids, const int64_t *arrivals, size_t len);
size_t oracle_state_get_chain(const oracle_miner_state *s, uint32_t *ids, int64_t *arrivals, size_t cap);
int oracle_state_stale(const oracle_miner_state *s);
void oracle_state_found_block(oracle_miner_state *s, int64_t block_time, size_t best_chain_size);
void oracle_state_notify(oracle_miner_state *s, const uint32_t *ids, const int64_t *arrivals, size_t len, int64_t t);
int64_t oracle_selfish_arrival(void);
void oracle_pick_counts_w(const uint64_t *perc, int n_miners, uint64_t total_weight, uint64_t seed, uint64_t n,
                          uint64_t *out);
void oracle_interval_moments(uint64_t seed, uint64_t n, uint64_t *out);
void oracle_log1p_array(const double *x, double *out, size_t n);
void oracle_interval_of_array(const uint64_t *u, int64_t *out, size_t n);
uint32_t oracle_genesis_id(void);

#ifdef __cplusplus
}
#endif
#endif
