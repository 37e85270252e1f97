/*
 * oracle_cli.c — command-line driver for the CPU oracle (test infrastructure only).
 *
 *   oracle_cli kat                      print SURVEY Appendix B known-answer values
 *   oracle_cli hash PROP_MS RUNS        FNV-1a-64 over per-run {found, bits(share), bits(stale_rate)}
 *   oracle_cli time PRESET RUNS THREADS time RUNS run-years of a preset on THREADS threads
 *                                        (PRESET: c1 | c2 | c3 | c5 | default)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "msim_oracle.h"

#define MONTHS12_MS 31556952000LL /* main.cpp:7 SIM_DURATION = months{12} */

#define C5_M 1026
#define C5_W 102400u

/* SURVEY Appendix C (BASELINE configs[4]): pools 30720, 29696 and 1024 miners of weight 41, W = 102400. */
static uint64_t preset(const char *name, oracle_miner *m, int *n)
{
    if (!strcmp(name, "c5")) {
        *n = C5_M;
        for (int k = 0; k < C5_M; ++k) {
            m[k].id = (uint32_t)k;
            m[k].perc = k == 0 ? 30720u : (k == 1 ? 29696u : 41u);
            m[k].propagation_ms = 1000;
            m[k].is_selfish = 0;
        }
        return C5_W;
    }
    static const uint64_t honest[9] = {30, 29, 12, 11, 8, 5, 3, 1, 1};
    static const uint64_t selfish[9] = {40, 19, 12, 11, 8, 5, 3, 1, 1};
    int64_t prop = 1000;
    const uint64_t *p = honest;
    int s0 = 0;
    if (!strcmp(name, "c1")) prop = 10000;
    else if (!strcmp(name, "c2")) prop = 100;
    else if (!strcmp(name, "c3")) { p = selfish; s0 = 1; }
    *n = 9;
    for (int k = 0; k < 9; ++k) {
        m[k].id = (uint32_t)k;
        m[k].perc = p[k];
        m[k].propagation_ms = prop;
        m[k].is_selfish = (k == 0) ? s0 : 0;
    }
    return 100u;
}

static uint64_t fnv(uint64_t h, uint64_t w) { return (h ^ w) * 0x100000001b3ULL; }

int main(int argc, char **argv)
{
    if (argc < 2) { fprintf(stderr, "usage: oracle_cli kat|hash|time ...\n"); return 2; }
    if (!strcmp(argv[1], "kat")) {
        uint64_t seeds[3] = {0, 1, 4294967295ULL};
        for (int s = 0; s < 3; ++s) {
            oracle_rng r;
            oracle_rng_seed(&r, seeds[s]);
            printf("RNG{%llu}:", (unsigned long long)seeds[s]);
            for (int i = 0; i < 3; ++i) printf(" %016llx", (unsigned long long)oracle_rng_rand64(&r));
            printf("\n");
        }
        oracle_rng r;
        oracle_rng_seed(&r, 1);
        printf("NextBlockInterval(RNG{1}):");
        for (int i = 0; i < 6; ++i) printf(" %lld", (long long)oracle_next_block_interval(&r));
        printf("\n");
        uint64_t perc[9] = {30, 29, 12, 11, 8, 5, 3, 1, 1};
        oracle_rng_seed(&r, 7);
        printf("PickFinder(default9, RNG{7}):");
        for (int i = 0; i < 10; ++i) printf(" %d", oracle_pick_finder(perc, 9, &r));
        printf("\n");
        return 0;
    }
    if (!strcmp(argv[1], "hash") && argc >= 4) {
        oracle_miner m[9];
        int n;
        preset("default", m, &n);
        const int64_t prop = atoll(argv[2]);
        const uint64_t runs = strtoull(argv[3], NULL, 10);
        for (int k = 0; k < n; ++k) m[k].propagation_ms = prop;
        oracle_run_stats *pr = calloc(runs * (uint64_t)n, sizeof(*pr));
        int rc = oracle_run_batch(m, n, MONTHS12_MS, 0, runs, 1000, 8, pr, NULL);
        if (rc) { fprintf(stderr, "rc=%d\n", rc); return 1; }
        uint64_t h = 0xcbf29ce484222325ULL;
        for (uint64_t r = 0; r < runs; ++r)
            for (int k = 0; k < n; ++k) {
                const oracle_run_stats *o = &pr[r * (uint64_t)n + (uint64_t)k];
                uint64_t b1, b2;
                memcpy(&b1, &o->blocks_share, 8);
                memcpy(&b2, &o->stale_rate, 8);
                h = fnv(h, (uint64_t)o->blocks_found);
                h = fnv(h, b1);
                h = fnv(h, b2);
            }
        printf("hash %016llx\nrun0:", (unsigned long long)h);
        for (int k = 0; k < n; ++k) printf(" %lld/%lld", (long long)pr[k].blocks_found, (long long)pr[k].stale_blocks);
        printf("\n");
        free(pr);
        return 0;
    }
    if (!strcmp(argv[1], "time") && argc >= 5) {
        static oracle_miner m[C5_M];
        int n;
        const uint64_t W = preset(argv[2], m, &n);
        const uint64_t runs = strtoull(argv[3], NULL, 10);
        const int threads = atoi(argv[4]);
        static oracle_stats_sum sums[C5_M];
        struct timespec a, b;
        clock_gettime(CLOCK_MONOTONIC, &a);
        int rc = oracle_run_batch_w(m, n, MONTHS12_MS, W, 0, runs, 1000, threads, NULL, sums);
        clock_gettime(CLOCK_MONOTONIC, &b);
        if (rc) { fprintf(stderr, "rc=%d\n", rc); return 1; }
        const double dt = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
        printf("{\"preset\": \"%s\", \"runs\": %llu, \"threads\": %d, \"seconds\": %.4f, \"run_years_per_s\": %.3f}\n",
               argv[2], (unsigned long long)runs, threads, dt, (double)runs / dt);
        for (int k = 0; k < n && k < 9; ++k)
            printf("  miner %d: found %lld share %.6g%% stale %.6g%%\n", k, (long long)(sums[k].blocks_found / (int64_t)runs),
                   sums[k].blocks_share * 100 / (double)runs, sums[k].stale_rate * 100 / (double)runs);
        return 0;
    }
    fprintf(stderr, "bad arguments\n");
    return 2;
}
