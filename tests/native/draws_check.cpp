// draws_check.cpp — TEST INFRASTRUCTURE: checks msim_draws.h (the product's host/device draw code)
// bit-for-bit against glibc's log1p/llround, i.e. against exactly what the reference calls
// (xoroshiro128++.h:19, simulation.h:207-209).
//
//   draws_check N_RANDOM THREADS  -> prints mismatch counts as JSON
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <initializer_list>

#include "../../miningsimulation_amd/csrc/msim_draws.h"
#include "../../miningsimulation_amd/csrc/msim_fastdraw.h"

static msim::LogTab g_log;

static int64_t ref_interval(uint64_t u)
{
    const double e = -log1p((double)(u >> 11) * -0x1.0p-53);
    const long long ns = llround(msim::BLOCK_INTERVAL_NS * e);
    return (int64_t)(ns / 1000000LL);
}

struct Job {
    uint64_t n, seed, bad_log1p, bad_interval, first_bad_u, bad_fast, fallbacks;
    double max_err_ns;  // |fast 6e11*E + 0.5 - (fl(6e11*E_glibc) + 0.5)|
};

// The draw kernel's fast interval (msim_fastdraw.h) with its exact fallback, vs the reference.
static void check_fast(uint64_t u, Job *j)
{
    bool ok;
    const int32_t q = msim::interval_ms_fast(u, &g_log, ok);
    const int64_t fast = ok ? (int64_t)q : msim::interval_ms_of(u);
    if (!ok) j->fallbacks++;
    if (fast != ref_interval(u)) {
        j->bad_fast++;
        if (!j->first_bad_u) j->first_bad_u = u;
    }
    // error of the approximation itself (before the margin test), in ns of 6e11*E + 0.5
    const double e = -log1p((double)(u >> 11) * -0x1.0p-53);
    const double yref = msim::BLOCK_INTERVAL_NS * e + 0.5;
    const double err = fabs(msim::interval_fast_z(u, &g_log) * 1e6 - yref);
    if (err > j->max_err_ns) j->max_err_ns = err;
}

static int check_one(uint64_t u, Job *j)
{
    const double x = (double)(u >> 11) * -0x1.0p-53;
    const double a = log1p(x), b = msim::glibc_log1p(x);
    int bad = 0;
    if (memcmp(&a, &b, 8) != 0) {
        j->bad_log1p++;
        bad = 1;
    }
    if (ref_interval(u) != msim::interval_ms_of(u)) {
        j->bad_interval++;
        bad = 1;
    }
    if (bad && !j->first_bad_u) j->first_bad_u = u;
    check_fast(u, j);
    return bad;
}

// PickFinder (simulation.h:213-221) by its linear scan vs the draw kernel's table lookup.
static uint64_t check_picks(uint64_t seed)
{
    msim::Rng r = msim::rng_seed(seed);
    uint64_t bad = 0;
    for (int cfg = 0; cfg < 400; ++cfg) {
        const int m = 1 + (int)(msim::rng_next(r) % 15);
        uint64_t perc[15] = {0};
        int64_t prop[15] = {0};
        uint8_t self[15] = {0};
        int left = 100;
        for (int k = 0; k < m - 1; ++k) {
            perc[k] = msim::rng_next(r) % (uint64_t)(left + 1);
            left -= (int)perc[k];
        }
        perc[m - 1] = (uint64_t)left;
        for (int k = 0; k < m; ++k) prop[k] = (int64_t)(msim::rng_next(r) % 40000);  // < FTHR_CAP
        msim::PickTab tab;
        msim::build_pick_table(perc, prop, self, m, &tab);
        auto scan = [&](uint64_t u) {
            uint64_t i = 0;
            for (int k = 0; k < m; ++k) {
                i += perc[k] * msim::PERC_MULTIPLIER;
                if (i > u) return k;
            }
            return 15;
        };
        auto test = [&](uint64_t u) {
            const uint32_t info = msim::pick_info(u, &tab);
            bool rare;
            const uint32_t qf = msim::pick_q_fast(u, rare);
            if (!rare && tab.info[qf] != info) bad++;  // the fast index is exact whenever it claims to be
            const int k = (int)msim::info_finder(info);
            const uint32_t fthr = msim::info_fthr(info);
            const uint32_t want_thr = k < 15 ? (uint32_t)prop[k] : msim::FTHR_CAP;
            if (k != scan(u) || fthr != want_thr) bad++;
        };
        for (int i = 0; i < 20000; ++i) test(msim::rng_next(r));
        for (uint64_t c = 0; c <= 100; ++c) {
            const uint64_t t = c * msim::PERC_MULTIPLIER;
            for (int64_t d = -3; d <= 3; ++d) test(t + (uint64_t)d);
        }
        test(~0ull);
        test(~0ull - 15);
        test(~0ull - 16);
        for (uint64_t c = 1; c <= 100; ++c) {  // u_hi just below the point where 100 u_hi / 2^32 reaches c
            const uint64_t h = ((c << 32) + 99) / 100 - 1;
            for (int64_t dh = -2; dh <= 0; ++dh)
                for (uint64_t lo : {0ull, 1ull, 0x7FFFFFFFull, 0xFFFFFFF0ull, 0xFFFFFFFFull}) test(((h + dh) << 32) | lo);
        }
    }
    return bad;
}

// Inputs whose 6e11*E + 0.5 lies within a few ns of a millisecond boundary (the fallback's domain).
static void near_boundaries(Job *j, uint64_t *count)
{
    msim::Rng r = msim::rng_seed(99);
    for (int i = 0; i < 200000; ++i) {
        const double qms = (double)(msim::rng_next(r) % 22000000ull);
        const double off = ((double)(int64_t)(msim::rng_next(r) % 8001) - 4000.0) * 1e-3;  // +-4 ns
        const double y = qms * 1e6 - 0.5 + off;
        if (y <= 0) continue;
        const double v = exp(-y / msim::BLOCK_INTERVAL_NS);
        const double m = (1.0 - v) * 0x1.0p53;
        if (!(m >= 0 && m < 9007199254740991.0)) continue;
        const uint64_t mb = (uint64_t)m;
        for (int64_t d = -2; d <= 2; ++d) {
            const uint64_t mm = mb + (uint64_t)d;
            if (mm >= (1ull << 53)) continue;
            check_one((mm << 11) | (msim::rng_next(r) & 0x7FF), j);
            (*count)++;
        }
    }
}

static void *worker(void *p)
{
    Job *j = (Job *)p;
    msim::Rng r = msim::rng_seed(j->seed);
    for (uint64_t i = 0; i < j->n; ++i) check_one(msim::rng_next(r), j);
    return nullptr;
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000000ull;
    const int th = argc > 2 ? atoi(argv[2]) : 8;
    msim::build_log_table(&g_log);
    Job *jobs = (Job *)calloc((size_t)th, sizeof(Job));
    pthread_t *t = (pthread_t *)calloc((size_t)th, sizeof(pthread_t));
    for (int i = 0; i < th; ++i) {
        jobs[i].n = n / (uint64_t)th;
        jobs[i].seed = 0x51ed5eedull + (uint64_t)i;
        pthread_create(&t[i], nullptr, worker, &jobs[i]);
    }
    uint64_t bl = 0, bi = 0, first = 0, total = 0, bf = 0, fb = 0;
    double maxerr = 0;
    for (int i = 0; i < th; ++i) {
        pthread_join(t[i], nullptr);
        bl += jobs[i].bad_log1p;
        bi += jobs[i].bad_interval;
        bf += jobs[i].bad_fast;
        fb += jobs[i].fallbacks;
        if (jobs[i].max_err_ns > maxerr) maxerr = jobs[i].max_err_ns;
        total += jobs[i].n;
        if (!first) first = jobs[i].first_bad_u;
    }
    // Structured sweep: every branch boundary of the fdlibm algorithm and the domain ends.
    Job s = {};
    const uint64_t edges_hi[] = {0x3e200000u, 0x3c900000u, 0xbfd2bec3u, 0xbfd2bec4u, 0xbfd2bec5u,
                                 0xbe200000u, 0xbc900000u, 0xbfefffffu, 0xbfe6a09eu, 0xbfe00000u};
    uint64_t structured = 0;
    for (uint64_t u11 = 0; u11 < 4096; ++u11) {  // smallest and largest (u>>11)
        check_one(u11 << 11, &s);
        check_one(((0x1FFFFFFFFFFFFFull - u11) << 11) | 0x7FF, &s);
        structured += 2;
    }
    for (uint64_t e = 0; e < sizeof(edges_hi) / sizeof(edges_hi[0]); ++e)
        for (int64_t d = -2048; d <= 2048; ++d) {
            // u such that x = -(u>>11)*2^-53 has the given |high word| neighbourhood
            const uint64_t xb = ((edges_hi[e] & 0x7fffffffu) << 32) + (uint64_t)(d * 977);
            double ax;
            memcpy(&ax, &xb, 8);
            const double m = ax * 0x1.0p53;  // (u>>11) as a double
            if (!(m >= 0.0 && m < 9007199254740992.0)) continue;
            const uint64_t q = (uint64_t)m;
            check_one(q << 11, &s);
            structured++;
        }
    uint64_t nb = 0;
    near_boundaries(&s, &nb);
    const uint64_t bp = check_picks(4242);
    if (s.max_err_ns > maxerr) maxerr = s.max_err_ns;
    printf("{\"random\": %llu, \"structured\": %llu, \"near_boundary\": %llu, \"bad_log1p\": %llu, "
           "\"bad_interval\": %llu, \"bad_fast_interval\": %llu, \"fast_fallbacks\": %llu, \"fast_max_err_ns\": %.6g, "
           "\"bad_picks\": %llu, \"first_bad_u\": %llu}\n",
           (unsigned long long)total, (unsigned long long)structured, (unsigned long long)nb,
           (unsigned long long)(bl + s.bad_log1p), (unsigned long long)(bi + s.bad_interval),
           (unsigned long long)(bf + s.bad_fast), (unsigned long long)(fb + s.fallbacks), maxerr,
           (unsigned long long)bp, (unsigned long long)(first ? first : s.first_bad_u));
    return (bl + bi + bf + bp + s.bad_log1p + s.bad_interval + s.bad_fast) ? 1 : 0;
}
