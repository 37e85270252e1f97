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

#include "../../miningsimulation_amd/csrc/msim_draws.h"

static int64_t ref_interval(uint64_t u)
{
    const double e = -log1p((double)(u >> 11) * -0x1.0p-53);
    const long long ns = llround(msim::BLOCK_INTERVAL_NS * e);
    return (int64_t)(ns / 1000000LL);
}

struct Job {
    uint64_t n, seed, bad_log1p, bad_interval, first_bad_u;
};

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
    return bad;
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
    Job *jobs = (Job *)calloc((size_t)th, sizeof(Job));
    pthread_t *t = (pthread_t *)calloc((size_t)th, sizeof(pthread_t));
    for (int i = 0; i < th; ++i) {
        jobs[i].n = n / (uint64_t)th;
        jobs[i].seed = 0x51ed5eedull + (uint64_t)i;
        pthread_create(&t[i], nullptr, worker, &jobs[i]);
    }
    uint64_t bl = 0, bi = 0, first = 0, total = 0;
    for (int i = 0; i < th; ++i) {
        pthread_join(t[i], nullptr);
        bl += jobs[i].bad_log1p;
        bi += jobs[i].bad_interval;
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
    printf("{\"random\": %llu, \"structured\": %llu, \"bad_log1p\": %llu, \"bad_interval\": %llu, \"first_bad_u\": %llu}\n",
           (unsigned long long)total, (unsigned long long)structured, (unsigned long long)(bl + s.bad_log1p),
           (unsigned long long)(bi + s.bad_interval), (unsigned long long)(first ? first : s.first_bad_u));
    return (bl + bi + s.bad_log1p + s.bad_interval) ? 1 : 0;
}
