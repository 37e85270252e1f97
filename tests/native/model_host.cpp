// model_host.cpp — TEST INFRASTRUCTURE: a host (CPU) build of the product's compact state machine
// (miningsimulation_amd/csrc/msim_model.h) so its algorithm can be checked against the oracle on
// machines without a GPU. It is never part of the product path (libmsim.so is GPU-only).
#include <stdint.h>

#include "../../miningsimulation_amd/csrc/msim_dispatch.h"

using namespace msim;

template <int M, bool SELF, bool DEEP>
static void run_one(const SimParams &p, uint32_t si, uint32_t sp, RunResult &r)
{
    Sim<M, SELF, DEEP> s;
    s.run(p, rng_seed(si), rng_seed(sp), r);
}

extern "C" int model_run(const uint64_t *perc, const int64_t *prop, const uint8_t *selfish, int m,
                         int64_t duration_ms, uint32_t seed_i, uint32_t seed_p, int deep, uint32_t *found,
                         uint32_t *stale, uint32_t *best_height, uint32_t *err)
{
    SimParams p;
    const int rc = make_params(perc, prop, selfish, m, duration_ms, &p);
    if (rc) return rc;
    RunResult r;
    const bool self = p.selfish >= 0;
    const bool dp = deep != 0 || self;
#define CASE(MM)                                                                     \
    case MM:                                                                         \
        if (self) run_one<MM, true, true>(p, seed_i, seed_p, r);                     \
        else if (dp) run_one<MM, false, true>(p, seed_i, seed_p, r);                 \
        else run_one<MM, false, false>(p, seed_i, seed_p, r);                        \
        break;
    switch (m) { MSIM_FOR_EACH_M(CASE) default: return -1; }
#undef CASE
    for (int k = 0; k < m; ++k) {
        found[k] = r.found[k];
        stale[k] = r.stale[k];
    }
    *best_height = r.best_height;
    *err = r.err;
    return 0;
}
