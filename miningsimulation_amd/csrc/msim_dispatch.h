// msim_dispatch.h — maps a runtime miner count to the compile-time instantiation of the model.
#pragma once
#include "msim_model.h"

// MSIM_FOR_EACH_M(X) expands X(M) for every supported miner count.
#define MSIM_FOR_EACH_M(X) \
    X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

namespace msim {

// Build the kernel parameter block from a reference-style miner list (SetupMiners, main.cpp:44-65):
// perc -> cumulative perc*PERC_MULTIPLIER (simulation.h:217). Returns 0 or a negative error.
static inline int make_params(const uint64_t *perc, const int64_t *prop, const uint8_t *selfish, int m,
                              int64_t duration_ms, SimParams *out)
{
    if (m < 1 || m > MAXM) return -1;
    if (duration_ms < 0) return -1;
    uint64_t total = 0;
    int s = -1;
    for (int k = 0; k < MAXM; ++k) {
        out->prop[k] = 0;
        out->thresh[k] = ~0ull;
    }
    for (int k = 0; k < m; ++k) {
        if (perc[k] > 100u) return -2;
        total += perc[k];
        if (total > 100u) return -2;  // keeps the cumulative table monotone (no u64 wrap)
        if (prop[k] < 0) return -1;
        out->prop[k] = prop[k];
        out->thresh[k] = total * PERC_MULTIPLIER;
        if (selfish[k]) {
            if (s >= 0) return -3;  // at most one selfish miner on the device path
            s = k;
        }
    }
    out->m = m;
    out->selfish = s;
    out->duration_ms = duration_ms;
    return 0;
}

}  // namespace msim
