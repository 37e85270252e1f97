// sel_host.cpp — TEST INFRASTRUCTURE: a host (CPU) build of the product's entity engine
// (miningsimulation_amd/csrc/msim_sel.h) so its algorithm can be checked against the oracle on machines
// without a GPU. Never part of the product path (libmsim.so is GPU-only).
#include <stdint.h>
#include <string.h>

#include "../../miningsimulation_amd/csrc/msim_dispatch.h"
#include "../../miningsimulation_amd/csrc/msim_sel.h"
#include "../../miningsimulation_amd/csrc/msim_selm.h"

using namespace msim;

namespace {

uint32_t g_fold_every = 0;

struct HostEnv {
    const int64_t *props;
    uint32_t c[4][MAXM];
    ColdAct cs[8];
    int64_t prop(uint32_t k) const { return props[k]; }
    int64_t prop_tab(uint32_t k) const { return props[k]; }
    uint32_t get(int a, uint32_t k) const { return c[a][k]; }
    void add(int a, uint32_t k, uint32_t v) { c[a][k] += v; }
    void set(int a, uint32_t k, uint32_t v) { c[a][k] = v; }
    ColdAct cold(int i) const { return cs[i]; }
    void cold_put(int i, const ColdAct &r) { cs[i] = r; }
    uint32_t fold_every;  // 0: fold when due; else also fold at every n-th event (as the device folds early)
    uint32_t nev = 0;
    bool fold_vote(bool due) { return due || (fold_every && ++nev % fold_every == 0); }
};

// Draws exactly as the reference's loop makes them (simulation.h:205-221): finder = first k with
// cum_k > q, q = floor(u / MULT) (weights summing to W; W = 100 is PickFinder with PERC_MULTIPLIER),
// behind the device's draw FIFO (msim_selm.h SelFifo), so the held-draw bookkeeping of the in-lane path
// is exercised too.
struct HostDraw {
    Rng ri, rp;
    const uint64_t *cum;  // cumulative weights
    int m;
    uint64_t W, mult;
    void draw(uint32_t &I, uint32_t &k)
    {
        I = (uint32_t)next_interval(ri);
        const uint64_t u = rng_next(rp);
        const uint64_t q = u / mult;
        uint32_t f = 0;
        while ((int)f < m && cum[f] <= q) ++f;
        k = f;  // == m: fell through (simulation.h:220)
    }
};
using HostSrc = SelFifo<HostDraw>;

template <int M, int NS, int NA, int NG, int NQ, int NC>
void run_one(const int64_t *prop, const uint32_t *sids, HostSrc &src, int64_t D, SelOut &o)
{
    HostEnv env;
    env.props = prop;
    memset(env.c, 0, sizeof(env.c));
    memset(env.cs, 0, sizeof(env.cs));
    env.fold_every = g_fold_every;
    Sel<M, NS, NA, NG, NQ, NC> s;
    s.init((uint32_t)M, sids);
    s.run(env, src, D, o);
}

// The device E1 schedule for one lane (msim_sel_kernels.hip): the settled-state form (msim_selm.h) while
// it applies, the entity engine from a find that needs it until the network is quiet again.
struct MixStats {
    uint64_t macro_steps, exact_steps, entries;
};
MixStats g_mix;
struct LutInit {  // the four-find table (msim_selm.h sp_lut_entry), as the kernels keep it in LDS
    uint32_t t[SP_LUT];
    LutInit()
    {
        for (int i = 0; i < SP_LUT; ++i) t[i] = sp_lut_entry((uint32_t)i / 16u, (uint32_t)i % 16u);
    }
};
const LutInit g_lut_init;
const uint32_t *g_lut = g_lut_init.t;

template <int M, int NS, int NA, int NG, int NQ, int NC>
void run_mixed(const int64_t *prop, const uint32_t *sids, HostSrc &src, int64_t D, SelOut &o)
{
    HostEnv env;
    env.props = prop;
    memset(env.c, 0, sizeof(env.c));
    memset(env.cs, 0, sizeof(env.cs));
    env.fold_every = g_fold_every;
    Sel<M, NS, NA, NG, NQ, NC> s;
    SelMacro<M> mc;
    s.init((uint32_t)M, sids);
    const uint32_t sid = sids[0];
    int64_t thrmax = 0;  // as msim_sel_kernels.hip sel_mixed
    for (int j = 0; j < M; ++j)
        if ((uint32_t)j != sid) thrmax = prop[j] + prop[sid] > thrmax ? prop[j] + prop[sid] : thrmax;
    if (!mc.begin(src)) {
        o.err = SERR_DRAWS;
        return;
    }
    bool macro = true;
    if (mc.T >= D) {
        mc.finish(env, sid, o);
        return;
    }
    for (;;) {
        if (macro) {
            ++g_mix.macro_steps;
            const int r = mc.step4(env, src, D, sid, prop[sid], thrmax, g_lut);
            if (r == 2) {
                mc.finish(env, sid, o);
                return;
            }
            if (r == 1) {
                ++g_mix.entries;
                mc.to_exact(env, s, (uint32_t)M, sids);
                macro = false;
            }
        } else {
            ++g_mix.exact_steps;
            if (!s.step(env, src, D)) {
                s.finish(env, D, o);
                return;
            }
            if (mc.take_back(env, s, sid)) {
                if (mc.T >= D) {
                    mc.finish(env, sid, o);
                    return;
                }
                src.fill();
                macro = true;
            }
        }
    }
}

template <int M, int NS>
void run_caps(int caps, const int64_t *prop, const uint32_t *sids, HostSrc &src, int64_t D, SelOut &o)
{
    // 0: the device E1 capacities (msim_sel_launch.h), 3: a wider register class, 1: retry capacities,
    // 2: one hot slot of everything (the cold paths run constantly), 4: no cold slots (error paths)
    if (caps >= 10 && NS == 1) {  // the mixed schedule (settled form + engine), engine capacities caps - 10
        bool ok = true;
        for (int k = 0; k < M; ++k) ok = ok && prop[k] >= 1;
        if (ok) {
            if (caps == 10) run_mixed<M, NS, 2, 4, 2, 4>(prop, sids, src, D, o);
            else if (caps == 11) run_mixed<M, NS, 1, 2, 1, 4>(prop, sids, src, D, o);
            else run_mixed<M, NS, 1, 4, 1, 4>(prop, sids, src, D, o);
            return;
        }
        caps -= 10;
    }
    if (caps >= 10) caps -= 10;
    if (caps == 0) run_one<M, NS, 2, 4, 2, 4>(prop, sids, src, D, o);
    else if (caps == 1) run_one<M, NS, 4, 16, 4, 6>(prop, sids, src, D, o);
    else if (caps == 2) run_one<M, NS, 1, 4, 1, 6>(prop, sids, src, D, o);
    else if (caps == 3) run_one<M, NS, 3, 8, 3, 4>(prop, sids, src, D, o);
    else run_one<M, NS, 1, 1, 1, 0>(prop, sids, src, D, o);
}

}  // namespace

// Early folds in every later sel_run: 0 = only when due, n = also at every n-th event.
extern "C" void sel_set_fold_every(uint32_t n) { g_fold_every = n; }

// Counters of the mixed schedule since the last call (macro steps, engine steps, hand-overs).
extern "C" void sel_mix_stats(uint64_t *out)
{
    out[0] = g_mix.macro_steps;
    out[1] = g_mix.exact_steps;
    out[2] = g_mix.entries;
    g_mix = MixStats{0, 0, 0};
}

// weights[m] summing to W, prop[m], selfish[m]; caps: see run_caps.
extern "C" int sel_run(const uint64_t *weights, const int64_t *prop, const uint8_t *selfish, int m, uint64_t W,
                       int64_t duration_ms, uint32_t seed_i, uint32_t seed_p, int caps, uint32_t *found,
                       uint32_t *stale, uint32_t *best_height, uint32_t *err)
{
    if (m < 1 || m > MAXM || W == 0) return -1;
    uint64_t cum[MAXM];
    uint64_t c = 0;
    uint32_t sids[SEL_MAXS];
    int ns = 0;
    for (int k = 0; k < SEL_MAXS; ++k) sids[k] = SEL_NONE;
    for (int k = 0; k < m; ++k) {
        c += weights[k];
        cum[k] = c;
        if (selfish[k]) {
            if (ns == SEL_MAXS) return -3;
            sids[ns++] = (uint32_t)k;
        }
    }
    if (c != W) return -2;
    HostSrc src;
    src.d.ri = rng_seed(seed_i);
    src.d.rp = rng_seed(seed_p);
    src.d.cum = cum;
    src.d.m = m;
    src.d.W = W;
    src.d.mult = 0xFFFFFFFFFFFFFFFFull / W;
    src.n = 0;
    SelOut o;
    memset(&o, 0, sizeof(o));
#define CASE(MM)                                                                                 \
    case MM:                                                                                       \
        if (ns == 0) run_caps<MM, 0>(caps, prop, sids, src, duration_ms, o);                      \
        else if (ns == 1) run_caps<MM, 1>(caps, prop, sids, src, duration_ms, o);                 \
        else if (ns == 2) run_caps<MM, 2>(caps, prop, sids, src, duration_ms, o);                 \
        else run_caps<MM, 4>(caps, prop, sids, src, duration_ms, o);                              \
        break;
    switch (m) { MSIM_FOR_EACH_M(CASE) default: return -1; }
#undef CASE
    for (int k = 0; k < m; ++k) {
        found[k] = o.found[k];
        stale[k] = o.stale[k];
    }
    *best_height = o.best_height;
    *err = o.err;
    return 0;
}
