// msim_model.h — the per-run simulation loop as a compact, register-resident state machine.
//
// Replaces, for one run per GPU lane, the reference's
//   RunSimulation                  /root/reference/main.cpp:128-192
//   BestChain / EarliestArrival    /root/reference/main.cpp:68-82, 99-112
//   MinerStats                     /root/reference/main.cpp:13-30
//   Miner::FoundBlock / MaybeReorg / MaybeSelfishReveal / NotifyBestChain / PublishedChain /
//   UnpublishedBlocks / NextArrival / SelfishBlocks                /root/reference/simulation.h:62-180
// with per-run integer counters bit-identical to the reference for identical seeds.
//
// Why a compact state is exact:
//  * every chain is a root path of one block tree, and (owner, height) identifies a block because a
//    miner's tip height strictly increases (simulation.h:126 reorgs only to strictly longer chains,
//    FoundBlock appends one block) — so MaybeReorg's value comparison (simulation.h:130) is a
//    comparison of owners at equal heights, and two chains that differ at height h differ above h;
//  * blocks common to all chains and already published can never be popped and are in the final
//    best chain: they are folded into per-owner counters F[];
//  * the unsettled heights are a 16-height WINDOW; each chain keeps its owners there as 4-bit
//    nibbles in one u64, so a reorg's fork point is ctz(str_k ^ str_B) and its stale count is a
//    popcount of nibble matches;
//  * during a selfish-mining episode the network can split into at most two long branches (measured:
//    SURVEY Q5 / DESIGN.md); blocks below the window on each branch are folded into two per-owner
//    "deep segment" counters DA[], DB[] and each chain carries a 1-bit branch tag.
// Anything outside these capacities sets an error bit for the run (never silently diverges);
// the host re-runs such runs with the larger-capacity instantiation or reports them.
#pragma once
#include "msim_draws.h"

namespace msim {

constexpr int MAXM = 15;       // nibble 0xF is reserved for "no block"
constexpr int WIN = 16;        // window heights (nibbles per u64)
constexpr int NX_FAST = 4;     // extra in-flight honest blocks (beyond one per miner), fast kernel
constexpr int NG_FAST = 4;     // in-flight reveal groups of the selfish miner, fast kernel
constexpr int NX_WIDE = 12;    // ... retry kernel
constexpr int NG_WIDE = 12;
constexpr int FOLD_AT = WIN - 4;
constexpr int64_t T_INF = 0x7FFFFFFFFFFFFFFFll;

enum : uint32_t {
    ERR_WINDOW = 1u,  // an honest chain outgrew the window (long same-branch fork)
    ERR_EXTRA = 2u,   // too many simultaneously in-flight honest blocks
    ERR_GROUPS = 4u,  // too many in-flight reveal groups
    ERR_PICK = 8u,    // PickFinder fell through its table (simulation.h:220 assert)
    ERR_DRAWS = 16u,  // an episode ran past the pre-generated draws of its run
};

// Outcome of one episode (Sim::episode): the run's state machine started from a quiet state at
// block `start` and ran until it was quiet again (end = next unconsumed block) or until the end of
// the run (ended). F are per-owner block-count DELTAS: +1 per episode block in the chain, -1 per
// block consumed (modular u32; see msim_pipeline.h for how they combine).
template <int M>
struct EpisodeOut {
    uint32_t F[M];
    uint32_t S[M];  // stale_blocks increments (simulation.h:133)
    uint32_t end;
    uint32_t ended;
    uint32_t err;
};

struct SimParams {
    int64_t duration_ms;     // main.cpp:7 SIM_DURATION
    int64_t prop[MAXM];      // Miner::propagation (ms), simulation.h:47
    uint64_t thresh[MAXM];   // cumulative perc*PERC_MULTIPLIER, simulation.h:217
    int32_t m;               // number of miners
    int32_t selfish;         // index of the selfish miner or -1 (simulation.h:55 is_selfish)
};

struct RunResult {
    uint32_t found[MAXM];  // MinerStats::blocks_found (main.cpp:24-26)
    uint32_t stale[MAXM];  // Miner::stale_blocks (simulation.h:53, 133)
    uint32_t best_height;  // |best chain| - 1 (main.cpp:28 denominator)
    uint32_t err;
};

// ---------------------------------------------------------------- nibble-string helpers
MSIM_HD uint64_t nib_upto(int hi)  // nibble positions [0, hi]; hi in [-1, 15+]
{
    return hi >= 15 ? ~0ull : (hi < 0 ? 0ull : ((1ull << (4 * (hi + 1))) - 1ull));
}
MSIM_HD uint64_t nib_range(int lo, int hi) { return nib_upto(hi) & ~nib_upto(lo - 1); }
MSIM_HD int count_nib(uint64_t s, uint32_t k, uint64_t range)
{
    const uint64_t x = s ^ (0x1111111111111111ull * (uint64_t)k);
    const uint64_t z = ~(((x & 0x7777777777777777ull) + 0x7777777777777777ull) | x) & 0x8888888888888888ull;
    return __builtin_popcountll(z & range);
}
// Lowest nibble position in [0, hi] where a and b differ, or hi+1.
MSIM_HD int first_diff(uint64_t a, uint64_t b, int hi)
{
    const uint64_t x = (a ^ b) & nib_upto(hi);
    return x ? (__builtin_ctzll(x) >> 2) : hi + 1;
}
MSIM_HD int imin(int a, int b) { return a < b ? a : b; }
MSIM_HD int64_t lmin(int64_t a, int64_t b) { return a < b ? a : b; }

// PickFinder (simulation.h:213-221): first k with cumulative threshold > u. The table is monotone
// (weights validated to sum to <= 100 on the host), so "first k with T_k > u" = #{k : T_k <= u}.
template <int M>
MSIM_HD int pick_finder(const SimParams &p, uint64_t u)
{
    int k = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) k += (p.thresh[i] <= u) ? 1 : 0;
    return k;
}

template <int M, bool SELF, bool DEEP, int NX = NX_FAST, int NG = NG_FAST>
struct Sim {
    static_assert(M >= 1 && M <= MAXM, "miner count");
    uint64_t str[M];   // owners at window heights wb..wb+15 (0xF = none)
    int32_t rt[M];     // tip height - wb   (selfish tip may exceed the window: implicit own run)
    int32_t rp[M];     // published height - wb (PublishedChain, simulation.h:118-121)
    int64_t pa[M];     // arrival of the published tip (BestChain first-seen key, main.cpp:75)
    int64_t na[M];     // honest: arrival of the lowest in-flight own block (NextArrival), T_INF if none
    uint32_t F[M];     // settled per-owner block counts
    uint32_t stl[M];   // stale_blocks
    uint32_t DA[DEEP ? M : 1], DB[DEEP ? M : 1];  // per-owner counts of the two deep branches
    uint32_t grp;      // bit k set: chain k lies on deep branch B
    bool deep;
    int64_t xa[NX];    // extra honest in-flight blocks: arrival
    uint32_t xk[NX];   // key (abs height << 4 | owner), 0xFFFFFFFF = free
    int32_t w;         // selfish withheld count (SelfishBlocks, simulation.h:105-115)
    int32_t gc[NG];    // selfish in-flight reveal groups, oldest first: block count
    int64_t ga[NG];    //   ... and their common arrival
    int32_t ng;
    uint32_t wb;       // absolute height of window position 0
    int32_t bpub;      // previous event's best-chain tip - wb  (best_chain_size - 1, main.cpp:171)
    uint32_t err;

    MSIM_HD void init()
    {
#pragma unroll
        for (int k = 0; k < M; ++k) {
            str[k] = ~0ull;
            rt[k] = -1;
            rp[k] = -1;
            pa[k] = 0;  // Genesis arrival 0 (simulation.h:31-33)
            na[k] = T_INF;
            F[k] = 0;
            stl[k] = 0;
            if (DEEP) {
                DA[k] = 0;
                DB[k] = 0;
            }
        }
        grp = 0;
        deep = false;
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            xa[i] = T_INF;
            xk[i] = 0xFFFFFFFFu;
        }
        w = 0;
#pragma unroll
        for (int i = 0; i < NG; ++i) {
            gc[i] = 0;
            ga[i] = T_INF;
        }
        ng = 0;
        wb = 1;     // genesis (height 0) is settled
        bpub = -1;  // best_chain_size = 1 (main.cpp:149)
        err = 0;
    }

    MSIM_HD bool in_b(int k) const { return DEEP && ((grp >> k) & 1u); }

    MSIM_HD void push_group(int32_t cnt, int64_t arr)
    {
        bool done = false;
#pragma unroll
        for (int i = 0; i < NG; ++i)
            if (!done && i == ng) {
                gc[i] = cnt;
                ga[i] = arr;
                done = true;
            }
        if (done) ng++;
        else err |= ERR_GROUPS;
    }
    MSIM_HD void pop_group()
    {
#pragma unroll
        for (int i = 0; i + 1 < NG; ++i) {
            gc[i] = gc[i + 1];
            ga[i] = ga[i + 1];
        }
        gc[NG - 1] = 0;
        ga[NG - 1] = T_INF;
        ng--;
    }
    MSIM_HD void push_extra(uint32_t key, int64_t arr)
    {
        bool done = false;
#pragma unroll
        for (int i = 0; i < NX; ++i)
            if (!done && xk[i] == 0xFFFFFFFFu) {
                xk[i] = key;
                xa[i] = arr;
                done = true;
            }
        if (!done) err |= ERR_EXTRA;
    }
    MSIM_HD int64_t take_extra(uint32_t key)
    {
        int64_t a = T_INF;
#pragma unroll
        for (int i = 0; i < NX; ++i)
            if (xk[i] == key) {
                a = xa[i];
                xk[i] = 0xFFFFFFFFu;
            }
        if (a == T_INF) err |= ERR_EXTRA;
        return a;
    }
    MSIM_HD void drop_extras(int k)
    {
#pragma unroll
        for (int i = 0; i < NX; ++i)
            if (xk[i] != 0xFFFFFFFFu && (int)(xk[i] & 0xFu) == k) xk[i] = 0xFFFFFFFFu;
    }

    // Slide the window up by s heights (1 <= s <= 15).
    MSIM_HD void shift_all(int s, int sidx)
    {
        wb += (uint32_t)s;
        bpub -= s;
        const uint64_t fill = ~0ull << (64 - 4 * s);
#pragma unroll
        for (int k = 0; k < M; ++k) {
            str[k] = (str[k] >> (4 * s)) | fill;
            rt[k] -= s;
            rp[k] -= s;
            if (SELF && k == sidx && rt[k] >= WIN - s) {
                // heights that enter the window from the selfish miner's implicit own run
                const uint64_t mk = nib_range(WIN - s, imin(rt[k], WIN - 1));
                str[k] = (str[k] & ~mk) | (mk & (0x1111111111111111ull * (uint64_t)k));
            }
        }
    }

    // Fold the lowest window heights that every chain holds and that are published into the
    // settled counters (or, during a two-branch episode, into the two deep-branch counters).
    MSIM_HD void fold(int sidx)
    {
        int minrp = rp[0];
#pragma unroll
        for (int k = 1; k < M; ++k) minrp = imin(minrp, rp[k]);
        if (minrp < 0) return;
        const int cap = imin(minrp + 1, WIN - 1);
        if (!deep) {
            int s = cap;
#pragma unroll
            for (int k = 1; k < M; ++k) s = imin(s, first_diff(str[k], str[0], cap - 1));
            if (s > 0) {
                const uint64_t r = nib_upto(s - 1);
#pragma unroll
                for (int kk = 0; kk < M; ++kk) F[kk] += (uint32_t)count_nib(str[0], (uint32_t)kk, r);
                shift_all(s, sidx);
                return;
            }
            if (!DEEP) return;
            // The chains disagree at the lowest height: split them into two long branches.
            const uint32_t o0 = (uint32_t)(str[0] & 0xFu);
            uint32_t ob = 0xFu, gb = 0;
            bool three = false;
#pragma unroll
            for (int k = 1; k < M; ++k) {
                const uint32_t ok = (uint32_t)(str[k] & 0xFu);
                if (ok != o0) {
                    gb |= 1u << k;
                    if (ob == 0xFu) ob = ok;
                    else if (ok != ob) three = true;
                }
            }
            if (three) return;
            deep = true;
            grp = gb;
        }
        if (DEEP && deep) {
            uint64_t sa = 0, sb = 0;
            bool ha = false, hb = false;
#pragma unroll
            for (int k = 0; k < M; ++k) {
                if (in_b(k)) {
                    if (!hb) sb = str[k];
                    hb = true;
                } else {
                    if (!ha) sa = str[k];
                    ha = true;
                }
            }
            int s = cap;
#pragma unroll
            for (int k = 0; k < M; ++k) s = imin(s, first_diff(str[k], in_b(k) ? sb : sa, cap - 1));
            if (s > 0) {
                const uint64_t r = nib_upto(s - 1);
#pragma unroll
                for (int kk = 0; kk < M; ++kk) {
                    DA[kk] += (uint32_t)count_nib(sa, (uint32_t)kk, r);
                    DB[kk] += (uint32_t)count_nib(sb, (uint32_t)kk, r);
                }
                shift_all(s, sidx);
            }
        }
    }

    // Miner::FoundBlock (simulation.h:62-76) for miner k at time t.
    MSIM_HD void found_block(int k, int64_t t, const SimParams &p)
    {
#pragma unroll
        for (int kk = 0; kk < M; ++kk) {
            if (kk != k) continue;
            if (SELF && kk == p.selfish) {
                const bool is_race = (w == 1) && (bpub == rt[kk]);  // simulation.h:66
                if (is_race) {
                    w = 0;
                    push_group(2, t + p.prop[kk]);  // simulation.h:68-69
                } else {
                    w += 1;  // simulation.h:71
                }
                rt[kk] += 1;
                if (rt[kk] < WIN) str[kk] = (str[kk] & ~(0xFull << (4 * rt[kk]))) | ((uint64_t)kk << (4 * rt[kk]));
            } else {
                if (rt[kk] >= WIN - 1) fold(p.selfish);
                if (rt[kk] >= WIN - 1) {
                    err |= ERR_WINDOW;
                    return;
                }
                rt[kk] += 1;
                str[kk] = (str[kk] & ~(0xFull << (4 * rt[kk]))) | ((uint64_t)kk << (4 * rt[kk]));
                const int64_t arr = t + p.prop[kk];  // simulation.h:74
                if (rt[kk] - rp[kk] == 1) na[kk] = arr;
                else push_extra(((wb + (uint32_t)rt[kk]) << 4) | (uint32_t)kk, arr);
            }
        }
    }

    // Blocks whose arrival is <= t join their chain's published prefix (UnpublishedBlocks, 79-89).
    MSIM_HD void publish(int64_t t, int sidx)
    {
#pragma unroll
        for (int k = 0; k < M; ++k) {
            if (SELF && k == sidx) {
                while (ng > 0 && ga[0] <= t) {
                    rp[k] += gc[0];
                    pa[k] = ga[0];
                    pop_group();
                }
            } else {
                while (na[k] <= t) {
                    rp[k] += 1;
                    pa[k] = na[k];
                    na[k] = (rp[k] < rt[k]) ? take_extra(((wb + (uint32_t)rp[k] + 1u) << 4) | (uint32_t)k) : T_INF;
                }
            }
        }
    }

    // BestChain (main.cpp:68-82): longest published chain, first-seen tie-break, index order.
    MSIM_HD void best(int &bj, int32_t &bl, int64_t &ba, uint64_t &bs, bool &bb) const
    {
        bj = 0;
        bl = rp[0];
        ba = pa[0];
#pragma unroll
        for (int k = 1; k < M; ++k) {
            if (rp[k] > bl || (rp[k] == bl && pa[k] < ba)) {
                bj = k;
                bl = rp[k];
                ba = pa[k];
            }
        }
        bs = str[0];
        bb = in_b(0);
#pragma unroll
        for (int k = 1; k < M; ++k)
            if (k == bj) {
                bs = str[k];
                bb = in_b(k);
            }
    }

    // NotifyBestChain for every miner (main.cpp:165-167 -> simulation.h:177-180).
    MSIM_HD void notify(int64_t t, int32_t bl, int64_t ba, uint64_t bs, bool bb, const SimParams &p)
    {
        const uint64_t bmask = nib_upto(bl);
        const uint64_t bstr = (bs & bmask) | ~bmask;
#pragma unroll
        for (int k = 0; k < M; ++k) {
            const bool selfish = SELF && k == p.selfish;
            if (selfish && bl <= rt[k]) {
                // MaybeSelfishReveal (simulation.h:149-174)
                const int32_t sc = w, lead = rt[k] - bl;
                if (sc > lead) {
                    int32_t rc = sc - lead;
                    if (sc > 1 && lead == 1) rc = sc;
                    push_group(rc, t + p.prop[k]);
                    w -= rc;
                }
            }
            if (bl > rt[k]) {
                // MaybeReorg (simulation.h:124-142): pop to the fork point, count own pops as stale.
                int popped;
                if (DEEP && deep && in_b(k) != bb) {
                    const int hi = imin(rt[k], WIN - 1);
                    popped = (int)(in_b(k) ? DB[k] : DA[k]) + count_nib(str[k], (uint32_t)k, nib_upto(hi)) +
                             (rt[k] > WIN - 1 ? rt[k] - (WIN - 1) : 0);
                } else {
                    const int d = first_diff(str[k], bstr, rt[k]);
                    popped = count_nib(str[k], (uint32_t)k, nib_range(d, rt[k]));
                }
                stl[k] += (uint32_t)popped;
                str[k] = bstr;
                rt[k] = bl;
                rp[k] = bl;
                pa[k] = ba;
                if (selfish) {
                    w = 0;
                    ng = 0;
#pragma unroll
                    for (int i = 0; i < NG; ++i) {
                        gc[i] = 0;
                        ga[i] = T_INF;
                    }
                } else {
                    na[k] = T_INF;
                    drop_extras(k);
                }
                if (DEEP) grp = (grp & ~(1u << k)) | ((bb ? 1u : 0u) << k);
            }
        }
        if (DEEP && deep) {
            const uint32_t all = (1u << M) - 1u;
            if (grp == 0u || grp == all) {  // one branch left: it is common to all chains
#pragma unroll
                for (int k = 0; k < M; ++k) F[k] += grp ? DB[k] : DA[k];
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    DA[k] = 0;
                    DB[k] = 0;
                }
                deep = false;
                grp = 0;
            }
        }
    }

    // EarliestArrival (main.cpp:99-112) over NextArrival (simulation.h:92-102).
    MSIM_HD int64_t earliest_arrival(int64_t t, int sidx) const
    {
        int64_t ea = T_INF;
#pragma unroll
        for (int k = 0; k < M; ++k) {
            if (SELF && k == sidx) {
                if (ng > 0 && ga[0] > t) ea = lmin(ea, ga[0]);
            } else {
                ea = lmin(ea, na[k]);
            }
        }
        return ea;
    }

    // RunSimulation (main.cpp:128-192) for one run; returns the MinerStats inputs.
    MSIM_HD void run(const SimParams &p, Rng ri, Rng rpk, RunResult &out)
    {
        init();
        const int sidx = SELF ? p.selfish : -1;
        const int64_t D = p.duration_ms;
        int64_t nbt = next_interval(ri);  // main.cpp:138
        int64_t t = 0;
        while (t < D && err == 0) {  // main.cpp:150
            while (t == nbt) {       // main.cpp:153-157
                const int k = pick_finder<M>(p, rng_next(rpk));
                if (k >= M) {
                    err |= ERR_PICK;
                    break;
                }
                found_block(k, t, p);
                nbt += next_interval(ri);
            }
            publish(t, sidx);
            int bj;
            int32_t bl;
            int64_t ba;
            uint64_t bs;
            bool bb;
            best(bj, bl, ba, bs, bb);     // main.cpp:164
            notify(t, bl, ba, bs, bb, p);  // main.cpp:165-167
            bpub = bl;                     // main.cpp:171
            if (bl >= FOLD_AT) fold(sidx);
            const int64_t ea = earliest_arrival(t, sidx);  // main.cpp:176-182
            t = lmin(nbt, ea);
        }
        // main.cpp:185-189: BestChain at the end of the run, no notify.
        publish(D, sidx);
        int bj;
        int32_t bl;
        int64_t ba;
        uint64_t bs;
        bool bb;
        best(bj, bl, ba, bs, bb);
        const uint64_t r = nib_upto(bl);
#pragma unroll
        for (int k = 0; k < M; ++k) {
            uint32_t f = F[k] + (uint32_t)count_nib(bs, (uint32_t)k, r);
            if (DEEP && deep) f += bb ? DB[k] : DA[k];
            out.found[k] = f;
            out.stale[k] = stl[k];
        }
        out.best_height = wb + (uint32_t)bl;
        out.err = err;
    }

    // All chains identical and published, nothing withheld or in flight (caller checked ea == T_INF).
    MSIM_HD bool is_quiet() const
    {
        if (DEEP && deep) return false;
        if (SELF && (w != 0 || ng != 0)) return false;
        bool q = true;
#pragma unroll
        for (int k = 1; k < M; ++k) q = q && rt[k] == rt[0] && str[k] == str[0];
#pragma unroll
        for (int k = 0; k < M; ++k) q = q && rp[k] == rt[k];
        return q;
    }

    // One episode of RunSimulation (main.cpp:150-182) that starts in the quiet state at the find of
    // block `src.index` (time T0) and stops at the first event after which the network is quiet
    // again, or at the end of the run (then it also evaluates main.cpp:185-189 like run()).
    // Src: uint32_t word() = (I << 5 | fast << 4 | k) of the current block; bool advance(); index.
    template <class Src>
    MSIM_HD void episode(const SimParams &p, Src &src, int64_t T0, EpisodeOut<M> &out)
    {
        init();
        const int sidx = SELF ? p.selfish : -1;
        const int64_t D = p.duration_ms;
        int64_t nbt = T0, t = T0;
        bool quiet = false;
        while (t < D && err == 0) {
            while (t == nbt) {  // main.cpp:153-157
                const int k = (int)(src.word() & 15u);
                if (k >= M) {
                    err |= ERR_PICK;
                    break;
                }
                found_block(k, t, p);
#pragma unroll
                for (int kk = 0; kk < M; ++kk) F[kk] -= (kk == k) ? 1u : 0u;  // consumed (re-added by the caller)
                if (!src.advance()) {
                    err |= ERR_DRAWS;
                    break;
                }
                nbt += (int64_t)(src.word() >> 5);
            }
            if (err) break;
            publish(t, sidx);
            int bj;
            int32_t bl;
            int64_t ba;
            uint64_t bs;
            bool bb;
            best(bj, bl, ba, bs, bb);
            notify(t, bl, ba, bs, bb, p);
            bpub = bl;
            if (bl >= FOLD_AT) fold(sidx);
            const int64_t ea = earliest_arrival(t, sidx);
            if (ea == T_INF && is_quiet()) {
                quiet = true;
                break;
            }
            t = lmin(nbt, ea);
        }
        out.err = err;
        out.end = src.index;
        out.ended = quiet ? 0u : 1u;
        if (err) return;
        if (quiet) {
            const uint64_t r = nib_upto(rt[0]);
#pragma unroll
            for (int k = 0; k < M; ++k) out.F[k] = F[k] + (uint32_t)count_nib(str[0], (uint32_t)k, r);
        } else {
            publish(D, sidx);  // main.cpp:185: BestChain at the end of the run, no notify
            int bj;
            int32_t bl;
            int64_t ba;
            uint64_t bs;
            bool bb;
            best(bj, bl, ba, bs, bb);
            const uint64_t r = nib_upto(bl);
#pragma unroll
            for (int k = 0; k < M; ++k) {
                uint32_t f = F[k] + (uint32_t)count_nib(bs, (uint32_t)k, r);
                if (DEEP && deep) f += bb ? DB[k] : DA[k];
                out.F[k] = f;
            }
        }
#pragma unroll
        for (int k = 0; k < M; ++k) out.S[k] = stl[k];
    }
};

// Per-run seeds: run r uses rd()-equivalents (base + 2r, base + 2r + 1) mod 2^32;
// the first seeds the interval stream, the second the picker (main.cpp:134).
MSIM_HD uint32_t seed_interval(uint32_t base, uint64_t run) { return (uint32_t)(base + 2u * (uint32_t)run); }
MSIM_HD uint32_t seed_picker(uint32_t base, uint64_t run) { return (uint32_t)(base + 2u * (uint32_t)run + 1u); }

}  // namespace msim
