// msim_sel.h — the entity engine: RunSimulation for networks with selfish miners (and any <= 15-miner
// network), one run per lane, exact.
//
// Replaces, per run, the reference's
//   RunSimulation                  /root/reference/main.cpp:128-192
//   BestChain / EarliestArrival    /root/reference/main.cpp:68-82, 99-112
//   Miner::FoundBlock / MaybeReorg / MaybeSelfishReveal / NotifyBestChain / PublishedChain /
//   UnpublishedBlocks / NextArrival / SelfishBlocks                /root/reference/simulation.h:62-180
//
// The per-lane kernel of msim_model.h keeps one chain per MINER and walks all of them at every event
// (measured 4 970 VALU lane-ops per simulated block at 9 miners). Here state is kept per ENTITY:
//   P       the passive class: every honest miner whose chain is the common chain. Its members share one
//           chain, see the same BestChain and apply the same MaybeReorg (simulation.h:124-142), hold only
//           published blocks, and in BestChain (main.cpp:68-82: index order, strict comparisons) act as
//           one candidate at the lowest member index;
//   S_i     one entity per selfish miner (simulation.h:55): withheld count (SelfishBlocks, 105-115) and
//           the in-flight reveal groups (MaybeSelfishReveal, 149-174);
//   A_j     active honest miners: a miner leaves P when it finds a block (FoundBlock, 73-75) and rejoins
//           it as soon as its chain is the common chain again, all published.
// BestChain is the lexicographic maximum of (published length, -tip arrival, -miner index) over the
// entities, which is what the reference's strict-comparison scan over miners in index order returns.
//
// Chains use msim_model.h's exact compact form ((owner, height) identifies a block): a
// 16-height window of 4-bit owners per entity above settled per-owner counters, two deep-branch counter
// sets for long selfish episodes, and an implicit single-owner run above the window (a selfish miner's
// withheld run, or anything that adopted it). Per-owner counters live in the Env (LDS on the device).
//
// Hot and cold slots. P, the selfish entities and NA active slots live in registers. A miner that
// becomes active when the NA slots are taken, or whose in-flight queue outgrows NQ, moves to one of NC
// COLD slots kept in the Env (global memory on the device) with a deeper queue. Cold slots are touched
// only when some lane of a wave has one (measured: the second active slot is needed in 8-11 % of wave
// iterations at 1 s, a third far less), so the common path stays short and register-resident while a run
// practically never exceeds a capacity. Anything that does (all cold slots taken, a window that cannot
// fold) sets an error bit and the run is recomputed with wider capacities: results never depend on them.
#pragma once
#include "msim_model.h"

// Region markers for the host SIMT probe (tests/native); no code in product builds.
#ifndef SEL_HIT
#define SEL_HIT(region)
#endif
// Engine-step section timing (diagnostic device builds only, -DSEL_ENGPROF=1): cycles per section of step(),
// accumulated per lane in sel_engprof[] (the kernel prints them).
#if defined(__HIP_DEVICE_COMPILE__) && defined(SEL_ENGPROF) && SEL_ENGPROF
namespace msim {
__device__ void sel_engprof_acc(int i, uint64_t c);
}
#define SEL_EP_DECL uint64_t ep_t = clock64()
#define SEL_EP(i)                                      \
    do {                                               \
        const uint64_t ep_n = clock64();               \
        sel_engprof_acc(i, ep_n - ep_t);               \
        ep_t = ep_n;                                   \
    } while (0)
#else
#define SEL_EP_DECL
#define SEL_EP(i)
#endif

namespace msim {

constexpr uint32_t SEL_NONE = 0xFu;  // "no owner" (miner ids are < 15)
constexpr int SEL_MAXS = 4;          // selfish miners per network supported by the entity engine
constexpr int SEL_NQC = 6;           // in-flight blocks of a cold active slot
enum : uint32_t {
    SERR_WIN = 2u,     // a chain outgrew the window and could not fold
    SERR_PICK = 4u,    // PickFinder fell through (simulation.h:220 assert)
    SERR_DRAWS = 8u,   // the run outlasted its pre-generated draws
    SERR_ACT = 16u,    // active slots (hot and cold) exhausted
    SERR_GRP = 32u,    // reveal groups exhausted
    SERR_QUE = 64u,    // in-flight queue of a cold active slot exhausted
    SERR_CAP = SERR_ACT | SERR_GRP | SERR_QUE,
};
// Counter arrays of the Env: settled found, stale_blocks, deep branch A, deep branch B.
enum : int { C_F = 0, C_S = 1, C_A = 2, C_B = 3 };

struct SelOut {
    uint32_t found[MAXM];
    uint32_t stale[MAXM];
    uint32_t best_height;
    uint32_t err;
};

// One chain: owners at window heights wb..wb+15 (0xF above the tip), tip and published tip heights
// relative to wb (heights WIN..rt are owned by xo, the implicit run), arrival of the published tip
// (BestChain's first-seen key, main.cpp:75), deep branch (0 = A, 1 = B).
struct Ent {
    uint64_t s;
    int32_t rt, rp;
    int64_t pa;
    uint32_t xo, br;
};

// A cold active slot (Env storage).
struct ColdAct {
    Ent x;
    uint32_t aid;  // its miner
    int32_t nq;
    int64_t q[SEL_NQC];  // own in-flight blocks, lowest first
};

// The best chain of one event: published tip height, tip arrival, window string truncated at the tip,
// implicit run owner (heights >= WIN), deep branch.
struct SelBest {
    int32_t l;
    int64_t a;
    uint64_t s;
    uint32_t x, br;
};

MSIM_HD void ent_reset(Ent &x)
{
    x.s = ~0ull;
    x.rt = -1;  // genesis (height 0) is settled: wb = 1
    x.rp = -1;
    x.pa = 0;   // Genesis arrival (simulation.h:31-33)
    x.xo = SEL_NONE;
    x.br = 0;
}

// Room for a block of owner o at height rt + 1: inside the window, the first implicit-run height, or an
// implicit run of the same owner.
MSIM_HD bool ent_room(const Ent &x, uint32_t o) { return (x.rt + 1 <= WIN) | (x.xo == o); }

MSIM_HD void ent_append(Ent &x, uint32_t o)
{
    const int h = x.rt + 1;
    if (h < WIN) x.s = (x.s & ~(0xFull << (4 * h))) | ((uint64_t)o << (4 * h));
    else if (h == WIN) x.xo = o;
    x.rt = h;
}

MSIM_HD void ent_shift(Ent &x, int s, uint64_t fill)
{
    x.s = (x.s >> (4 * s)) | fill;
    x.rt -= s;
    x.rp -= s;
    if (x.rt >= WIN - s && x.xo != SEL_NONE) {  // heights entering the window from the implicit run
        const uint64_t mk = nib_range(WIN - s, imin(x.rt, WIN - 1));
        x.s = (x.s & ~mk) | (mk & (0x1111111111111111ull * (uint64_t)x.xo));
    }
    if (x.rt < WIN) x.xo = SEL_NONE;
}

// c ? a : b field by field. A conditional whole-struct copy would become a copy through a selected
// pointer, which keeps both structs out of registers.
MSIM_HD Ent ent_pick(bool c, const Ent &a, const Ent &b)
{
    Ent r;
    r.s = c ? a.s : b.s;
    r.rt = c ? a.rt : b.rt;
    r.rp = c ? a.rp : b.rp;
    r.pa = c ? a.pa : b.pa;
    r.xo = c ? a.xo : b.xo;
    r.br = c ? a.br : b.br;
    return r;
}

// An active miner whose chain is the class's chain again, all published, rejoins the class.
MSIM_HD bool ent_same_as_p(const Ent &x, const Ent &P)
{
    // bitwise, not short-circuit: these run for most lanes of every wave iteration (no branches)
    return (x.rp == x.rt) & (x.rt == P.rt) & (x.s == P.s) & (x.xo == P.xo) & (x.br == P.br);
}

// Env: int64_t prop(uint32_t k); int64_t prop_tab(uint32_t k) (same value, as a table read); uint32_t get(int arr, uint32_t k); void add(int arr, uint32_t k, uint32_t v);
//      void set(int arr, uint32_t k, uint32_t v); ColdAct cold(int c); void cold_put(int c, const ColdAct &);
//      bool fold_vote(bool due)  (fold now: at least `due`; may be true when not due).
// Src: bool next(uint32_t &interval_ms, uint32_t &finder)  (finder >= M: PickFinder fell through).
template <int M, int NS, int NA, int NG, int NQ, int NC>
struct Sel {
    static_assert(M >= 1 && M <= MAXM, "miner count");
    static_assert(NS >= 0 && NS <= SEL_MAXS && NA >= 1 && NG >= 1 && NQ >= 1 && NC >= 0 && NC <= 7, "capacities");
    static constexpr int NSA = NS > 0 ? NS : 1;

    Ent P;
    Ent S[NSA];
    Ent A[NA];
    uint32_t sidv[NSA];
    int32_t w[NSA];    // withheld blocks (SelfishBlocks)
    int32_t ng[NSA];   // in-flight reveal groups, oldest first
    int32_t gc[NSA][NG];
    int64_t ga[NSA][NG];
    uint32_t aid[NA];  // miner of each hot active slot
    int32_t nq[NA];    // own in-flight blocks, lowest first (only own blocks are ever unpublished)
    int64_t q[NA][NQ];
    uint32_t sv, av, cm;  // valid selfish entities / hot active slots / occupied cold slots
    uint32_t caid;     // miner of each cold slot, 4 bits per slot
    uint32_t am, hm, sm;  // active / honest / selfish miner masks
    uint32_t wb;       // absolute height of window position 0
    int32_t bpub;      // previous event's best tip - wb (best_chain_size - 1, main.cpp:171)
    bool deep;
    uint32_t err;

    MSIM_HD bool sval(int si) const { return (sv >> si) & 1u; }
    MSIM_HD bool aval(int a) const { return (av >> a) & 1u; }
    MSIM_HD bool cval(int c) const { return (cm >> c) & 1u; }
    MSIM_HD uint32_t cold_aid(int c) const { return (caid >> (4 * c)) & 15u; }

    // sids: NSA selfish miner ids in index order (SEL_NONE for unused entries); m miners.
    MSIM_HD void init(uint32_t m, const uint32_t *sids)
    {
        sm = 0;
        sv = 0;
        ent_reset(P);
#pragma unroll
        for (int si = 0; si < NSA; ++si) {
            sidv[si] = NS > 0 ? sids[si] : SEL_NONE;
            if (sidv[si] != SEL_NONE) {
                sm |= 1u << sidv[si];
                sv |= 1u << si;
            }
            ent_reset(S[si]);
            w[si] = 0;
            ng[si] = 0;
#pragma unroll
            for (int i = 0; i < NG; ++i) {
                gc[si][i] = 0;
                ga[si][i] = T_INF;
            }
        }
        hm = ((1u << m) - 1u) & ~sm;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            ent_reset(A[a]);
            aid[a] = SEL_NONE;
            nq[a] = 0;
#pragma unroll
            for (int i = 0; i < NQ; ++i) q[a][i] = T_INF;
        }
        av = 0;
        cm = 0;
        caid = 0;
        am = 0;
        wb = 1;
        bpub = -1;  // best_chain_size = 1 (main.cpp:149)
        deep = false;
        err = 0;
    }

    MSIM_HD void push_group(int si, int32_t c, int64_t arr)
    {
        if (ng[si] >= NG) {
            err |= SERR_GRP;
            return;
        }
        // unconditional selects: a predicated store per slot would become a store through a selected
        // pointer and keep the queue out of registers
#pragma unroll
        for (int i = 0; i < NG; ++i) {
            const bool me = i == ng[si];
            gc[si][i] = me ? c : gc[si][i];
            ga[si][i] = me ? arr : ga[si][i];
        }
        ng[si]++;
    }

    // ------------------------------------------------------------------ cold slots
    MSIM_HD int free_cold() const
    {
        int c = -1;
#pragma unroll
        for (int i = NC - 1; i >= 0; --i)
            if (!cval(i)) c = i;
        return c;
    }
    MSIM_HD void take_cold(int c, uint32_t k)
    {
        cm |= 1u << c;
        caid = (caid & ~(15u << (4 * c))) | (k << (4 * c));
    }

    // ------------------------------------------------------------------ Miner::FoundBlock
    // simulation.h:62-76 for miner k at time T. A passive miner leaves the class with its chain.
    template <class Env>
    MSIM_HD void found(Env &env, uint32_t k, int64_t T)
    {
        const int64_t arr = T + env.prop(k);
        if ((sm >> k) & 1u) {
            SEL_HIT(1);
#pragma unroll
            for (int si = 0; si < NS; ++si) {
                if (sidv[si] != k) continue;
                if (!ent_room(S[si], k)) {
                    err |= SERR_WIN;
                    return;
                }
                const bool race = (w[si] == 1) & (bpub == S[si].rt);  // simulation.h:66
                if (race) {
                    w[si] = 0;
                    push_group(si, 2, arr);  // simulation.h:68-69: both blocks arrive at T + prop
                } else {
                    w[si] += 1;  // simulation.h:71 (SELFISH_ARRIVAL)
                }
                ent_append(S[si], k);
            }
            return;
        }
        // An honest miner: its hot slot, a free hot slot (leaving the class), or the cold path.
        int at = -1;
        const bool was_active = (am >> k) & 1u;
        if (was_active) {
            SEL_HIT(2);
#pragma unroll
            for (int a = 0; a < NA; ++a)
                if (aval(a) && aid[a] == k) at = a;
        } else {
            SEL_HIT(3);
#pragma unroll
            for (int a = NA - 1; a >= 0; --a)
                if (!aval(a)) at = a;
        }
        bool hot = at >= 0;
        int32_t qn = 0;
#pragma unroll
        for (int a = 0; a < NA; ++a)
            if (a == at) qn = was_active ? nq[a] : 0;
        if (hot && qn >= NQ) hot = false;  // a hot slot whose queue is full moves to a cold slot
        if (hot) {
            // selects over the slots (see push_group)
            Ent x = P;
#pragma unroll
            for (int a = 0; a < NA; ++a) x = ent_pick(a == at && was_active, A[a], x);
            if (!ent_room(x, k)) {
                err |= SERR_WIN;
                return;
            }
            ent_append(x, k);
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                const bool me = a == at;
                A[a].s = me ? x.s : A[a].s;
                A[a].rt = me ? x.rt : A[a].rt;
                A[a].rp = me ? x.rp : A[a].rp;
                A[a].pa = me ? x.pa : A[a].pa;
                A[a].xo = me ? x.xo : A[a].xo;
                A[a].br = me ? x.br : A[a].br;
                aid[a] = me ? k : aid[a];
#pragma unroll
                for (int i = 0; i < NQ; ++i) q[a][i] = (me && i == qn) ? arr : q[a][i];  // simulation.h:74
                nq[a] = me ? qn + 1 : nq[a];
            }
            av |= 1u << at;
            am |= 1u << k;
            return;
        }
        found_cold(env, k, at, was_active, arr);
    }

    // The cold path of found(): miner k is in a cold slot, or needs one (no free hot slot, or its hot
    // slot `at` has a full queue and moves).
    template <class Env>
    MSIM_HD void found_cold(Env &env, uint32_t k, int at, bool was_active, int64_t arr)
    {
        SEL_HIT(19);
        int c = -1;
        ColdAct r;
        if (at >= 0) {  // migrate hot slot `at`
            c = free_cold();
            if (c < 0) {
                err |= SERR_ACT;
                return;
            }
            r.x = P;
            r.nq = 0;
#pragma unroll
            for (int i = 0; i < SEL_NQC; ++i) r.q[i] = T_INF;
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                const bool me = a == at;
                r.x = ent_pick(me, A[a], r.x);
                r.nq = me ? nq[a] : r.nq;
#pragma unroll
                for (int i = 0; i < NQ; ++i) r.q[i] = me ? q[a][i] : r.q[i];
            }
            r.aid = k;
            av &= ~(1u << at);
            take_cold(c, k);
        } else if (was_active) {  // already cold
#pragma unroll
            for (int i = 0; i < NC; ++i)
                if (cval(i) && cold_aid(i) == k) c = i;
            r = env.cold(c);
        } else {  // leaves the class into a cold slot
            c = free_cold();
            if (c < 0) {
                err |= SERR_ACT;
                return;
            }
            r.x = P;
            r.aid = k;
            r.nq = 0;
#pragma unroll
            for (int i = 0; i < SEL_NQC; ++i) r.q[i] = T_INF;
            take_cold(c, k);
            am |= 1u << k;
        }
        if (!ent_room(r.x, k)) {
            err |= SERR_WIN;
            return;
        }
        if (r.nq >= SEL_NQC) {
            err |= SERR_QUE;
            return;
        }
        ent_append(r.x, k);
#pragma unroll
        for (int i = 0; i < SEL_NQC; ++i) r.q[i] = i == r.nq ? arr : r.q[i];  // simulation.h:74
        r.nq++;
        env.cold_put(c, r);
    }

    // ------------------------------------------------------------------ window maintenance
    template <class Env>
    MSIM_HD void add_nibs(Env &env, int arr, uint64_t s, int n)
    {
        for (int j = 0; j < n; ++j) {
            const uint32_t o = (uint32_t)(s >> (4 * j)) & 15u;
            if (o < (uint32_t)M) env.add(arr, o, 1u);
        }
    }

    template <class Env>
    MSIM_HD void shift(Env &env, int s)
    {
        wb += (uint32_t)s;
        bpub -= s;
        const uint64_t fill = ~0ull << (64 - 4 * s);
        ent_shift(P, s, fill);
#pragma unroll
        for (int si = 0; si < NSA; ++si) ent_shift(S[si], s, fill);
#pragma unroll
        for (int a = 0; a < NA; ++a) ent_shift(A[a], s, fill);
        if (cm) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (cval(c)) {
                    ColdAct r = env.cold(c);
                    ent_shift(r.x, s, fill);
                    env.cold_put(c, r);
                }
        }
    }

    // Visits every entity slot with f(const Ent &, bool valid): the register-resident slots without a
    // branch (f selects on `valid`), the cold slots only when the lane has any.
    template <class Env, class F>
    MSIM_HD void each(Env &env, F f) const
    {
        f(P, true);
#pragma unroll
        for (int si = 0; si < NS; ++si) f(S[si], sval(si));
#pragma unroll
        for (int a = 0; a < NA; ++a) f(A[a], aval(a));
        if (cm) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (cval(c)) {
                    const ColdAct r = env.cold(c);
                    f(r.x, true);
                }
        }
    }

    // Fold the lowest window heights that every chain holds (all published) into the settled counters,
    // or, during a two-branch episode, into the deep-branch counters of each branch.
    // An early fold (not `due`) only shifts: splitting into deep mode waits until the lane needs room.
    template <class Env>
    MSIM_HD void fold(Env &env, bool due)
    {
        SEL_HIT(14);
        if (deep) SEL_HIT(18);
        int minrp = P.rt;
        each(env, [&](const Ent &x, bool v) { minrp = v ? imin(minrp, x.rp) : minrp; });
        if (minrp < 0) return;
        const int cap = imin(minrp + 1, WIN - 1);
        if (!deep) {
            int s = cap;
            each(env, [&](const Ent &x, bool v) { s = v ? imin(s, first_diff(x.s, P.s, cap - 1)) : s; });
            if (s > 0) {
                SEL_HIT(17);
                add_nibs(env, C_F, P.s, s);
                shift(env, s);
                return;
            }
            if (!due) return;
            // The chains disagree at the lowest height: split them into two long branches.
            const uint32_t o0 = (uint32_t)(P.s & 15u);
            uint32_t ob = SEL_NONE;
            bool three = false;
            each(env, [&](const Ent &x, bool v) {
                const uint32_t oe = (uint32_t)(x.s & 15u);
                const bool d = v & (oe != o0);
                three = three | (d & (ob != SEL_NONE) & (oe != ob));
                ob = (d & (ob == SEL_NONE)) ? oe : ob;
            });
            if (three || ob == SEL_NONE) return;
            SEL_HIT(16);
            deep = true;
            set_branches(env, o0);
        }
        uint64_t sa = P.s, sb = 0;
        bool ha = false, hb = false;
        each(env, [&](const Ent &x, bool v) {
            const bool b = x.br != 0u;
            sb = (v & b & !hb) ? x.s : sb;
            sa = (v & !b & !ha) ? x.s : sa;
            hb = hb | (v & b);
            ha = ha | (v & !b);
        });
        if (!ha || !hb) return;  // cannot happen: resolve() ends deep mode when one branch is left
        int s = cap;
        each(env, [&](const Ent &x, bool v) { s = v ? imin(s, first_diff(x.s, x.br ? sb : sa, cap - 1)) : s; });
        if (s > 0) {
            SEL_HIT(15);
            add_nibs(env, C_A, sa, s);
            add_nibs(env, C_B, sb, s);
            shift(env, s);
        }
    }

    // Entering deep mode: branch B = every entity whose lowest window owner differs from o0.
    template <class Env>
    MSIM_HD void set_branches(Env &env, uint32_t o0)
    {
        P.br = 0;
#pragma unroll
        for (int si = 0; si < NSA; ++si) S[si].br = (uint32_t)(S[si].s & 15u) != o0 ? 1u : 0u;
#pragma unroll
        for (int a = 0; a < NA; ++a) A[a].br = (uint32_t)(A[a].s & 15u) != o0 ? 1u : 0u;
        if (cm) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (cval(c)) {
                    ColdAct r = env.cold(c);
                    r.x.br = (uint32_t)(r.x.s & 15u) != o0 ? 1u : 0u;
                    env.cold_put(c, r);
                }
        }
    }

    // Fold when the best chain or any chain nears the top of the window (honest chains need room for the
    // next find; an implicit run only extends with its own owner).
    template <class Env>
    MSIM_HD bool fold_due(Env &env, int32_t bl) const
    {
        int32_t r = bl;
        each(env, [&](const Ent &x, bool v) { r = (v & (x.rt < WIN) & (x.rt > r)) ? x.rt : r; });
        return r >= FOLD_AT;
    }

    // One branch left: its deep blocks are common to every chain.
    template <class Env>
    MSIM_HD void resolve(Env &env)
    {
        if (!deep) return;
        uint32_t any = 0, all = 1;
        each(env, [&](const Ent &x, bool v) {
            any |= v ? x.br : 0u;
            all &= v ? x.br : 1u;
        });
        if (any && !all) return;
        SEL_HIT(13);
        const int src = all ? C_B : C_A;
#pragma unroll
        for (int k = 0; k < M; ++k) {
            env.add(C_F, (uint32_t)k, env.get(src, (uint32_t)k));
            env.set(C_A, (uint32_t)k, 0u);
            env.set(C_B, (uint32_t)k, 0u);
        }
        deep = false;
        P.br = 0;
#pragma unroll
        for (int si = 0; si < NSA; ++si) S[si].br = 0;
#pragma unroll
        for (int a = 0; a < NA; ++a) A[a].br = 0;
        if (cm) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (cval(c)) {
                    ColdAct r = env.cold(c);
                    r.x.br = 0;
                    env.cold_put(c, r);
                }
        }
    }

    // Blocks whose arrival is <= t join their chain's published prefix (UnpublishedBlocks, 79-89).
    template <class Env>
    MSIM_HD void publish(Env &env, int64_t t)
    {
        // One pop per queue is branch-free (most lanes of a wave need it); further pops are rare.
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            for (int rep = 0;; ++rep) {
                const bool p = aval(a) & (nq[a] > 0) & (q[a][0] <= t);
                if (rep > 0 && !p) break;
                if (p) SEL_HIT(4);
                A[a].rp += p ? 1 : 0;
                A[a].pa = p ? q[a][0] : A[a].pa;
#pragma unroll
                for (int i = 0; i + 1 < NQ; ++i) q[a][i] = p ? q[a][i + 1] : q[a][i];
                q[a][NQ - 1] = p ? T_INF : q[a][NQ - 1];
                nq[a] -= p ? 1 : 0;
                if (!(aval(a) & (nq[a] > 0) & (q[a][0] <= t))) break;
            }
        }
#pragma unroll
        for (int si = 0; si < NS; ++si) {
            for (int rep = 0;; ++rep) {
                const bool p = sval(si) & (ng[si] > 0) & (ga[si][0] <= t);
                if (rep > 0 && !p) break;
                if (p) SEL_HIT(5);
                S[si].rp += p ? gc[si][0] : 0;
                S[si].pa = p ? ga[si][0] : S[si].pa;
#pragma unroll
                for (int i = 0; i + 1 < NG; ++i) {
                    gc[si][i] = p ? gc[si][i + 1] : gc[si][i];
                    ga[si][i] = p ? ga[si][i + 1] : ga[si][i];
                }
                gc[si][NG - 1] = p ? 0 : gc[si][NG - 1];
                ga[si][NG - 1] = p ? T_INF : ga[si][NG - 1];
                ng[si] -= p ? 1 : 0;
                if (!(sval(si) & (ng[si] > 0) & (ga[si][0] <= t))) break;
            }
        }
        if (cm) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (cval(c)) {
                    ColdAct r = env.cold(c);
                    if (r.nq > 0 && r.q[0] <= t) {
                        while (r.nq > 0 && r.q[0] <= t) {
                            r.x.rp += 1;
                            r.x.pa = r.q[0];
#pragma unroll
                            for (int i = 0; i + 1 < SEL_NQC; ++i) r.q[i] = r.q[i + 1];
                            r.q[SEL_NQC - 1] = T_INF;
                            r.nq--;
                        }
                        env.cold_put(c, r);
                    }
                }
        }
    }

    // BestChain (main.cpp:68-82).
    template <class Env>
    MSIM_HD SelBest best(Env &env) const
    {
        const uint32_t pas = hm & ~am;
        SelBest b;
        b.l = -3;
        b.a = 0;
        b.s = ~0ull;
        b.x = SEL_NONE;
        b.br = 0;
        uint32_t bi = 99u;
        auto consider = [&](const Ent &x, uint32_t idx, int32_t L, bool v) {
            const bool better = v & ((L > b.l) | ((L == b.l) & ((x.pa < b.a) | ((x.pa == b.a) & (idx < bi)))));
            b.l = better ? L : b.l;
            b.a = better ? x.pa : b.a;
            bi = better ? idx : bi;
            b.s = better ? x.s : b.s;
            b.x = better ? x.xo : b.x;
            b.br = better ? x.br : b.br;
        };
        consider(P, pas ? (uint32_t)__builtin_ctz(pas) : 99u, P.rt, pas != 0u);
#pragma unroll
        for (int si = 0; si < NS; ++si) consider(S[si], sidv[si], S[si].rp, sval(si));
#pragma unroll
        for (int a = 0; a < NA; ++a) consider(A[a], aid[a], A[a].rp, aval(a));
        if (cm) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (cval(c)) {
                    const ColdAct r = env.cold(c);
                    consider(r.x, r.aid, r.x.rp, true);
                }
        }
        b.s = b.l >= WIN - 1 ? b.s : ((b.s & nib_upto(b.l)) | ~nib_upto(b.l));
        b.x = b.l >= WIN ? b.x : SEL_NONE;
        return b;
    }

    // MaybeReorg (simulation.h:124-142) of a chain to a strictly longer best chain: pop to the fork point,
    // counting popped own blocks as stale (for the class: blocks of its members, `pas`), then adopt.
    template <class Env>
    MSIM_HD void reorg_ent(Env &env, Ent &x, bool is_p, uint32_t own, const SelBest &B, uint32_t pas)
    {
        const bool same = (!deep) | (x.br == B.br);
        const int top = imin(x.rt, WIN - 1);
        const int d = same ? first_diff(x.s, B.s, top) : 0;
        const int32_t beyond = x.rt >= WIN ? x.rt - (WIN - 1) : 0;
        const bool popb = (beyond > 0) & ((!same) | (d <= top) | (x.xo != B.x));
        if (!same) SEL_HIT(11);
        if (is_p) {
            SEL_HIT(7);
            if (d <= top) SEL_HIT(8);
            for (int j = d; j <= top; ++j) {
                const uint32_t o = (uint32_t)(x.s >> (4 * j)) & 15u;
                if ((pas >> o) & 1u) env.add(C_S, o, 1u);
            }
            if (popb && ((pas >> x.xo) & 1u)) env.add(C_S, x.xo, (uint32_t)beyond);
            if (!same) {
#pragma unroll
                for (int k = 0; k < M; ++k)
                    if ((pas >> k) & 1u) env.add(C_S, (uint32_t)k, env.get(x.br ? C_B : C_A, (uint32_t)k));
            }
        } else {
            SEL_HIT(9);
            uint32_t c = (uint32_t)count_nib(x.s, own, nib_range(d, top));
            if (popb && x.xo == own) c += (uint32_t)beyond;
            if (!same) c += env.get(x.br ? C_B : C_A, own);
            if (c) {
                SEL_HIT(10);
                env.add(C_S, own, c);
            }
        }
        x.s = B.s;
        x.rt = B.l;
        x.rp = B.l;
        x.pa = B.a;
        x.xo = B.x;
        x.br = B.br;
    }

    // NotifyBestChain for every miner (main.cpp:165-167 -> simulation.h:177-180): Reveal, then Reorg.
    template <class Env>
    MSIM_HD void notify(Env &env, int64_t t, const SelBest &B)
    {
#pragma unroll
        for (int si = 0; si < NS; ++si) {
            if (sval(si) && B.l <= S[si].rt) {  // MaybeSelfishReveal (simulation.h:149-174)
                const int32_t sc = w[si], lead = S[si].rt - B.l;
                if (sc > lead) {
                    SEL_HIT(6);
                    int32_t rc = sc - lead;
                    if (sc > 1 && lead == 1) rc = sc;
                    push_group(si, rc, t + env.prop(sidv[si]));
                    w[si] -= rc;
                }
            }
        }
        const uint32_t pas = hm & ~am;
        if (B.l > P.rt) reorg_ent(env, P, true, 0u, B, pas);
#pragma unroll
        for (int si = 0; si < NS; ++si)
            if (sval(si) && B.l > S[si].rt) {
                reorg_ent(env, S[si], false, sidv[si], B, pas);
                w[si] = 0;
                ng[si] = 0;
            }
#pragma unroll
        for (int a = 0; a < NA; ++a)
            if (aval(a) && B.l > A[a].rt) {
                reorg_ent(env, A[a], false, aid[a], B, pas);
                nq[a] = 0;
            }
        if (cm) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (cval(c)) {
                    ColdAct r = env.cold(c);
                    if (B.l > r.x.rt) {
                        reorg_ent(env, r.x, false, r.aid, B, pas);
                        r.nq = 0;
                        env.cold_put(c, r);
                    }
                }
        }
    }

    // Active miners whose chain is the class's chain again rejoin the class.
    template <class Env>
    MSIM_HD void merge(Env &env)
    {
#pragma unroll
        for (int a = 0; a < NA; ++a)
            if (aval(a) && ent_same_as_p(A[a], P)) {
                SEL_HIT(12);
                av &= ~(1u << a);
                am &= ~(1u << aid[a]);
                nq[a] = 0;
            }
        if (cm) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (cval(c)) {
                    const ColdAct r = env.cold(c);
                    if (ent_same_as_p(r.x, P)) {
                        cm &= ~(1u << c);
                        am &= ~(1u << r.aid);
                    }
                }
        }
    }

    // EarliestArrival (main.cpp:99-112) over NextArrival (simulation.h:92-102); withheld blocks
    // (SELFISH_ARRIVAL) never bring the next event forward.
    template <class Env>
    MSIM_HD int64_t earliest(Env &env, int64_t t) const
    {
        int64_t ea = T_INF;
#pragma unroll
        for (int a = 0; a < NA; ++a)
            if (aval(a) && nq[a] > 0) ea = lmin(ea, q[a][0]);
#pragma unroll
        for (int si = 0; si < NS; ++si)
            if (sval(si) && ng[si] > 0 && ga[si][0] > t) ea = lmin(ea, ga[si][0]);
        if (cm) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (cval(c)) {
                    const ColdAct r = env.cold(c);
                    if (r.nq > 0) ea = lmin(ea, r.q[0]);
                }
        }
        return ea;
    }

    // RunSimulation (main.cpp:128-192) for one run, as begin / step (one event) / finish so that a
    // kernel can interleave its own work between events.
    int64_t t_, nbt_;
    uint32_t kn_;
    template <class Src>
    MSIM_HD void begin(Src &src)
    {
        uint32_t I = 0;
        kn_ = 0;
        if (!src.next(I, kn_)) err |= SERR_DRAWS;
        nbt_ = (int64_t)I;  // main.cpp:138
        t_ = 0;
    }
    // One iteration of main.cpp:150-182 at cur_time = t_. Returns false once the loop has ended.
    template <class Env, class Src>
    MSIM_HD bool step(Env &env, Src &src, int64_t D)
    {
        if (!(t_ < D && err == 0)) return false;  // main.cpp:150
        const int64_t t = t_;
        SEL_EP_DECL;
        while (t == nbt_) {  // main.cpp:153-157
            SEL_HIT(0);
            if (kn_ >= (uint32_t)M) {
                err |= SERR_PICK;
                break;
            }
            found(env, kn_, t);
            uint32_t I = 0;
            if (!src.next(I, kn_)) {
                err |= SERR_DRAWS;
                break;
            }
            nbt_ += (int64_t)I;
        }
        if (err) return false;
        SEL_EP(0);
        publish(env, t);
        SEL_EP(1);
        const SelBest B = best(env);  // main.cpp:164
        SEL_EP(2);
        notify(env, t, B);            // main.cpp:165-167
        SEL_EP(3);
        merge(env);
        bpub = B.l;                   // main.cpp:171
        resolve(env);
        SEL_EP(4);
        // Folding is a change of representation only, so a lane may fold before it is due: the device
        // folds every lane of a wave when any lane is due (one wave-uniform branch, and lanes that folded
        // together are due again later, together).
        const bool due = fold_due(env, B.l);
        if (env.fold_vote(due)) fold(env, due);
        SEL_EP(5);
        t_ = lmin(nbt_, earliest(env, t));  // main.cpp:176-182
        SEL_EP(6);
        return true;
    }
    // main.cpp:185-189: BestChain at the end of the run, no notify.
    template <class Env>
    MSIM_HD void finish(Env &env, int64_t D, SelOut &out)
    {
        publish(env, D);
        const SelBest B = best(env);
        const int top = imin(B.l, WIN - 1);
#pragma unroll
        for (int k = 0; k < M; ++k) {
            uint32_t f = env.get(C_F, (uint32_t)k) + (uint32_t)count_nib(B.s, (uint32_t)k, nib_upto(top));
            if (B.x == (uint32_t)k) f += (uint32_t)(B.l - (WIN - 1));
            if (deep) f += env.get(B.br ? C_B : C_A, (uint32_t)k);
            out.found[k] = f;
            out.stale[k] = env.get(C_S, (uint32_t)k);
        }
        out.best_height = wb + (uint32_t)B.l;
        out.err = err;
    }
    template <class Env, class Src>
    MSIM_HD void run(Env &env, Src &src, int64_t D, SelOut &out)
    {
        begin(src);
        while (step(env, src, D)) {
        }
        finish(env, D, out);
    }
};

}  // namespace msim
