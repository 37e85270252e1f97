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
// Capacities (active slots, reveal groups, in-flight blocks, window) only ever set an error bit; the
// caller recomputes such runs with larger capacities, so results never depend on them.
#pragma once
#include "msim_model.h"

namespace msim {

constexpr uint32_t SEL_NONE = 0xFu;  // "no owner" (miner ids are < 15)
constexpr int SEL_MAXS = 4;          // selfish miners per network supported by the entity engine
enum : uint32_t {
    SERR_CAP = 1u,    // active slots / reveal groups / in-flight queue exhausted
    SERR_WIN = 2u,    // a chain outgrew the window and could not fold
    SERR_PICK = 4u,   // PickFinder fell through (simulation.h:220 assert)
    SERR_DRAWS = 8u,  // the run outlasted its pre-generated draws
};
// Counter arrays of the Env: settled found, stale_blocks, deep branch A, deep branch B.
enum : int { C_F = 0, C_S = 1, C_A = 2, C_B = 3 };

struct SelOut {
    uint32_t found[MAXM];
    uint32_t stale[MAXM];
    uint32_t best_height;
    uint32_t err;
};

// The best chain of one event: entity, published tip height, tip arrival, window string (owners above
// the tip = 0xF), implicit run owner (heights >= WIN), deep branch.
struct SelBest {
    int e;
    int32_t l;
    int64_t a;
    uint64_t s;
    uint32_t x;
    uint32_t br;
};

// Env: int64_t prop(uint32_t k); uint32_t get(int arr, uint32_t k); void add(int arr, uint32_t k, uint32_t v);
//      void set(int arr, uint32_t k, uint32_t v).
// Src: bool next(uint32_t &interval_ms, uint32_t &finder)  (finder >= M: PickFinder fell through).
template <int M, int NS, int NA, int NG, int NQ>
struct Sel {
    static_assert(M >= 1 && M <= MAXM, "miner count");
    static_assert(NS >= 0 && NS <= SEL_MAXS && NA >= 1 && NG >= 1 && NQ >= 1, "capacities");
    static constexpr int NSA = NS > 0 ? NS : 1;
    static constexpr int E0A = 1 + NS;  // first active entity
    static constexpr int NE = 1 + NS + NA;

    uint64_t str[NE];  // owners at window heights wb..wb+15 (0xF above the tip)
    int32_t rt[NE];    // tip height - wb (>= WIN: heights WIN..rt are owned by xo)
    int32_t rp[NE];    // published tip height - wb (PublishedChain, simulation.h:118-121)
    int64_t pa[NE];    // arrival of the published tip (BestChain's first-seen key, main.cpp:75)
    uint32_t xo[NE];   // owner of the implicit run above the window (SEL_NONE when rt < WIN)
    uint32_t vm;       // valid entities
    uint32_t bm;       // deep branch of each entity (bit e set: branch B)
    uint32_t sidv[NSA];
    int32_t w[NSA];    // withheld blocks (SelfishBlocks)
    int32_t ng[NSA];   // in-flight reveal groups, oldest first
    int32_t gc[NSA][NG];
    int64_t ga[NSA][NG];
    uint32_t aid[NA];  // miner of each active slot (SEL_NONE = free)
    int32_t nq[NA];    // own in-flight blocks, lowest first (only own blocks are ever unpublished)
    int64_t q[NA][NQ];
    uint32_t am, hm, sm;  // active / honest / selfish miner masks
    uint32_t wb;       // absolute height of window position 0
    int32_t bpub;      // previous event's best tip - wb (best_chain_size - 1, main.cpp:171)
    bool deep;
    uint32_t err;

    MSIM_HD bool valid(int e) const { return (vm >> e) & 1u; }
    MSIM_HD uint32_t ebr(int e) const { return (bm >> e) & 1u; }
    MSIM_HD uint32_t owner(int e) const { return e == 0 ? SEL_NONE : (e < E0A ? sidv[e - 1] : aid[e - E0A]); }

    // sids: NSA selfish miner ids in index order (SEL_NONE for unused entries); m miners.
    MSIM_HD void init(uint32_t m, const uint32_t *sids)
    {
        sm = 0;
#pragma unroll
        for (int si = 0; si < NSA; ++si) {
            sidv[si] = NS > 0 ? sids[si] : SEL_NONE;
            if (sidv[si] != SEL_NONE) sm |= 1u << sidv[si];
            w[si] = 0;
            ng[si] = 0;
#pragma unroll
            for (int i = 0; i < NG; ++i) {
                gc[si][i] = 0;
                ga[si][i] = T_INF;
            }
        }
        hm = ((1u << m) - 1u) & ~sm;
        vm = 1u;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            str[e] = ~0ull;
            rt[e] = -1;  // genesis (height 0) is settled: wb = 1
            rp[e] = -1;
            pa[e] = 0;   // Genesis arrival (simulation.h:31-33)
            xo[e] = SEL_NONE;
            if (e >= 1 && e < E0A && sidv[e - 1] != SEL_NONE) vm |= 1u << e;
        }
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            aid[a] = SEL_NONE;
            nq[a] = 0;
#pragma unroll
            for (int i = 0; i < NQ; ++i) q[a][i] = T_INF;
        }
        am = 0;
        bm = 0;
        wb = 1;
        bpub = -1;  // best_chain_size = 1 (main.cpp:149)
        deep = false;
        err = 0;
    }

    MSIM_HD void push_group(int si, int32_t c, int64_t arr)
    {
        if (ng[si] >= NG) {
            err |= SERR_CAP;
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
    MSIM_HD void enqueue(int a, int64_t arr)
    {
        if (nq[a] >= NQ) {
            err |= SERR_CAP;
            return;
        }
#pragma unroll
        for (int i = 0; i < NQ; ++i) q[a][i] = (i == nq[a]) ? arr : q[a][i];
        nq[a]++;
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

    MSIM_HD void shift(int s)
    {
        wb += (uint32_t)s;
        bpub -= s;
        const uint64_t fill = ~0ull << (64 - 4 * s);
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            str[e] = (str[e] >> (4 * s)) | fill;
            rt[e] -= s;
            rp[e] -= s;
            if (rt[e] >= WIN - s && xo[e] != SEL_NONE) {  // heights entering the window from the implicit run
                const uint64_t mk = nib_range(WIN - s, imin(rt[e], WIN - 1));
                str[e] = (str[e] & ~mk) | (mk & (0x1111111111111111ull * (uint64_t)xo[e]));
            }
            if (rt[e] < WIN) xo[e] = SEL_NONE;
        }
    }

    // Fold the lowest window heights that every chain holds (all published) into the settled counters,
    // or, during a two-branch episode, into the deep-branch counters of each branch.
    template <class Env>
    MSIM_HD void fold(Env &env)
    {
        int minrp = rt[0];
#pragma unroll
        for (int e = 1; e < NE; ++e)
            if (valid(e)) minrp = imin(minrp, rp[e]);
        if (minrp < 0) return;
        const int cap = imin(minrp + 1, WIN - 1);
        if (!deep) {
            int s = cap;
#pragma unroll
            for (int e = 1; e < NE; ++e)
                if (valid(e)) s = imin(s, first_diff(str[e], str[0], cap - 1));
            if (s > 0) {
                add_nibs(env, C_F, str[0], s);
                shift(s);
                return;
            }
            // The chains disagree at the lowest height: split them into two long branches.
            const uint32_t o0 = (uint32_t)(str[0] & 15u);
            uint32_t ob = SEL_NONE, nb = 0;
            bool three = false;
#pragma unroll
            for (int e = 1; e < NE; ++e)
                if (valid(e)) {
                    const uint32_t oe = (uint32_t)(str[e] & 15u);
                    if (oe != o0) {
                        nb |= 1u << e;
                        if (ob == SEL_NONE) ob = oe;
                        else if (oe != ob) three = true;
                    }
                }
            if (three || nb == 0) return;
            deep = true;
            bm = nb;
        }
        uint64_t sa = 0, sb = 0;
        bool ha = false, hb = false;
#pragma unroll
        for (int e = 0; e < NE; ++e)
            if (valid(e)) {
                if (ebr(e)) {
                    if (!hb) sb = str[e];
                    hb = true;
                } else {
                    if (!ha) sa = str[e];
                    ha = true;
                }
            }
        int s = cap;
#pragma unroll
        for (int e = 0; e < NE; ++e)
            if (valid(e)) s = imin(s, first_diff(str[e], ebr(e) ? sb : sa, cap - 1));
        if (s > 0) {
            add_nibs(env, C_A, sa, s);
            add_nibs(env, C_B, sb, s);
            shift(s);
        }
    }

    // One branch left: its deep blocks are common to every chain.
    template <class Env>
    MSIM_HD void resolve(Env &env)
    {
        if (!deep) return;
        uint32_t any = 0, all = 1;
#pragma unroll
        for (int e = 0; e < NE; ++e)
            if (valid(e)) {
                any |= ebr(e);
                all &= ebr(e);
            }
        if (any && !all) return;
        const int src = all ? C_B : C_A;
#pragma unroll
        for (int k = 0; k < M; ++k) {
            env.add(C_F, (uint32_t)k, env.get(src, (uint32_t)k));
            env.set(C_A, (uint32_t)k, 0u);
            env.set(C_B, (uint32_t)k, 0u);
        }
        deep = false;
        bm = 0;
    }

    // ------------------------------------------------------------------ Miner::FoundBlock
    // simulation.h:62-76 for miner k at time T. A passive miner leaves the class with its chain.
    template <class Env>
    MSIM_HD void found(Env &env, uint32_t k, int64_t T)
    {
        int et = -1;
        if ((sm >> k) & 1u) {
#pragma unroll
            for (int si = 0; si < NS; ++si)
                if (sidv[si] == k) et = 1 + si;
        } else if ((am >> k) & 1u) {
#pragma unroll
            for (int a = 0; a < NA; ++a)
                if (aid[a] == k) et = E0A + a;
        } else {
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                const int e = E0A + a;
                const bool me = et < 0 && aid[a] == SEL_NONE;
                et = me ? e : et;
                str[e] = me ? str[0] : str[e];
                rt[e] = me ? rt[0] : rt[e];
                rp[e] = me ? rt[0] : rp[e];
                pa[e] = me ? pa[0] : pa[e];
                xo[e] = me ? xo[0] : xo[e];
                bm = me ? ((bm & ~(1u << e)) | (ebr(0) << e)) : bm;
                aid[a] = me ? k : aid[a];
                nq[a] = me ? 0 : nq[a];
                vm = me ? (vm | (1u << e)) : vm;
            }
            if (et >= 0) am |= 1u << k;
        }
        if (et < 0) {
            err |= SERR_CAP;
            return;
        }
        // Room for height rt+1: inside the window, the first implicit-run height, or the run's owner.
        int32_t r = 0;
        uint32_t x = SEL_NONE;
#pragma unroll
        for (int e = 0; e < NE; ++e)
            if (e == et) {
                r = rt[e];
                x = xo[e];
            }
        if (r + 1 > WIN && x != k) {
            fold(env);
#pragma unroll
            for (int e = 0; e < NE; ++e)
                if (e == et) {
                    r = rt[e];
                    x = xo[e];
                }
            if (r + 1 > WIN && x != k) {
                err |= SERR_WIN;
                return;
            }
        }
        const int64_t arr = T + env.prop(k);
        // Append at height r + 1 of entity et (selects over the entities, see push_group).
        const int h = r + 1;
        const uint64_t nmask = h < WIN ? (0xFull << (4 * h)) : 0ull;
        const uint64_t nval = h < WIN ? ((uint64_t)k << (4 * h)) : 0ull;
#pragma unroll
        for (int e = 1; e < NE; ++e) {
            const bool me = e == et;
            str[e] = me ? ((str[e] & ~nmask) | nval) : str[e];
            xo[e] = (me && h == WIN) ? k : xo[e];
            rt[e] = me ? h : rt[e];
        }
#pragma unroll
        for (int si = 0; si < NS; ++si) {
            if (et != 1 + si) continue;
            const bool race = (w[si] == 1) && (bpub == r);  // simulation.h:66
            if (race) {
                w[si] = 0;
                push_group(si, 2, arr);  // simulation.h:68-69: both blocks arrive at T + prop
            } else {
                w[si] += 1;  // simulation.h:71 (SELFISH_ARRIVAL)
            }
        }
#pragma unroll
        for (int a = 0; a < NA; ++a)
            if (et == E0A + a) enqueue(a, arr);  // simulation.h:74
    }

    // Blocks whose arrival is <= t join their chain's published prefix (UnpublishedBlocks, 79-89).
    MSIM_HD void publish(int64_t t)
    {
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const int e = E0A + a;
            if (!valid(e)) continue;
            while (nq[a] > 0 && q[a][0] <= t) {
                rp[e] += 1;
                pa[e] = q[a][0];
#pragma unroll
                for (int i = 0; i + 1 < NQ; ++i) q[a][i] = q[a][i + 1];
                q[a][NQ - 1] = T_INF;
                nq[a]--;
            }
        }
#pragma unroll
        for (int si = 0; si < NS; ++si) {
            const int e = 1 + si;
            if (!valid(e)) continue;
            while (ng[si] > 0 && ga[si][0] <= t) {
                rp[e] += gc[si][0];
                pa[e] = ga[si][0];
#pragma unroll
                for (int i = 0; i + 1 < NG; ++i) {
                    gc[si][i] = gc[si][i + 1];
                    ga[si][i] = ga[si][i + 1];
                }
                gc[si][NG - 1] = 0;
                ga[si][NG - 1] = T_INF;
                ng[si]--;
            }
        }
    }

    // BestChain (main.cpp:68-82).
    MSIM_HD SelBest best() const
    {
        const uint32_t pas = hm & ~am;
        const uint32_t pmin = pas ? (uint32_t)__builtin_ctz(pas) : 99u;
        SelBest b;
        b.e = 0;
        b.l = -3;
        b.a = 0;
        uint32_t bi = 99u;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const bool cand = valid(e) && (e != 0 || pas != 0u);
            const uint32_t idx = e == 0 ? pmin : owner(e);
            const int32_t L = rp[e];
            const int64_t A = pa[e];
            const bool better = L > b.l || (L == b.l && (A < b.a || (A == b.a && idx < bi)));
            if (cand && better) {
                b.e = e;
                b.l = L;
                b.a = A;
                bi = idx;
            }
        }
        uint64_t s = 0;
        uint32_t x = SEL_NONE, br = 0;
#pragma unroll
        for (int e = 0; e < NE; ++e)
            if (e == b.e) {
                s = str[e];
                x = xo[e];
                br = ebr(e);
            }
        b.s = b.l >= WIN - 1 ? s : ((s & nib_upto(b.l)) | ~nib_upto(b.l));
        b.x = b.l >= WIN ? x : SEL_NONE;
        b.br = br;
        return b;
    }

    // MaybeReorg (simulation.h:124-142) of entity e to a strictly longer best chain: pop to the fork
    // point, counting popped own blocks as stale (for P: blocks of its members), then adopt.
    template <class Env>
    MSIM_HD void reorg(Env &env, int e, const SelBest &B, uint32_t pas)
    {
        const bool same = !deep || ebr(e) == B.br;
        const int top = imin(rt[e], WIN - 1);
        const int d = same ? first_diff(str[e], B.s, top) : 0;
        const int32_t beyond = rt[e] >= WIN ? rt[e] - (WIN - 1) : 0;
        const bool popb = beyond > 0 && (!same || d <= top || xo[e] != B.x);
        if (e == 0) {
            for (int j = d; j <= top; ++j) {
                const uint32_t o = (uint32_t)(str[0] >> (4 * j)) & 15u;
                if ((pas >> o) & 1u) env.add(C_S, o, 1u);
            }
            if (popb && ((pas >> xo[0]) & 1u)) env.add(C_S, xo[0], (uint32_t)beyond);
            if (!same) {
#pragma unroll
                for (int k = 0; k < M; ++k)
                    if ((pas >> k) & 1u) env.add(C_S, (uint32_t)k, env.get(ebr(0) ? C_B : C_A, (uint32_t)k));
            }
        } else {
            const uint32_t o = owner(e);
            uint32_t c = (uint32_t)count_nib(str[e], o, nib_range(d, top));
            if (popb && xo[e] == o) c += (uint32_t)beyond;
            if (!same) c += env.get(ebr(e) ? C_B : C_A, o);
            if (c) env.add(C_S, o, c);
        }
        str[e] = B.s;
        rt[e] = B.l;
        rp[e] = B.l;
        pa[e] = B.a;
        xo[e] = B.x;
        bm = (bm & ~(1u << e)) | (B.br << e);
        if (e >= 1 && e < E0A) {
            w[e - 1] = 0;
            ng[e - 1] = 0;
        } else if (e >= E0A) {
            nq[e - E0A] = 0;
        }
    }

    // NotifyBestChain for every miner (main.cpp:165-167 -> simulation.h:177-180): Reveal, then Reorg.
    template <class Env>
    MSIM_HD void notify(Env &env, int64_t t, const SelBest &B)
    {
#pragma unroll
        for (int si = 0; si < NS; ++si) {
            const int e = 1 + si;
            if (valid(e) && B.l <= rt[e]) {  // MaybeSelfishReveal (simulation.h:149-174)
                const int32_t sc = w[si], lead = rt[e] - B.l;
                if (sc > lead) {
                    int32_t rc = sc - lead;
                    if (sc > 1 && lead == 1) rc = sc;
                    push_group(si, rc, t + env.prop(sidv[si]));
                    w[si] -= rc;
                }
            }
        }
        const uint32_t pas = hm & ~am;
#pragma unroll
        for (int e = 0; e < NE; ++e)
            if (valid(e) && B.l > rt[e]) reorg(env, e, B, pas);
    }

    // An active miner whose chain is the class's chain again, all published, rejoins the class.
    MSIM_HD void merge()
    {
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const int e = E0A + a;
            if (valid(e) && rp[e] == rt[e] && rt[e] == rt[0] && str[e] == str[0] && xo[e] == xo[0] &&
                ebr(e) == ebr(0)) {
                vm &= ~(1u << e);
                am &= ~(1u << aid[a]);
                aid[a] = SEL_NONE;
                nq[a] = 0;
            }
        }
    }

    // EarliestArrival (main.cpp:99-112) over NextArrival (simulation.h:92-102); withheld blocks
    // (SELFISH_ARRIVAL) never bring the next event forward.
    MSIM_HD int64_t earliest(int64_t t) const
    {
        int64_t ea = T_INF;
#pragma unroll
        for (int a = 0; a < NA; ++a)
            if (valid(E0A + a) && nq[a] > 0) ea = lmin(ea, q[a][0]);
#pragma unroll
        for (int si = 0; si < NS; ++si)
            if (valid(1 + si) && ng[si] > 0 && ga[si][0] > t) ea = lmin(ea, ga[si][0]);
        return ea;
    }

    // RunSimulation (main.cpp:128-192) for one run.
    template <class Env, class Src>
    MSIM_HD void run(Env &env, Src &src, int64_t D, SelOut &out)
    {
        uint32_t I = 0, kn = 0;
        if (!src.next(I, kn)) err |= SERR_DRAWS;
        int64_t nbt = (int64_t)I;  // main.cpp:138
        int64_t t = 0;
        while (t < D && err == 0) {  // main.cpp:150
            while (t == nbt) {       // main.cpp:153-157
                if (kn >= (uint32_t)M) {
                    err |= SERR_PICK;
                    break;
                }
                found(env, kn, t);
                if (!src.next(I, kn)) {
                    err |= SERR_DRAWS;
                    break;
                }
                nbt += (int64_t)I;
            }
            if (err) break;
            publish(t);
            const SelBest B = best();  // main.cpp:164
            notify(env, t, B);         // main.cpp:165-167
            merge();
            bpub = B.l;                // main.cpp:171
            resolve(env);
            if (B.l >= FOLD_AT) fold(env);
            t = lmin(nbt, earliest(t));  // main.cpp:176-182
        }
        // main.cpp:185-189: BestChain at the end of the run, no notify.
        publish(D);
        const SelBest B = best();
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
};

}  // namespace msim
