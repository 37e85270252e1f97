// msim_selm.h — the settled-state ("macro") form of a run with ONE selfish miner, exact, and its hand-over
// to and from the entity engine (msim_sel.h).
//
// Why. With one selfish miner (simulation.h:55) and every propagation delay >= 1 ms, a find whose
// consequences (the honest block's arrival at T + prop_k, the selfish reveal it triggers, arriving
// prop_s later — simulation.h:149-174, main.cpp:164-167) are all over before the next find leaves
// the network in one of few SETTLED states, and the whole event sequence of that find collapses into one
// transition of a small Markov chain (the 2013 paper's state machine with gamma = 0, as the reference
// implements it):
//   F   the common prefix (every miner's chain agrees up to height F, all published),
//   h   the length of a published tie fork above F: the honest miners' branch (h honest blocks) and the
//       selfish miner's published branch (h selfish blocks); the honest branch arrived first, so it is
//       BestChain's pick (main.cpp:75 first-seen) and the honest miners stay on it,
//   w   the selfish miner's withheld blocks on top of its branch (SelfishBlocks, simulation.h:105-115).
// A settled state always has the selfish published branch as long as the honest one, so FoundBlock's
// 1-block-race case (simulation.h:66) never applies. Transitions for a find by miner k:
//   selfish                       w += 1                                    (simulation.h:71)
//   honest, w == 0                the honest branch (+ k's block) wins: F += h + 1; the selfish miner's h
//                                 tie blocks are stale (MaybeReorg, simulation.h:124-142)
//   honest, w == 1 or w >= 3      one block is revealed (lead w - 1, simulation.h:160-163) and ties the
//                                 new honest block: h += 1, w -= 1
//   honest, w == 2                lead 1: everything is revealed (simulation.h:166-168) and the selfish
//                                 branch (h + 2 blocks) wins: F += h + 2; the honest branch is stale
// The transition is exact when the find is selfish (nothing is published) or when the next find comes
// strictly after prop_k (+ prop_s if w > 0) and that settle time is before the end of the run D; every
// other find is handed to the entity engine, which runs the reference's event loop until the network is
// quiet again (a common published chain, only withheld blocks on top) and hands the run back.
//
// Counters: found[k] is counted provisionally at every find (the LDS C_F array); blocks that later leave
// the best chain (stale honest branches: stp[], stale selfish tie blocks: sst; the honest branch's
// composition is kept as 16-bit counts per miner in pend[]) are subtracted when they are flushed.
#pragma once
#include "msim_sel.h"

namespace msim {

// The settled-form transitions (msim_selm.h SelMacro::transition) of four blocks with selfish pattern s4 (bit i:
// block i is the selfish miner's; the others honest) from lead class cls (w = cls; cls 6 stands for any
// w >= 6, from which no resolution can happen within four blocks), as one 27-bit table entry:
//   bits 0-3   w after the four blocks (cls 6: the change + 4)
//   bit 4      some resolution (honest find at w == 0: the honest branch wins; at w == 2: the selfish one)
//   bit 5      the first resolution is a selfish win (the honest branch open before the half is stale)
//   bits 6-8   ties since the last resolution (none: since the half's start)
//   bits 9-12  F's increase beyond the entering h (which the first resolution adds)
//   bits 13-15 selfish stale blocks beyond the entering h (which a first resolution by an honest win adds)
//   bits 16-19 honest blocks of the half made stale by selfish wins
//   bits 20-23 w != 0 before block i (a candidate there needs the engine)
//   bits 24-26 one past the last resolution's block (0: none)
MSIM_HD uint32_t sp_lut_entry(uint32_t cls, uint32_t s4)
{
    uint32_t w = cls, hrel = 0, rs = 0, fsw = 0, dF = 0, dsst = 0, st = 0, wnz = 0, lrs = 0, rstart = 0;
    for (uint32_t i = 0; i < 4; ++i) {
        if (w != 0) wnz |= 1u << i;
        if ((s4 >> i) & 1u) {
            w += 1;
            continue;
        }
        if (w == 0 || w == 2) {
            const bool res = w == 0;
            dF += hrel + (res ? 1u : 2u);
            if (res) dsst += hrel;
            else
                for (uint32_t j = rstart; j <= i; ++j)
                    if (!((s4 >> j) & 1u)) st |= 1u << j;
            if (!rs) fsw = res ? 0u : 1u;
            rs = 1;
            hrel = 0;
            w = 0;
            rstart = i + 1;
            lrs = i + 1;
        } else {
            hrel += 1;
            w -= 1;
        }
    }
    const uint32_t wf = cls < 6 ? w : w + 4u - 6u;
    return wf | (rs << 4) | (fsw << 5) | (hrel << 6) | (dF << 9) | (dsst << 13) | (st << 16) | (wnz << 20) | (lrs << 24);
}
constexpr int SP_LUT = 7 * 16;

// A FIFO of up to four held draws in front of a drawer that makes the reference's draws in-lane
// (void D::draw(uint32_t &interval_ms, uint32_t &finder)). The settled form's four-find step (step4) tops it up
// to four (draws from streams that advance whatever the steps' outcomes, so the draw arithmetic has no
// dependency on the transitions it runs beside); the one-find step (step1) takes a held draw. A
// lane that leaves the form keeps its held draws for the engine, which takes them first (next/peek), then
// draws on demand.
template <class D>
struct SelFifo {
    D d;
    uint32_t I0, k0, I1, k1, I2, k2, I3, k3;
    uint32_t n;  // held draws
    MSIM_HD bool peek(uint32_t &I, uint32_t &k)
    {
        if (n == 0u) {
            d.draw(I0, k0);
            n = 1u;
        }
        I = I0;
        k = k0;
        return true;
    }
    MSIM_HD void pop()
    {
        I0 = I1;
        k0 = k1;
        I1 = I2;
        k1 = k2;
        I2 = I3;
        k2 = k3;
        n -= 1u;
    }
    MSIM_HD void pop_if(bool p)
    {
        I0 = p ? I1 : I0;
        k0 = p ? k1 : k0;
        I1 = p ? I2 : I1;
        k1 = p ? k2 : k1;
        I2 = p ? I3 : I2;
        k2 = p ? k3 : k2;
        n -= p ? 1u : 0u;
    }
    // step4: four held draws (from at least two)
    MSIM_HD void top4()
    {
        if (n < 3u) d.draw(I2, k2);
        if (n < 4u) d.draw(I3, k3);
        n = 4u;
    }
    MSIM_HD bool next(uint32_t &I, uint32_t &k)
    {
        peek(I, k);
        pop();
        return true;
    }
    MSIM_HD void fill()
    {
        if (n == 0u) {
            d.draw(I0, k0);
            n = 1u;
        }
        if (n == 1u) {
            d.draw(I1, k1);
            n = 2u;
        }
    }
    MSIM_HD void prefetch() {}
    MSIM_HD void settle() {}
    // step4 consumed the four held draws (three finds and the new pending one)
    MSIM_HD void took4() { n = 0u; }
};

template <int M>
struct SelMacro {
    // The honest branch's composition and the honest stale blocks not yet flushed are kept per HONEST slot
    // (miner j's slot is j minus 1 if j is above the selfish miner), 16 bits per slot, four slots per
    // 64-bit word: one shift and one 64-bit add per find, one add per resolution.
    static constexpr int NP = M > 1 ? (M + 2) / 4 : 1;
    int64_t T;             // time of the pending find
    uint32_t k;            // its finder
    uint32_t F, h, w;      // settled state (see above)
    uint64_t pend[NP];     // honest branch: blocks per honest slot
    uint64_t stp[NP];      // honest stale blocks not yet flushed to C_S, same packing
    uint32_t sst;          // selfish stale blocks not yet flushed
    uint32_t Ff;           // F at the last flush (stale added since <= F - Ff keeps stp's fields < 2^16)

    // The state as NW words at p[0], p[stride], ... (a lane's LDS column while the wave runs engine steps).
    static constexpr int NW = 8 + 4 * NP;
    MSIM_HD void save(uint32_t *p, int stride) const
    {
        p[0] = (uint32_t)T;
        p[stride] = (uint32_t)((uint64_t)T >> 32);
        p[2 * stride] = k;
        p[3 * stride] = F;
        p[4 * stride] = h;
        p[5 * stride] = w;
        p[6 * stride] = sst;
        p[7 * stride] = Ff;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            p[(8 + 2 * i) * stride] = (uint32_t)pend[i];
            p[(9 + 2 * i) * stride] = (uint32_t)(pend[i] >> 32);
            p[(8 + 2 * NP + 2 * i) * stride] = (uint32_t)stp[i];
            p[(9 + 2 * NP + 2 * i) * stride] = (uint32_t)(stp[i] >> 32);
        }
    }
    MSIM_HD void load(const uint32_t *p, int stride)
    {
        T = (int64_t)(((uint64_t)p[stride] << 32) | p[0]);
        k = p[2 * stride];
        F = p[3 * stride];
        h = p[4 * stride];
        w = p[5 * stride];
        sst = p[6 * stride];
        Ff = p[7 * stride];
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            pend[i] = ((uint64_t)p[(9 + 2 * i) * stride] << 32) | p[(8 + 2 * i) * stride];
            stp[i] = ((uint64_t)p[(9 + 2 * NP + 2 * i) * stride] << 32) | p[(8 + 2 * NP + 2 * i) * stride];
        }
    }

    MSIM_HD static uint32_t slot(uint32_t j, uint32_t sid) { return j - (j > sid ? 1u : 0u); }
    MSIM_HD static uint32_t field(const uint64_t (&a)[NP], uint32_t s)
    {
        uint64_t v = 0;
#pragma unroll
        for (int i = 0; i < NP; ++i) v = (s >> 2) == (uint32_t)i ? a[i] : v;
        return (uint32_t)(v >> (16 * (s & 3u))) & 0xFFFFu;
    }
    MSIM_HD static void field_add(uint64_t (&a)[NP], uint32_t s, uint32_t v)
    {
        const uint64_t x = (uint64_t)v << (16 * (s & 3u));
#pragma unroll
        for (int i = 0; i < NP; ++i) a[i] += (s >> 2) == (uint32_t)i ? x : 0ull;
    }
    MSIM_HD uint32_t pend_of(uint32_t j, uint32_t sid) const { return field(pend, slot(j, sid)); }

    // Start of a run (main.cpp:138, 149): the first find, at the first interval; genesis is the prefix.
    template <class Src>
    MSIM_HD bool begin(Src &src)
    {
        F = 0;
        h = 0;
        w = 0;
        sst = 0;
        Ff = 0;
#pragma unroll
        for (int i = 0; i < NP; ++i) pend[i] = stp[i] = 0;
        uint32_t I = 0;
        if (!src.peek(I, k)) return false;
        src.pop();
        T = (int64_t)I;
        src.fill();
        return true;
    }

    // The settled-state transition of a find by miner k (is_s: k is the selfish miner), applied only when ok
    // (branch-free: every update is masked). It touches no counter: found blocks are counted by the caller
    // (step: one provisional count per find).
    MSIM_HD void transition(uint32_t k, bool is_s, bool ok, uint32_t sid)
    {
        const bool hon = ok & !is_s;
        const bool sf = ok & is_s;
        const bool res = hon & (w == 0u);     // the honest branch wins (h == 0: a plain honest block)
        const bool swin = hon & (w == 2u);    // the selfish branch wins
        const bool tie = hon & !res & !swin;  // one more tied block each
        const bool rs = res | swin;
        // k's block joins the honest branch (a resolving branch is cleared below)
        field_add(pend, slot(k, sid), hon ? 1u : 0u);
#pragma unroll
        for (int i = 0; i < NP; ++i) stp[i] += swin ? pend[i] : 0ull;
        sst += res ? h : 0u;
        F += res ? h + 1u : (swin ? h + 2u : 0u);
        h = rs ? 0u : h + (tie ? 1u : 0u);
        w = sf ? w + 1u : (rs ? 0u : w - (tie ? 1u : 0u));
#pragma unroll
        for (int i = 0; i < NP; ++i) pend[i] = rs ? 0ull : pend[i];
    }

    // One find from held draws (the FIFO holds at least one). Returns 0 (next find pending), 1 (this find
    // needs the entity engine), 2 (run over: the next find is at or after D). A find needs the engine when
    // it is honest and the next interval does not clear its propagation threshold (prop_k, plus prop_s while
    // the selfish miner leads), or when a 16-bit field could overflow (h, or the honest stale blocks added to
    // stp since the last flush, bounded by F - Ff: the engine's hand-over flushes).
    template <class Env, class Src>
    MSIM_HD int step1(Env &env, Src &src, int64_t D, uint32_t sid, int64_t ps)
    {
        const int64_t pk = env.prop_tab(k < (uint32_t)M ? k : 0u);
        uint32_t I = 0, kn = 0;
        src.peek(I, kn);
        const bool is_s = k == sid;
        const int64_t thr = is_s ? 0 : pk + (w != 0u ? ps : 0);
        const bool ok = (k < (uint32_t)M) & (h < 0xFFFFu) & (F - Ff < 0xFF00u) & (is_s | (((int64_t)I > thr) & (T + thr < D)));
        transition(k, is_s, ok, sid);
        env.add(C_F, k < (uint32_t)M ? k : 0u, ok ? 1u : 0u);
        src.pop_if(ok);
        T += ok ? (int64_t)I : 0;
        k = ok ? kn : k;
        return ok ? (T < D ? 0 : 2) : 1;
    }

    // Four finds at once when none of them can need the engine: the pending find and the next three, from four
    // held draws (src: SelFifo; topped up here). The transitions come from the four-block table (lut:
    // sp_lut_entry, SP_LUT entries) indexed by the lead class and the selfish pattern; the honest branch's
    // composition follows the table's resolution points. A find needs the engine iff it is honest and
    // I_next <= prop_k + (w != 0 ? prop_s : 0) (step), i.e. B (I_next <= prop_k) or A (<= prop_k + prop_s) with
    // w != 0, which the table's "w != 0 before block i" bits decide for all four; the settle times are all
    // below D when the fourth find's plus the largest threshold (thrmax) is. Otherwise one find by step1.
    // Returns as step1().
    template <class Env, class Src>
    MSIM_HD int step4(Env &env, Src &src, int64_t D, uint32_t sid, int64_t ps, int64_t thrmax, const uint32_t *lut)
    {
        src.top4();
        const uint32_t kk[4] = {k, src.k0, src.k1, src.k2};
        const uint32_t In[4] = {src.I0, src.I1, src.I2, src.I3};
        uint32_t s4 = 0, a4 = 0, b4 = 0;
        bool valid = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            valid &= kk[j] < (uint32_t)M;
            const bool is_s = kk[j] == sid;
            const int64_t pk = env.prop_tab(kk[j] < (uint32_t)M ? kk[j] : 0u);
            s4 |= (is_s ? 1u : 0u) << j;
            a4 |= (((!is_s) & ((int64_t)In[j] <= pk + ps)) ? 1u : 0u) << j;
            b4 |= (((!is_s) & ((int64_t)In[j] <= pk)) ? 1u : 0u) << j;
        }
        const int64_t T3 = T + (int64_t)In[0] + (int64_t)In[1] + (int64_t)In[2];
        const uint32_t cls = w < 6u ? w : 6u;
        const uint32_t e = lut[cls * 16 + s4];
        const bool fast = valid & ((b4 | (a4 & ((e >> 20) & 15u))) == 0u) & (T3 + thrmax < D) & (h < 0xFFF0u) &
                          (F - Ff < 0xFEF0u);
        if (!fast) return step1(env, src, D, sid, ps);
        const uint32_t rs = (e >> 4) & 1u, fsw = (e >> 5) & 1u, hl = (e >> 6) & 7u, st4 = (e >> 16) & 15u,
                       lrs = (e >> 24) & 7u;
        F += (rs ? h : 0u) + ((e >> 9) & 15u);
        sst += ((rs & (fsw ^ 1u)) ? h : 0u) + ((e >> 13) & 7u);
        h = rs ? hl : h + hl;
        w = cls == 6u ? w + (e & 15u) - 4u : (e & 15u);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            stp[i] += fsw ? pend[i] : 0ull;
            pend[i] = rs ? 0ull : pend[i];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool hon = ((s4 >> j) & 1u) == 0u;
            const uint32_t sl = slot(kk[j], sid);
            field_add(stp, sl, (hon & (((st4 >> j) & 1u) != 0u)) ? 1u : 0u);  // made stale by a selfish win
            field_add(pend, sl, (hon & ((uint32_t)j >= lrs)) ? 1u : 0u);      // the honest branch after the last resolution
            env.add(C_F, kk[j], 1u);
        }
        T = T3 + (int64_t)In[3];
        k = src.k3;
        src.took4();
        src.fill();
        return T < D ? 0 : 2;
    }

    template <class Env>
    MSIM_HD void flush_stale(Env &env, uint32_t sid)
    {
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const uint32_t v = (uint32_t)j == sid ? 0u : field(stp, slot((uint32_t)j, sid));
            if (v) {
                env.add(C_S, (uint32_t)j, v);
                env.add(C_F, (uint32_t)j, 0u - v);
            }
        }
#pragma unroll
        for (int i = 0; i < NP; ++i) stp[i] = 0;
        Ff = F;
        if (sst) {
            env.add(C_S, sid, sst);
            env.add(C_F, sid, 0u - sst);
            sst = 0;
        }
    }

    // main.cpp:185-189 from a settled state: the honest branch is the best chain (first seen), the selfish
    // tie blocks and withheld blocks are not in it.
    template <class Env>
    MSIM_HD void finish(Env &env, uint32_t sid, SelOut &out)
    {
        flush_stale(env, sid);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            out.found[j] = env.get(C_F, (uint32_t)j) - ((uint32_t)j == sid ? h + w : 0u);
            out.stale[j] = env.get(C_S, (uint32_t)j);
        }
        out.best_height = F + h;
        out.err = 0;
    }

    // Hand the run to the entity engine at the pending find. The tie fork becomes the engine's two-branch
    // ("deep") form: window base F + h + 1, honest branch counts in C_A, the selfish branch in C_B. Tip
    // arrivals only order chains of equal length (main.cpp:75); every settled tip arrived before T and
    // every later block arrives after T, so T - 2 (honest tip) < T - 1 (selfish published tip) keeps
    // every comparison the reference makes.
    template <class Env, int NS, int NA, int NG, int NQ, int NC>
    MSIM_HD void to_exact(Env &env, Sel<M, NS, NA, NG, NQ, NC> &s, uint32_t m, const uint32_t *sids)
    {
        const uint32_t sid = sids[0];
        flush_stale(env, sid);
        s.init(m, sids);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const uint32_t p = (uint32_t)j == sid ? 0u : pend_of((uint32_t)j, sid);
            if (p) {
                env.add(C_F, (uint32_t)j, 0u - p);
                env.set(C_A, (uint32_t)j, p);
            }
        }
        env.add(C_F, sid, 0u - (h + w));
        if (h) env.set(C_B, sid, h);
        s.wb = F + h + 1u;
        s.deep = h != 0u;
        s.P.pa = h ? T - 2 : T - 1;
        Ent &X = s.S[0];
        X.pa = T - 1;
        X.br = h ? 1u : 0u;
        X.rp = -1;
        X.rt = (int32_t)w - 1;
        const int top = imin((int)w, WIN) - 1;
        X.s = (nib_upto(top) & (0x1111111111111111ull * (uint64_t)sid)) | ~nib_upto(top);
        X.xo = w > (uint32_t)WIN ? sid : SEL_NONE;
        s.w[0] = (int32_t)w;
        s.bpub = -1;
        s.t_ = T;
        s.nbt_ = T;
        s.kn_ = k;
    }

    // Take the run back from the engine when its state is settled (see above): nothing in flight, every
    // honest miner in the passive class on a published chain, the selfish miner on a published chain of the
    // same length plus withheld blocks, and either one common chain (a quiet network) or a tie fork whose
    // honest branch holds only honest blocks, whose selfish branch holds only the selfish miner's blocks,
    // and whose honest tip wins BestChain's tie-break (main.cpp:75). The fork's blocks may sit in the
    // window or, during a two-branch episode, partly in the deep-branch counters. Returns false (and
    // changes nothing) otherwise.
    template <class Env, int NS, int NA, int NG, int NQ, int NC>
    MSIM_HD bool take_back(Env &env, Sel<M, NS, NA, NG, NQ, NC> &s, uint32_t sid)
    {
        const Ent &P = s.P, &X = s.S[0];
        const bool calm = ((s.av | s.cm | s.am) == 0u) & (s.ng[0] == 0) & (s.err == 0u) & (s.t_ == s.nbt_);
        const bool shape = (P.rp == P.rt) & (P.rt < WIN) & (X.rp == P.rt) & (s.w[0] == X.rt - X.rp);
        if (!(calm & shape)) return false;
        // withheld blocks: the selfish miner's own (window part and implicit run)
        const int wtop = imin(X.rt, WIN - 1);
        if (count_nib(X.s, sid, nib_range(X.rp + 1, wtop)) != wtop - X.rp) return false;
        if (X.rt >= WIN && X.xo != sid) return false;
        const bool split = s.deep & (X.br != P.br);
        if (s.deep & !split) return false;  // (resolve() ends a one-branch deep episode within the step)
        int d = 0;  // lowest window height of the fork
        uint32_t below = 0;  // fork blocks below the window (per branch)
        if (!split) {
            d = first_diff(X.s, P.s, P.rt);
        } else {
            const int pa = P.br ? C_B : C_A, xa = X.br ? C_B : C_A;
            for (int j = 0; j < M; ++j) {
                const uint32_t cp = env.get(pa, (uint32_t)j), cx = env.get(xa, (uint32_t)j);
                if (((uint32_t)j == sid && cp) || ((uint32_t)j != sid && cx)) return false;
                below += cp;
            }
        }
        const int n = P.rt - d + 1;  // fork heights inside the window
        if (count_nib(P.s, sid, nib_range(d, P.rt)) != 0 || count_nib(X.s, sid, nib_range(d, P.rt)) != n) return false;
        const uint32_t hh = below + (uint32_t)n;
        if (hh) {
            if (hh >= 0xFFFFu) return false;
            const uint32_t pas = s.hm;  // every honest miner is passive
            const uint32_t pi = pas ? (uint32_t)__builtin_ctz(pas) : 99u;
            if (!((P.pa < X.pa) | ((P.pa == X.pa) & (pi < sid)))) return false;
        }
        // convert: the common part joins the settled counters, the fork's blocks and the withheld ones are
        // counted provisionally, the honest branch's composition goes to pend[]
#pragma unroll
        for (int i = 0; i < NP; ++i) pend[i] = 0;
        if (split) {
            const int pa = P.br ? C_B : C_A;
            for (int j = 0; j < M; ++j) {
                const uint32_t cp = env.get(pa, (uint32_t)j);
                if ((uint32_t)j != sid) field_add(pend, slot((uint32_t)j, sid), cp);
                env.add(C_F, (uint32_t)j, cp);
                env.set(C_A, (uint32_t)j, 0u);
                env.set(C_B, (uint32_t)j, 0u);
            }
        }
        for (int j = 0; j <= P.rt; ++j) {
            const uint32_t o = (uint32_t)(P.s >> (4 * j)) & 15u;
            env.add(C_F, o, 1u);
            if (j >= d) field_add(pend, slot(o, sid), 1u);
        }
        const uint32_t wn = (uint32_t)s.w[0];
        if (wn + hh) env.add(C_F, sid, wn + hh);
        F = s.wb + (uint32_t)P.rt - hh;
        h = hh;
        w = wn;
        sst = 0;
        Ff = F;
#pragma unroll
        for (int i = 0; i < NP; ++i) stp[i] = 0;
        T = s.nbt_;
        k = s.kn_;
        return true;
    }
};

}  // namespace msim
