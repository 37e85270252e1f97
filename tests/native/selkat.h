// selkat.h — TEST INFRASTRUCTURE: the reference's TestSelfishStrategy (/root/reference/test.cpp:213-367,
// tests/golden/selfish_strategy_kats.json) replayed on the PRODUCT's two selfish state machines, as lane
// functions that the host build (selkat_host.cpp) and a gfx950 kernel (selkat_dev.hip) both run:
//
//   kat_sel    the entity engine (miningsimulation_amd/csrc/msim_sel.h). The KAT's chain becomes the selfish
//              entity S[0] (window owners, published tip and its arrival, in-flight reveal groups, withheld
//              count); the op is Sel::found (Miner::FoundBlock, simulation.h:62-76, with best_chain_size as the
//              previous event's best tip, bpub) or Sel::notify (NotifyBestChain, simulation.h:177-180, with the
//              KAT's best chain as BestChain's pick). The resulting entity is written back as a chain: owners at
//              every height, W for withheld blocks, the arrival of every in-flight block and of the published
//              tip. The arrivals of published blocks below the tip are not carried by the engine (a block is
//              identified by (owner, height); UnpublishedBlocks stops at the first published block
//              from the top and BestChain reads only the tip's arrival, main.cpp:68-82): those come back as -1
//              and the test checks that the reference's block there is published.
//   kat_macro  the settled form (miningsimulation_amd/csrc/msim_selm.h SelMacro::transition). It holds a run
//              only between finds whose consequences have settled: a common prefix F, a published tie fork of h
//              blocks per branch, w withheld blocks. A KAT whose chain is such a state (no fork, no block in
//              flight) is entered as (F, 0, w); a found op is the selfish miner's transition, a notify op one
//              honest transition per new block of the best chain. The result is the settled tuple
//              (F, h, w, the honest branch's miner-1 count, the selfish stale blocks), which the test compares
//              with the tuple the reference's expected chain settles to.
#pragma once
#include <stdint.h>

#include "../../miningsimulation_amd/csrc/msim_sel.h"
#include "../../miningsimulation_amd/csrc/msim_selm.h"

namespace msim {

constexpr int KAT_MAXB = 16;        // blocks per chain (genesis excluded)
constexpr int64_t KAT_W = -2;       // SELFISH_ARRIVAL in KatIn / KatOut
constexpr int64_t KAT_UNSEEN = -1;  // a published block whose arrival the engine does not carry
constexpr uint32_t KAT_M = 2;       // the KATs' two ids: the selfish miner 0 and "the others" 1

struct KatIn {
    uint32_t op;        // 0: FoundBlock by the selfish miner at t; 1: NotifyBestChain(best, t)
    uint32_t bcs;       // found: best_chain_size (genesis included)
    int64_t t;
    int64_t prop;       // the selfish miner's propagation (ms)
    uint32_t n, bn;     // blocks of chain / best (genesis excluded)
    uint32_t own[KAT_MAXB], bown[KAT_MAXB];
    int64_t arr[KAT_MAXB], barr[KAT_MAXB];
};

struct KatOut {
    // entity engine
    uint32_t n, err, stale_s;
    uint32_t own[KAT_MAXB + 2];
    int64_t arr[KAT_MAXB + 2];
    // settled form (rep == 0: the KAT's chain is not a settled state)
    uint32_t rep, F, h, w, pend1, sst;
};

struct KatEnv {
    int64_t p[KAT_M];
    uint32_t c[4][MAXM];
    ColdAct cs[8];
    MSIM_HD int64_t prop(uint32_t k) const { return p[k < KAT_M ? k : 0]; }
    MSIM_HD int64_t prop_tab(uint32_t k) const { return p[k < KAT_M ? k : 0]; }
    MSIM_HD uint32_t get(int a, uint32_t k) const { return c[a][k]; }
    MSIM_HD void add(int a, uint32_t k, uint32_t v) { c[a][k] += v; }
    MSIM_HD void set(int a, uint32_t k, uint32_t v) { c[a][k] = v; }
    MSIM_HD ColdAct cold(int i) const { return cs[i]; }
    MSIM_HD void cold_put(int i, const ColdAct &r) { cs[i] = r; }
    MSIM_HD bool fold_vote(bool due) { return due; }
};

using KatSel = Sel<KAT_M, 1, 1, 4, 1, 4>;

MSIM_HD void kat_env(const KatIn &in, KatEnv &env)
{
    env.p[0] = in.prop;
    env.p[1] = in.prop;
    for (int a = 0; a < 4; ++a)
        for (int k = 0; k < MAXM; ++k) env.c[a][k] = 0;
}

MSIM_HD void kat_sel(const KatIn &in, KatOut &out)
{
    KatEnv env;
    kat_env(in, env);
    const uint32_t sids[SEL_MAXS] = {0u, SEL_NONE, SEL_NONE, SEL_NONE};
    KatSel s;
    s.init(KAT_M, sids);
    Ent &X = s.S[0];
    // the chain: owners from height 1 (window position 0, wb = 1), then what is published at t, in flight, withheld
    int rp = -1;
    int32_t w = 0;
    for (uint32_t i = 0; i < in.n; ++i) {
        ent_append(X, in.own[i]);
        if (in.arr[i] == KAT_W) ++w;
        else if (in.arr[i] <= in.t) rp = (int)i;
    }
    X.rp = rp;
    X.pa = rp >= 0 ? in.arr[rp] : 0;  // Genesis arrives at 0 (simulation.h:31-33)
    for (int i = rp + 1; i < (int)in.n && in.arr[i] != KAT_W;) {
        int j = i;
        while (j + 1 < (int)in.n && in.arr[j + 1] == in.arr[i]) ++j;
        s.push_group(0, j - i + 1, in.arr[i]);
        i = j + 1;
    }
    s.w[0] = w;
    if (in.op == 0) {
        s.bpub = (int32_t)in.bcs - 2;  // best_chain_size - 1 - wb
        s.found(env, 0u, in.t);
    } else {
        SelBest B;
        B.l = (int32_t)in.bn - 1;
        B.s = ~0ull;
        for (uint32_t i = 0; i < in.bn && i < (uint32_t)WIN; ++i)
            B.s = (B.s & ~(0xFull << (4 * i))) | ((uint64_t)in.bown[i] << (4 * i));
        B.a = in.bn ? in.barr[in.bn - 1] : 0;
        B.x = SEL_NONE;
        B.br = 0;
        s.notify(env, in.t, B);
    }
    // back to a chain
    out.err = s.err;
    out.n = (uint32_t)(X.rt + 1);
    int g = 0, gl = s.ng[0] > 0 ? s.gc[0][0] : 0;
    for (int i = 0; i <= X.rt && i < KAT_MAXB + 2; ++i) {
        out.own[i] = i < WIN ? (uint32_t)(X.s >> (4 * i)) & 15u : X.xo;
        if (i < X.rp) out.arr[i] = KAT_UNSEEN;
        else if (i == X.rp) out.arr[i] = X.pa;
        else if (i > X.rt - s.w[0]) out.arr[i] = KAT_W;
        else {  // in flight: the reveal groups in order
            while (gl == 0 && g + 1 < s.ng[0]) gl = s.gc[0][++g];
            out.arr[i] = g < s.ng[0] ? s.ga[0][g] : KAT_UNSEEN - 100;
            --gl;
        }
    }
    out.stale_s = env.get(C_S, 0u);
}

MSIM_HD void kat_macro(const KatIn &in, KatOut &out)
{
    // a settled state: a published chain, then withheld blocks, nothing in flight and no race
    uint32_t pub = 0, w = 0;
    bool rep = true;
    for (uint32_t i = 0; i < in.n; ++i) {
        if (in.arr[i] == KAT_W) ++w;
        else if (w != 0 || in.arr[i] > in.t) rep = false;
        else ++pub;
    }
    if (in.op == 0) rep = rep & (in.bcs == pub + 1);  // the public chain is the selfish miner's published one
    else {
        rep = rep & (in.bn > pub);  // the best chain extends the published chain
        for (uint32_t i = 0; i < pub && rep; ++i) rep = in.bown[i] == in.own[i] && in.barr[i] == in.arr[i];
    }
    out.rep = rep ? 1u : 0u;
    if (!rep) return;
    SelMacro<KAT_M> mc;
    mc.T = in.t;
    mc.k = 0;
    mc.F = pub;
    mc.h = 0;
    mc.w = w;
    mc.sst = 0;
    mc.Ff = 0;
    for (int i = 0; i < SelMacro<KAT_M>::NP; ++i) mc.pend[i] = mc.stp[i] = 0;
    if (in.op == 0) mc.transition(0u, true, true, 0u);
    else
        for (uint32_t i = pub; i < in.bn; ++i) mc.transition(in.bown[i], in.bown[i] == 0u, true, 0u);
    out.F = mc.F;
    out.h = mc.h;
    out.w = mc.w;
    out.pend1 = mc.pend_of(1u, 0u);
    out.sst = mc.sst;
}

}  // namespace msim
