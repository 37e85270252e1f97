// msim_selpipe.h — the selfish pipeline: networks with ONE selfish miner (BASELINE configs[2]), integer
// percentages and every propagation delay >= 1 ms, split into a draw kernel and a state kernel.
//
// The settled-state form (msim_selm.h) makes a network with one selfish miner a small Markov chain per
// find: selfish finds grow the withheld lead, honest finds resolve or extend a tie, and only a find whose
// consequences overlap the next find needs the entity engine (msim_sel.h). E1 (msim_sel_kernels.hip) runs
// that chain with the draws made in-lane, ~230 VALU instructions per block at two waves per SIMD. Here
// the draws leave the chain:
//
//   K1<NIB>  msim_draws_kernel (msim_drawgen.hip, the honest pipeline's draw kernel, msim_pipeline.h):
//            (run, segment) workers jumped to their segment, every block drawn as the reference draws it
//            (simulation.h:205-221); per block it stores the finder as a 4-bit nibble ([nb/8][nr] words)
//            and counts it per owner; it lists a block (with both RNG states after the next block) when
//            its finder is honest and the next interval is <= prop_k + prop_s: only such a "candidate"
//            can need the engine (msim_selm.h step: an honest find settles iff I_next > prop_k, or
//            > prop_k + prop_s when the selfish miner withholds blocks). Selfish finds are never listed.
//   S2       msim_selpipe_kernel (msim_sel_kernels.hip): one lane per run, the settled-state transition
//            for every block from its nibble alone (no draw, no counter: ~40 instructions per block), the
//            candidates checked against the state, and the engine for those that need it, drawing its
//            episode from the candidate's stored RNG states. The block where the nibble form stops, B (the
//            first block with T_B >= D - max(prop_k + prop_s)), is found in the prologue from K1's band sums
//            and one group redrawn from its stored RNG states; the run then ends right after B - 1 (T_B >= D,
//            ~99.7 % of runs at 1 s) or the engine finishes it from B with draws from the same group record,
//            so every comparison with D is the reference's.
//
// Counting. E1 counts every find provisionally in the settled form (C_F += 1) and the engine counts the
// blocks of its chains. S2 omits the provisional +1: K1's per-owner counts of blocks [0, B) are added at
// the end, and every block below B that the engine consumes is subtracted as it is consumed (SpSrc), so the
// totals equal E1's run for run.
//
// Exactness of the nibble form: every pending block i < B has T_i + prop_k + prop_s < D and T_{i+1} < D
// (checked for i = B - 1, whose next find is T_B), so the settled step's conditions reduce to "not a
// candidate, or a candidate whose I_next exceeds the state's threshold" — both known without the time. Runs
// that outgrow a capacity (candidate slots, list, pre-generated blocks) are flagged and recomputed by E2 from
// their seeds.
#pragma once
#include <math.h>

#include "msim_pipeline.h"
#include "msim_selm.h"

namespace msim {

constexpr uint32_t SP_NONE = 0xFFFFFFFFu;
constexpr double SP_MAX_RHO = 0.02;  // candidate rate above which E1 (in-lane draws) serves the network
enum : uint32_t { SERR_SP = 128u };  // the pipeline's capacities (slots, list, band): recomputed by E2

// P(block is a candidate) = sum over honest k of share_k * P(I_next <= prop_k + prop_s).
inline double sp_rho(const uint64_t *perc, const int64_t *prop, const uint8_t *self, int m)
{
    int sid = -1;
    for (int k = 0; k < m; ++k)
        if (self[k]) sid = k;
    const double ps = sid >= 0 ? (double)prop[sid] : 0.0;
    double rho = 0;
    for (int k = 0; k < m; ++k)
        if (!self[k]) rho += (double)perc[k] / 100.0 * (1.0 - exp(-((double)prop[k] + ps + 1.0) / 599999.5));
    return rho;
}

// The honest pipeline's layout (msim_pipeline.h) sized for the candidate rate, plus the nibbles.
struct SpLayout {
    PipeLayout L;
    size_t nib_off, total;
};
inline SpLayout sp_layout_for(double rho, uint32_t m, int64_t duration_ms, uint64_t n_runs, double budget,
                              uint32_t slots)
{
    SpLayout s;
    s.L = pipe_layout_for(rho, m, duration_ms, n_runs, budget, slots);
    const double nib = (double)s.L.nr * s.L.nb / 2.0;
    if ((double)s.L.total + nib > budget)  // shrink the slice so that both fit
        s.L = pipe_layout_for(rho, m, duration_ms, n_runs, budget * (double)s.L.total / ((double)s.L.total + nib), slots);
    s.nib_off = (s.L.total + 255) / 256 * 256;
    s.total = s.nib_off + ((size_t)s.L.nb / 8 * s.L.nr * 4 + 255) / 256 * 256;
    return s;
}

// K1<NIB>'s pick table: finder as in build_pick_table; fthr = prop_k + prop_s + 1 for honest finders (a
// block is listed when I_next < fthr), 0 for the selfish miner (never listed); PickFinder's fall-through
// carries FTHR_CAP (listed; the lane flags its run when it meets owner 15).
inline void build_pick_table_sp(const uint64_t *perc, const int64_t *prop, const uint8_t *selfish, int m, PickTab *out)
{
    int64_t ps = 0;
    for (int k = 0; k < m; ++k)
        if (selfish[k]) ps = prop[k];
    for (int q = 0; q < 128; ++q) {
        uint64_t cum = 0;
        int k = 15;
        for (int i = 0; i < m && q < PICK_TAB; ++i) {
            cum += perc[i];
            if (cum > (uint64_t)q) {
                k = i;
                break;
            }
        }
        uint32_t fthr = FTHR_CAP;
        if (k < 15) {
            const int64_t t = selfish[k] ? 0 : prop[k] + ps + 1;
            fthr = t < (int64_t)FTHR_CAP ? (uint32_t)t : FTHR_CAP;
        }
        out->info[q] = make_info((uint32_t)k, fthr);
    }
}

// What S2 reads of K1's output (one slice).
struct SpArgs {
    uint32_t nr, seg, gps, nsg, nseg, nb, cap, band_lo, lcap;
    const uint64_t *segsum;  // [nseg][nr]
    const uint32_t *segcnt;  // [nseg][8][nr] packed u16 owner counts
    const uint32_t *nslow;   // [nseg][nr] candidates per segment
    const uint32_t *slots;   // [nseg][cap][nr] list indices, block order
    const uint32_t *gsum;    // [nband][gps][nr]
    const uint64_t *gend;    // [nband][nsg][nr]
    const uint32_t *gcum;    // [nband][gps][8][nr]
    const GroupRec *grec;    // [nband][gps][nr]
    const EpEntry *list;
    const uint32_t *nib;     // [nb/8][nr]
};

// The nibble-mode cursor of one run (saved to LDS around engine phases on the device).
struct SpCur {
    uint32_t pos;          // pending block (the next find the settled form applies)
    uint32_t B;            // the first block with T_B >= D - max(prop_k + prop_s): the nibble form stops there
    uint32_t cseg, ci, cn; // candidate cursor: segment, next slot, candidates of that segment
    uint32_t c0, w0, i0;   // next candidate: block, next block's word (I << 5 | k), list index
    uint32_t c1, w1, i1;   // the one after it (prefetched)
    uint32_t sg;           // segment of pos
    uint64_t Tseg;         // time of the last block before segment sg (sum of the segment sums below it)
    uint64_t TB;           // T_B
    uint32_t gE;           // band position of B's group: jb * gps + g
    uint32_t err;
    static constexpr int NW = 18;
    MSIM_HD void save(uint32_t *p, int st) const
    {
        const uint32_t v[NW] = {pos, B, cseg, ci, cn, c0, w0, i0, c1, w1, i1, sg, (uint32_t)Tseg, (uint32_t)(Tseg >> 32),
                                (uint32_t)TB, (uint32_t)(TB >> 32), gE, err};
#pragma unroll
        for (int i = 0; i < NW; ++i) p[i * st] = v[i];
    }
    MSIM_HD void load(const uint32_t *p, int st)
    {
        pos = p[0];
        B = p[st];
        cseg = p[2 * st];
        ci = p[3 * st];
        cn = p[4 * st];
        c0 = p[5 * st];
        w0 = p[6 * st];
        i0 = p[7 * st];
        c1 = p[8 * st];
        w1 = p[9 * st];
        i1 = p[10 * st];
        sg = p[11 * st];
        Tseg = (uint64_t)p[12 * st] | ((uint64_t)p[13 * st] << 32);
        TB = (uint64_t)p[14 * st] | ((uint64_t)p[15 * st] << 32);
        gE = p[16 * st];
        err = p[17 * st];
    }
};

// Next candidate of run r after the cursor (block SP_NONE when the run has no more).
MSIM_HD void sp_fetch(const SpArgs &a, uint32_t r, SpCur &c, uint32_t &blk, uint32_t &wn, uint32_t &idx)
{
    while (c.ci >= c.cn) {
        if (++c.cseg >= a.nseg) {
            blk = SP_NONE;
            wn = 0;
            idx = SP_NONE;
            return;
        }
        c.cn = a.nslow[(size_t)c.cseg * a.nr + r];
        c.ci = 0;
        if (c.cn > a.cap) c.err |= SERR_SP;
    }
    idx = a.slots[((size_t)c.cseg * a.cap + c.ci) * a.nr + r];
    c.ci++;
    if (idx >= a.lcap || c.err) {
        c.err |= SERR_SP;
        blk = SP_NONE;
        wn = 0;
        return;
    }
    blk = a.list[idx].block;
    wn = a.list[idx].w1;
}

// Drop the next candidate (consumed), pull the prefetched one forward.
MSIM_HD void sp_pop(const SpArgs &a, uint32_t r, SpCur &c)
{
    c.c0 = c.c1;
    c.w0 = c.w1;
    c.i0 = c.i1;
    sp_fetch(a, r, c, c.c1, c.w1, c.i1);
}

// Resume the nibble form at block pos: the candidates below it were consumed by the engine, and the
// segment time follows pos.
MSIM_HD void sp_seek(const SpArgs &a, uint32_t r, SpCur &c, uint32_t pos)
{
    c.pos = pos;
    while (c.c0 != SP_NONE && c.c0 < pos) sp_pop(a, r, c);
    while (pos >= (c.sg + 1) * a.seg) {
        c.Tseg += a.segsum[(size_t)c.sg * a.nr + r];
        c.sg++;
    }
}

// Prologue of run r: B, the first block with T_B >= D - thr (thr = max over honest k of prop_k + prop_s), and
// T_B — from K1's band sums (super-group ends, then group sums) and B's group redrawn from its record (the
// group's first block word and both RNG states after it; drw: the lane's exact drawer, msim_selm.h) — and the
// first two candidates.
template <class Drw>
MSIM_HD void sp_begin(const SpArgs &a, uint32_t r, int64_t D, int64_t thr, Drw &drw, SpCur &c)
{
    c.err = 0;
    c.pos = 0;
    c.sg = 0;
    c.Tseg = 0;
    uint64_t Tb = 0;  // time of the last block before the band
    for (uint32_t s = 0; s < a.band_lo; ++s) Tb += a.segsum[(size_t)s * a.nr + r];
    const int64_t Dth = D - thr;
    c.B = SP_NONE;
    c.TB = 0;
    c.gE = 0;
    uint64_t Tj = Tb;
    if ((int64_t)Tb >= Dth) c.err |= SERR_SP;  // the run ends before the band (P ~ 1e-15): recomputed by E2
    for (uint32_t jb = 0; !c.err && jb + a.band_lo < a.nseg; ++jb) {
        // super-group ends: time from the segment's start to the end of every SGROUP-th group
        uint32_t sg = a.nsg;
        for (uint32_t q = 0; q < a.nsg; ++q) {
            const uint64_t e = a.gend[((size_t)jb * a.nsg + q) * a.nr + r];
            if (sg == a.nsg && (int64_t)(Tj + e) >= Dth) sg = q;
        }
        if (sg == a.nsg) {
            Tj += a.segsum[(size_t)(a.band_lo + jb) * a.nr + r];
            continue;
        }
        uint64_t t = Tj + (sg ? a.gend[((size_t)jb * a.nsg + sg - 1) * a.nr + r] : 0ull);
        const uint32_t g0 = sg * SGROUP, g1 = g0 + SGROUP < a.gps ? g0 + SGROUP : a.gps;
        for (uint32_t g = g0; g < g1; ++g) {
            const uint32_t gs = a.gsum[((size_t)jb * a.gps + g) * a.nr + r];
            if ((int64_t)(t + gs) >= Dth) {
                // B is in group g: redraw it from its first block (T_{W-1} = t)
                const GroupRec gr = a.grec[((size_t)jb * a.gps + g) * a.nr + r];
                drw.ri = gr.ri;
                drw.rp = gr.rp;
                uint32_t b = (a.band_lo + jb) * a.seg + g * GROUP;
                uint64_t T = t + (gr.w0 >> 5);
                for (uint32_t i = 1; i < GROUP && (int64_t)T < Dth; ++i) {
                    uint32_t I, k;
                    drw.draw(I, k);
                    T += I;
                    ++b;
                }
                c.B = b;
                c.TB = T;
                c.gE = jb * a.gps + g;
                break;
            }
            t += gs;
        }
        break;
    }
    if (c.B == SP_NONE) c.err |= SERR_SP;  // the run outlasts the pre-generated blocks
    c.cseg = 0;
    c.ci = 0;
    c.cn = a.nslow[r];
    if (c.cn > a.cap) c.err |= SERR_SP;
    sp_fetch(a, r, c, c.c0, c.w0, c.i0);
    sp_fetch(a, r, c, c.c1, c.w1, c.i1);
}

// K1's per-owner counts of blocks [0, B): the segments below B's segment, the cumulative counts at the start of
// B's group (gcum), and the group's blocks before B (their finders from the nibbles).
template <int M>
MSIM_HD void sp_counts(const SpArgs &a, uint32_t r, const SpCur &c, uint32_t (&F)[M])
{
#pragma unroll
    for (int k = 0; k < M; ++k) F[k] = 0;
    const uint32_t jb = c.gE / a.gps;
    for (uint32_t s = 0; s < a.band_lo + jb; ++s) add_packed<M>(F, a.segcnt + (size_t)s * CNT_WORDS * a.nr + r, a.nr);
    add_packed<M>(F, a.gcum + (size_t)c.gE * CNT_WORDS * a.nr + r, a.nr);
    for (uint32_t b = c.B & ~(GROUP - 1u); b < c.B; ++b) {
        const uint32_t k = (a.nib[(size_t)(b >> 3) * a.nr + r] >> (4 * (b & 7u))) & 15u;
#pragma unroll
        for (int kk = 0; kk < M; ++kk) F[kk] += (uint32_t)kk == k ? 1u : 0u;
    }
}

// One nibble word of a lane in the nibble form: the settled-state transition of every block from
// max(pos, the word's first block) up to the word's end or B, from the block's finder alone. A candidate is
// checked against the state (msim_selm.h step: an honest find settles iff I_next > prop_k + (w ? prop_s : 0);
// candidates have I_next <= prop_k + prop_s, so with w != 0 they never settle). Returns the lane's mode:
// 0 (continue at the next word), 1 (cur.pos is a candidate that needs the engine), 4 (cur.pos == B: switch
// to the engine: T_B < D), 6 (the run ends after block B - 1: T_B >= D, finish the settled form), 3 (error
// in cur.err). vote(b): nonzero when b holds for some lane of the wave (host: b).
template <int M, class Env, class Vote>
MSIM_HD int sp_word(const SpArgs &a, uint32_t r, Env &env, Vote vote, SpCur &cur, SelMacro<M> &mc, uint32_t sid,
                    int64_t D)
{
    if (cur.pos >= (cur.sg + 1) * a.seg) {  // segments start at word boundaries (seg is a multiple of GROUP)
        cur.Tseg += a.segsum[(size_t)cur.sg * a.nr + r];
        cur.sg++;
    }
    const uint32_t wi = cur.pos >> 3, off = cur.pos & 7u, p = wi << 3;
    const uint32_t word = a.nib[(size_t)wi * a.nr + r];
    bool run = true;
    int mode = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t pj = p + j;
        bool act = run & (j >= off) & (pj < cur.B);
        const uint32_t k = (word >> (4 * j)) & 15u;
        const bool isc = act & (pj == cur.c0);
        if (vote(isc)) {
            if (isc) {
                const bool ok = (mc.w == 0u) & ((cur.w0 >> 5) > (uint32_t)env.prop_tab(k < (uint32_t)M ? k : 0u));
                if (ok) {
                    sp_pop(a, r, cur);
                } else {
                    run = false;
                    act = false;
                    mode = 1;
                    cur.pos = pj;
                }
            }
        }
        if (act & (k >= (uint32_t)M)) {  // PickFinder fell through (simulation.h:220 asserts)
            cur.err |= SERR_PICK;
            run = false;
            act = false;
            mode = 3;
        }
        mc.transition(k, k == sid, act, sid);
    }
    if (run) {
        cur.pos = p + 8 < cur.B ? p + 8 : cur.B;
        if (cur.pos == cur.B) mode = (int64_t)cur.TB >= D ? 6 : 4;
    }
    if (vote(mc.F - mc.Ff >= 0xF000u)) {  // stp's 16-bit fields: flush well before they could overflow
        if (mc.F - mc.Ff >= 0xF000u) mc.flush_stale(env, sid);
    }
    if ((mc.h >= 0xF000u) & (mode != 3)) {  // a tie longer than the packed fields hold (never at 1 year)
        cur.err |= SERR_SP;
        mode = 3;
    }
    if (cur.err && mode != 3) mode = 3;
    return mode;
}

// The engine's draw source in the selfish pipeline: E1's FIFO (msim_selm.h SelFifo) seeded from K1's stored
// RNG states, which tracks the block the engine has pending. Every block below B the engine consumes (the
// pending block at each next(): the reference's loop draws the next find right after FoundBlock, main.cpp:
// 153-157) was counted by K1, so its count is taken back here (msim_selpipe.h header).
// Holds the FIFO by value and a copy of the counter access (device: SelDevEnv, a few pointers; host: a
// forwarding reference type): a member reference would take the FIFO's address and keep it in scratch.
template <class Fifo, class Env>
struct SpSrc {
    Fifo f;
    Env env;
    uint32_t pidx, pk, B;  // pending block and its finder (pidx = SP_NONE once the lane draws); the switch block
    MSIM_HD bool next(uint32_t &I, uint32_t &k)
    {
        if (pidx < B) env.add(C_F, pk, 0xFFFFFFFFu);
        f.next(I, k);
        if (pidx != SP_NONE) pidx += 1;
        pk = k;
        return true;
    }
    MSIM_HD void prefetch() {}
    MSIM_HD void settle() {}
};

// A lane leaves the nibble form for the engine: mode 1 (its candidate cur.c0 needs the engine: the FIFO is
// seeded from the candidate's list entry) or mode 4 (it reached B with T_B < D: the FIFO is seeded by redrawing
// B's group from its record). The settled state is handed to the engine (msim_selm.h to_exact). Returns the
// new mode (2: engine, 3: error in cur.err). src: SpSrc (its FIFO, the pending block and finder).
template <int M, class Src, class SelT, class Env>
MSIM_HD int sp_enter(const SpArgs &a, uint32_t r, int mode, SpCur &cur, SelMacro<M> &mc, Src &src, SelT &s, Env &env,
                     uint32_t m, const uint32_t *sids)
{
    auto &fifo = src.f;
    if (mode == 1) {
        const EpEntry &e = a.list[cur.i0];
        mc.T = (int64_t)(cur.Tseg + e.offset);
        mc.k = e.w0 & 31u;
        fifo.d.ri = e.ri;
        fifo.d.rp = e.rp;
        fifo.I0 = e.w1 >> 5;
        fifo.k0 = e.w1 & 31u;
        src.pidx = cur.c0;
    } else {
        const uint32_t jb = cur.gE / a.gps, g = cur.gE % a.gps;
        const GroupRec gr = a.grec[(size_t)cur.gE * a.nr + r];
        fifo.d.ri = gr.ri;
        fifo.d.rp = gr.rp;
        uint32_t I = gr.w0 >> 5, k = gr.w0 & 31u;  // the group's first block
        uint32_t kB = k;
        for (uint32_t b = (a.band_lo + jb) * a.seg + g * GROUP; b <= cur.B; ++b) {  // draws up to block B + 1
            kB = k;
            fifo.d.draw(I, k);
        }
        if (kB >= (uint32_t)M) {
            cur.err |= SERR_PICK;
            return 3;
        }
        mc.T = (int64_t)cur.TB;
        mc.k = kB;
        fifo.I0 = I;
        fifo.k0 = k;
        src.pidx = SP_NONE;  // nothing past B was counted by K1
    }
    fifo.n = 1;
    fifo.fill();
    src.pk = mc.k;
    mc.to_exact(env, s, m, sids);
    return 2;
}

// A lane in the engine steps it (msim_sel.h step) until the run is over (finish) or the engine hands the run
// back to the settled form below B (msim_selm.h take_back: the nibble form resumes at the source's pending
// block, sp_seek); past B the engine keeps the run to its end (only the last ~prop_k + prop_s of a run is
// there). The kernel writes this step inline (msim_sel_kernels.hip msim_selpipe_kernel, and the host driver in
// tests/native/selpipe_host.cpp): as a helper taking the finish record and the taken-back state by reference,
// both stayed live across the engine step and the engine loop spilled ~3x more.

}  // namespace msim
