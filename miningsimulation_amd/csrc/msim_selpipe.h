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
//            (simulation.h:205-221); per block it stores the finder as a 4-bit nibble (a 16-byte chunk of 32
//            blocks per run, [nb/32][nr] chunks, so S2 reads a run's chunk with one 16-byte load)
//            and counts it per owner; it lists a block (with both RNG states after the next block) when
//            its finder is honest and the next interval is <= prop_k + prop_s: only such a "candidate"
//            can need the engine (msim_selm.h step: an honest find settles iff I_next > prop_k, or
//            > prop_k + prop_s when the selfish miner withholds blocks). Selfish finds are never listed.
//            Per 32-block chunk it also writes two candidate masks: A (the block is listed) and B (its
//            I_next <= prop_k: it never settles), so S2 decides every candidate from its chunk alone.
//   S2       msim_selpipe_kernel (msim_sel_kernels.hip): one lane per run, the settled-state transition
//            for every block from its nibble and mask bits alone (no draw, no counter, no memory access but
//            one 16-byte chunk and one mask pair per 32 blocks, loaded a chunk ahead), and the engine for
//            the candidates that need it, drawing the episode from the candidate's stored RNG states (found
//            through the run's slot list only then). The block where the nibble form stops, B (the
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
    size_t nib_off, cmask_off, total;
};
inline SpLayout sp_layout_for(double rho, uint32_t m, int64_t duration_ms, uint64_t n_runs, double budget,
                              uint32_t slots)
{
    SpLayout s;
    const double mu = (double)duration_ms / 599999.5;
    // >= nb / 2 bytes of nibbles and nb / 4 bytes of candidate masks per run
    const double nib = (mu + 8.0 * sqrt(mu > 1.0 ? mu : 1.0) + 64.0 + GROUP * 256.0) * 0.75;
    s.L = pipe_layout_for(rho, m, duration_ms, n_runs, budget, slots, false, nib);
    s.nib_off = (s.L.total + 255) / 256 * 256;
    s.cmask_off = s.nib_off + ((size_t)s.L.nb / 8 * s.L.nr * 4 + 255) / 256 * 256;
    s.total = s.cmask_off + ((size_t)s.L.nb / 32 * s.L.nr * 8 + 255) / 256 * 256;
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
    uint32_t nr, seg, nsg, nseg, nb, cap, band_lo, lcap;
    const uint64_t *segsum;  // [nseg][nr]
    const uint32_t *segcnt;  // [nseg][8][nr] packed u16 owner counts
    const uint32_t *nslow;   // [nseg][nr] candidates per segment
    const uint32_t *slots;   // [nseg][cap][nr] list indices, block order
    const uint64_t *gend;    // [nband][nsg][nr]: time from the segment's start to each super-group's end
    const uint32_t *gcum;    // [nband][nsg][8][nr]: counts before each super-group
    const GroupRec *grec;    // [nband][nsg][nr]: each super-group's first block and the streams after it
    const EpEntry *list;
    const uint32_t *nib;     // [nb/32][nr][4]: word w (blocks 8w .. 8w+7) of run r at ((w >> 2) * nr + r) * 4 + (w & 3)
    const CMask *cmask;      // [nb/32][nr]: per chunk (A: listed candidates, B: candidates with I_next <= prop_k)
};

// The u32 index of nibble word w of run r (the 16-byte chunk layout above; K1 writes it, S2 reads it).
MSIM_HD size_t sp_nib_index(uint32_t nr, uint32_t r, uint32_t w) { return ((size_t)(w >> 2) * nr + r) * 4 + (w & 3u); }

// The nibble-form cursor of one run (saved to LDS around engine phases on the device).
struct SpCur {
    uint32_t pos;          // pending block (the next find the settled form applies)
    uint32_t B;            // the first block with T_B >= D - max(prop_k + prop_s): the nibble form stops there
    uint32_t sg;           // segment of pos
    uint32_t ci;           // candidates of segment sg below pos (the slot of the next one)
    uint64_t Tseg;         // time of the last block before segment sg (sum of the segment sums below it)
    uint64_t TB;           // T_B
    uint32_t gE;           // band position of B's super-group: jb * nsg + q
    uint32_t err;
    uint32_t A[4], N[4];   // the nibble chunk of pos (blocks 32c .. 32c + 31) and the next one, loaded ahead
    CMask mA, mN;          // their candidate masks (not saved with the cursor: reloaded, sp_refill)
    static constexpr int NW = 10;
    MSIM_HD void save(uint32_t *p, int st) const
    {
        const uint32_t v[NW] = {pos, B, sg, ci, (uint32_t)Tseg, (uint32_t)(Tseg >> 32), (uint32_t)TB, (uint32_t)(TB >> 32),
                                gE, err};
#pragma unroll
        for (int i = 0; i < NW; ++i) p[i * st] = v[i];
    }
    MSIM_HD void load(const uint32_t *p, int st)
    {
        pos = p[0];
        B = p[st];
        sg = p[2 * st];
        ci = p[3 * st];
        Tseg = (uint64_t)p[4 * st] | ((uint64_t)p[5 * st] << 32);
        TB = (uint64_t)p[6 * st] | ((uint64_t)p[7 * st] << 32);
        gE = p[8 * st];
        err = p[9 * st];
    }
};

// Nibble chunk c (blocks 32c .. 32c + 31) of run r and its candidate masks (one 16-byte and one 8-byte load);
// beyond the pre-generated blocks, the last chunk.
MSIM_HD void sp_chunk_at(const SpArgs &a, uint32_t r, uint32_t c, uint32_t (&w)[4], CMask &m)
{
    const uint32_t last = a.nb / 32 - 1;
    c = c < last ? c : last;
    const uint32_t *q = a.nib + sp_nib_index(a.nr, r, c * 4);
#if defined(__HIP_DEVICE_COMPILE__)
    const uint4 v = *(const uint4 *)q;  // one global_load_dwordx4
    w[0] = v.x;
    w[1] = v.y;
    w[2] = v.z;
    w[3] = v.w;
#else
    for (int i = 0; i < 4; ++i) w[i] = q[i];
#endif
    m = a.cmask[(size_t)c * a.nr + r];
}

// The finder nibble of block b of run r.
MSIM_HD uint32_t sp_nib(const SpArgs &a, uint32_t r, uint32_t b)
{
    return (a.nib[sp_nib_index(a.nr, r, b >> 3)] >> (4 * (b & 7u))) & 15u;
}

// Load the chunk of pos and the next one (the nibble form reads a chunk per 32 blocks with the next one in
// flight, so its latency is hidden).
MSIM_HD void sp_refill(const SpArgs &a, uint32_t r, SpCur &c)
{
    sp_chunk_at(a, r, c.pos >> 5, c.A, c.mA);
    sp_chunk_at(a, r, (c.pos >> 5) + 1, c.N, c.mN);
}

// Candidates of run r among blocks [b0, b1) (their A mask bits; the chunks loaded here: rare paths only).
MSIM_HD uint32_t sp_count_cands(const SpArgs &a, uint32_t r, uint32_t b0, uint32_t b1)
{
    uint32_t n = 0;
    for (uint32_t c = b0 >> 5; c * 32 < b1; ++c) {
        uint32_t m = a.cmask[(size_t)c * a.nr + r].a;
        const uint32_t lo = b0 > c * 32 ? b0 - c * 32 : 0u, hi = b1 < c * 32 + 32 ? b1 - c * 32 : 32u;
        m &= (hi >= 32 ? 0xFFFFFFFFu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
        n += (uint32_t)__builtin_popcount(m);
    }
    return n;
}

// Resume the nibble form at block pos (after an engine episode that consumed blocks from cur.pos on): the
// segment time and the candidate count follow pos.
MSIM_HD void sp_seek(const SpArgs &a, uint32_t r, SpCur &c, uint32_t pos)
{
    uint32_t from = c.pos;
    while (pos >= (c.sg + 1) * a.seg) {
        c.Tseg += a.segsum[(size_t)c.sg * a.nr + r];
        c.sg++;
        c.ci = 0;
        from = c.sg * a.seg;
    }
    c.ci += sp_count_cands(a, r, from, pos);
    c.pos = pos;
    sp_refill(a, r, c);
}

// First block of band super-group gE.
MSIM_HD uint32_t sp_sg_block(const SpArgs &a, uint32_t gE)
{
    return (a.band_lo + gE / a.nsg) * a.seg + (gE % a.nsg) * (SGROUP * GROUP);
}

// Prologue of run r: B, the first block with T_B >= D - thr (thr = max over honest k of prop_k + prop_s), and
// T_B — from K1's super-group ends and B's super-group redrawn from its record (its first block's word and
// both RNG states after it; drw: the lane's exact drawer, msim_selm.h; at most SGROUP * GROUP draws, once per
// run) — and the first chunks. A run whose candidates outgrew a segment's slots is flagged (E2 recomputes it).
template <class Drw>
MSIM_HD void sp_begin(const SpArgs &a, uint32_t r, int64_t D, int64_t thr, Drw &drw, SpCur &c)
{
    c.err = 0;
    c.pos = 0;
    c.sg = 0;
    c.ci = 0;
    c.Tseg = 0;
    uint64_t Tb = 0;  // time of the last block before the band
    for (uint32_t s = 0; s < a.nseg; ++s) {
        if (s < a.band_lo) Tb += a.segsum[(size_t)s * a.nr + r];
        if (a.nslow[(size_t)s * a.nr + r] > a.cap) c.err |= SERR_SP;
    }
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
        // B is in super-group sg: redraw it from its first block (T of the block before it = t)
        const uint64_t t = Tj + (sg ? a.gend[((size_t)jb * a.nsg + sg - 1) * a.nr + r] : 0ull);
        c.gE = jb * a.nsg + sg;
        const GroupRec gr = a.grec[(size_t)c.gE * a.nr + r];
        drw.ri = gr.ri;
        drw.rp = gr.rp;
        uint32_t b = sp_sg_block(a, c.gE);
        uint64_t T = t + (gr.w0 >> 5);
        for (uint32_t i = 1; i < SGROUP * GROUP && (int64_t)T < Dth; ++i) {
            uint32_t I, k;
            drw.draw(I, k);
            T += I;
            ++b;
        }
        c.B = b;
        c.TB = T;
        break;
    }
    if (c.B == SP_NONE) c.err |= SERR_SP;  // the run outlasts the pre-generated blocks
    sp_refill(a, r, c);
}

// K1's per-owner counts of blocks [0, B): the segments below B's segment, the cumulative counts at the start of
// B's super-group (gcum), and the super-group's blocks before B (their finders from the nibbles).
template <int M>
MSIM_HD void sp_counts(const SpArgs &a, uint32_t r, const SpCur &c, uint32_t (&F)[M])
{
#pragma unroll
    for (int k = 0; k < M; ++k) F[k] = 0;
    const uint32_t jb = c.gE / a.nsg;
    for (uint32_t s = 0; s < a.band_lo + jb; ++s) add_packed<M>(F, a.segcnt + (size_t)s * CNT_WORDS * a.nr + r, a.nr);
    add_packed<M>(F, a.gcum + (size_t)c.gE * CNT_WORDS * a.nr + r, a.nr);
    for (uint32_t b = sp_sg_block(a, c.gE); b < c.B; ++b) {
        const uint32_t k = sp_nib(a, r, b);
#pragma unroll
        for (int kk = 0; kk < M; ++kk) F[kk] += (uint32_t)kk == k ? 1u : 0u;
    }
}

// One nibble word (blocks 8 wi .. 8 wi + 7) of a lane in the nibble form: the settled-state transition of every
// block from max(pos, 8 wi) up to the word's end or B, from the block's finder and candidate bits alone
// (mA, mB: the word's bits of the chunk masks; a block whose finder fell through PickFinder is left to the
// error check). A candidate settles (msim_selm.h step: an honest find settles
// iff I_next > prop_k + (w ? prop_s : 0); a candidate has I_next <= prop_k + prop_s) iff its B bit is clear
// and w == 0. Returns the lane's mode: 0 (continue), 1 (cur.pos is a candidate that needs the engine), 4
// (cur.pos == B: to the engine, T_B < D), 6 (the run ends after block B - 1: T_B >= D, finish the settled
// form), 3 (error in cur.err). vote(b): nonzero when b holds for some lane of the wave (host: b).
template <int M, class Vote>
MSIM_HD int sp_word(Vote vote, SpCur &cur, SelMacro<M> &mc, uint32_t sid, int64_t D, uint32_t word,
                    uint32_t mA, uint32_t mB, uint32_t wi)
{
    const uint32_t off = cur.pos & 7u, p = wi << 3;
    bool run = true;
    int mode = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t pj = p + j;
        bool act = run & (j >= off) & (pj < cur.B);
        const uint32_t k = (word >> (4 * j)) & 15u;
        const bool cand = act & (((mA >> j) & 1u) != 0u);
#if SP_DIAG_NOENG
        const bool need = false;
#else
        const bool need = cand & (k < (uint32_t)M) & ((((mB >> j) & 1u) != 0u) | (mc.w != 0u));
#endif
        if (vote(need)) {
            if (need) {
                run = false;
                act = false;
                mode = 1;
                cur.pos = pj;
            }
        }
        cur.ci += (cand & act) ? 1u : 0u;  // a candidate the settled form takes
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
    return mode;
}

// One 32-block chunk of a lane in the nibble form (from pos to the chunk's end; the four words of cur.A in
// order), then the next chunk moves up and the one after it is loaded. Returns the lane's mode (sp_word).
template <int M, class Env, class Vote>
MSIM_HD int sp_chunk(const SpArgs &a, uint32_t r, Env &env, Vote vote, SpCur &cur, SelMacro<M> &mc, uint32_t sid,
                     int64_t D)
{
    if (cur.pos >= (cur.sg + 1) * a.seg) {  // segments start at chunk boundaries (seg is a multiple of GROUP)
        cur.Tseg += a.segsum[(size_t)cur.sg * a.nr + r];
        cur.sg++;
        cur.ci = 0;
    }
    const uint32_t c = cur.pos >> 5;
    int mode = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        if ((mode == 0) & ((cur.pos >> 3) == c * 4 + j))
            mode = sp_word<M>(vote, cur, mc, sid, D, cur.A[j], (cur.mA.a >> (8 * j)) & 0xFFu,
                              (cur.mA.b >> (8 * j)) & 0xFFu, c * 4 + j);
    if (vote(mc.F - mc.Ff >= 0xF000u)) {  // stp's 16-bit fields: flush well before they could overflow
        if (mc.F - mc.Ff >= 0xF000u) mc.flush_stale(env, sid);
    }
    if ((mc.h >= 0xF000u) & (mode != 3)) {  // a tie longer than the packed fields hold (never at 1 year)
        cur.err |= SERR_SP;
        mode = 3;
    }
    if (mode == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) cur.A[j] = cur.N[j];
        cur.mA = cur.mN;
        sp_chunk_at(a, r, c + 2, cur.N, cur.mN);
    }
    return mode;
}

// The engine's draw source in the selfish pipeline: E1's FIFO (msim_selm.h SelFifo) seeded from K1's stored
// RNG states, which tracks the block the engine has pending. Every block below B the engine consumes (the
// pending block at each next(): the reference's loop draws the next find right after FoundBlock, main.cpp:
// 153-157) was counted by K1, so its count is taken back here (msim_selpipe.h header).
// Holds the FIFO by value and the lane's found-counter access (Cnt: add(k, v) on C_F; device: one LDS pointer):
// a member reference would take the FIFO's address and keep it in scratch.
template <class Fifo, class Cnt>
struct SpSrc {
    Fifo f;
    Cnt cnt;
    uint32_t pidx, pk, B;  // pending block and its finder (pidx = SP_NONE once the lane draws); the switch block
    MSIM_HD bool next(uint32_t &I, uint32_t &k)
    {
        if (pidx < B) cnt.add(pk, 0xFFFFFFFFu);
        f.next(I, k);
        if (pidx != SP_NONE) pidx += 1;
        pk = k;
        return true;
    }
    MSIM_HD void prefetch() {}
    MSIM_HD void settle() {}
};

// A lane leaves the nibble form for the engine: mode 1 (its candidate at cur.pos needs the engine: the FIFO is
// seeded from the candidate's list entry, found through the segment's slots) or mode 4 (it reached B with
// T_B < D: the FIFO is seeded by redrawing B's super-group from its record). The settled state is handed to the
// engine (msim_selm.h to_exact). Returns the new mode (2: engine, 3: error in cur.err). src: SpSrc.
template <int M, class Src, class SelT, class Env>
MSIM_HD int sp_enter(const SpArgs &a, uint32_t r, int mode, SpCur &cur, SelMacro<M> &mc, Src &src, SelT &s, Env &env,
                     uint32_t m, const uint32_t *sids)
{
    auto &fifo = src.f;
    if (mode == 1) {
        const uint32_t idx = a.slots[((size_t)cur.sg * a.cap + cur.ci) * a.nr + r];
        if (idx >= a.lcap || a.list[idx].block != cur.pos) {
            cur.err |= SERR_SP;  // the list overflowed (its entry was not stored)
            return 3;
        }
        const EpEntry &e = a.list[idx];
        mc.T = (int64_t)(cur.Tseg + e.offset);
        mc.k = e.w0 & 31u;
        fifo.d.ri = e.ri;
        fifo.d.rp = e.rp;
        fifo.I0 = e.w1 >> 5;
        fifo.k0 = e.w1 & 31u;
        src.pidx = cur.pos;
    } else {
        const GroupRec gr = a.grec[(size_t)cur.gE * a.nr + r];
        fifo.d.ri = gr.ri;
        fifo.d.rp = gr.rp;
        uint32_t I = gr.w0 >> 5, k = gr.w0 & 31u;  // the group's first block
        uint32_t kB = k;
        for (uint32_t b = sp_sg_block(a, cur.gE); b <= cur.B; ++b) {  // draws up to block B + 1
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
