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
    size_t nib_off, cmask_off, stale_off, total;
};
inline SpLayout sp_layout_for(double rho, uint32_t m, int64_t duration_ms, uint64_t n_runs, double budget,
                              uint32_t slots)
{
    SpLayout s;
    const double mu = (double)duration_ms / 599999.5;
    // >= nb / 2 bytes of nibbles, nb / 4 of candidate masks and nb / 8 of stale masks per run
    const double nib = (mu + 8.0 * sqrt(mu > 1.0 ? mu : 1.0) + 64.0 + GROUP * 256.0) * 0.875;
    s.L = pipe_layout_for(rho, m, duration_ms, n_runs, budget, slots, false, nib);
    s.nib_off = (s.L.total + 255) / 256 * 256;
    s.cmask_off = s.nib_off + ((size_t)s.L.nb / 8 * s.L.nr * 4 + 255) / 256 * 256;
    s.stale_off = s.cmask_off + ((size_t)s.L.nb / 32 * s.L.nr * 8 + 255) / 256 * 256;
    s.total = s.stale_off + ((size_t)s.L.nb / 32 * s.L.nr * 4 + 255) / 256 * 256;
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
    uint32_t *stale;         // [nb/32][nr]: S2's stale honest blocks per chunk (zeroed before S2; SpSt)
    uint32_t xth;            // waiting lanes that start an engine phase (msim_sel_kernels.hip msim_selpipe_kernel)
};


// The u32 index of nibble word w of run r (the 16-byte chunk layout above; K1 writes it, S2 reads it).
MSIM_HD size_t sp_nib_index(uint32_t nr, uint32_t r, uint32_t w) { return ((size_t)(w >> 2) * nr + r) * 4 + (w & 3u); }

// Chunks the nibble form keeps loaded: a ring of SP_PF, the chunk at ring slot S being the one the lane's S-th
// table step (mod SP_PF) since the last refill reads. All lanes of a nibble phase step together and every phase
// starts from a refill, so the slot is wave-uniform and each step names its registers at compile time: a ring
// shifted by register moves made the compiler wait for the load just issued (a move of a pending load's
// destination), which left every chunk waiting on memory (measured: ~18k cycles per chunk).
#ifndef MSIM_SP_PF
#define MSIM_SP_PF 4
#endif
constexpr int SP_PF = MSIM_SP_PF;
static_assert(SP_PF == 1 || SP_PF == 2 || SP_PF == 4, "the kernel steps four ring slots per pass");

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
    uint32_t A[SP_PF][4];  // the nibble chunk of pos (blocks 32c .. 32c + 31) and the next ones, loaded ahead
    CMask mA[SP_PF];       // their candidate masks (not saved with the cursor: reloaded, sp_refill)
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

// The settled state of a run in the nibble form: msim_selm.h's (F, h, w) and unflushed selfish stale blocks,
// with the honest branch kept as a block RANGE instead of per-miner counts. Every honest block the nibble form
// applies after the last resolution is in the honest branch, so the branch is the honest blocks of
// [prs, pos) (plus, after an engine hand-back, the blocks the engine handed over: their per-miner counts wait
// in the lane's C_A counters, pxf). When the selfish branch wins (an honest find at w == 2) those blocks are
// stale: they are marked in a per-chunk bit mask (smask for the current chunk, SpArgs::stale for the chunks
// behind it) and counted per miner once, at the end of the run (sp_stale_counts). No per-miner state is
// touched per block, which is what lets four blocks at a time go through one table entry (sp_lut_entry).
struct SpSt {
    uint32_t F, h, w, sst;
    uint32_t prs;     // first block of the honest branch's range
    uint32_t pxf;     // the branch also holds engine-handed blocks (C_A)
    uint32_t smask;   // stale honest blocks of chunk schunk marked so far (bit i: block 32 schunk + i)
    uint32_t schunk;
    uint32_t hbits;   // honest blocks of chunk schunk the form has applied
    static constexpr int NW = 9;
    MSIM_HD void save(uint32_t *p, int st) const
    {
        const uint32_t v[NW] = {F, h, w, sst, prs, pxf, smask, schunk, hbits};
#pragma unroll
        for (int i = 0; i < NW; ++i) p[i * st] = v[i];
    }
    MSIM_HD void load(const uint32_t *p, int st)
    {
        F = p[0];
        h = p[st];
        w = p[2 * st];
        sst = p[3 * st];
        prs = p[4 * st];
        pxf = p[5 * st];
        smask = p[6 * st];
        schunk = p[7 * st];
        hbits = p[8 * st];
    }
};

// Nibble-lsb bits (bit 4i) of the nibbles of `word` equal to k.
MSIM_HD uint32_t sp_nibeq(uint32_t word, uint32_t k)
{
    const uint32_t x = word ^ (k * 0x11111111u);
    return ~(x | (x >> 1) | (x >> 2) | (x >> 3)) & 0x11111111u;
}
// Nibble-lsb bits of one half word (bits 0, 4, 8, 12) packed to bits 0..3: the four partial products of
// z * 0x1248 land on distinct bit positions (no carries), bits 12..15 holding the packed value.
MSIM_HD uint32_t sp_pack4(uint32_t z) { return (((z & 0x1111u) * 0x1248u) >> 12) & 15u; }

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

// Load the chunk of pos and the SP_PF - 1 after it (the nibble form reads a chunk per 32 blocks with the next
// ones in flight, so their latency is hidden).
MSIM_HD void sp_refill(const SpArgs &a, uint32_t r, SpCur &c)
{
#pragma unroll
    for (int i = 0; i < SP_PF; ++i) sp_chunk_at(a, r, (c.pos >> 5) + (uint32_t)i, c.A[i], c.mA[i]);
}

// Bits [lo, hi) of a chunk word (lo <= hi <= 32).
MSIM_HD uint32_t sp_bits(uint32_t lo, uint32_t hi)
{
    const uint32_t up = hi >= 32u ? 0xFFFFFFFFu : ((1u << hi) - 1u);
    return lo >= 32u ? 0u : up & ~((1u << lo) - 1u);
}

// Candidates of run r among blocks [b0, b1) (their A mask bits; the chunks loaded here: rare paths only).
MSIM_HD uint32_t sp_count_cands(const SpArgs &a, uint32_t r, uint32_t b0, uint32_t b1)
{
    uint32_t n = 0;
    for (uint32_t c = b0 >> 5; c * 32 < b1; ++c) {
        const uint32_t lo = b0 > c * 32 ? b0 - c * 32 : 0u, hi = b1 < c * 32 + 32 ? b1 - c * 32 : 32u;
        n += (uint32_t)__builtin_popcount(a.cmask[(size_t)c * a.nr + r].a & sp_bits(lo, hi));
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
    // the super-group's blocks before B, a word at a time (eight loads in flight per batch)
    const uint32_t b0 = sp_sg_block(a, c.gE);
    for (uint32_t w0 = b0 >> 3; w0 * 8 < c.B; w0 += 8) {
        uint32_t wd[8];
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) wd[q] = (w0 + q) * 8 < c.B ? a.nib[sp_nib_index(a.nr, r, w0 + q)] : 0u;
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
            const uint32_t p = (w0 + q) * 8;
            const uint32_t in = p < c.B ? sp_bits(0u, c.B - p < 8u ? c.B - p : 8u) : 0u;  // b0 is word-aligned
#pragma unroll
            for (int kk = 0; kk < M; ++kk) {
                const uint32_t z = sp_nibeq(wd[q], (uint32_t)kk);
                F[kk] += (uint32_t)__builtin_popcount((sp_pack4(z) | (sp_pack4(z >> 16) << 4)) & in);
            }
        }
    }
}


// ---------------------------------------------------------------- the settled form over nibbles

// The form moves to chunk c: the stale mask of the chunk it leaves is stored (SpArgs::stale starts zeroed, so
// chunks with no stale block, and chunks the engine consumed, are never written).
MSIM_HD void sp_to_chunk(const SpArgs &a, uint32_t r, SpSt &st, uint32_t c)
{
    if (st.schunk == c) return;
    if (st.smask) a.stale[(size_t)st.schunk * a.nr + r] = st.smask;
    st.schunk = c;
    st.smask = 0;
    st.hbits = 0;
}

// Honest blocks of [lo, 32 schunk) are stale (a selfish win whose honest branch began in an earlier chunk; rare):
// their chunks' masks, already stored, get the bits.
MSIM_HD void sp_mark_prev(const SpArgs &a, uint32_t r, const SpSt &st, uint32_t lo, uint32_t sid)
{
    for (uint32_t c = lo >> 5; c < st.schunk; ++c) {
        uint32_t w[4];
        CMask m;
        sp_chunk_at(a, r, c, w, m);
        uint32_t hb = 0;
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t z = sp_nibeq(w[j], sid);
            hb |= ((~(sp_pack4(z) | (sp_pack4(z >> 16) << 4))) & 0xFFu) << (8 * j);
        }
        hb &= sp_bits(lo > c * 32 ? lo - c * 32 : 0u, 32u);
        if (hb) a.stale[(size_t)c * a.nr + r] |= hb;
    }
}

// The honest branch's engine-handed blocks (C_A) at the first resolution after the hand-back: stale when the
// selfish branch wins (moved to C_S, out of C_F), in the best chain otherwise.
template <int M, class Env>
MSIM_HD void sp_pend_resolve(Env &env, bool swin, SpSt &st)
{
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const uint32_t v = env.get(C_A, (uint32_t)j);
        if (v) {
            if (swin) {
                env.add(C_S, (uint32_t)j, v);
                env.add(C_F, (uint32_t)j, 0u - v);
            }
            env.set(C_A, (uint32_t)j, 0u);
        }
    }
    st.pxf = 0;
}

// One block in the settled form, block by block (the paths around engine entries, hand-backs and B): a find
// by k at block `pos` of chunk st.schunk (msim_selm.h SelMacro::transition, with the branch as a range).
template <int M, class Env>
MSIM_HD void sp_blk(const SpArgs &a, uint32_t r, Env &env, SpSt &st, uint32_t pos, uint32_t k, uint32_t sid)
{
    if (k == sid) {
        st.w += 1;
        return;
    }
    st.hbits |= 1u << (pos & 31u);
    if ((st.w == 0u) | (st.w == 2u)) {
        const bool sw = st.w == 2u;
        if (sw) {  // the honest branch [prs, pos] is stale
            const uint32_t c0 = st.schunk * 32;
            if (st.prs < c0) sp_mark_prev(a, r, st, st.prs, sid);
            st.smask |= st.hbits & sp_bits(st.prs > c0 ? st.prs - c0 : 0u, (pos & 31u) + 1u);
        }
        if (st.pxf) sp_pend_resolve<M>(env, sw, st);
        st.F += st.h + (sw ? 2u : 1u);
        st.sst += sw ? 0u : st.h;
        st.h = 0;
        st.w = 0;
        st.prs = pos + 1;
    } else {
        st.h += 1;
        st.w -= 1;
    }
}

// The nibble form block by block from cur.pos to the end of its word: the word that the table path left
// (a candidate that needs the engine, B, a finder that fell through PickFinder) or the rest of a word the
// engine handed back in. Returns the lane's mode: 0 (word done: cur.pos at the next word), 1 (cur.pos is a
// candidate that needs the engine: an honest find settles iff I_next > prop_k + (w ? prop_s : 0), a candidate
// has I_next <= prop_k + prop_s, and its B bit says I_next <= prop_k), 4 (cur.pos == B, T_B < D: to the
// engine), 6 (cur.pos == B, T_B >= D: the run ends after block B - 1), 3 (error in cur.err).
template <int M, class Env>
MSIM_HD int sp_slow_word(const SpArgs &a, uint32_t r, Env &env, SpCur &cur, SpSt &st, uint32_t sid, int64_t D)
{
    while (cur.pos >= (cur.sg + 1) * a.seg) {  // segments start at chunk boundaries
        cur.Tseg += a.segsum[(size_t)cur.sg * a.nr + r];
        cur.sg++;
        cur.ci = 0;
    }
    sp_to_chunk(a, r, st, cur.pos >> 5);
    const uint32_t wi = cur.pos >> 3, p = wi << 3;
    const uint32_t word = a.nib[sp_nib_index(a.nr, r, wi)];
    const CMask m = a.cmask[(size_t)(wi >> 2) * a.nr + r];
    const uint32_t sh = 8u * (wi & 3u), mA = (m.a >> sh) & 0xFFu, mB = (m.b >> sh) & 0xFFu;
    for (uint32_t j = cur.pos & 7u; j < 8; ++j) {
        const uint32_t pj = p + j;
        if (pj >= cur.B) {
            cur.pos = cur.B;
            return (int64_t)cur.TB >= D ? 6 : 4;
        }
        const uint32_t k = (word >> (4 * j)) & 15u;
        if (k >= (uint32_t)M) {  // PickFinder fell through (simulation.h:220 asserts)
            cur.pos = pj;
            cur.err |= SERR_PICK;
            return 3;
        }
        const bool cand = ((mA >> j) & 1u) != 0u;
        if (cand & ((((mB >> j) & 1u) != 0u) | (st.w != 0u))) {
            cur.pos = pj;
            return 1;
        }
        cur.ci += cand ? 1u : 0u;  // a candidate that settles
        sp_blk<M>(a, r, env, st, pj, k, sid);
    }
    cur.pos = p + 8;
    return 0;
}

// Applies table entry e of a half word (lead class cls, selfish pattern s4) at chunk bit hoff / block hs. The
// rare parts (a selfish win whose branch began in an earlier chunk, engine-handed blocks) go through vote(b)
// (nonzero when b holds for some lane; host: b).
template <int M, class Env, class Vote>
MSIM_HD void sp_apply(const SpArgs &a, uint32_t r, Env &env, Vote vote, SpSt &st, uint32_t e, uint32_t cls, uint32_t s4,
                      uint32_t hoff, uint32_t hs, uint32_t sid)
{
    const uint32_t rs = (e >> 4) & 1u, fsw = (e >> 5) & 1u, hl = (e >> 6) & 7u;
    st.w = cls == 6u ? st.w + (e & 15u) - 4u : (e & 15u);
    st.F += (rs ? st.h : 0u) + ((e >> 9) & 15u);
    st.sst += ((rs & (fsw ^ 1u)) ? st.h : 0u) + ((e >> 13) & 7u);
    st.h = rs ? hl : st.h + hl;
    const uint32_t c0 = st.schunk * 32;
    // a selfish win first: the honest branch open before the half, [prs, hs), is stale too
    st.smask |= fsw ? st.hbits & sp_bits(st.prs > c0 ? st.prs - c0 : 0u, hoff) : 0u;
    if (vote((fsw != 0u) & (st.prs < c0))) {
        if (fsw && st.prs < c0) sp_mark_prev(a, r, st, st.prs, sid);
    }
    if (vote((rs != 0u) & (st.pxf != 0u))) {
        if (rs && st.pxf) sp_pend_resolve<M>(env, fsw != 0u, st);
    }
    st.smask |= ((e >> 16) & 15u) << hoff;
    st.hbits |= (~s4 & 15u) << hoff;
    st.prs = rs ? hs + ((e >> 24) & 7u) : st.prs;
}

// The nibble form over the rest of cur's chunk (ring slot S), a whole word at a time: the word's selfish pattern, two table
// entries (lut: SP_LUT entries, LDS on the device), and the word is applied when none of its candidates needs
// the engine, it ends before B and no finder fell through; otherwise the lane stops at the word (mode 9: the
// block-by-block path, sp_slow_word, runs it among the engine phase's lanes). At the chunk's end the next chunk
// moves up and the one after it is loaded. Returns the lane's mode (0: continue, 9: a word for the slow path).
template <int M, int S, class Env, class Vote>
MSIM_HD int sp_chunk(const SpArgs &a, uint32_t r, Env &env, Vote vote, const uint32_t *lut, SpCur &cur, SpSt &st,
                     uint32_t sid)
{
    if (cur.pos >= (cur.sg + 1) * a.seg) {  // segments start at chunk boundaries (seg is a multiple of GROUP)
        cur.Tseg += a.segsum[(size_t)cur.sg * a.nr + r];
        cur.sg++;
        cur.ci = 0;
    }
    const uint32_t c = cur.pos >> 5;
    sp_to_chunk(a, r, st, c);
    int mode = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t p = (c * 4 + j) * 8;
        if ((mode == 0) & (cur.pos == p)) {
            const uint32_t word = cur.A[S][j];
            const uint32_t z = sp_nibeq(word, sid), s8 = sp_pack4(z) | (sp_pack4(z >> 16) << 4);
            const uint32_t c0 = st.w < 6u ? st.w : 6u;
            const uint32_t e0 = lut[c0 * 16 + (s8 & 15u)];
            const uint32_t w1 = c0 == 6u ? st.w + (e0 & 15u) - 4u : (e0 & 15u);
            const uint32_t c1 = w1 < 6u ? w1 : 6u;
            const uint32_t e1 = lut[c1 * 16 + (s8 >> 4)];
            const uint32_t mA = (cur.mA[S].a >> (8 * j)) & 0xFFu, mB = (cur.mA[S].b >> (8 * j)) & 0xFFu;
            const uint32_t wnz = ((e0 >> 20) & 15u) | (((e1 >> 20) & 15u) << 4);
            const bool slow = ((mA & (mB | wnz)) != 0u) | (p + 8 > cur.B) | (sp_nibeq(word, 15u) != 0u);
            if (slow) {
                mode = 9;
            } else {
                sp_apply<M>(a, r, env, vote, st, e0, c0, s8 & 15u, 8 * j, p, sid);
                sp_apply<M>(a, r, env, vote, st, e1, c1, s8 >> 4, 8 * j + 4, p + 4, sid);
                cur.ci += (uint32_t)__builtin_popcount(mA);
                cur.pos = p + 8;
            }
        }
    }
    if ((st.h >= 0xF000u) & (mode == 0)) {  // a tie longer than the hand-over's 16-bit fields (never at 1 year)
        cur.err |= SERR_SP;
        mode = 3;
    }
    if (mode == 0) sp_chunk_at(a, r, c + SP_PF, cur.A[S], cur.mA[S]);
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
// engine (msim_selm.h to_exact) with the honest branch's composition counted from the nibbles of [prs, pos) and
// the engine-handed blocks (C_A). Returns the new mode (2: engine, 3: error in cur.err). src: SpSrc.
template <int M, class Src, class SelT, class Env>
MSIM_HD int sp_enter(const SpArgs &a, uint32_t r, int mode, SpCur &cur, SpSt &st, Src &src, SelT &s, Env &env,
                     uint32_t m, const uint32_t *sids)
{
    const uint32_t sid = sids[0];
    SelMacro<M> mc;
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
        uint32_t I = gr.w0 >> 5, k = gr.w0 & 31u;  // the super-group's first block
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
    // the settled state, its honest branch as per-miner counts
    mc.F = st.F;
    mc.h = st.h;
    mc.w = st.w;
    mc.sst = st.sst;
    mc.Ff = st.F;
#pragma unroll
    for (int i = 0; i < SelMacro<M>::NP; ++i) mc.pend[i] = mc.stp[i] = 0;
    if (st.pxf) {
#pragma unroll
        for (int j = 0; j < M; ++j)
            if ((uint32_t)j != sid) SelMacro<M>::field_add(mc.pend, SelMacro<M>::slot((uint32_t)j, sid), env.get(C_A, (uint32_t)j));
    }
    // the honest blocks of [prs, pos), a word at a time (the words' loads issued together)
    for (uint32_t w0 = st.prs >> 3; w0 * 8 < cur.pos; w0 += 4) {
        uint32_t wd[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) wd[q] = (w0 + q) * 8 < cur.pos ? a.nib[sp_nib_index(a.nr, r, w0 + q)] : 0u;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t p = (w0 + q) * 8;
            if (p >= cur.pos) continue;
            const uint32_t lo = st.prs > p ? st.prs - p : 0u, hi = cur.pos - p < 8u ? cur.pos - p : 8u;
            const uint32_t in = sp_bits(lo, hi);  // blocks of the word inside the range
#pragma unroll
            for (int j = 0; j < M; ++j) {
                if ((uint32_t)j == sid) continue;
                const uint32_t z = sp_nibeq(wd[q], (uint32_t)j);
                const uint32_t n = (uint32_t)__builtin_popcount((sp_pack4(z) | (sp_pack4(z >> 16) << 4)) & in);
                if (n) SelMacro<M>::field_add(mc.pend, SelMacro<M>::slot((uint32_t)j, sid), n);
            }
        }
    }
    st.sst = 0;
    mc.to_exact(env, s, m, sids);
    return 2;
}

// The engine hands the run back to the nibble form at block pidx (msim_selm.h take_back gave tb): the fork's
// honest branch composition waits in C_A (take_back left the deep counters zero) and the range restarts at pidx.
template <int M, class Env>
MSIM_HD void sp_handback(Env &env, const SelMacro<M> &tb, SpSt &st, uint32_t pidx, uint32_t sid)
{
    st.F = tb.F;
    st.h = tb.h;
    st.w = tb.w;
    st.sst = tb.sst;
    uint32_t any = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const uint32_t v = (uint32_t)j == sid ? 0u : tb.pend_of((uint32_t)j, sid);
        env.set(C_A, (uint32_t)j, v);
        any |= v;
    }
    st.pxf = any ? 1u : 0u;
    st.prs = pidx;
}

// main.cpp:185-189 from a settled state (msim_selm.h SelMacro::finish): the honest branch is the best chain
// (first seen), the selfish tie and withheld blocks are not in it.
template <int M, class Env>
MSIM_HD void sp_finish(Env &env, const SpSt &st, uint32_t sid, SelOut &out)
{
    if (st.sst) {
        env.add(C_S, sid, st.sst);
        env.add(C_F, sid, 0u - st.sst);
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {
        out.found[j] = env.get(C_F, (uint32_t)j) - ((uint32_t)j == sid ? st.h + st.w : 0u);
        out.stale[j] = env.get(C_S, (uint32_t)j);
    }
    out.best_height = st.F + st.h;
    out.err = 0;
}

// The run's honest stale blocks of the nibble form, per miner: the stale masks of chunks [0, st.schunk) from
// SpArgs::stale and st.smask for the current chunk, against the chunks' finder nibbles (end of the run).
// Eight chunks' loads in flight per batch (it runs once per run, at its end).
template <int M>
MSIM_HD void sp_stale_counts(const SpArgs &a, uint32_t r, const SpSt &st, uint32_t sid, uint32_t (&cnt)[M])
{
#pragma unroll
    for (int j = 0; j < M; ++j) cnt[j] = 0;
    for (uint32_t c0 = 0; c0 <= st.schunk; c0 += 8) {
        uint32_t sm[8];
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            const uint32_t c = c0 + i;
            sm[i] = c < st.schunk ? a.stale[(size_t)c * a.nr + r] : (c == st.schunk ? st.smask : 0u);
        }
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            if (!sm[i]) continue;
            uint32_t w[4];
            CMask m;
            sp_chunk_at(a, r, c0 + i, w, m);
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                const uint32_t b8 = (sm[i] >> (8 * q)) & 0xFFu;
#pragma unroll
                for (int j = 0; j < M; ++j) {
                    if ((uint32_t)j == sid) continue;
                    const uint32_t z = sp_nibeq(w[q], (uint32_t)j);
                    cnt[j] += (uint32_t)__builtin_popcount((sp_pack4(z) | (sp_pack4(z >> 16) << 4)) & b8);
                }
            }
        }
    }
}

// The engine phase (msim_sel.h step until the run is over or the engine hands it back below B, msim_selm.h
// take_back) is written inline in the kernel (msim_sel_kernels.hip msim_selpipe_kernel, and the host driver in
// tests/native/selpipe_host.cpp): as a helper taking the finish record and the taken-back state by reference,
// both stayed live across the engine step and the engine loop spilled ~3x more.

}  // namespace msim
