// msim_pipeline.h — the event-skipping pipeline for honest networks.
//
// RunSimulation (/root/reference/main.cpp:128-192) spends almost every event in one state: all
// chains identical and published ("quiet"). From a quiet state, a block i found at T_i by an honest
// miner k whose successor comes later than its arrival (I_{i+1} > prop_k) is adopted by everyone at
// T_i + prop_k and leaves the network quiet again — a "fast" block. Everything else is an EPISODE,
// a pure function of the draws from its first block on (translation-invariant in time apart from the
// end of the run). So one run is computed as
//
//   K1 msim_draws_kernel    (run, segment) workers, jump-ahead to draw j*SEG, draw every block
//                           (interval, finder, fast bit), keep per-segment time and per-owner counts,
//                           and append every non-fast block to a dense episode list together with both
//                           RNG states there; nothing is stored per block (the band where a run can end
//                           keeps per-group sums, counts and the RNG states at each group start);
//   K2 msim_episode_kernel  one lane per listed block: the full state machine (msim_model.h) from a
//                           quiet state at that block, until quiet again or the end of the run;
//   K3 msim_combine_kernel  one lane per run: locate the end of the run (first T_i >= D), chain the
//                           episodes that start from a quiet state, and combine
//                              found_k = #{i < n_end : finder_i = k} + sum(episode deltas)
//                           stale_k = sum(episode stale counts).
// Runs that hit any capacity (draw budget, slots, list) are flagged and recomputed by the per-lane
// retry kernel, so results never depend on these capacities.
#pragma once
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "msim_fastdraw.h"
#include "msim_model.h"

namespace msim {

// K2's state machine comes in three sizes (KIND). Lean (0: networks with rho <= K2_LEAN_RHO): 2 extra in-flight
// blocks and no deep-branch counters; at rho <= 0.002 an episode that needs more is < 1e-3 of the runs of a
// 12-month simulation; configs[1] (rho = 1.7e-4): K2 125 -> 77 us per launch (no spills instead of 134 VGPR
// spills; profiles/r04/k2v). Mid (1: every other pipeline network, rho <= PIPE_MAX_RHO): 4 extra blocks, no
// deep branches — a fork deeper than the 16-height window needs 16 finds inside one propagation delay, which
// no network the pipeline takes (delays up to ~50 s) makes in practice, and an episode that would is flagged
// and its run recomputed by the retry kernel. Full (2): deep branches too (kept for A/B builds).
// An episode that outgrows its capacities flags its run for the retry kernel: results never depend on them.
constexpr double K2_LEAN_RHO = 0.002;
#ifndef MSIM_K2_KIND_HI
#define MSIM_K2_KIND_HI 1  // K2 above K2_LEAN_RHO: 1 mid, 2 full (A/B builds)
#endif
constexpr uint32_t K2_KIND_HI = MSIM_K2_KIND_HI;
constexpr uint32_t GROUP = 32;          // blocks per group (end-of-run search metadata)
constexpr uint32_t SGROUP = 8;          // groups per super-group (K3 searches super-group ends, then groups)
constexpr uint32_t MIN_SEG = 512;       // shortest K1 worker (keeps the jump-ahead cost < 5 %)
constexpr uint32_t CNT_WORDS = 8;       // per-owner counters packed as u16 pairs (<= 16 owners)
#ifndef MSIM_K1_QB
#define MSIM_K1_QB 4  // blocks drawn together by K1 (one exactness branch per batch)
#endif
constexpr int K1_QB = MSIM_K1_QB;

constexpr uint32_t EP_HOLE = 0xFFFFFFFFu;  // EpEntry::run of a list slot K1 reserved but did not use

struct EpEntry {
    uint32_t run;     // slice-local run (EP_HOLE: an unused slot of a wave's reserved chunk)
    uint32_t block;   // block index within the run
    uint64_t offset;  // T_block - (start time of its segment), ms
    uint32_t w0, w1;  // (interval << 5 | finder) of the block and of the next one
    uint32_t skip;    // draws from ri / rp's position to the block after w1 (1-4)
    uint32_t pad;
    Rng ri, rp;       // both streams at the start of K1's quad of w1's block: `skip` draws before the block after w1
};

// A group of the band (where a run can end): the first block's word and both streams after it.
struct GroupRec {
    Rng ri, rp;
    uint32_t w0;
    uint32_t pad;
};

struct PipeLayout {
    uint32_t nr;       // runs in a slice (multiple of 256)
    uint32_t seg;      // blocks per K1 worker (multiple of GROUP)
    uint32_t gps;      // groups per segment (seg / GROUP)
    uint32_t nsg;      // super-groups per segment (ceil(gps / SGROUP))
    uint32_t nseg;     // segments (K1 workers) per run
    uint32_t nb;       // nseg * seg pre-generated blocks per run
    uint32_t cap;      // slow-block slots per (run, segment)
    uint32_t band_lo;  // first segment with group metadata (where the run can end)
    uint32_t nband;
    uint32_t lcap;     // episode list capacity
    uint32_t lchunk;   // list slots a K1 wave reserves at a time (one atomic per chunk, not per append)
    uint32_t rec_words;
    uint32_t k2_kind;  // K2's state machine: 0 lean (rho <= K2_LEAN_RHO), 1 mid, 2 full (msim_kernels.hip)
    size_t segsum_off, segcnt_off, nslow_off, slots_off, gsum_off, gend_off, gcum_off, grec_off, list_off, recs_off,
        count_off, total;
};

// Device tables (per config, per device): pick table, log table, jump matrices.
struct PipeTables {
    const PickTab *pick;
    const LogTab *logt;
    const uint32_t *jump;  // nseg * 128 columns of 4 words
};

struct DrawArgs {
    PipeTables tab;
    uint64_t run_begin;   // absolute index of the slice's first run
    uint32_t n;           // valid runs in the slice
    uint32_t seed_base;
    uint32_t nr, seg, gps, nseg, cap, band_lo, lcap, lchunk;
    uint64_t *segsum;     // [nseg][nr]
    uint32_t *segcnt;     // [nseg][8][nr]
    uint32_t *nslow;      // [nseg][nr]
    uint32_t *slots;      // [nseg][cap][nr]
    uint32_t *gsum;       // [nband][gps][nr]
    uint64_t *gend;       // [nband][nsg][nr]: time from the segment's start to the end of each super-group
    uint32_t *gcum;       // [nband][gps][8][nr]
    GroupRec *grec;       // [nband][gps][nr]
    EpEntry *list;        // [lcap]
    uint32_t *list_count;
};

struct PipeArgs {  // K2 / K3
    uint32_t nr, seg, gps, nseg, nb, cap, band_lo, lcap, rec_words;
    PipeTables tab;       // K2 / K3 redraw blocks from stored RNG states
    const uint64_t *segsum;
    const uint32_t *segcnt;
    const uint32_t *nslow;
    const uint32_t *slots;
    const uint32_t *gsum;
    const uint64_t *gend;
    const uint32_t *gcum;
    const GroupRec *grec;
    const EpEntry *list;
    const uint32_t *list_count;
    uint32_t *recs;       // [lcap][rec_words]: end, flags, F[M], S[M], first block
};

enum : uint32_t { REC_ENDED = 1u, REC_ERR = 2u, REC_SKIP = 4u };

// ---------------------------------------------------------------- sizing (host)
// Every capacity has a >= 8-sigma margin; a run that exceeds one anyway is recomputed by the retry
// kernel, so the sizes only affect speed, never results. rho = P(block is not fast).
// `slots` = wave slots of K1 on the device (CUs x resident waves per CU). The run is cut into `nseg`
// workers of `seg` blocks so that the K1 grid fills the device in whole rounds: every wave does the
// same work, so a partial last round would leave SIMDs idle.
// The layout of a slice of exactly nr runs (a multiple of 256): K2's episode records, band records per group.
inline PipeLayout pipe_layout_nr(double rho, uint32_t m, int64_t duration_ms, uint32_t nr, uint32_t slots)
{
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    PipeLayout L;
    const double D = (double)duration_ms;
    const double mu = D / 599999.5, sd = sqrt(mu > 1.0 ? mu : 1.0);
    const double need = mu + 8.0 * sd + 64.0;  // blocks to pre-generate (P(more) < 1e-15 per run)
    L.rec_words = 3 + 2 * m;
    L.k2_kind = rho <= K2_LEAN_RHO ? 0u : K2_KIND_HI;
    L.nr = nr;
    // workers per run: minimise rounds(w) * (seg(w) + jump cost), jump ~ 25 blocks of work
    const double rows = L.nr / 64.0;
    if (slots < 1) slots = 1;
    uint32_t best_w = 1;
    double best_f = 1e300;
    for (uint32_t w = 1; w <= 256; ++w) {
        const uint32_t sg = (uint32_t)ceil(need / w / GROUP) * GROUP;
        if (sg < MIN_SEG && w > 1) break;
        const double rounds = ceil(rows * w / slots);
        const double f = rounds * (sg + 25.0);
        if (f < best_f * 0.999) {
            best_f = f;
            best_w = w;
        }
    }
    L.nseg = best_w;
    L.seg = (uint32_t)ceil(need / best_w / GROUP) * GROUP;
    if (L.seg < GROUP) L.seg = GROUP;
    L.gps = L.seg / GROUP;
    L.nsg = (L.gps + SGROUP - 1) / SGROUP;
    L.nb = L.nseg * L.seg;
    const double lo = mu - 8.0 * sd - 64.0;
    L.band_lo = lo > 0 ? (uint32_t)floor(lo / L.seg) : 0u;
    if (L.band_lo >= L.nseg) L.band_lo = L.nseg - 1;
    L.nband = L.nseg - L.band_lo;
    const double lam = rho * L.seg;
    L.cap = (uint32_t)ceil(lam + 8.0 * sqrt(lam) + 8.0);
    const double ent = (double)L.nr * rho * L.nb;
    // A K1 wave reserves list slots a chunk at a time: one same-address atomic per chunk instead of one per
    // append (at rho = 1.7 % — configs[0] — the per-append atomics serialised K1 to 30x its draw time). The
    // chunk follows a wave's expected appends; its unused tail (< lchunk slots per wave) is marked EP_HOLE.
    const double per_wave = 64.0 * rho * L.seg;
    L.lchunk = 16;
    while (L.lchunk < 256 && L.lchunk < per_wave / 4.0) L.lchunk *= 2;
    const double holes = (double)(L.nr / 64) * L.nseg * L.lchunk;
    L.lcap = (uint32_t)ceil(ent + 8.0 * sqrt(ent) + 1024.0 + holes);
    size_t o = 0;
    L.segsum_off = o;
    o = al(o + (size_t)L.nseg * L.nr * 8);
    L.segcnt_off = o;
    o = al(o + (size_t)L.nseg * CNT_WORDS * L.nr * 4);
    L.nslow_off = o;
    o = al(o + (size_t)L.nseg * L.nr * 4);
    L.slots_off = o;
    o = al(o + (size_t)L.nseg * L.cap * L.nr * 4);
    const size_t grp = L.gps;  // band records per segment
    L.gsum_off = o;
    o = al(o + (size_t)L.nband * L.gps * L.nr * 4);
    L.gend_off = o;
    o = al(o + (size_t)L.nband * L.nsg * L.nr * 8);
    L.gcum_off = o;
    o = al(o + (size_t)L.nband * grp * CNT_WORDS * L.nr * 4);
    L.grec_off = o;
    o = al(o + (size_t)L.nband * grp * L.nr * sizeof(GroupRec));
    L.list_off = o;
    o = al(o + (size_t)L.lcap * sizeof(EpEntry));
    L.recs_off = o;
    o = al(o + (size_t)L.lcap * L.rec_words * 4);
    L.count_off = o;
    o = al(o + 4);
    L.total = o;
    return L;
}

// The largest slice (all n_runs, or fewer) whose layout, plus extra_per_run bytes per run, fits the budget.
inline PipeLayout pipe_layout_for(double rho, uint32_t m, int64_t duration_ms, uint64_t n_runs, double budget,
                                  uint32_t slots, double extra_per_run = 0.0)
{
    uint64_t nr = (n_runs + 255) / 256 * 256;
    for (;;) {
        const PipeLayout L = pipe_layout_nr(rho, m, duration_ms, (uint32_t)nr, slots);
        const double tot = (double)L.total + extra_per_run * (double)nr;
        if (tot <= budget || nr <= 256) return L;
        uint64_t next = (uint64_t)((double)nr * budget / tot * 0.98) / 256 * 256;
        if (next >= nr) next = nr - 256;
        nr = next < 256 ? 256 : next;
    }
}

// ---------------------------------------------------------------- K1 lane body (shared host/device)
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __noinline__ int32_t interval_ms_exact_dev(uint64_t u);
#endif

MSIM_HD uint32_t draw_interval(Rng &ri, const LogTab *__restrict__ lt, FdConsts kc = MSIM_FD_DEFAULT)
{
    const uint64_t u = rng_next(ri);
    bool ok;
    const int32_t q = interval_ms_fast(u, lt, ok, kc);
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)(ok ? q : interval_ms_exact_dev(u));
#else
    return (uint32_t)(ok ? q : (int32_t)interval_ms_of(u));
#endif
}

// Both draws of one block as a word: interval << 5 | finder (pick_info's low nibble).
MSIM_HD uint32_t draw_word(Rng &ri, Rng &rp, const LogTab *__restrict__ lt, const PickTab *__restrict__ pt)
{
    const uint32_t I = draw_interval(ri, lt);
    return (I << 5) | info_finder(pick_info(rng_next(rp), pt));
}

// Episode draw source (K2): the stored words of its first two blocks, then the streams redrawn.
struct EpSrc {
    const LogTab *lt;
    const PickTab *pt;
    Rng ri, rp;
    uint32_t nb, index, cur, nxt;
    bool have_nxt;
    MSIM_HD uint32_t word() const { return cur; }
    MSIM_HD bool advance()
    {
        if (index + 1 >= nb) return false;  // past the pre-generated budget: the run is retried
        ++index;
        if (have_nxt) {
            cur = nxt;
            have_nxt = false;
        } else {
            cur = draw_word(ri, rp, lt, pt);
        }
        return true;
    }
};

// The draws of four consecutive blocks, each by its fast path, with their exactness checks folded into
// one flag; the rare quad that needs an exact path (an interval within 1 ns of a millisecond boundary,
// or a PickFinder index the high word cannot settle: ~8e-6 of quads) is redrawn by draw_quad_exact from
// the streams at its start. Batching four draws lets their table reads be in flight together.
MSIM_HD bool draw_quad_fast(Rng &ri, Rng &rp, const LogTab *__restrict__ lt, const PickTab *__restrict__ pt,
                            FdConsts kc, uint32_t (&I)[K1_QB], uint32_t (&info)[K1_QB])
{
    uint32_t ki = 0, kp = 0;  // largest acceptance keys of the quad
#pragma unroll
    for (int q = 0; q < K1_QB; ++q) {
        const uint64_t ui = rng_next(ri), up = rng_next(rp);
        uint32_t a, b;
        I[q] = (uint32_t)interval_ms_fast_key(ui, lt, a, kc);
        info[q] = pt->info[pick_q_fast_key(up, b)];
        ki = a > ki ? a : ki;
        kp = b > kp ? b : kp;
    }
    return ki >= FD_OK_RANGE || kp >= PICK_RARE_LO;
}
MSIM_HD void draw_quad_exact(Rng ri, Rng rp, const LogTab *__restrict__ lt, const PickTab *__restrict__ pt,
                             uint32_t (&I)[K1_QB], uint32_t (&info)[K1_QB])
{
#pragma unroll
    for (int q = 0; q < K1_QB; ++q) {
        I[q] = draw_interval(ri, lt);  // the exact glibc sequence stays out of line (interval_ms_exact_dev)
        info[q] = pt->info[pick_q_exact(rng_next(rp))];
    }
}

// One (run, segment) worker: SEG blocks from the jumped RNG states. Ctx supplies the side effects:
//   count(info)                       per-owner counter of this lane (+1 for owner info_finder(info))
//   vote(s)                           nonzero when s holds for some active lane of the wave (host: s)
//   slow(s, block, offset, w0, w1, ri, rp, skip)
//                                     called after a nonzero vote: records a non-fast block when s
//                                     (offset = its find time minus the segment's start; its word, the
//                                     next one; both streams at the quad's start, `skip` draws before the
//                                     block after the next one: the consumer steps them, not the wave)
//   group(g, sum, end)                band only: sum of the group's intervals, and the time from the segment's
//                                     start to the group's end
//   quad()                            start of a quad of blocks
//   group_start(g, w0, ri, rp)        band only: before group g's first block (its word and the streams
//                                     after it; snapshot the counters)
// Blocks are drawn four at a time (draw_quad_fast); the streams after a block inside a quad, needed only
// by the rare non-fast block, are re-stepped from the quad's start. Time is summed per group in 32 bits
// (32 intervals < 2^25 ms each) and folded into 64 bits per group.
template <class Ctx>
MSIM_HD uint64_t draw_segment(Ctx &cx, Rng &ri, Rng &rp, const LogTab *__restrict__ lt,
                              const PickTab *__restrict__ pt, uint32_t b0, uint32_t seg, bool band)
{
#if defined(__HIP_DEVICE_COMPILE__)
    FdConsts kc{FD_C1, FD_C2, FD_C3, FD_C4, FD_C5};  // all five in SGPRs; c5 reaches a VGPR per quad (below)
    asm("" : "+s"(kc.c1));
    asm("" : "+s"(kc.c2));
    asm("" : "+s"(kc.c3));
    asm("" : "+s"(kc.c4));
    asm("" : "+s"(kc.c5));
#else
    const FdConsts kc = fd_consts();
#endif
    uint32_t Icur = draw_interval(ri, lt, kc);
    uint32_t infocur = pick_info(rng_next(rp), pt);
    uint64_t tsum = 0;
    for (uint32_t g = 0; g < seg / GROUP; ++g) {
        if (band) cx.group_start(g, (Icur << 5) | info_finder(infocur), ri, rp);
        uint32_t gacc = 0;
        for (uint32_t q4 = 0; q4 < GROUP / K1_QB; ++q4) {
            uint32_t I[K1_QB], info[K1_QB];
            cx.quad();  // per-quad values the context rebuilds rather than holding across the loop
#if defined(__HIP_DEVICE_COMPILE__)
            // the polynomial's leading coefficient, a VGPR operand (one VOP3 reads at most one SGPR), copied
            // from its SGPR each quad (one v_mov_b64) instead of being held across the loop, where the register
            // budget of K1 sent it to scratch
            FdConsts kq = kc;
            asm volatile("v_mov_b64 %0, %1" : "=v"(kq.c5) : "s"(kc.c5));
#else
            const FdConsts kq = kc;
#endif
            // The quad's start states are read only on the two rare paths below; at K1's register budget (96
            // VGPRs at 5 waves per SIMD, msim_drawgen.hip) the compiler keeps them in scratch, written once per quad.
            // Measured on MI355X: recovering them by inverse stepping instead (no scratch, 84 VGPRs) made K1
            // 11 % slower at the same occupancy (profiles/r03/INDEX.md, k1 A/B).
            const Rng ri0 = ri, rp0 = rp;
            if (draw_quad_fast(ri, rp, lt, pt, kq, I, info)) draw_quad_exact(ri0, rp0, lt, pt, I, info);
#pragma unroll
            for (int q = 0; q < K1_QB; ++q) {
                gacc += Icur;
                const bool slow = I[q] <= info_fthr(infocur);  // I_{i+1} vs the finder's delay
                cx.count(infocur);
                if (cx.vote(slow))  // the streams after block i+1 are the quad's start + q + 1 draws (K2 steps them)
                    cx.slow(slow, b0 + g * GROUP + q4 * K1_QB + (uint32_t)q, tsum + gacc, (Icur << 5) | info_finder(infocur),
                            (I[q] << 5) | info_finder(info[q]), ri0, rp0, (uint32_t)q + 1u);
                Icur = I[q];
                infocur = info[q];
            }
        }
        if (band) cx.group(g, gacc, tsum + gacc);
        tsum += gacc;
    }
    return tsum;
}

// ---------------------------------------------------------------- K3 lane body (shared host/device)
// Adds the M owner counters of a packed row; returns PickFinder's fall-through count (owner 15).
template <int M>
MSIM_HD uint32_t add_packed(uint32_t (&F)[M], const uint32_t *__restrict__ src, size_t stride)
{
#pragma unroll
    for (int w = 0; w < (M + 1) / 2; ++w) {
        const uint32_t c = src[(size_t)w * stride];
        F[2 * w] += c & 0xFFFFu;
        if (2 * w + 1 < M) F[2 * w + 1] += c >> 16;
    }
    return src[(size_t)(CNT_WORDS - 1) * stride] >> 16;
}

// K3 phase timing (diagnostic builds only, -DK3_PROF=1: scripts/build_variant.sh): clock at each phase of
// combine_run for the first lane of a few workgroups.
#if defined(__HIP_DEVICE_COMPILE__) && defined(K3_PROF) && K3_PROF
#define K3T(i) k3t[i] = clock64()
#define K3T_DECL uint64_t k3t[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}; K3T(0)
#define K3T_PRINT                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x % 16 == 0)                                                               \
        printf("K3PROF blk %u seg %llu cnt %llu idxhdr %llu groups %llu chain %llu redraw %llu prevgrp %llu eps %llu\n", \
               blockIdx.x, (unsigned long long)(k3t[1] - k3t[0]), (unsigned long long)(k3t[2] - k3t[1]),       \
               (unsigned long long)(k3t[3] - k3t[2]), (unsigned long long)(k3t[4] - k3t[3]),                    \
               (unsigned long long)(k3t[5] - k3t[4]), (unsigned long long)(k3t[6] - k3t[5]),                    \
               (unsigned long long)(k3t[7] - k3t[6]), (unsigned long long)(k3t[8] - k3t[7]))
#else
#define K3T(i)
#define K3T_DECL
#define K3T_PRINT
#endif

// Combine one run r of a slice. Returns false when the run must be recomputed by the retry path.
// nsw: K3_SCRATCH words of per-run scratch at stride nss (device: the lane's LDS column): the list counts of
// the run's segments (later the first blocks of the candidate episodes), the candidates' record indices, and
// their (end << 2 | ended << 1 | unusable) words.
//
// K3 is latency-bound (one lane per run, a fraction of a wave per SIMD): its time is set by its dependent
// memory rounds and by single-wave instruction latency. The reads are ordered so that independent ones share a
// round and the episode reads stay in flight behind the end-of-run search: (1) segment sums; (2) list counts +
// per-owner counts; (3) slot indices; (4) episode headers + super-group ends; (5) group sums; (6) the end
// group's records + the first candidates' deltas, which land while the end group is redrawn. The episode
// chain is built from the headers without the end block (the episodes are in block order, so the end only
// truncates it) and cut once the redraw found it.
#ifndef MSIM_K3_EP_MAX
#define MSIM_K3_EP_MAX 32  // 24: 76.8 us, 16: 99.1 us vs 67.7 us per c2 launch (more runs on the one-read-at-a-time path)
#endif
constexpr uint32_t K3_SEG_MAX = 32, K3_EP_MAX = MSIM_K3_EP_MAX, K3_SCRATCH = K3_SEG_MAX + 2 * K3_EP_MAX;
// combine_run keeps its candidate starts in the segment-count rows (nsw[na * nss], na < K3_EP_MAX): a larger
// K3_EP_MAX would overwrite the record indices at rows K3_SEG_MAX + t before they are read
static_assert(K3_EP_MAX <= K3_SEG_MAX, "MSIM_K3_EP_MAX must not exceed K3_SEG_MAX");
template <int M>
MSIM_HD bool combine_run(const SimParams &p, const PipeArgs &a, uint32_t r, uint32_t (&F)[M], uint32_t (&S)[M],
                         uint32_t *nsw, size_t nss)
{
    const int64_t D = p.duration_ms;
    K3T_DECL;
#pragma unroll
    for (int k = 0; k < M; ++k) {
        F[k] = 0;
        S[k] = 0;
    }
    // 1. Segment containing the end of the run: the first whose last block is found at >= D. The sums are
    // loaded KB at a time (independent loads in flight together), then scanned.
    constexpr uint32_t KB = 16;
    int64_t T = 0;
    int e = -1;
    for (uint32_t j0 = 0; j0 < a.nseg && e < 0; j0 += KB) {
        uint64_t ss[KB];
#pragma unroll
        for (uint32_t j = 0; j < KB; ++j) {  // unconditional (clamped) loads: all KB in flight together
            const uint32_t jj = j0 + j < a.nseg ? j0 + j : a.nseg - 1;
            ss[j] = a.segsum[(size_t)jj * a.nr + r];
        }
#pragma unroll
        for (uint32_t j = 0; j < KB; ++j) {
            if (e < 0 && j0 + j < a.nseg) {
                if (T + (int64_t)ss[j] >= D) e = (int)(j0 + j);
                else T += (int64_t)ss[j];
            }
        }
    }
    K3T(1);
    if (e < (int)a.band_lo) return false;  // past the pre-generated draws or outside the band
    constexpr uint32_t EP_MAX = K3_EP_MAX, SEG_MAX = K3_SEG_MAX;
    const bool fits = (uint32_t)e < SEG_MAX;
    // 2. List counts of segments 0..e (issued first) and per-owner counts of the segments before e, in one
    // round (no early exit between them: a fall-through in any segment is checked once at the end).
    uint32_t nsv[SEG_MAX];
    if (fits) {
#pragma unroll
        for (uint32_t j = 0; j < SEG_MAX; ++j) nsv[j] = a.nslow[(size_t)(j <= (uint32_t)e ? j : (uint32_t)e) * a.nr + r];
    }
    {
        uint32_t ft = 0;
        for (int j0 = 0; j0 < e; j0 += (int)KB) {
            uint32_t c[KB][CNT_WORDS];
#pragma unroll
            for (uint32_t j = 0; j < KB; ++j) {
                const int jj = j0 + (int)j < e ? j0 + (int)j : e - 1;  // clamped: unconditional loads, masked below
#pragma unroll
                for (uint32_t w = 0; w < CNT_WORDS; ++w) {
                    const uint32_t v = (w < (uint32_t)(M + 1) / 2 || w == CNT_WORDS - 1)
                                           ? a.segcnt[((size_t)jj * CNT_WORDS + w) * a.nr + r]
                                           : 0u;
                    c[j][w] = j0 + (int)j < e ? v : 0u;
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < KB; ++j) {
#pragma unroll
                for (int w = 0; w < (M + 1) / 2; ++w) {
                    F[2 * w] += c[j][w] & 0xFFFFu;
                    if (2 * w + 1 < M) F[2 * w + 1] += c[j][w] >> 16;
                }
                ft |= c[j][CNT_WORDS - 1] >> 16;
            }
        }
        if (ft) return false;  // PickFinder fell through (owner 15): the retry kernel reports it
    }
    uint32_t tot = 0;
    if (fits) {
#pragma unroll
        for (uint32_t j = 0; j < SEG_MAX; ++j) {
            const uint32_t v = j <= (uint32_t)e ? nsv[j] : 0u;
            if (v > a.cap) return false;
            tot += v;
            nsw[j * nss] = v;  // read back below at data-dependent positions
        }
    }
    K3T(2);
    // 3. The run's episodes in block order (segments 0..e): record indices, then headers. The header loads
    // are not waited for here: they stay in flight through the group search.
    const bool batched = fits && tot <= EP_MAX;
    uint32_t st[EP_MAX], en[EP_MAX], fl[EP_MAX];
    bool bad_idx = false;
    if (batched) {
        // entry t -> (segment, slot): a walk over the counts in LDS, no memory reads; then every slot index and
        // every header is loaded without a branch (entries past tot read slot 0 / record 0 and are masked), so
        // no load waits behind a divergent block for the ones issued before it
        uint32_t pos[EP_MAX];
        {
            uint32_t j = 0, c = 0, nj = nsw[0];  // (segment, slot) of entry t; nj = count of segment j
#pragma unroll
            for (uint32_t t = 0; t < EP_MAX; ++t) {
                uint32_t v = 0;
                if (t < tot) {
                    while (c >= nj) {
                        ++j;
                        c = 0;
                        nj = nsw[j * nss];
                    }
                    v = j * a.cap + c;
                    ++c;
                }
                pos[t] = v;
            }
        }
        uint32_t idx[EP_MAX];
#pragma unroll
        for (uint32_t t = 0; t < EP_MAX; ++t) idx[t] = a.slots[(size_t)pos[t] * a.nr + r];
#pragma unroll
        for (uint32_t t = 0; t < EP_MAX; ++t) {
            const bool in = t < tot;
            bad_idx |= in && idx[t] >= a.lcap;
            const uint32_t i = in && idx[t] < a.lcap ? idx[t] : 0u;
            const uint32_t *rec = a.recs + (size_t)i * a.rec_words;
            st[t] = rec[2 + 2 * M];  // the episode's first block (K2 copies it from the list entry)
            en[t] = rec[0];
            fl[t] = rec[1];
            nsw[(SEG_MAX + t) * nss] = i;
        }
    }
    K3T(3);
    // 4. Group, then block, where T first reaches D: n_end = #{i : T_i < D} (main.cpp:150,153). Two rounds: the
    // ends of the segment's super-groups (time from the segment's start, KS at a time), then the SGROUP group
    // sums of the super-group that reaches D.
    const size_t gb = (size_t)(e - (int)a.band_lo) * a.gps;
    const uint32_t nsg = (a.gps + SGROUP - 1) / SGROUP;
    const size_t sb = (size_t)(e - (int)a.band_lo) * nsg;
    constexpr uint32_t KS = 24;
    uint32_t sg = nsg;
    uint64_t base = 0;  // time from the segment's start to the start of super-group sg
    for (uint32_t s0 = 0; s0 < nsg && sg == nsg; s0 += KS) {
        uint64_t ps[KS];
#pragma unroll
        for (uint32_t j = 0; j < KS; ++j) ps[j] = a.gend[(sb + (s0 + j < nsg ? s0 + j : nsg - 1)) * a.nr + r];
#pragma unroll
        for (uint32_t j = 0; j < KS; ++j) {
            if (sg == nsg && s0 + j < nsg) {
                if (T + (int64_t)ps[j] >= D) sg = s0 + j;
                else base = ps[j];
            }
        }
    }
    if (sg == nsg) return false;
    T += (int64_t)base;
    uint32_t G = a.gps;
    {
        const uint32_t g0 = sg * SGROUP;
        uint32_t gs[SGROUP];
#pragma unroll
        for (uint32_t g = 0; g < SGROUP; ++g) gs[g] = a.gsum[(gb + (g0 + g < a.gps ? g0 + g : a.gps - 1)) * a.nr + r];
#pragma unroll
        for (uint32_t g = 0; g < SGROUP; ++g) {
            if (G == a.gps && g0 + g < a.gps) {
                if (T + (int64_t)gs[g] >= D) G = g0 + g;
                else T += (int64_t)gs[g];
            }
        }
    }
    if (G == a.gps || bad_idx) return false;
    K3T(4);
    // 5. The end group's stream record and counters are issued, then the candidate chain is built from the
    // headers (an episode is a candidate when its first block is reached quiet, ignoring the end of the run),
    // then the first APPLY_B candidates' deltas are issued; the group redraw waits for the stream record only.
    const GroupRec gr = a.grec[(gb + G) * a.nr + r];
    uint32_t gc[CNT_WORDS];
#pragma unroll
    for (uint32_t w = 0; w < CNT_WORDS; ++w)
        gc[w] = (w < (uint32_t)(M + 1) / 2 || w == CNT_WORDS - 1) ? a.gcum[((gb + G) * CNT_WORDS + w) * a.nr + r] : 0u;
    constexpr uint32_t APPLY_B = 8;
    uint32_t na = 0;
    uint32_t d[APPLY_B][2 * M];
    if (batched) {
        uint32_t cursor = 0;
        bool stop = false;
#pragma unroll
        for (uint32_t t = 0; t < EP_MAX; ++t) {
            if (stop || t >= tot || st[t] < cursor) continue;  // consumed by the previous candidate
            const bool ended = (fl[t] & REC_ENDED) != 0u;
            nsw[na * nss] = st[t];
            nsw[(SEG_MAX + na) * nss] = nsw[(SEG_MAX + t) * nss];  // na <= t: compacts in place
            nsw[(SEG_MAX + EP_MAX + na) * nss] =
                (en[t] << 2) | (ended ? 2u : 0u) | ((fl[t] & (REC_ERR | REC_SKIP)) ? 1u : 0u);
            ++na;
            cursor = en[t];
            stop = ended;  // the run ended inside this episode
        }
        if (na) {
#pragma unroll
            for (uint32_t b = 0; b < APPLY_B; ++b) {
                const uint32_t t = b < na ? b : na - 1;  // clamped: unconditional loads, masked below
                const uint32_t *rec = a.recs + (size_t)nsw[(SEG_MAX + t) * nss] * a.rec_words;
#pragma unroll
                for (int k = 0; k < 2 * M; ++k) d[b][k] = rec[2 + k];
            }
        }
    }
    K3T(5);
#pragma unroll
    for (int w = 0; w < (M + 1) / 2; ++w) {
        F[2 * w] += gc[w] & 0xFFFFu;
        if (2 * w + 1 < M) F[2 * w + 1] += gc[w] >> 16;
    }
    if (gc[CNT_WORDS - 1] >> 16) return false;
    const uint32_t bg = (uint32_t)e * a.seg + G * GROUP;
    uint32_t n_end = 0, klast = 15u;
    int64_t t_last = 0;
    bool done = false;
    {  // redraw the group from its first block's stored streams, four blocks at a time as K1 drew them
       // (draw_quad_fast, the exact form for a flagged quad): the four draws' table reads and interval
       // polynomials are independent, so they overlap instead of forming one chain of 31 draws
        Rng ri = gr.ri, rp = gr.rp;
        uint32_t Ic = gr.w0 >> 5, kc = gr.w0 & 15u;  // the current block (q) and its finder
        for (uint32_t q0 = 0; q0 < GROUP && !done; q0 += K1_QB) {
            uint32_t I[K1_QB], info[K1_QB];
            const Rng ri0 = ri, rp0 = rp;
            if (draw_quad_fast(ri, rp, a.tab.logt, a.tab.pick, MSIM_FD_DEFAULT, I, info))
                draw_quad_exact(ri0, rp0, a.tab.logt, a.tab.pick, I, info);
#pragma unroll
            for (uint32_t b = 0; b < K1_QB; ++b) {
                if (done) continue;
                const int64_t Tn = T + (int64_t)Ic;
                if (Tn >= D) {
                    done = true;
                    n_end = bg + q0 + b;
                    t_last = T;
                    continue;
                }
                T = Tn;
                klast = kc;
                if (klast == 15u) return false;  // PickFinder fell through (simulation.h:220): the retry reports it
#pragma unroll
                for (int kk = 0; kk < M; ++kk) F[kk] += (klast == (uint32_t)kk) ? 1u : 0u;
                Ic = I[b];
                kc = info_finder(info[b]);
            }
        }
    }
    if (!done) return false;
    K3T(6);
    if (n_end == bg && n_end > 0) {  // the block before the end is the previous group's last one
        size_t pg;
        if (G > 0) pg = gb + G - 1;
        else if (e > (int)a.band_lo) pg = gb - 1;
        else return false;
        const GroupRec gp = a.grec[pg * a.nr + r];
        // only the finder of its last block is needed: the picker stream alone, stepped to block GROUP - 1
        Rng rp = gp.rp;
        for (uint32_t q = 1; q + 1 < GROUP; ++q) rng_next(rp);
        klast = info_finder(pick_info(rng_next(rp), a.tab.pick));
    }
    K3T(7);
    // 6. Episodes: the candidates that start before the end apply (a prefix of the chain).
    uint32_t cursor = 0;  // first block not consumed yet; ~0 once the run ended inside an episode
    if (batched) {
        uint32_t naf = 0;
        for (uint32_t t = 0; t < na && nsw[t * nss] < n_end; ++t) {
            const uint32_t x = nsw[(SEG_MAX + EP_MAX + t) * nss];
            if (x & 1u) return false;  // an applied episode K2 could not finish, or one it skipped
            cursor = (x & 2u) ? 0xFFFFFFFFu : (x >> 2);
            ++naf;
        }
#pragma unroll
        for (uint32_t b = 0; b < APPLY_B; ++b)
#pragma unroll
            for (int k = 0; k < M; ++k) {
                F[k] += b < naf ? d[b][k] : 0u;
                S[k] += b < naf ? d[b][M + k] : 0u;
            }
        for (uint32_t t0 = APPLY_B; t0 < naf; t0 += APPLY_B) {  // more than APPLY_B applied episodes (rare)
            uint32_t dd[APPLY_B][2 * M];
#pragma unroll
            for (uint32_t b = 0; b < APPLY_B; ++b) {
                const uint32_t t = t0 + b < naf ? t0 + b : naf - 1;
                const uint32_t *rec = a.recs + (size_t)nsw[(SEG_MAX + t) * nss] * a.rec_words;
#pragma unroll
                for (int k = 0; k < 2 * M; ++k) dd[b][k] = rec[2 + k];
            }
#pragma unroll
            for (uint32_t b = 0; b < APPLY_B; ++b)
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    F[k] += t0 + b < naf ? dd[b][k] : 0u;
                    S[k] += t0 + b < naf ? dd[b][M + k] : 0u;
                }
        }
    } else {  // more than EP_MAX episodes up to the end segment (never at BASELINE sizes): one read at a time
        bool stop = false;
        for (int j = 0; j <= e && !stop; ++j) {
            const uint32_t ns = a.nslow[(size_t)j * a.nr + r];
            if (ns > a.cap) return false;
            for (uint32_t c = 0; c < ns; ++c) {
                const uint32_t idx = a.slots[((size_t)j * a.cap + c) * a.nr + r];
                if (idx >= a.lcap) return false;
                const uint32_t *rec = a.recs + (size_t)idx * a.rec_words;
                const uint32_t s0 = rec[2 + 2 * M];
                if (s0 >= n_end) {
                    stop = true;
                    break;
                }
                if (s0 < cursor) continue;
                const uint32_t f0 = rec[1];
                if (f0 & (REC_ERR | REC_SKIP)) return false;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    F[k] += rec[2 + k];
                    S[k] += rec[2 + M + k];
                }
                cursor = rec[0];
                if (f0 & REC_ENDED) {
                    cursor = 0xFFFFFFFFu;
                    stop = true;
                    break;
                }
            }
        }
    }
    K3T(8);
    K3T_PRINT;
    // 7. The run ended quiet and its last block was a fast one: it counts only if it arrived by D.
    if (cursor != 0xFFFFFFFFu && n_end > 0 && cursor < n_end) {
        const uint32_t k = klast;
        int64_t pk = 0;
#pragma unroll
        for (int kk = 0; kk < M; ++kk)
            if ((uint32_t)kk == k) pk = p.prop[kk];
        if (t_last + pk > D) {
#pragma unroll
            for (int kk = 0; kk < M; ++kk) F[kk] -= ((uint32_t)kk == k) ? 1u : 0u;
        }
    }
    return true;
}

// ---------------------------------------------------------------- K2 lane body (shared host/device)
template <int M, int KIND>
MSIM_HD void episode_entry(const SimParams &p, const PipeArgs &a, uint32_t idx)
{
    const EpEntry e = a.list[idx];
    if (e.run == EP_HOLE) return;  // never referenced by a run's slots
    uint32_t *rec = a.recs + (size_t)idx * a.rec_words;
    rec[2 + 2 * M] = e.block;
    const uint32_t seg = e.block / a.seg;
    int64_t T = (int64_t)e.offset;
    // the segment sums before the episode's segment, 8 independent loads at a time
    for (uint32_t j0 = 0; j0 < seg; j0 += 8) {
        uint64_t ss[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) ss[j] = a.segsum[(size_t)(j0 + j < seg ? j0 + j : seg - 1) * a.nr + e.run];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) T += j0 + j < seg ? (int64_t)ss[j] : 0;  // clamped loads, masked
    }
    if (T >= p.duration_ms) {  // beyond the end of the run: never applied
        rec[1] = REC_SKIP;
        return;
    }
    EpSrc src;
    src.lt = a.tab.logt;
    src.pt = a.tab.pick;
    src.ri = e.ri;
    src.rp = e.rp;
    for (uint32_t t = 0; t < e.skip; ++t) {  // K1 stored its quad's start states (EpEntry::skip)
        rng_next(src.ri);
        rng_next(src.rp);
    }
    src.nb = a.nb;
    src.index = e.block;
    src.cur = e.w0;
    src.nxt = e.w1;
    src.have_nxt = true;
    // K2's capacities (K2_LEAN_RHO above); the retry kernel recomputes a flagged run with NX_WIDE and deep branches
    Sim<M, false, KIND == 2, KIND == 0 ? 2 : NX_FAST, NG_FAST> s;
    EpisodeOut<M> o;
    s.episode(p, src, T, o);
    rec[0] = o.end;
    rec[1] = (o.ended ? REC_ENDED : 0u) | (o.err ? REC_ERR : 0u);
#pragma unroll
    for (int k = 0; k < M; ++k) {
        rec[2 + k] = o.F[k];
        rec[2 + M + k] = o.S[k];
    }
}

}  // namespace msim
