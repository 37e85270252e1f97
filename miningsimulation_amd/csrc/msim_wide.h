// msim_wide.h — the event-skipping pipeline for LARGE honest networks (BASELINE configs[4]: two pools
// and 1 024 small miners; any honest network with up to WIDE_MAX_M miners).
//
// The reference's RunSimulation (/root/reference/main.cpp:128-192) is unchanged in meaning; what changes
// with M is where the per-miner state can live. The narrow pipeline (msim_pipeline.h) keeps one run per
// lane and nine counters per lane; with M = 1 026 a run's counters are 4 KiB, so here
//
//   W1 msim_wide_draws_kernel    ONE WAVE PER RUN. Lane l draws a contiguous segment of the run's blocks
//                                (both xoroshiro128++ streams jumped to draw l*S0 by a per-lane GF(2)
//                                matrix, msim_jump.h); every block adds 1 to its finder's counter in the
//                                wave's LDS histogram (M u32); every non-fast block (I_{i+1} <= prop of
//                                its finder) is appended, with both RNG states, to the run's candidate
//                                list. A wave prefix-sum of the lane time sums locates the end of the run
//                                (the first T_i >= D, main.cpp:150-153); the run's tail is drawn in short
//                                64 x ST chunks so that only a few blocks past D are drawn, and the
//                                blocks past D are taken out of the histogram again.
//   W2 msim_wide_episode_kernel  one lane per candidate: the honest state machine from a quiet state
//                                (wide_episode below: explicit block tree, active miners + one class for
//                                all miners that have not found a block in the episode), until quiet
//                                again or the end of the run; sparse per-miner deltas.
//   W3 msim_wide_combine_kernel  one wave per run: order the candidates, chain the episodes whose first
//                                block is reached quiet, apply their deltas to the histogram, the last
//                                block's arrival correction, then MinerStats (main.cpp:22-30) for every
//                                miner into order-independent fixed-point workgroup sums.
//
// PickFinder for integer weights w_k summing to W (W = 100 is exactly the reference's
// percentages, simulation.h:18,213-221): q = floor(u / MULT), MULT = (2^64-1)/W, finder = first k with
// cum_k > q. q is p1 = floor(u*W / 2^64) or p1 + 1 (one 64x64 high multiply and one compare, as in
// msim_fastdraw.h); the first candidate k comes from a 4 096-entry u16 bucket table indexed by u's top
// bits, then a short scan of the packed cumulative-weight / fast-threshold table in LDS.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "msim_pipeline.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define MSIM_HDN __host__ __device__
#else
#define MSIM_HDN inline
#endif

namespace msim {

constexpr uint32_t WIDE_MAX_M = 4096;   // LDS histogram of 4 waves: 64 KiB; bucket entries are u16
constexpr int WB_BITS = 12;
constexpr uint32_t WB_N = 1u << WB_BITS;  // pick buckets
constexpr uint32_t WIDE_ST = 16;        // tail blocks per lane per chunk
// Episode capacities (blocks, miners that found one) of W2's two passes: every candidate with the small ones
// (its arrays fit in registers at 104 VGPRs, 4 waves per SIMD), the ones that outgrew them with the record
// format's full WA entries. Measured on configs[4] (profiles/r04/w2v, w2v3): first pass with 12 / 6 1.43 ms,
// 8 / 4 0.94 ms, 6 / 3 0.78 ms per launch, retry pass 0.09-0.14 ms; a middle pass (12 / 6) between them cost
// more than it saved.
#ifndef MSIM_WE_FAST
#define MSIM_WE_FAST 6
#endif
#ifndef MSIM_WA_FAST
#define MSIM_WA_FAST 3
#endif
constexpr int WE_FAST = MSIM_WE_FAST, WA_FAST = MSIM_WA_FAST;
constexpr int WE = 48;
constexpr int WA = 16;
constexpr uint32_t WREC_WORDS = 4 + 3 * WA;
constexpr uint32_t WIDE_NONE = 0xFFFFFFFFu;

enum : uint32_t {
    WERR_PICK = 1u,   // PickFinder fell through (simulation.h:220 assert) before the end of the run
    WERR_CAND = 2u,   // candidate list of the run overflowed
    WERR_DRAWS = 4u,  // the run outlasted the pre-planned tail chunks
    WERR_EP = 8u,     // an episode exceeded WE blocks / WA miners
};
enum : uint32_t { WREC_ENDED = 1u, WREC_ERR = 2u, WREC_SKIP = 4u, WREC_RETRY = 8u };

// One non-fast block of a run, with everything an episode needs to replay the run from there.
struct WideCand {
    uint32_t block;   // block index s within the run
    uint32_t f;       // its finder
    uint32_t inext;   // I_{s+1} (ms)
    uint32_t fnext;   // finder of block s+1
    uint32_t phase;   // 0 = main segments, 1 + c = tail chunk c
    uint32_t lane_seq;  // lane << 16 | rank among the lane's candidates in this phase
    uint64_t offset;  // T_s - (start time of the lane's segment)
    Rng ri, rp;       // both streams after drawing block s+1
};

// Per (run, phase, lane): the time of the last block before the lane's segment and the lane's
// candidate count in that phase.
struct WideLane {
    uint64_t t0;
    uint32_t count;
    uint32_t pad;
};

// Pick table entry k (k = 0..m; entry m is a sentinel): cumulative weight of miners 0..k in the low
// word, the fast threshold of miner k (its propagation, clamped to FTHR_NEVER) in the high word, so
// the scan's last load also yields the finder's threshold. Sentinel: cumulative 0xFFFFFFFF > any q.
MSIM_HD uint32_t wide_pick(uint64_t u, const uint64_t *__restrict__ cf, const uint16_t *__restrict__ bucket,
                           uint32_t W, uint64_t mult, uint32_t &fthr)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const uint64_t p1 = __umul64hi(u, (uint64_t)W);
#else
    const uint64_t p1 = (uint64_t)(((unsigned __int128)u * W) >> 64);
#endif
    const uint32_t q = (uint32_t)(u >= (p1 + 1) * mult ? p1 + 1 : p1);
    uint32_t k = bucket[u >> (64 - WB_BITS)];
    uint64_t e = cf[k];
    while ((uint32_t)e <= q) e = cf[++k];
    fthr = (uint32_t)(e >> 32);
    return k;  // == m: fell through (the reference asserts, simulation.h:220)
}

// ---------------------------------------------------------------- host table builders
// weights: m integer weights summing to W (validated by the caller, W < 2^31); fthr: m thresholds.
// cf: m + 1 entries; bucket: WB_N entries = first miner whose range can contain q for u in the bucket.
inline void build_wide_pick(const uint64_t *w, const uint32_t *fthr, uint32_t m, uint32_t W, uint64_t *cf,
                            uint16_t *bucket)
{
    uint64_t c = 0;
    for (uint32_t k = 0; k < m; ++k) {
        c += w[k];
        cf[k] = (uint64_t)(uint32_t)c | ((uint64_t)fthr[k] << 32);
    }
    cf[m] = 0xFFFFFFFFull;
    const uint64_t mult = 0xFFFFFFFFFFFFFFFFull / W;
    uint32_t k = 0;
    for (uint32_t b = 0; b < WB_N; ++b) {
        const uint64_t qlo = ((uint64_t)b << (64 - WB_BITS)) / mult;
        while (k < m && (uint32_t)cf[k] <= qlo) ++k;
        bucket[b] = (uint16_t)k;
    }
}

// Geometry of W1 for a run duration D: main segments of S0 blocks per lane (up to ~mu - 3 sigma blocks),
// then up to nch tail chunks of 64 x ST blocks (through mu + 8 sigma + 64).
struct WideGeom {
    uint32_t S0, ST, nch;
    uint64_t B0;
};
inline WideGeom wide_geom(int64_t duration_ms)
{
    WideGeom g;
    const double mu = (double)duration_ms / 599999.5, sd = sqrt(mu > 1.0 ? mu : 1.0);
    const double lo = mu - 3.0 * sd;
    g.S0 = lo > 64.0 ? (uint32_t)floor(lo / 64.0) : 0u;
    g.B0 = (uint64_t)g.S0 * 64u;
    g.ST = WIDE_ST;
    const double need = mu + 8.0 * sd + 64.0 - (double)g.B0;
    const double ch = ceil(need / (64.0 * g.ST));
    g.nch = ch < 1.0 ? 1u : (uint32_t)ch;
    return g;
}

// ---------------------------------------------------------------- W2: one episode (honest network)
// Draw source of one run from a candidate on: both streams, exact interval (draw_interval), wide pick.
struct WideSrc {
    Rng ri, rp;
    const LogTab *lt;
    const uint64_t *cf;
    const uint16_t *bucket;
    uint32_t W;
    uint64_t mult;
    MSIM_HD void next(uint32_t &I, uint32_t &f)
    {
        I = draw_interval(ri, lt);
        uint32_t th;
        f = wide_pick(rng_next(rp), cf, bucket, W, mult, th);
    }
};

struct WideEpOut {
    uint32_t end;    // next unconsumed block
    uint32_t flags;  // WREC_ENDED / WREC_ERR
    uint32_t ne;     // entries
    uint32_t gid[WA];
    uint32_t dF[WA];  // + blocks in the final chain - blocks consumed (modular u32)
    uint32_t dS[WA];  // stale_blocks increments (simulation.h:133)
};

// The honest event loop of RunSimulation (main.cpp:150-182) from a quiet state at the find time T_s
// of block s (finder fs; block s+1 is (inext, fnext); later blocks from src), until every miner holds
// the same, fully published chain again (quiet) or the run ends (cur_time >= D).
//
// State: the episode's blocks as a tree over the quiet tip (the base, index -1): parent, owner, arrival
// (Miner::FoundBlock honest branch, simulation.h:74), height above the base. Each miner that found a
// block in the episode is "active" with its own tip (= its chain, a root path: SURVEY Q2, (owner, height)
// identifies a block) and stale counter. All other miners ("passive") hold one common chain: they start
// equal, see the same BestChain and apply the same MaybeReorg (simulation.h:124-142), and hold only
// published blocks; in BestChain (main.cpp:68-82, index order, strict comparisons) they act as one
// candidate at the position of the lowest passive index.
// CE / CA: capacities of this instantiation; exceeding one sets WREC_RETRY (recompute with larger ones)
// instead of WREC_ERR.
template <int CE, int CA, class Src>
MSIM_HDN void wide_episode(const int64_t *__restrict__ prop, uint32_t m, int64_t D, uint32_t s, int64_t Ts,
                           uint32_t fs, uint32_t inext, uint32_t fnext, Src &src, WideEpOut &o)
{
    static_assert(CA <= WA, "record holds WA entries");
    int32_t par[CE];
    uint32_t own[CE];
    int64_t arr[CE];
    int32_t hgt[CE];
    uint32_t gid[CA];  // active miners, sorted by index
    int32_t tip[CA];
    uint32_t stl[CA], nf[CA];
    uint32_t cap = 0;
    int na = 0, nb = 0, ptip = -1;
    uint32_t err = 0, consumed = 0;
    int64_t Tn = Ts;
    uint32_t fn = fs;
    bool have1 = true, ended = false;
    int64_t cur = Ts;
    auto H = [&](int b) { return b < 0 ? 0 : hgt[b]; };
    auto pub = [&](int b, int64_t t) {  // PublishedChain (simulation.h:118-121): drop blocks arriving after t
        while (b >= 0 && arr[b] > t) b = par[b];
        return b;
    };
    int best = -1;
    for (;;) {
        if (cur >= D) {  // main.cpp:150
            ended = true;
            break;
        }
        while (cur == Tn) {  // main.cpp:153-157
            if (fn >= m) {
                err |= WERR_PICK;
                break;
            }
            int a = -1;
            for (int i = 0; i < na; ++i)
                if (gid[i] == fn) a = i;
            if (a < 0) {  // a passive miner finds a block: it leaves the class with the class's chain
                if (na == CA) {
                    cap = 1;
                    break;
                }
                a = na;
                while (a > 0 && gid[a - 1] > fn) {
                    gid[a] = gid[a - 1];
                    tip[a] = tip[a - 1];
                    stl[a] = stl[a - 1];
                    nf[a] = nf[a - 1];
                    --a;
                }
                gid[a] = fn;
                tip[a] = ptip;
                stl[a] = 0;
                nf[a] = 0;
                ++na;
            }
            if (nb == CE) {
                cap = 1;
                break;
            }
            par[nb] = tip[a];  // Miner::FoundBlock, honest (simulation.h:73-75)
            own[nb] = fn;
            arr[nb] = Tn + prop[fn];
            hgt[nb] = H(tip[a]) + 1;
            tip[a] = nb;
            ++nb;
            ++nf[a];
            ++consumed;
            if (have1) {  // next_block_time += NextBlockInterval (main.cpp:156)
                Tn += inext;
                fn = fnext;
                have1 = false;
            } else {
                uint32_t I, f;
                src.next(I, f);
                Tn += I;
                fn = f;
            }
        }
        if (err || cap) break;
        // BestChain(cur) (main.cpp:68-82): candidates in index order; the passive class sits at the lowest
        // index that is not active.
        uint32_t pmin = 0;
        for (int i = 0; i < na; ++i)
            if (gid[i] == pmin) ++pmin;
        const bool passive = pmin < m;
        best = -2;
        int bl = -1;
        int64_t ba = 0;
        // merged walk: actives (sorted) with the passive candidate inserted before the first gid > pmin
        {
            bool pdone = !passive;
            int ai = 0;
            while (ai < na || !pdone) {
                int t;
                if (!pdone && (ai == na || gid[ai] > pmin)) {
                    t = ptip;
                    pdone = true;
                } else {
                    t = pub(tip[ai], cur);
                    ++ai;
                }
                const int L = H(t);
                const int64_t A = t < 0 ? 0 : arr[t];
                if (best == -2 || L > bl || (L == bl && A < ba)) {  // more_work || first_seen
                    best = t;
                    bl = L;
                    ba = A;
                }
            }
        }
        // NotifyBestChain -> MaybeReorg (simulation.h:124-142, 177-180): adopt a strictly longer chain,
        // popping to the fork point and counting own popped blocks as stale.
        for (int a = 0; a < na; ++a) {
            int x = tip[a];
            if (bl <= H(x)) continue;
            int y = best;
            while (H(y) > H(x)) y = par[y];
            while (x != y) {
                if (own[x] == gid[a]) ++stl[a];
                x = par[x];
                y = par[y];
            }
            tip[a] = best;
        }
        if (bl > H(ptip)) ptip = best;
        // Quiet again: every miner on one chain whose tip has arrived.
        {
            const int t0 = passive ? ptip : tip[0];
            bool q = true;
            for (int a = 0; a < na; ++a) q = q && tip[a] == t0;
            if (q && (t0 < 0 || arr[t0] <= cur)) {
                best = t0;
                break;
            }
        }
        // EarliestArrival (main.cpp:99-112): the lowest unpublished block of any chain (only own blocks
        // can be unpublished), then cut through to the next event (main.cpp:176-182).
        int64_t ea = Tn;
        for (int a = 0; a < na; ++a) {
            int b = tip[a];
            while (b >= 0 && arr[b] > cur) {
                if (arr[b] < ea) ea = arr[b];
                b = par[b];
            }
        }
        cur = ea;
    }
    if (cap) {
        o.end = s;
        o.flags = WREC_RETRY;
        o.ne = 0;
        return;
    }
    if (ended && !err) {
        // BestChain(duration_time) (main.cpp:185), no notification.
        uint32_t pmin = 0;
        for (int i = 0; i < na; ++i)
            if (gid[i] == pmin) ++pmin;
        const bool passive = pmin < m;
        bool pdone = !passive, first = true;
        int ai = 0, bl = -1;
        int64_t ba = 0;
        while (ai < na || !pdone) {
            int t;
            if (!pdone && (ai == na || gid[ai] > pmin)) {
                t = ptip;
                pdone = true;
            } else {
                t = pub(tip[ai], D);
                ++ai;
            }
            const int L = H(t);
            const int64_t A = t < 0 ? 0 : arr[t];
            if (first || L > bl || (L == bl && A < ba)) {
                best = t;
                bl = L;
                ba = A;
                first = false;
            }
        }
    }
    o.end = s + consumed;
    o.flags = (ended ? WREC_ENDED : 0u) | (err ? WREC_ERR : 0u);
    o.ne = err ? 0u : (uint32_t)na;
    if (err) return;
#pragma unroll
    for (int a = 0; a < CA; ++a) {  // static indices into o: its arrays stay in registers
        if (a >= na) continue;
        uint32_t inch = 0;
        for (int b = best; b >= 0; b = par[b]) inch += own[b] == gid[a] ? 1u : 0u;
        o.gid[a] = gid[a];
        o.dF[a] = inch - nf[a];
        o.dS[a] = stl[a];
    }
}

}  // namespace msim
