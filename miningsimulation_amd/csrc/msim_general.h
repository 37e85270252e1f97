// msim_general.h — the general engine (G): RunSimulation for ANY network the reference accepts, one run
// per lane, exact, with the reference's own data model (one explicit chain per miner) held in a bounded
// window of global memory.
//
// Replaces, per run, /root/reference/main.cpp:128-192 (RunSimulation, BestChain 68-82, EarliestArrival
// 99-112) and simulation.h:62-180 (FoundBlock, UnpublishedBlocks, NextArrival, SelfishBlocks,
// PublishedChain, MaybeReorg, MaybeSelfishReveal, NotifyBestChain), with the draws of simulation.h:205-221
// made exactly as the reference makes them (glibc log1p sequence, PickFinder over integer weights).
//
// Why it exists. The fast engines are specialised: the event-skipping pipelines (honest networks), the
// settled form + entity engine (<= 15 miners, <= 4 selfish miners, 16-height nibble window). G serves what
// they cannot: selfish miners in networks of more than 15 miners, more than 4 selfish miners, and every run
// that outgrows a fast engine's capacities (a majority selfish miner whose withheld chain grows for the
// whole run). It is slower per block — it walks every miner at every event, like the reference — and is
// used only where nothing faster is exact.
//
// The window. Every chain is a vector of (owner index, arrival) from genesis up (simulation.h:22-39,
// 57-59). Blocks that are in EVERY miner's chain at the same height, and already arrived, can never leave
// any chain: a chain only changes by appending (FoundBlock), by revealing its own trailing withheld blocks
// (MaybeSelfishReveal), or by MaybeReorg to a strictly longer chain of another miner, which shares that
// prefix; MaybeReorg's walk stops at the first equal block, above it. So when a chain runs out of room, the
// common arrived prefix below its top block is folded into per-owner counters (`pre`) and every window is
// shifted down by the same amount (`base` keeps the absolute height). The windows' block comparisons
// (MaybeReorg) and arrival reads (BestChain's first-seen key, UnpublishedBlocks, NextArrival) never reach
// below the common prefix, so the fold changes nothing the reference computes. A run that cannot fold
// enough room is flagged (GERR_CAP) and the host recomputes it with a larger window; the last tier's window
// holds every block a run can have, so results never depend on the window size.
#pragma once
#include <stdint.h>

#include "msim_draws.h"

namespace msim {

constexpr uint32_t GEN_GENESIS = 0xFFFFFFFFu;       // owner of Genesis (simulation.h:32, id = UINT_MAX)
constexpr int64_t GEN_SELFISH = 0x7FFFFFFFFFFFFFFFll;  // SELFISH_ARRIVAL = milliseconds::max() (simulation.h:20)
enum : uint32_t {
    GERR_CAP = 1u,   // a chain outgrew its window and the common prefix could not be folded
    GERR_PICK = 2u,  // PickFinder fell through (simulation.h:220 assert): weights not summing to W
};

// One network (a sweep point). Weights are integers summing to W; W = 100 is the reference's percentages
// with PERC_MULTIPLIER = UINT64_MAX / 100 (simulation.h:18), any other W is SURVEY Appendix C's
// generalisation (multiplier UINT64_MAX / W).
//
// Miner ids. The reference identifies a block's creator by Miner::id, not by the miner's position: a
// block is (miner_id, arrival) (simulation.h:22-38), MaybeReorg's walk compares blocks by that pair and
// counts a popped block as stale when its miner_id is the miner's own id (simulation.h:130-133), and
// MinerStats counts the best chain's blocks whose miner_id equals the miner's id (main.cpp:24-26), Genesis
// (id UINT_MAX, simulation.h:31-33) included. So two miners that share an id share their blocks' identity,
// their stale counting and their found counts. G stores as a block's owner the id's CLASS: the lowest index
// of a miner with that id (cls[k]); owners are then equal exactly when the reference's ids are, and the
// per-owner counters of a class hold the blocks of every miner with that id. The class whose id is
// UINT_MAX (umax, or GEN_GENESIS when no miner has it) also owns Genesis in MinerStats.
struct GenParams {
    int64_t duration_ms;
    uint64_t mult;         // UINT64_MAX / W
    uint32_t m;            // miners
    uint32_t umax;         // class of id UINT_MAX, or GEN_GENESIS
    const uint64_t *cum;   // [m] cumulative weights
    const int64_t *prop;   // [m] propagation (ms)
    const uint8_t *self;   // [m] 1: selfish (simulation.h:55)
    const uint32_t *cls;   // [m] id class: lowest index with the same Miner::id
};

// PickFinder (simulation.h:213-221): the first miner k whose cumulative weight * mult exceeds u. With
// q = floor(u / mult) that is the first k with cum_k > q (cum_k * mult > u <=> cum_k >= q + 1), found by
// bisection. Returns m when it falls through.
MSIM_HD uint32_t gen_pick(uint64_t u, const GenParams &g)
{
    const uint64_t q = u / g.mult;
    uint32_t lo = 0, hi = g.m;  // first index in [lo, hi) with cum > q, or m
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (g.cum[mid] > q) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// Store: the run's chains and per-miner counters.
//   uint32_t own(k, i); int64_t arr(k, i); void put(k, i, owner, arrival); void set_arr(k, i, arrival)
//   uint32_t size(k); void set_size(k, n); void add_stale(k); uint32_t stale(k);
//   void add_pre(k, v); uint32_t pre(k); uint32_t cap
struct GenOut {
    uint32_t best_len;  // window length of the final best chain
    int32_t best;       // its miner
    uint32_t base;      // absolute height of window index 0
    uint32_t err;
};

template <class St>
struct Gen {
    St &st;
    const GenParams &g;
    uint32_t base;   // absolute height of window index 0
    int32_t bcs;     // best_chain_size of the previous event (main.cpp:149, 171), window-relative; negative
                     // when a fold took blocks that arrived after that event (one miner, zero delays)
    int64_t now;     // the current time (a fold only takes blocks that arrived by now)
    uint32_t err;

    MSIM_HD Gen(St &s, const GenParams &gp) : st(s), g(gp), base(0), bcs(1), now(0), err(0) {}

    // Fold the common arrived prefix of every chain below its top block into `pre` (see the header).
    // Returns the number of heights folded.
    MSIM_HD uint32_t fold()
    {
        uint32_t c = st.size(0);
        for (uint32_t k = 1; k < g.m; ++k) c = st.size(k) < c ? st.size(k) : c;
        uint32_t i = 0;
        for (; i < c; ++i) {
            const uint32_t o = st.own(0, i);
            const int64_t a = st.arr(0, i);
            if (a > now) break;
            bool same = true;
            for (uint32_t k = 1; k < g.m && same; ++k) same = st.own(k, i) == o && st.arr(k, i) == a;
            if (!same) break;
        }
        if (i < 2) return 0;
        const uint32_t s = i - 1;  // keep the last common block as window index 0
        for (uint32_t j = 0; j < s; ++j) {
            const uint32_t o = st.own(0, j);
            if (o != GEN_GENESIS) st.add_pre(o, 1u);
        }
        for (uint32_t k = 0; k < g.m; ++k) {
            const uint32_t n = st.size(k);
            for (uint32_t j = s; j < n; ++j) st.put(k, j - s, st.own(k, j), st.arr(k, j));
            st.set_size(k, n - s);
        }
        base += s;
        bcs -= (int32_t)s;
        return s;
    }

    // chain.push_back with room made by a fold; a fold that frees less than an eighth of the window
    // flags the run for a larger window instead of folding again and again.
    MSIM_HD bool push(uint32_t k, uint32_t o, int64_t a)
    {
        if (st.size(k) >= st.cap) {
            const uint32_t s = fold();
            if (s < (st.cap >> 3) || st.size(k) >= st.cap) {
                err |= GERR_CAP;
                return false;
            }
        }
        const uint32_t n = st.size(k);
        st.put(k, n, o, a);
        st.set_size(k, n + 1);
        return true;
    }

    // simulation.h:62-76 FoundBlock. A selfish miner's block races when it is the one withheld block
    // (SelfishBlocks() == 1) on a chain as long as the last best chain.
    MSIM_HD bool found_block(uint32_t k, int64_t t)
    {
        const int64_t p = g.prop[k];
        if (g.self[k]) {
            const uint32_t n = st.size(k);
            const bool one = n >= 1 && st.arr(k, n - 1) == GEN_SELFISH && (n < 2 || st.arr(k, n - 2) != GEN_SELFISH);
            if (one && bcs == (int32_t)n) {
                st.set_arr(k, n - 1, t + p);
                return push(k, g.cls[k], t + p);
            }
            return push(k, g.cls[k], GEN_SELFISH);
        }
        return push(k, g.cls[k], t + p);
    }

    // simulation.h:118-121 PublishedChain length: the chain minus UnpublishedBlocks(t) (simulation.h:79-89).
    MSIM_HD uint32_t pub_len(uint32_t k, int64_t t) const
    {
        uint32_t n = st.size(k);
        while (n > 0 && st.arr(k, n - 1) > t) --n;
        return n;
    }

    // main.cpp:68-82 BestChain: index order, strictly more work or strictly earlier tip arrival.
    MSIM_HD void best_chain(int64_t t, int32_t &bk, uint32_t &bl) const
    {
        bk = -1;
        bl = 0;
        int64_t ba = 0;
        for (uint32_t k = 0; k < g.m; ++k) {
            const uint32_t pl = pub_len(k, t);
            if (pl == 0) continue;
            const int64_t a = st.arr(k, pl - 1);
            if (pl > bl || (pl == bl && a < ba)) {
                bk = (int32_t)k;
                bl = pl;
                ba = a;
            }
        }
    }

    // simulation.h:105-115 SelfishBlocks: trailing blocks with SELFISH_ARRIVAL.
    MSIM_HD uint32_t selfish_blocks(uint32_t k) const
    {
        uint32_t n = st.size(k), c = 0;
        while (n > 0 && st.arr(k, n - 1) == GEN_SELFISH) {
            --n;
            ++c;
        }
        return c;
    }

    // simulation.h:149-174 MaybeSelfishReveal.
    MSIM_HD void selfish_reveal(uint32_t k, uint32_t bl, int64_t t)
    {
        if (!g.self[k]) return;
        const uint32_t n = st.size(k);
        if (bl > n) return;
        const uint32_t sc = selfish_blocks(k);
        const uint32_t lead = n - bl;
        if (sc > lead) {
            uint32_t rc = sc - lead;
            if (sc > 1 && lead == 1) rc = sc;
            for (uint32_t i = 0; i < rc; ++i) st.set_arr(k, n - sc + i, t + g.prop[k]);
        }
    }

    // simulation.h:124-142 MaybeReorg onto miner bk's first bl blocks.
    MSIM_HD bool reorg(uint32_t k, int32_t bk, uint32_t bl)
    {
        uint32_t n = st.size(k);
        if (bl <= n) return true;
        for (uint32_t i = n; i > 0; --i) {
            const uint32_t o = st.own(k, n - 1);
            if (o == st.own((uint32_t)bk, i - 1) && st.arr(k, n - 1) == st.arr((uint32_t)bk, i - 1)) break;
            if (o == g.cls[k]) st.add_stale(k);  // chain.back().miner_id == id
            --n;
        }
        if (bl > st.cap) {
            err |= GERR_CAP;
            return false;
        }
        for (uint32_t i = n; i < bl; ++i) st.put(k, i, st.own((uint32_t)bk, i), st.arr((uint32_t)bk, i));
        st.set_size(k, bl);
        return true;
    }

    // simulation.h:92-102 NextArrival: the lowest block of the trailing run that has not arrived by t.
    MSIM_HD bool next_arrival(uint32_t k, int64_t t, int64_t &out) const
    {
        uint32_t n = st.size(k);
        bool have = false;
        while (n > 0 && st.arr(k, n - 1) > t) {
            out = st.arr(k, n - 1);
            have = true;
            --n;
        }
        return have;
    }

    // main.cpp:128-192 RunSimulation. Returns false on an error (out.err).
    MSIM_HD bool run(Rng ri, Rng rp, GenOut &out)
    {
        for (uint32_t k = 0; k < g.m; ++k) {
            st.put(k, 0, GEN_GENESIS, 0);  // simulation.h:57-59: chain = {Genesis}
            st.set_size(k, 1);
        }
        const int64_t D = g.duration_ms;
        int64_t nbt = next_interval(ri);  // main.cpp:138
        bcs = 1;                          // main.cpp:149
        for (int64_t cur = 0; cur < D;) {
            now = cur;
            while (cur == nbt) {  // main.cpp:153-157
                const uint32_t k = gen_pick(rng_next(rp), g);
                if (k >= g.m) {
                    err |= GERR_PICK;
                    break;
                }
                if (!found_block(k, nbt)) break;
                nbt += next_interval(ri);
            }
            if (err) break;
            int32_t bk;
            uint32_t bl;
            best_chain(cur, bk, bl);  // main.cpp:164
            for (uint32_t k = 0; k < g.m && !err; ++k) {  // main.cpp:165-167
                selfish_reveal(k, bl, cur);
                reorg(k, bk, bl);
            }
            if (err) break;
            bcs = (int32_t)bl;  // main.cpp:171
            bool have = false;  // main.cpp:176-182 EarliestArrival
            int64_t ea = 0;
            for (uint32_t k = 0; k < g.m; ++k) {
                int64_t a;
                if (next_arrival(k, cur, a)) {
                    ea = have ? (a < ea ? a : ea) : a;
                    have = true;
                }
            }
            cur = nbt;
            if (have && ea < cur) cur = ea;
        }
        out.err = err;
        if (err) return false;
        best_chain(D, out.best, out.best_len);  // main.cpp:185
        out.base = base;
        return true;
    }

    // main.cpp:22-26: blocks of miner k in the final best chain (folded prefix + window): the blocks of
    // its id class, plus Genesis when its id is UINT_MAX.
    MSIM_HD uint32_t found(uint32_t k, const GenOut &o) const
    {
        const uint32_t c = g.cls[k];
        uint32_t f = st.pre(c) + (c == g.umax ? 1u : 0u);
        for (uint32_t i = 0; i < o.best_len; ++i) f += st.own((uint32_t)o.best, i) == c ? 1u : 0u;
        return f;
    }
    // The same for every miner in one pass: the window of the final best chain is added to `pre`, which
    // then holds every id class's blocks (found_after_count gives a miner's blocks_found).
    MSIM_HD void count_best(const GenOut &o)
    {
        for (uint32_t i = 0; i < o.best_len; ++i) {
            const uint32_t ow = st.own((uint32_t)o.best, i);
            if (ow != GEN_GENESIS) st.add_pre(ow, 1u);
        }
    }
    MSIM_HD uint32_t found_after_count(uint32_t k) const
    {
        const uint32_t c = g.cls[k];
        return st.pre(c) + (c == g.umax ? 1u : 0u);
    }
    // the best chain's length minus Genesis (main.cpp:28's best_chain.size() - 1)
    MSIM_HD static uint32_t best_height(const GenOut &o) { return o.base + o.best_len - 1u; }
};

}  // namespace msim
