// msim_general_launch.h — host/device interface of G, the general engine (msim_general.h).
//
// G runs in up to three tiers of growing windows. Tier 1 takes its runs from a list (the runs the entity
// engine's retry kernel E2 could not finish) or from an index range (networks only G serves: selfish miners
// in networks of more than 15 miners, more than 4 selfish miners); a run whose chains outgrow the window is
// appended to the next tier's list. The last tier's window holds every block a run can have (gen_tiers).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>

#include "msim_general.h"

namespace msim {

// Counter words of a launch's workspace shared by the entity-engine path and G (u32 each):
//   [0] runs E1 flagged for E2, [1] runs that failed everywhere, [2..4] G tier lists 1..3
enum : uint32_t { GEN_C_FLAG = 0, GEN_C_FAIL = 1, GEN_C_L1 = 2, GEN_C_L2 = 3, GEN_C_L3 = 4, GEN_C_WORDS = 8 };

struct GenArgs {
    const GenParams *pts;      // per point (device)
    uint32_t rpp;              // runs per point (a code is point * rpp + rel)
    uint32_t max_m;            // sums / counter stride
    uint64_t run_begin;
    uint32_t seed_base;
    const uint32_t *list;      // codes of this tier's runs, or null: codes 0 .. n_items - 1
    const uint32_t *list_count;
    uint32_t list_cap;
    uint32_t n_items;
    uint32_t *next;            // the next tier's list (null in the last tier)
    uint32_t *next_count;
    uint32_t cap;              // window (blocks per chain)
    size_t lanes;
    uint32_t *owners;          // [lanes][M][cap]
    int64_t *arrivals;         // [lanes][M][cap]
    uint32_t *sizes;           // 3 x [max_m][lanes]: size, stale, folded prefix
    uint64_t *sums;            // [n_points][6 * max_m] (atomic adds)
    uint32_t *records;         // [n_points * rpp][M][2] or null
    uint32_t *best_h;          // [n_points * rpp] or null
    uint32_t *counts;          // GEN_C_WORDS u32
};

struct GenTier {
    uint32_t cap;
    size_t lanes;
};

// Window tiers for networks of up to max_m miners and runs of up to max_duration ms: 256 blocks (every
// honest or minority-selfish run folds well inside it), 4 096, and, when `full`, the largest chain a run can
// have (mu + 10 sigma + 64 blocks: a selfish miner that never reveals holds every block). `full` is set for
// networks with a selfish miner and for honest networks whose largest propagation delay could span a
// quarter of the 4 096-block window (gen_needs_full): an honest fork folds once its blocks have arrived
// everywhere, so the window needs about the blocks found within the largest delay. Any other honest network
// stops at 4 096 and does not reserve a window it never uses. Lanes per tier fill `budget` bytes: whole waves
// while a wave fits, down to ONE lane for a window too large for a wave (the last tier of a large selfish
// network: a run only reaches it with a selfish majority, and a lane serves its list in turn).
// One lane's chains may take up to a third of the MI355X's 288 GB of HBM; larger networks are rejected at
// config creation (MSIM_E_MINERS), and msim_run rejects a launch whose workspace exceeds the device's free
// memory with the same code (msim_api.hip).
constexpr double GEN_MAX_LANE_BYTES = 96.0 * 1024 * 1024 * 1024;
inline bool gen_needs_full(bool selfish, int64_t max_prop_ms)
{
    if (selfish) return true;
    const double mu = (double)max_prop_ms / 599999.5;
    return mu + 10.0 * sqrt(mu > 1.0 ? mu : 1.0) + 64.0 >= 1024.0;
}
inline double gen_lane_bytes(uint32_t max_m, uint32_t cap) { return (double)max_m * (cap * 12.0 + 12.0); }
inline uint32_t gen_last_cap(int64_t max_duration)
{
    const double mu = (double)max_duration / 599999.5, sd = sqrt(mu > 1.0 ? mu : 1.0);
    uint64_t top = (uint64_t)ceil(mu + 10.0 * sd + 64.0) + 2;
    top = (top + 255) / 256 * 256;
    return (uint32_t)(top > 4096 ? top : 4096);
}
inline int gen_tiers(uint32_t max_m, int64_t max_duration, double budget, GenTier (&t)[3], bool full)
{
    const uint32_t caps[3] = {256u, 4096u, gen_last_cap(max_duration)};
    const int nt = full && caps[2] > 4096u ? 3 : 2;
    for (int i = 0; i < nt; ++i) {
        double l = floor(budget / gen_lane_bytes(max_m, caps[i]));
        l = l >= 64.0 ? floor(l / 64.0) * 64.0 : (l >= 1.0 ? l : 1.0);
        if (l > 65536.0) l = 65536.0;
        t[i].cap = caps[i];
        t[i].lanes = (size_t)l;
    }
    return nt;
}
// Whether G can hold a network of m miners and runs of duration_ms (one lane of its last window).
inline bool gen_fits(uint32_t m, int64_t duration_ms, bool full)
{
    return gen_lane_bytes(m, full ? gen_last_cap(duration_ms) : 4096u) <= GEN_MAX_LANE_BYTES;
}

// Workspace of G: the tier lists and the largest tier's chains and counters.
struct GenWs {
    GenTier tier[3];
    int nt;
    uint32_t list_cap;
    size_t lists_off, sizes_off, owners_off, arrivals_off, total;
};

inline GenWs gen_ws_layout(uint32_t max_m, int64_t max_duration, uint32_t list_cap, double budget, bool full)
{
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    GenWs w;
    w.nt = gen_tiers(max_m, max_duration, budget, w.tier, full);
    w.list_cap = list_cap;
    size_t lanes = 0, chain = 0;
    for (int i = 0; i < w.nt; ++i) {
        lanes = w.tier[i].lanes > lanes ? w.tier[i].lanes : lanes;
        const size_t c = w.tier[i].lanes * (size_t)max_m * w.tier[i].cap;
        chain = c > chain ? c : chain;
    }
    w.lists_off = 0;
    w.sizes_off = al(3 * (size_t)list_cap * 4);
    w.owners_off = al(w.sizes_off + 3 * (size_t)max_m * lanes * 4);
    w.arrivals_off = al(w.owners_off + chain * 4);
    w.total = al(w.arrivals_off + chain * 8);
    return w;
}

hipError_t launch_gen(const GenArgs &a, hipStream_t s);
hipError_t launch_gen_status(const uint32_t *counts, uint32_t *status, hipStream_t s);

// All tiers over one workspace: tier 1 from `first` (list + count, or null for codes 0 .. n_items - 1).
inline hipError_t launch_gen_tiers(GenArgs a, const GenWs &w, char *gws, const uint32_t *first, const uint32_t *first_count,
                                   uint32_t n_items, hipStream_t s)
{
    uint32_t *lists = (uint32_t *)(gws + w.lists_off);
    a.sizes = (uint32_t *)(gws + w.sizes_off);
    a.owners = (uint32_t *)(gws + w.owners_off);
    a.arrivals = (int64_t *)(gws + w.arrivals_off);
    a.list_cap = w.list_cap;
    for (int i = 0; i < w.nt; ++i) {
        a.cap = w.tier[i].cap;
        a.lanes = w.tier[i].lanes;
        if (i == 0) {
            a.list = first;
            a.list_count = first_count;
            a.n_items = n_items;
        } else {
            a.list = lists + (size_t)(i - 1) * w.list_cap;
            a.list_count = a.counts + GEN_C_L1 + i;
        }
        a.next = i + 1 < w.nt ? lists + (size_t)i * w.list_cap : nullptr;
        a.next_count = i + 1 < w.nt ? a.counts + GEN_C_L1 + i + 1 : nullptr;
        const hipError_t e = launch_gen(a, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace msim
