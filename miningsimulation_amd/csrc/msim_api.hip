// msim_api.hip — the C ABI declared in include/msim.h.
//
// msim_run replaces main()'s batch loop (/root/reference/main.cpp:195-220): the reference starts one
// std::async thread per RunSimulation call, in barrier-synchronised batches of hardware_concurrency(),
// and sums MinerStats in run order on the main thread. Here one launch runs a whole shard of runs,
// one run per lane, and the per-miner sums are reduced on the device in integers.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/msim.h"
#include "msim_general_launch.h"
#include "msim_jump.h"
#include "msim_kernels.h"
#include "msim_sel_launch.h"
#include "msim_wide_launch.h"

namespace {
constexpr int MAX_DEVICES = 64;
}

// A network as the general engine reads it (msim_general.h): integer weights summing to W.
struct GenHost {
    int64_t duration_ms = 0;
    uint64_t W = 100;
    std::vector<uint64_t> w;
    std::vector<int64_t> prop;
    std::vector<uint8_t> self;
    std::vector<uint32_t> ids;  // Miner::id (msim_general.h: blocks are identified by id class)
};

// Id classes of a miner list (msim_general.h GenParams::cls): the lowest index with the same id; the class
// of id UINT_MAX (Genesis's id, simulation.h:31-33) or GEN_GENESIS.
static void gen_id_classes(const std::vector<uint32_t> &ids, std::vector<uint32_t> &cls, uint32_t *umax)
{
    const size_t m = ids.size();
    std::vector<uint32_t> ord(m);
    for (size_t k = 0; k < m; ++k) ord[k] = (uint32_t)k;
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return ids[a] < ids[b]; });
    cls.assign(m, 0);
    *umax = msim::GEN_GENESIS;
    for (size_t i = 0; i < m; ++i) {
        const uint32_t k = ord[i];
        cls[k] = (i > 0 && ids[ord[i - 1]] == ids[k]) ? cls[ord[i - 1]] : k;  // stable: the lowest index first
        if (ids[k] == 0xFFFFFFFFu) *umax = cls[k];
    }
}

struct msim_config {
    msim::SimParams p;
    uint32_t n;
    uint32_t ids[MSIM_MAX_MINERS];
    uint64_t perc[MSIM_MAX_MINERS];
    int64_t prop[MSIM_MAX_MINERS];
    uint8_t self[MSIM_MAX_MINERS];
    double rho;      // probability that a block is not "fast" (msim_pipeline.h)
    bool pipe_ok;    // event-skipping pipeline eligible (honest network, rare forks)
    uint32_t jobs = 1;  // launches the caller keeps in flight at once (msim_config_set_concurrent_launches)
    std::mutex mu;
    struct Tab {
        int dev;
        uint32_t seg, nseg;
        void *ptr;
    };
    std::vector<Tab> tables;  // per (device, segment length) pipeline tables, lazily uploaded
    // Large honest networks (msim_wide.h): any miner count up to WIDE_MAX_M, integer weights summing to W.
    bool wide = false;
    uint64_t total_weight = 100;
    std::vector<uint32_t> wids;
    std::vector<uint64_t> wperc;
    std::vector<int64_t> wprop;
    std::vector<std::pair<int, void *>> wtables;  // per device: pick, fast-threshold, prop, log, jump tables
    // Networks with selfish miners (msim_sel.h entity engine): parameter block.
    bool sel = false;
    msim::SelParams sp;
    std::vector<std::pair<int, void *>> stables;  // per device: SelParams + point list {0}
    // The segment-parallel form of E1 (msim_selseg.h: SW workers + ST stitch) serves it when asked for
    // (MSIM_SELSEG): one selfish miner, the settled form applies, long runs, rare cuts (seg_rate: expected cuts
    // per find).
    bool seg_ok = false;
    double seg_rate = 0;
    // Every network, as the general engine reads it: G finishes the runs the entity engine cannot, and
    // serves alone (`general`) the networks no fast engine covers: selfish miners in networks of more than
    // MSIM_MAX_MINERS miners, more than SEL_MAXS selfish miners, large honest networks whose fork rate the
    // wide combine cannot hold.
    GenHost gh;
    bool general = false;
    bool selfish = false;   // some miner is selfish
    bool gen_full = false;  // G keeps its full last window tier (msim_general_launch.h gen_needs_full)
    std::vector<std::pair<int, void *>> gtables;  // per device: GenParams + arrays
};

// A parameter sweep (BASELINE configs[3]): the points' parameter blocks, uploaded per device on first use.
struct msim_sweep {
    std::vector<msim::SimParams> pts;
    uint32_t m;
    bool self;
    std::mutex mu;
    std::vector<std::pair<int, void *>> dev;  // (device, SimParams[n_points])
    // Entity-engine sweeps (some point has a selfish miner): every point's SelParams, the points grouped
    // by selfish class, one draw pass per slice shared by all points.
    bool sel = false;
    int64_t max_duration = 0;
    std::vector<msim::SelParams> sps;
    struct Group {
        uint32_t nscls;
        std::vector<uint32_t> points;
    };
    std::vector<Group> groups;
    std::vector<std::pair<int, void *>> sdev;  // (device, SelParams[n_points] + point lists)
    // General-engine view of every point (G finishes what E2 cannot; a sweep with a general point runs on G)
    bool general = false;
    bool gen_full = false;  // some point needs G's full last window tier (gen_needs_full)
    std::vector<GenHost> gens;
    std::vector<std::pair<int, void *>> gdev;  // (device, GenParams[n_points] + arrays)
};

namespace {

uint32_t err_cap_for(uint64_t n)
{
    uint64_t c = n < 65536 ? n : 65536;
    if (c < 256) c = 256;
    return (uint32_t)((c + 255) / 256 * 256);
}

struct WsLayout {
    size_t partials_off, counts_off, list_off, total;
    uint32_t err_cap;
};

WsLayout ws_layout(uint32_t m, uint64_t n)
{
    WsLayout l;
    l.err_cap = err_cap_for(n);
    l.partials_off = 0;
    l.counts_off = msim::partials_words(m, (uint32_t)n, l.err_cap) * sizeof(uint64_t);
    l.list_off = l.counts_off + 2 * sizeof(uint32_t);
    l.total = l.list_off + (size_t)l.err_cap * sizeof(uint32_t);
    l.total = (l.total + 255) / 256 * 256;
    return l;
}

constexpr uint64_t MAX_LAUNCH_RUNS = 1ull << 26;

// Sweep workspace: per-workgroup partials, per-point retry sums, counters, retry list.
struct SweepLayout {
    size_t partials_off, retry_off, counts_off, list_off, total;
    uint32_t wpp, err_cap;
};
SweepLayout sweep_layout(uint32_t m, uint32_t n_points, uint64_t rpp)
{
    SweepLayout l;
    l.wpp = (uint32_t)((rpp + msim::TPB - 1) / msim::TPB);
    l.err_cap = err_cap_for(rpp * n_points);
    const size_t nv = 6 * (size_t)m;
    l.partials_off = 0;
    l.retry_off = (size_t)n_points * l.wpp * nv * 8;
    l.counts_off = l.retry_off + (size_t)n_points * nv * 8;
    l.list_off = l.counts_off + 256;
    l.total = (l.list_off + (size_t)l.err_cap * 4 + 255) / 256 * 256;
    return l;
}
constexpr double PIPE_MAX_RHO = 0.08;           // above this the per-lane kernel is cheaper
constexpr double PIPE_SLICE_BUDGET = 16.0 * (1ull << 30);  // pipeline workspace per slice (bytes)

// K1 wave slots of the current device (CUs x resident K1 waves per CU); 8192 if it cannot be queried.
uint32_t draw_slots()
{
    if (const char *e = getenv("MSIM_K1_SLOTS")) return (uint32_t)atoi(e);  // A/B override (measurement only)
    int dev = 0, cus = 0, blocks = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        msim::draws_blocks_per_cu(&blocks) != hipSuccess || cus <= 0 || blocks <= 0)
        return 8192;
    return (uint32_t)(cus * blocks * 4);
}

// K1's grid is planned for the launches in flight: one launch gets three rounds of resident waves (more,
// shorter segments: later rounds fill the earlier ones' ragged ends), two launches on two streams one round
// each (the other launch fills it). Measured on MI355X, c2 serial (profiles/r06/k1slots/): 3.31 / 3.13 / 3.08 /
// 3.21 / 3.21 ms per step with 1 / 2 / 3 / 5 / 6 rounds (more segments also cost K2 and K3); two streams 2.82 ms
// per step with one round each against 2.89 with 1.5 and two.
msim::PipeLayout pipe_layout(const msim_config *c, uint64_t n_runs)
{
    const uint32_t jobs = c->jobs ? c->jobs : 1u;
    uint32_t slots = jobs == 1u ? draw_slots() * 3u : draw_slots() * 2u / jobs;
    if (slots < 1u) slots = 1u;
    return msim::pipe_layout_for(c->rho, c->n, c->p.duration_ms, n_runs, PIPE_SLICE_BUDGET, slots);
}

// Pipeline tables for this config on the current device: pick table, log table, jump matrices for
// draw offsets j * seg.
int device_tables(msim_config *c, uint32_t seg, uint32_t nseg, msim::PipeTables *out)
{
    using namespace msim;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return MSIM_E_HIP;
    std::lock_guard<std::mutex> g(c->mu);
    const size_t pick_b = sizeof(PickTab), log_b = sizeof(LogTab);
    void *d = nullptr;
    for (const auto &t : c->tables)
        if (t.dev == dev && t.seg == seg && t.nseg >= nseg) d = t.ptr;
    if (!d) {
        const size_t jump_b = (size_t)nseg * 128 * 16;
        std::vector<char> h(pick_b + log_b + jump_b);
        build_pick_table(c->perc, c->prop, c->self, (int)c->n, (PickTab *)h.data());
        build_log_table((LogTab *)(h.data() + pick_b));
        build_jump_table(nseg, seg, (uint32_t *)(h.data() + pick_b + log_b));
        if (hipMalloc(&d, h.size()) != hipSuccess) return MSIM_E_HIP;
        if (hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            return MSIM_E_HIP;
        }
        c->tables.push_back({dev, seg, nseg, d});
    }
    const char *b = (const char *)d;
    out->pick = (const PickTab *)b;
    out->logt = (const LogTab *)(b + pick_b);
    out->jump = (const uint32_t *)(b + pick_b + log_b);
    return MSIM_OK;
}

// Stage timing (msim_timing_enable / msim_timing_read): HIP events recorded on the launch stream.
struct Timing {
    std::mutex mu;
    bool on = false;
    std::vector<hipEvent_t> k1;      // (begin, end) pairs around K1
    std::vector<hipEvent_t> launch;  // (begin, end) pairs around msim_launch
    std::vector<hipEvent_t> engine;  // (begin, end) pairs around the entity engine (E1) of each slice
    uint32_t launches = 0;
};
Timing &timing()
{
    static Timing t;
    return t;
}

void destroy_events(std::vector<hipEvent_t> &v)
{
    for (auto e : v) (void)hipEventDestroy(e);
    v.clear();
}

// Process-wide log table (msim_fastdraw.h) per device, for msim_device_intervals.
int global_log_table(const msim::LogTab **out)
{
    static std::mutex mu;
    static void *tab[MAX_DEVICES] = {nullptr};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEVICES) return MSIM_E_HIP;
    std::lock_guard<std::mutex> g(mu);
    if (!tab[dev]) {
        msim::LogTab h;
        msim::build_log_table(&h);
        void *d = nullptr;
        if (hipMalloc(&d, sizeof(h)) != hipSuccess) return MSIM_E_HIP;
        if (hipMemcpy(d, &h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            return MSIM_E_HIP;
        }
        tab[dev] = d;
    }
    *out = (const msim::LogTab *)tab[dev];
    return MSIM_OK;
}

constexpr double WIDE_SLICE_BUDGET = 16.0 * (1ull << 30);

msim::WideLayout wide_layout(const msim_config *c, uint64_t n_runs)
{
    return msim::wide_layout_for(c->rho, c->n, c->p.duration_ms, n_runs, WIDE_SLICE_BUDGET);
}

// Device tables of a wide config (msim_wide_launch.h WideArgs) on the current device, uploaded once.
int wide_tables(msim_config *c, msim::WideArgs *a)
{
    using namespace msim;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return MSIM_E_HIP;
    const uint32_t m = c->n;
    const WideGeom g = wide_geom(c->p.duration_ms);
    const size_t o_cf = 0, o_bkt = o_cf + 8 * ((size_t)m + 1), o_prop = (o_bkt + 2 * (size_t)WB_N + 7) / 8 * 8;
    const size_t o_log = o_prop + 8 * (size_t)m;
    const size_t o_jm = (o_log + sizeof(LogTab) + 255) / 256 * 256, o_jt = o_jm + 64 * 2048,
                 o_js = o_jt + 64 * 2048, total = o_js + 2048;
    std::lock_guard<std::mutex> lk(c->mu);
    void *d = nullptr;
    for (const auto &t : c->wtables)
        if (t.first == dev) d = t.second;
    if (!d) {
        std::vector<char> h(total, 0);
        std::vector<uint32_t> fthr(m);
        for (uint32_t k = 0; k < m; ++k) {
            fthr[k] = c->wprop[k] < (int64_t)FTHR_NEVER ? (uint32_t)c->wprop[k] : FTHR_NEVER;
            ((int64_t *)(h.data() + o_prop))[k] = c->wprop[k];
        }
        build_wide_pick(c->wperc.data(), fthr.data(), m, (uint32_t)c->total_weight, (uint64_t *)(h.data() + o_cf),
                        (uint16_t *)(h.data() + o_bkt));
        build_log_table((LogTab *)(h.data() + o_log));
        // jmain[l] = T^(l*S0); jtail[l] = T^(B0 + l*ST); jstep = T^(63*ST - 1)
        auto store = [](const Mat128 &mm, uint32_t *w) {
            for (int col = 0; col < 128; ++col) {
                w[4 * col + 0] = (uint32_t)mm.lo[col];
                w[4 * col + 1] = (uint32_t)(mm.lo[col] >> 32);
                w[4 * col + 2] = (uint32_t)mm.hi[col];
                w[4 * col + 3] = (uint32_t)(mm.hi[col] >> 32);
            }
        };
        build_jump_table(64, g.S0, (uint32_t *)(h.data() + o_jm));
        {
            Mat128 step, cur, tmp;
            mat_pow(g.B0, cur);
            mat_pow(g.ST, step);
            for (uint32_t l = 0; l < 64; ++l) {
                store(cur, (uint32_t *)(h.data() + o_jt) + (size_t)l * 512);
                mat_mul(step, cur, tmp);
                cur = tmp;
            }
            mat_pow(63ull * g.ST - 1, tmp);
            store(tmp, (uint32_t *)(h.data() + o_js));
        }
        if (hipMalloc(&d, total) != hipSuccess) return MSIM_E_HIP;
        if (hipMemcpy(d, h.data(), total, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            return MSIM_E_HIP;
        }
        c->wtables.push_back({dev, d});
    }
    const char *b = (const char *)d;
    a->cf = (const uint64_t *)(b + o_cf);
    a->bucket = (const uint16_t *)(b + o_bkt);
    a->prop = (const int64_t *)(b + o_prop);
    a->logt = (const LogTab *)(b + o_log);
    a->jmain = (const uint32_t *)(b + o_jm);
    a->jtail = (const uint32_t *)(b + o_jt);
    a->jstep = (const uint32_t *)(b + o_js);
    a->m = m;
    a->W = (uint32_t)c->total_weight;
    a->mult = 0xFFFFFFFFFFFFFFFFull / c->total_weight;
    a->D = c->p.duration_ms;
    a->S0 = g.S0;
    a->ST = g.ST;
    a->nch = g.nch;
    a->B0 = g.B0;
    return MSIM_OK;
}

// ---------------------------------------------------------------- entity-engine path (msim_sel_launch.h)
// E1 draws in-lane (SelFastDraw) for a single network and for sweeps alike; round 2's shared per-block word
// stream (D1) is gone: on MI355X the configs[3] grid (360 points x 8192 runs) ran 2.92 s in-lane vs 3.63 s
// reading the word stream (profiles/r03/sweep_b_*.txt).
struct SelWs {
    uint32_t nr;  // runs per slice (per point)
    uint32_t wpp, err_cap;
    size_t cold_lanes;
    size_t counts_off, partials_off, retry_off, list_off, cold_off, gen_off, total;
    msim::GenWs g;  // G, for the runs E2 cannot finish
};

// Workspace of the general engine: 512 MiB of windows when it only finishes other engines' runs, 2 GiB
// when it serves a whole network (msim_general_launch.h gen_tiers).
constexpr double GEN_FALLBACK_BUDGET = 512.0 * (1 << 20);
constexpr double GEN_BUDGET = 2048.0 * (1 << 20);

SelWs sel_ws_layout(uint32_t m, uint32_t np, uint64_t rpp, int64_t duration_ms, uint32_t max_nr = 1u << 22)
{
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    SelWs w;
    // one slice of every run (up to 2^22 runs per point: cold slots ~1.4 GiB)
    const uint64_t want = (rpp + 255) / 256 * 256;
    w.nr = (uint32_t)(want < max_nr ? want : max_nr);
    w.wpp = (uint32_t)((rpp + msim::TPB - 1) / msim::TPB);
    w.err_cap = (uint32_t)(rpp * np);  // every lane can be retried: the list never overflows
    const size_t nv = 6 * (size_t)m;
    w.counts_off = 0;
    w.partials_off = 256;
    w.retry_off = al(w.partials_off + (size_t)np * w.wpp * nv * 8);
    w.list_off = al(w.retry_off + (size_t)np * nv * 8);
    // cold slots: one set per E1 lane of a slice (every point x the slice's runs, rounded to whole
    // workgroups) and per E2 lane
    const size_t e1 = (size_t)np * ((w.nr + msim::TPB - 1) / msim::TPB) * msim::TPB;
    w.cold_lanes = e1 > w.err_cap ? e1 : (size_t)w.err_cap;
    w.cold_off = al(w.list_off + (size_t)w.err_cap * 4);
    w.gen_off = al(w.cold_off + w.cold_lanes * msim::SEL_NC * sizeof(msim::ColdAct));
    w.g = msim::gen_ws_layout(m, duration_ms, w.err_cap, GEN_FALLBACK_BUDGET, true);
    w.total = al(w.gen_off + w.g.total);
    return w;
}

// Geometry of the segment-parallel form (msim_selseg.h) for slices of nr runs: nseg segments of seg blocks
// covering mu + 8 sigma + 64 blocks (as K1, msim_pipeline.h), cut into whole rounds of SW's resident waves (five
// per SIMD); cap subs per (run, segment) = the expected cuts + 6 sigma + 16 (a run that exceeds it is
// recomputed by E2), qcap checkpoints (msim_sel_launch.h seg_qcap; measured on configs[2]: ~1 700 per year-long
// run, ~2/3 of the room; beyond it a worker just stores no more). Records [nr][nseg][cap], checkpoints
// [nr][nseg][qcap], counts [nseg][nr].
constexpr double SEG_MAX_RATE = 0.004;             // expected cuts per find above which E1 serves the network
constexpr double SEG_MIN_BLOCKS = 4096.0;          // shorter runs: E1
constexpr double SEG_BUDGET = 24.0 * (1ull << 30);  // records of one slice
struct SegLayout {
    uint32_t nr, nseg, seg, cap, qcap;
    size_t recs_off, cnt_off, qrecs_off, qcnt_off, total;
};
SegLayout seg_layout_nr(uint32_t m, double rate, int64_t duration_ms, uint32_t nr)
{
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    SegLayout L;
    L.nr = nr;
    const double mu = (double)duration_ms / 599999.5, sd = sqrt(mu > 1.0 ? mu : 1.0);
    const double need = mu + 8.0 * sd + 64.0;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const double slots = (double)cus * 4.0 * 5.0, rows = ceil(nr / 64.0);
    uint32_t best = 1;
    double bestf = 1e300;
    for (uint32_t w = 1; w <= 64; ++w) {
        const double sg = ceil(need / w);
        if (sg < 1024.0 && w > 1) break;
        const double f = ceil(rows * w / slots) * (sg + 25.0);
        if (f < bestf * 0.999) {
            bestf = f;
            best = w;
        }
    }
    if (const char *e = getenv("MSIM_SEG_NSEG")) best = (uint32_t)atoi(e) > 0 ? (uint32_t)atoi(e) : best;
    L.nseg = best;
    L.seg = (uint32_t)ceil(need / best);
    const double lam = rate * L.seg;
    L.cap = (uint32_t)ceil(lam + 6.0 * sqrt(lam) + 16.0);
    L.qcap = msim::seg_qcap((uint32_t)ceil(lam), L.seg);
    L.recs_off = 0;
    L.cnt_off = al((size_t)nr * L.nseg * L.cap * msim::seg_rec_bytes(m));
    L.qrecs_off = al(L.cnt_off + (size_t)L.nseg * nr * 4);
    L.qcnt_off = al(L.qrecs_off + (size_t)nr * L.nseg * L.qcap * msim::seg_qrec_bytes(m));
    L.total = al(L.qcnt_off + (size_t)L.nseg * nr * 4);
    return L;
}
// Runs per slice of the segment-parallel form: the records of one slice within SEG_BUDGET.
uint32_t seg_max_nr(uint32_t m, double rate, int64_t duration_ms, uint64_t n_runs)
{
    uint64_t nr = (n_runs + 255) / 256 * 256;
    if (nr > (1u << 22)) nr = 1u << 22;
    for (;;) {  // the geometry depends on the slice size: shrink until one slice's records fit the budget
        const SegLayout L = seg_layout_nr(m, rate, duration_ms, (uint32_t)nr);
        if ((double)L.total <= SEG_BUDGET || nr <= 256) return (uint32_t)nr;
        uint64_t next = (uint64_t)((double)nr * SEG_BUDGET / (double)L.total * 0.98) / 256 * 256;
        nr = next >= nr ? nr - 256 : (next < 256 ? 256 : next);
    }
}

// The E1 workspace of a single-network launch, plus the segment-parallel form's records when it serves the config.
struct SelCfgWs {
    SelWs w;
    bool seg;
    SegLayout L;
    size_t total;
};
SelCfgWs sel_cfg_layout(const msim_config *cfg, uint64_t n_runs)
{
    SelCfgWs c;
    c.seg = cfg->seg_ok;
    const uint32_t max_nr = c.seg ? seg_max_nr(cfg->n, cfg->seg_rate, cfg->p.duration_ms, n_runs) : (1u << 22);
    c.w = sel_ws_layout(cfg->n, 1, n_runs, cfg->p.duration_ms, max_nr);
    c.total = c.w.total;
    if (c.seg) {
        c.L = seg_layout_nr(cfg->n, cfg->seg_rate, cfg->p.duration_ms, c.w.nr);
        c.total += c.L.total;
    }
    return c;
}

#ifndef MSIM_XTH_MID
#define MSIM_XTH_MID 32  // engine-phase threshold for delays of 2-10 s (build_sel_params)
#endif
#ifndef MSIM_XTH_HI
#define MSIM_XTH_HI 48  // and above 10 s
#endif

// One SelParams for a validated network (weights summing to W, <= MSIM_MAX_MINERS miners).
void build_sel_params(const msim_miner *miners, uint32_t n, int64_t duration_ms, uint64_t W, msim::SelParams *sp)
{
    using namespace msim;
    memset(sp, 0, sizeof(*sp));
    sp->duration_ms = duration_ms;
    sp->W = (uint32_t)W;
    sp->mult = 0xFFFFFFFFFFFFFFFFull / W;
    sp->m = n;
    for (int i = 0; i < SEL_MAXS; ++i) sp->sids[i] = SEL_NONE;
    uint64_t c = 0;
    for (uint32_t k = 0; k < n; ++k) {
        c += miners[k].perc;
        sp->cum[k] = c;
        sp->prop[k] = miners[k].propagation_ms;
        if (miners[k].is_selfish) sp->sids[sp->ns++] = k;
    }
    for (int k = 0; k < MAXM; ++k)
        sp->ccum[k] = (uint32_t)k < n ? (W == 100 ? (uint32_t)sp->cum[k] : (uint32_t)k + 1u) : 0xFFFFFFFFu;
    sp->uniform_prop = 1;
    for (uint32_t k = 1; k < n; ++k)
        if (miners[k].propagation_ms != miners[0].propagation_ms) sp->uniform_prop = 0;
    sp->macro = sp->ns == 1 ? 1u : 0u;
    for (uint32_t k = 0; k < n; ++k)
        if (miners[k].propagation_ms < 1) sp->macro = 0;
    if (getenv("MSIM_SEL_NO_MACRO")) sp->macro = 0;  // A/B switch: the entity engine for every find
    // Engine phases start when this many lanes of a wave wait. Long delays send more finds to the engine,
    // and larger batches then pay (measured on MI355X, SEL_XTH A/B: configs[2] at 1 s fastest with 16, the
    // configs[3] grid up to 30 s with 32; profiles/r02/xth_v.txt).
    int64_t pmax = 0;
    for (uint32_t k = 0; k < n; ++k) pmax = miners[k].propagation_ms > pmax ? miners[k].propagation_ms : pmax;
    sp->xth = pmax <= 2000 ? 16u : (pmax <= 10000 ? (uint32_t)MSIM_XTH_MID : (uint32_t)MSIM_XTH_HI);
    if (const char *e = getenv("MSIM_SEL_XTH")) sp->xth = (uint32_t)atoi(e);  // A/B override
}

struct SelGroupDev {
    uint32_t nscls, nlist;
    const uint32_t *plist;
    uint32_t uni;  // every point of the group has a uniform propagation delay
};

// The segment-parallel form's device arguments for one launch (msim_selseg.h).
struct SegPlan {
    msim::SegArgs g;
};

// The slice loop of one launch: E1 per group (or SW + ST for a single network the segment-parallel form serves)
// -> E2 (retries) -> G (what E2 cannot finish) -> F.
int sel_launch_impl(uint32_t m, uint32_t np, const msim::SelParams *d_pts, const msim::GenParams *d_gpts,
                    const std::vector<SelGroupDev> &groups, const msim::LogTab *logt, const SelWs &w, char *ws,
                    uint64_t run_begin, uint64_t rpp, uint32_t seed_base, void *d_sums, void *d_per_run,
                    void *d_best_height, void *d_status, hipStream_t s, std::vector<hipEvent_t> *engine_events,
                    const SegPlan *seg = nullptr)
{
    using namespace msim;
    uint32_t *counts = (uint32_t *)(ws + w.counts_off);
    uint64_t *retry = (uint64_t *)(ws + w.retry_off);
    if (hipMemsetAsync(counts, 0, msim::GEN_C_WORDS * sizeof(uint32_t), s) != hipSuccess ||
        hipMemsetAsync(retry, 0, (size_t)np * 6 * m * 8, s) != hipSuccess)
        return MSIM_E_HIP;
    char *gws = ws + w.gen_off;
    uint32_t *gen_first = (uint32_t *)(gws + w.g.lists_off) + 2 * (size_t)w.g.list_cap;
    SelArgs a;
    a.pts = d_pts;
    a.rpp = (uint32_t)rpp;
    a.wpp = w.wpp;
    a.run_begin = run_begin;
    a.seed_base = seed_base;
    a.logt = logt;
    a.partials = (uint64_t *)(ws + w.partials_off);
    a.retry_sums = retry;
    a.records = (uint32_t *)d_per_run;
    a.best_h = (uint32_t *)d_best_height;
    a.counts = counts;
    a.err_list = (uint32_t *)(ws + w.list_off);
    a.err_cap = w.err_cap;
    a.force_retry = getenv("MSIM_SEL_FORCE_RETRY") != nullptr ? 1u : 0u;
    a.cold = (ColdAct *)(ws + w.cold_off);
    a.cold_lanes = w.cold_lanes;
    a.gen_list = gen_first;
    a.force_gen = getenv("MSIM_SEL_FORCE_GEN") != nullptr ? 1u : 0u;
    auto event = [&](std::vector<hipEvent_t> *v) -> hipEvent_t {
        hipEvent_t e = nullptr;
        if (v && hipEventCreate(&e) == hipSuccess) {
            v->push_back(e);
            (void)hipEventRecord(e, s);
        }
        return e;
    };
    uint32_t max_ns = 1;
    for (const auto &g : groups) max_ns = g.nscls > max_ns ? g.nscls : max_ns;
    for (uint64_t s0 = 0; s0 < rpp; s0 += w.nr) {
        const uint32_t sn = (uint32_t)((rpp - s0) < w.nr ? (rpp - s0) : w.nr);
        a.s0 = (uint32_t)s0;
        a.sn = sn;
        event(engine_events);
        if (seg) {  // one network: SW over (run, segment), then ST per run
            a.plist = groups[0].plist;
            a.nlist = 1;
            a.uni = groups[0].uni;
            if (launch_segwork(a, seg->g, m, s) != hipSuccess || launch_stitch(a, seg->g, m, s) != hipSuccess)
                return MSIM_E_HIP;
        }
        for (const auto &g : groups) {
            if (!g.nlist || seg) continue;
            a.plist = g.plist;
            a.nlist = g.nlist;
            a.uni = g.uni;
            if (launch_sel(a, m, g.nscls, s) != hipSuccess) return MSIM_E_HIP;
        }
        event(engine_events);
    }
    a.s0 = 0;
    a.sn = 0;
    if (launch_sel_retry(a, m, max_ns, s) != hipSuccess) return MSIM_E_HIP;
    GenArgs ga;
    memset(&ga, 0, sizeof(ga));
    ga.pts = d_gpts;
    ga.rpp = (uint32_t)rpp;
    ga.max_m = m;
    ga.run_begin = run_begin;
    ga.seed_base = seed_base;
    ga.sums = retry;
    ga.records = (uint32_t *)d_per_run;
    ga.best_h = (uint32_t *)d_best_height;
    ga.counts = counts;
    if (launch_gen_tiers(ga, w.g, gws, gen_first, counts + GEN_C_L1, 0, s) != hipSuccess) return MSIM_E_HIP;
    if (launch_sel_finalize(a.partials, np, w.wpp, 6 * m, retry, (uint64_t *)d_sums, counts, (uint32_t *)d_status, s) !=
        hipSuccess)
        return MSIM_E_HIP;
    return MSIM_OK;
}

// Device GenParams of a list of networks (one per point) and their weight / delay / selfish arrays, in one
// allocation whose pointers are device addresses.
int gen_tables_upload(const std::vector<const GenHost *> &hs, void **out)
{
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t np = hs.size();
    size_t off = al(np * sizeof(msim::GenParams));
    std::vector<size_t> o(np);
    for (size_t i = 0; i < np; ++i) {
        o[i] = off;
        off = al(off + hs[i]->w.size() * 21);
    }
    std::vector<char> h(off, 0);
    void *d = nullptr;
    if (hipMalloc(&d, off) != hipSuccess) return MSIM_E_HIP;
    for (size_t i = 0; i < np; ++i) {
        const GenHost &g = *hs[i];
        const size_t m = g.w.size();
        uint64_t *cum = (uint64_t *)(h.data() + o[i]);
        int64_t *prop = (int64_t *)(h.data() + o[i] + 8 * m);
        uint32_t *cls = (uint32_t *)(h.data() + o[i] + 16 * m);
        uint8_t *self = (uint8_t *)(h.data() + o[i] + 20 * m);
        std::vector<uint32_t> cv;
        uint32_t umax = msim::GEN_GENESIS;
        gen_id_classes(g.ids, cv, &umax);
        uint64_t c = 0;
        for (size_t k = 0; k < m; ++k) {
            cum[k] = (c += g.w[k]);
            prop[k] = g.prop[k];
            cls[k] = cv[k];
            self[k] = g.self[k];
        }
        msim::GenParams *gp = (msim::GenParams *)h.data() + i;
        gp->duration_ms = g.duration_ms;
        gp->mult = 0xFFFFFFFFFFFFFFFFull / g.W;
        gp->m = (uint32_t)m;
        gp->umax = umax;
        gp->cum = (const uint64_t *)((char *)d + o[i]);
        gp->prop = (const int64_t *)((char *)d + o[i] + 8 * m);
        gp->cls = (const uint32_t *)((char *)d + o[i] + 16 * m);
        gp->self = (const uint8_t *)((char *)d + o[i] + 20 * m);
    }
    if (hipMemcpy(d, h.data(), off, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return MSIM_E_HIP;
    }
    *out = d;
    return MSIM_OK;
}

// The per-device copy of a table list (lazily uploaded, cached under `mu`).
int gen_cached(std::mutex &mu, std::vector<std::pair<int, void *>> &cache, const std::vector<const GenHost *> &hs,
               const msim::GenParams **out)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return MSIM_E_HIP;
    std::lock_guard<std::mutex> g(mu);
    for (const auto &t : cache)
        if (t.first == dev) {
            *out = (const msim::GenParams *)t.second;
            return MSIM_OK;
        }
    void *d = nullptr;
    const int rc = gen_tables_upload(hs, &d);
    if (rc) return rc;
    cache.push_back({dev, d});
    *out = (const msim::GenParams *)d;
    return MSIM_OK;
}

// Workspace of a launch served by the general engine alone: counters, then G's lists and windows.
struct GenOnlyWs {
    msim::GenWs g;
    size_t gen_off, total;
};
GenOnlyWs gen_only_layout(uint32_t m, uint32_t np, uint64_t rpp, int64_t duration_ms, bool selfish)
{
    GenOnlyWs w;
    w.g = msim::gen_ws_layout(m, duration_ms, (uint32_t)(rpp * np), GEN_BUDGET, selfish);
    w.gen_off = 256;
    w.total = w.gen_off + w.g.total;
    return w;
}

// Every run of every point on G: codes point * rpp + rel, tier 1 over the whole range.
int gen_launch_impl(uint32_t m, uint32_t np, const msim::GenParams *d_gpts, const GenOnlyWs &w, char *ws,
                    uint64_t run_begin, uint64_t rpp, uint32_t seed_base, void *d_sums, void *d_per_run,
                    void *d_best_height, void *d_status, hipStream_t s)
{
    using namespace msim;
    uint32_t *counts = (uint32_t *)ws;
    if (hipMemsetAsync(counts, 0, GEN_C_WORDS * sizeof(uint32_t), s) != hipSuccess ||
        hipMemsetAsync(d_sums, 0, (size_t)np * 6 * m * 8, s) != hipSuccess)
        return MSIM_E_HIP;
    GenArgs ga;
    memset(&ga, 0, sizeof(ga));
    ga.pts = d_gpts;
    ga.rpp = (uint32_t)rpp;
    ga.max_m = m;
    ga.run_begin = run_begin;
    ga.seed_base = seed_base;
    ga.sums = (uint64_t *)d_sums;
    ga.records = (uint32_t *)d_per_run;
    ga.best_h = (uint32_t *)d_best_height;
    ga.counts = counts;
    if (launch_gen_tiers(ga, w.g, ws + w.gen_off, nullptr, nullptr, (uint32_t)(rpp * np), s) != hipSuccess ||
        launch_gen_status(counts, (uint32_t *)d_status, s) != hipSuccess)
        return MSIM_E_HIP;
    return MSIM_OK;
}

// Device copy of a config's SelParams and the point list {0}.
int sel_config_tables(msim_config *c, const msim::SelParams **pts, const uint32_t **plist)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return MSIM_E_HIP;
    std::lock_guard<std::mutex> g(c->mu);
    void *d = nullptr;
    for (const auto &t : c->stables)
        if (t.first == dev) d = t.second;
    const size_t pb = (sizeof(msim::SelParams) + 255) / 256 * 256;
    if (!d) {
        std::vector<char> h(pb + 256, 0);
        memcpy(h.data(), &c->sp, sizeof(msim::SelParams));
        if (hipMalloc(&d, h.size()) != hipSuccess) return MSIM_E_HIP;
        if (hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            return MSIM_E_HIP;
        }
        c->stables.push_back({dev, d});
    }
    *pts = (const msim::SelParams *)d;
    *plist = (const uint32_t *)((const char *)d + pb);
    return MSIM_OK;
}

// Validate a miner list with integer weights summing to total_weight and build the config.
int config_create_impl(const msim_miner *miners, uint32_t n, int64_t duration_ms, uint64_t total_weight,
                       msim_config **out)
{
    if (!miners || !out || n == 0 || duration_ms < 0 || total_weight == 0) return MSIM_E_INVALID;
    if (total_weight >= (1ull << 31)) return MSIM_E_WEIGHTS;
    // Ids only name a block's creator (simulation.h:22-38); the fast engines count blocks per miner INDEX,
    // which is the reference's per-id count exactly when every id is distinct and none is Genesis's id
    // UINT_MAX (simulation.h:31-33). Any other network (two miners sharing an id: shared blocks, stale
    // counting and found counts, main.cpp:24-26, simulation.h:133; an id UINT_MAX: Genesis counted as its
    // block) runs on the general engine, whose chains hold id classes (msim_general.h).
    bool id_quirk = false;
    {
        std::vector<uint32_t> ids(n);
        for (uint32_t k = 0; k < n; ++k) ids[k] = miners[k].id;
        std::sort(ids.begin(), ids.end());
        for (uint32_t k = 1; k < n; ++k) id_quirk = id_quirk || ids[k] == ids[k - 1];
        id_quirk = id_quirk || ids[n - 1] == 0xFFFFFFFFu;
    }
    uint64_t total = 0;
    uint32_t nself = 0;
    for (uint32_t k = 0; k < n; ++k) {
        if (miners[k].propagation_ms < 0) return MSIM_E_INVALID;
        if (miners[k].perc > total_weight) return MSIM_E_WEIGHTS;
        total += miners[k].perc;
        nself += miners[k].is_selfish ? 1u : 0u;
    }
    // "Must add up to 1" (main.cpp:43); anything else makes PickFinder assert (simulation.h:220).
    if (total != total_weight) return MSIM_E_WEIGHTS;
    // Selfish miners run on the entity engine (msim_sel.h): up to SEL_MAXS of them, in networks of up to
    // MSIM_MAX_MINERS miners with any integer weights. The large-network path is honest-only.
    // The entity engine takes up to SEL_MAXS selfish miners in networks of up to MSIM_MAX_MINERS miners; any
    // other network with selfish miners runs on the general engine (msim_general.h), as does any network when
    // MSIM_FORCE_GENERAL is set (test switch).
    // Honest networks of more than WIDE_MAX_M miners (beyond the large-network pipeline's LDS tables) also
    // run on G.
    const bool gen = nself > (uint32_t)msim::SEL_MAXS || (nself && n > MSIM_MAX_MINERS) || id_quirk ||
                     n > msim::WIDE_MAX_M || getenv("MSIM_FORCE_GENERAL") != nullptr;
    // G holds every miner's explicit chain: one lane of its last window must fit (msim_general_launch.h).
    int64_t max_prop = 0;
    for (uint32_t k = 0; k < n; ++k) max_prop = miners[k].propagation_ms > max_prop ? miners[k].propagation_ms : max_prop;
    const bool gen_full = msim::gen_needs_full(nself > 0, max_prop);
    if (gen && !msim::gen_fits(n, duration_ms, gen_full)) return MSIM_E_MINERS;
    const bool sel = nself > 0 && !gen;
    const bool narrow = n <= MSIM_MAX_MINERS && (total_weight == 100 || sel);
    const bool force_wide = getenv("MSIM_FORCE_WIDE") != nullptr && nself == 0;
    msim_config *c = new (std::nothrow) msim_config();
    if (!c) return MSIM_E_INVALID;
    c->n = n;
    c->total_weight = total_weight;
    c->general = gen;
    c->selfish = nself > 0;
    c->gen_full = gen_full;
    c->gh.duration_ms = duration_ms;
    c->gh.W = total_weight;
    for (uint32_t k = 0; k < n; ++k) {
        c->gh.w.push_back(miners[k].perc);
        c->gh.prop.push_back(miners[k].propagation_ms);
        c->gh.self.push_back(miners[k].is_selfish ? 1 : 0);
        c->gh.ids.push_back(miners[k].id);
    }
    c->p.duration_ms = duration_ms;
    c->p.m = (int32_t)n;
    c->p.selfish = -1;
    double rho = 0.0;
    for (uint32_t k = 0; k < n; ++k)
        rho += (double)miners[k].perc / (double)total_weight *
               (miners[k].is_selfish ? 1.0 : 1.0 - exp(-((double)miners[k].propagation_ms + 1.0) / 599999.5));
    c->rho = rho;
    if (gen && !narrow) {
        // G alone: nothing else to prepare (its tables are uploaded on first launch)
        c->pipe_ok = false;
    } else if (narrow && !force_wide) {
        for (uint32_t k = 0; k < n; ++k) {
            c->ids[k] = miners[k].id;
            c->perc[k] = miners[k].perc;
            c->prop[k] = miners[k].propagation_ms;
            c->self[k] = miners[k].is_selfish ? 1 : 0;
        }
        if (sel) {
            c->sel = true;
            build_sel_params(miners, n, duration_ms, total_weight, &c->sp);
            if (c->sp.macro && c->sp.ns == 1) {  // expected cuts per find (msim_selseg.h): honest finds that may
                const uint32_t sid = c->sp.sids[0];  // need the engine (next find within prop_k + prop_s)
                double rate = 0.0;
                for (uint32_t k = 0; k < n; ++k)
                    if (k != sid)
                        rate += (double)miners[k].perc / (double)total_weight *
                                (1.0 - exp(-((double)miners[k].propagation_ms + (double)miners[sid].propagation_ms + 1.0) /
                                           599999.5));
                c->seg_rate = rate;
                // opt-in (MSIM_SELSEG=1): exact, but slower than E1 on configs[2]
                c->seg_ok = rate <= SEG_MAX_RATE && (double)duration_ms / 599999.5 >= SEG_MIN_BLOCKS &&
                            getenv("MSIM_SELSEG") != nullptr;
            }
            c->p.duration_ms = duration_ms;
            c->p.m = (int32_t)n;
            c->p.selfish = (int32_t)c->sp.sids[0];
            for (int k = 0; k < msim::MAXM; ++k) {
                c->p.prop[k] = k < (int)n ? miners[k].propagation_ms : 0;
                c->p.thresh[k] = ~0ull;
            }
        } else if (gen) {
            c->p.m = (int32_t)n;
        } else {
            const int rc = msim::make_params(c->perc, c->prop, c->self, (int)n, duration_ms, &c->p);
            if (rc) {
                delete c;
                return rc == -3 ? MSIM_E_SELFISH : (rc == -2 ? MSIM_E_WEIGHTS : MSIM_E_INVALID);
            }
        }
        // the draw kernel's fast threshold holds delays below FTHR_CAP (262 s; msim_fastdraw.h)
        bool prop_ok = true;
        for (uint32_t k = 0; k < n; ++k) prop_ok = prop_ok && miners[k].propagation_ms < (int64_t)msim::FTHR_CAP;
        c->pipe_ok = !sel && !gen && prop_ok && rho <= PIPE_MAX_RHO && getenv("MSIM_NO_PIPELINE") == nullptr;
    } else {
        c->wide = true;
        c->pipe_ok = false;
        c->wids.resize(n);
        c->wperc.resize(n);
        c->wprop.resize(n);
        for (uint32_t k = 0; k < n; ++k) {
            c->wids[k] = miners[k].id;
            c->wperc[k] = miners[k].perc;
            c->wprop[k] = miners[k].propagation_ms;
        }
        const msim::WideLayout L = wide_layout(c, 1);
        if (msim::wide_w3_lds(n, L.rcap, L.g.nch) > 160 * 1024) c->general = true;  // fork rate too high for W3
    }
    *out = c;
    return MSIM_OK;
}

int launch_wide_cfg(const msim_config *cfg, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base, void *d_sums,
                    void *d_per_run, void *d_best_height, void *d_status, void *d_workspace, size_t workspace_bytes,
                    void *stream, std::vector<hipEvent_t> *w1_events)
{
    const msim::WideLayout L = wide_layout(cfg, n_runs);
    const size_t head = 256;
    if (workspace_bytes < head + L.total) return MSIM_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    char *ws = (char *)d_workspace;
    uint32_t *counts = (uint32_t *)ws;
    if (hipMemsetAsync(counts, 0, 2 * sizeof(uint32_t), s) != hipSuccess ||
        hipMemsetAsync(d_sums, 0, 6 * sizeof(uint64_t) * cfg->n, s) != hipSuccess)
        return MSIM_E_HIP;
    msim::WideArgs a;
    int rc = wide_tables(const_cast<msim_config *>(cfg), &a);
    if (rc) return rc;
    a.seed_base = seed_base;
    a.rcap = L.rcap;
    msim::WideOut o;
    o.sums = (uint64_t *)d_sums;
    o.records = (uint32_t *)d_per_run;
    o.best_h = (uint32_t *)d_best_height;
    o.fail = counts + 1;
    o.run_begin = run_begin;
    o.n_total = n_runs;
    o.rel_begin = 0;
    if (msim::launch_wide(a, L, ws + head, o, s, w1_events) != hipSuccess) return MSIM_E_HIP;
    if (d_status && hipMemcpyAsync(d_status, counts, 2 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s) != hipSuccess)
        return MSIM_E_HIP;
    return MSIM_OK;
}

}  // namespace

extern "C" {

int msim_config_create(const msim_miner *miners, uint32_t n, int64_t duration_ms, msim_config **out)
{
    return config_create_impl(miners, n, duration_ms, 100u, out);
}

int msim_config_create_weighted(const msim_miner *miners, uint32_t n, int64_t duration_ms, uint64_t total_weight,
                                msim_config **out)
{
    return config_create_impl(miners, n, duration_ms, total_weight, out);
}

int msim_config_is_wide(const msim_config *cfg) { return cfg && cfg->wide ? 1 : 0; }

int msim_config_set_concurrent_launches(msim_config *cfg, uint32_t n)
{
    if (!cfg || n < 1 || n > 64) return MSIM_E_INVALID;
    std::lock_guard<std::mutex> g(cfg->mu);
    cfg->jobs = n;
    return MSIM_OK;
}

void msim_config_destroy(msim_config *cfg)
{
    if (!cfg) return;
    for (const auto &t : cfg->tables) (void)hipFree(t.ptr);
    for (const auto &t : cfg->wtables) (void)hipFree(t.second);
    for (const auto &t : cfg->stables) (void)hipFree(t.second);
    for (const auto &t : cfg->gtables) (void)hipFree(t.second);
    delete cfg;
}

uint32_t msim_config_miner_count(const msim_config *cfg) { return cfg ? cfg->n : 0; }

size_t msim_workspace_bytes(const msim_config *cfg, uint64_t n_runs)
{
    if (!cfg || n_runs == 0 || n_runs > MAX_LAUNCH_RUNS) return 0;
    if (cfg->general) return gen_only_layout(cfg->n, 1, n_runs, cfg->p.duration_ms, cfg->gen_full).total;
    if (cfg->wide) return 256 + wide_layout(cfg, n_runs).total;
    if (cfg->sel)
        return sel_cfg_layout(cfg, n_runs).total;
    size_t t = ws_layout(cfg->n, n_runs).total;
    if (cfg->pipe_ok) t += pipe_layout(cfg, n_runs).total;
    return t;
}

int msim_launch(const msim_config *cfg, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base, void *d_sums,
                void *d_per_run, void *d_best_height, void *d_status, void *d_workspace, size_t workspace_bytes,
                void *stream)
{
    if (!cfg || !d_sums || !d_status || !d_workspace || n_runs == 0 || n_runs > MAX_LAUNCH_RUNS) return MSIM_E_INVALID;
    if (cfg->general) {
        const GenOnlyWs w = gen_only_layout(cfg->n, 1, n_runs, cfg->p.duration_ms, cfg->gen_full);
        if (workspace_bytes < w.total) return MSIM_E_INVALID;
        msim_config *c = const_cast<msim_config *>(cfg);
        const msim::GenParams *gp = nullptr;
        int rc = gen_cached(c->mu, c->gtables, {&cfg->gh}, &gp);
        if (rc) return rc;
        Timing &tm = timing();
        std::unique_lock<std::mutex> lk(tm.mu);
        hipEvent_t lb = nullptr, le = nullptr;
        hipStream_t s = (hipStream_t)stream;
        if (tm.on) {
            if (hipEventCreate(&lb) == hipSuccess && hipEventCreate(&le) == hipSuccess) {
                tm.launch.push_back(lb);
                tm.launch.push_back(le);
                (void)hipEventRecord(lb, s);
            }
            tm.launches++;
        } else {
            lk.unlock();
        }
        rc = gen_launch_impl(cfg->n, 1, gp, w, (char *)d_workspace, run_begin, n_runs, seed_base, d_sums, d_per_run,
                             d_best_height, d_status, s);
        if (le) (void)hipEventRecord(le, s);
        return rc;
    }
    if (cfg->wide) {
        Timing &tm = timing();
        std::unique_lock<std::mutex> lk(tm.mu);
        hipEvent_t lb = nullptr, le = nullptr;
        std::vector<hipEvent_t> *w1 = nullptr;
        if (tm.on) {
            w1 = &tm.k1;
            if (hipEventCreate(&lb) == hipSuccess && hipEventCreate(&le) == hipSuccess) {
                tm.launch.push_back(lb);
                tm.launch.push_back(le);
                (void)hipEventRecord(lb, (hipStream_t)stream);
            }
            tm.launches++;
        } else {
            lk.unlock();
        }
        const int rc = launch_wide_cfg(cfg, run_begin, n_runs, seed_base, d_sums, d_per_run, d_best_height, d_status,
                                       d_workspace, workspace_bytes, stream, w1);
        if (le) (void)hipEventRecord(le, (hipStream_t)stream);
        return rc;
    }
    if (cfg->sel) {
        const SelCfgWs cw = sel_cfg_layout(cfg, n_runs);
        const SelWs &w = cw.w;
        if (workspace_bytes < cw.total) return MSIM_E_INVALID;
        msim_config *c = const_cast<msim_config *>(cfg);
        SegPlan plan;
        if (cw.seg) {  // the segment-parallel form: jump matrices for offsets j * seg, records after E1's workspace
            msim::PipeTables tab;
            const int rt = device_tables(c, cw.L.seg, cw.L.nseg, &tab);
            if (rt) return rt;
            plan.g.jump = tab.jump;
            plan.g.recs = (char *)d_workspace + w.total + cw.L.recs_off;
            plan.g.cnt = (uint32_t *)((char *)d_workspace + w.total + cw.L.cnt_off);
            plan.g.qrecs = (char *)d_workspace + w.total + cw.L.qrecs_off;
            plan.g.qcnt = (uint32_t *)((char *)d_workspace + w.total + cw.L.qcnt_off);
            plan.g.nr = cw.L.nr;
            plan.g.nseg = cw.L.nseg;
            plan.g.seg = cw.L.seg;
            plan.g.cap = cw.L.cap;
            plan.g.qcap = cw.L.qcap;
            plan.g.xth = 16;
            if (const char *e = getenv("MSIM_SEG_XTH")) plan.g.xth = (uint32_t)atoi(e);
        }
        const msim::SelParams *pts = nullptr;
        const uint32_t *plist = nullptr;
        int rc = sel_config_tables(c, &pts, &plist);
        if (rc) return rc;
        const msim::GenParams *gp = nullptr;
        rc = gen_cached(c->mu, c->gtables, {&cfg->gh}, &gp);
        if (rc) return rc;
        const msim::LogTab *lt = nullptr;
        rc = global_log_table(&lt);
        if (rc) return rc;
        std::vector<SelGroupDev> groups{{msim::sel_ns_class(cfg->sp.ns), 1u, plist, cfg->sp.uniform_prop != 0 ? 1u : 0u}};
        Timing &tm = timing();
        std::unique_lock<std::mutex> lk(tm.mu);
        hipEvent_t lb = nullptr, le = nullptr;
        hipStream_t s = (hipStream_t)stream;
        const bool on = tm.on;
        if (on) {
            if (hipEventCreate(&lb) == hipSuccess && hipEventCreate(&le) == hipSuccess) {
                tm.launch.push_back(lb);
                tm.launch.push_back(le);
                (void)hipEventRecord(lb, s);
            }
            tm.launches++;
        } else {
            lk.unlock();
        }
        rc = sel_launch_impl(cfg->n, 1, pts, gp, groups, lt, w, (char *)d_workspace, run_begin, n_runs, seed_base, d_sums,
                             d_per_run, d_best_height, d_status, s, on ? &tm.engine : nullptr, cw.seg ? &plan : nullptr);
        if (le) (void)hipEventRecord(le, s);
        return rc;
    }
    const WsLayout l = ws_layout(cfg->n, n_runs);
    msim::PipeLayout pl;
    if (cfg->pipe_ok) pl = pipe_layout(cfg, n_runs);
    if (workspace_bytes < l.total + (cfg->pipe_ok ? pl.total : 0)) return MSIM_E_INVALID;
    char *ws = (char *)d_workspace;
    hipStream_t s = (hipStream_t)stream;
    uint32_t *counts = (uint32_t *)(ws + l.counts_off);
    if (hipMemsetAsync(counts, 0, 2 * sizeof(uint32_t), s) != hipSuccess) return MSIM_E_HIP;
    msim::LaunchArgs a;
    a.p = cfg->p;
    a.run_begin = run_begin;
    a.n = (uint32_t)n_runs;
    a.seed_base = seed_base;
    a.partials = (uint64_t *)(ws + l.partials_off);
    a.sums = (uint64_t *)d_sums;
    a.records = (uint32_t *)d_per_run;
    a.best_h = (uint32_t *)d_best_height;
    a.err_count = counts;
    a.fail_count = counts + 1;
    a.err_list = (uint32_t *)(ws + l.list_off);
    a.err_cap = l.err_cap;
    a.status = (uint32_t *)d_status;
    a.stream = s;
    a.pl = nullptr;
    a.pipe_ws = nullptr;
    a.k1_events = nullptr;
    if (cfg->pipe_ok) {
        const int rc = device_tables(const_cast<msim_config *>(cfg), pl.seg, pl.nseg, &a.tab);
        if (rc) return rc;
        a.pl = &pl;
        a.pipe_ws = ws + l.total;
    }
    Timing &tm = timing();
    std::unique_lock<std::mutex> lk(tm.mu);
    hipEvent_t lb = nullptr, le = nullptr;
    if (tm.on) {
        a.k1_events = &tm.k1;
        if (hipEventCreate(&lb) == hipSuccess && hipEventCreate(&le) == hipSuccess) {
            tm.launch.push_back(lb);
            tm.launch.push_back(le);
            (void)hipEventRecord(lb, s);
        }
        tm.launches++;
    } else {
        lk.unlock();
    }
    const int rc = msim::launch_runs(a) == hipSuccess ? MSIM_OK : MSIM_E_HIP;
    if (le) (void)hipEventRecord(le, s);
    return rc;
}

int msim_device_log1p(const double *d_x, double *d_out, uint64_t n, void *stream)
{
    if (!d_x || !d_out) return MSIM_E_INVALID;
    return msim::launch_log1p(d_x, d_out, n, (hipStream_t)stream) == hipSuccess ? MSIM_OK : MSIM_E_HIP;
}

int msim_device_intervals(const uint64_t *d_uniform, int64_t *d_out_ms, uint64_t n, void *stream)
{
    if (!d_uniform || !d_out_ms) return MSIM_E_INVALID;
    const msim::LogTab *lt = nullptr;
    const int rc = global_log_table(&lt);
    if (rc) return rc;
    return msim::launch_intervals(lt, d_uniform, d_out_ms, n, (hipStream_t)stream) == hipSuccess ? MSIM_OK : MSIM_E_HIP;
}

int msim_device_picks(const msim_config *cfg, const uint64_t *d_uniform, int32_t *d_out_index, uint64_t n, void *stream)
{
    if (!cfg || !d_uniform || !d_out_index) return MSIM_E_INVALID;
    if (cfg->wide) {
        msim::WideArgs a;
        const int rc = wide_tables(const_cast<msim_config *>(cfg), &a);
        if (rc) return rc;
        return msim::launch_wide_picks(a, d_uniform, d_out_index, n, (hipStream_t)stream) == hipSuccess ? MSIM_OK
                                                                                                         : MSIM_E_HIP;
    }
    msim::PipeTables t;
    const msim::PipeLayout pl = pipe_layout(cfg, 1);
    const int rc = device_tables(const_cast<msim_config *>(cfg), pl.seg, pl.nseg, &t);
    if (rc) return rc;
    return msim::launch_picks(t.pick, d_uniform, d_out_index, n, (hipStream_t)stream) == hipSuccess ? MSIM_OK : MSIM_E_HIP;
}

// A Q32.32 sum held as two limbs -> double with ONE rounding of the exact value (hi << 32) + lo, so the
// result does not depend on how runs were split into workgroups, slices, launches or ranks (each split
// moves value between the limbs but never changes the exact sum).
static double fx_value(uint64_t hi, uint64_t lo)
{
    const unsigned __int128 v = ((unsigned __int128)hi << 32) + lo;
    return (double)v * 0x1.0p-32;
}

void msim_sums_to_stats(const msim_sums *sums, uint32_t n, msim_stats *out)
{
    for (uint32_t k = 0; k < n; ++k) {
        out[k].blocks_found = sums[k].blocks_found;
        out[k].blocks_share = fx_value(sums[k].share_hi, sums[k].share_lo);
        out[k].stale_rate = fx_value(sums[k].rate_hi, sums[k].rate_lo);
    }
}

// Whether a workspace of `bytes` fits the current device's free memory (hipMemGetInfo).
static bool workspace_fits(size_t bytes)
{
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return true;  // let the allocation report it
    return bytes <= fr;
}

int msim_run(const msim_config *cfg, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base, int device,
             msim_stats *out_sums, msim_sums *opt_sums, msim_run_record *opt_per_run, uint32_t *opt_best_height)
{
    if (!cfg || !out_sums || n_runs == 0) return MSIM_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return MSIM_E_HIP;
    const uint32_t m = cfg->n;
    const uint64_t chunk = n_runs < MAX_LAUNCH_RUNS ? n_runs : MAX_LAUNCH_RUNS;
    const size_t wsb = msim_workspace_bytes(cfg, chunk);
    void *ws = nullptr, *sums = nullptr, *status = nullptr, *rec = nullptr, *bh = nullptr;
    const bool want_rec = opt_per_run != nullptr;
    const bool want_bh = want_rec || opt_best_height != nullptr;
    int rc = MSIM_OK;
    std::vector<uint32_t> bh_host;
    if (want_rec && !opt_best_height) bh_host.resize(n_runs);
    uint32_t *bh_out = opt_best_height ? opt_best_height : (want_rec ? bh_host.data() : nullptr);
    std::vector<uint64_t> acc(6 * (size_t)m, 0), part(6 * (size_t)m);
    uint32_t st[2];
    hipStream_t s = nullptr;
    // G's last window can need tens of GB for one lane of a large network (msim_general_launch.h): a
    // workspace larger than the device's free memory is the network's size limit, not a HIP failure
    if (cfg->general && !workspace_fits(wsb)) return MSIM_E_MINERS;
    if (hipMalloc(&ws, wsb) != hipSuccess || hipMalloc(&sums, 6 * sizeof(uint64_t) * m) != hipSuccess ||
        hipMalloc(&status, 2 * sizeof(uint32_t)) != hipSuccess ||
        (want_rec && hipMalloc(&rec, chunk * m * sizeof(msim_run_record)) != hipSuccess) ||
        (want_bh && hipMalloc(&bh, chunk * sizeof(uint32_t)) != hipSuccess) || hipStreamCreate(&s) != hipSuccess) {
        rc = MSIM_E_HIP;
        goto out;
    }
    for (uint64_t off = 0; off < n_runs && rc == MSIM_OK; off += chunk) {
        const uint64_t cn = (n_runs - off) < chunk ? (n_runs - off) : chunk;
        rc = msim_launch(cfg, run_begin + off, cn, seed_base, sums, rec, bh, status, ws, wsb, s);
        if (rc) break;
        if (hipMemcpyAsync(part.data(), sums, part.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(st, status, sizeof(st), hipMemcpyDeviceToHost, s) != hipSuccess ||
            (want_rec && hipMemcpyAsync(opt_per_run + off * m, rec, cn * m * sizeof(msim_run_record),
                                        hipMemcpyDeviceToHost, s) != hipSuccess) ||
            (want_bh && hipMemcpyAsync(bh_out + off, bh, cn * sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess) ||
            hipStreamSynchronize(s) != hipSuccess) {
            rc = MSIM_E_HIP;
            break;
        }
        if (st[1] != 0) {
            rc = MSIM_E_CAPACITY;
            break;
        }
        for (size_t i = 0; i < acc.size(); ++i) acc[i] += part[i];
    }
    if (rc == MSIM_OK) {
        msim_sums *fs = (msim_sums *)acc.data();
        if (opt_sums) memcpy(opt_sums, fs, sizeof(msim_sums) * m);
        msim_sums_to_stats(fs, m, out_sums);
        if (want_rec) {
            // Exact reference aggregation: per-run MinerStats (main.cpp:22-30) summed in run order
            // (main.cpp:211-217, MinerStats::operator+= 34-40).
            for (uint32_t k = 0; k < m; ++k) {
                out_sums[k].blocks_share = 0.0;
                out_sums[k].stale_rate = 0.0;
            }
            for (uint64_t r = 0; r < n_runs; ++r)
                for (uint32_t k = 0; k < m; ++k) {
                    const msim_run_record &x = opt_per_run[r * m + k];
                    const double share = x.found == 0 ? 0.0 : (double)x.found / (double)bh_out[r];
                    const double rate = x.found == 0 ? 0.0 : (double)x.stale / (double)x.found;
                    out_sums[k].blocks_share += share;
                    out_sums[k].stale_rate += rate;
                }
        }
    }
out:
    if (s) (void)hipStreamDestroy(s);
    (void)hipFree(ws);
    (void)hipFree(sums);
    (void)hipFree(status);
    (void)hipFree(rec);
    (void)hipFree(bh);
    return rc;
}

int msim_sweep_create(const msim_config *const *cfgs, uint32_t n_points, msim_sweep **out)
{
    if (!cfgs || !out || n_points == 0) return MSIM_E_INVALID;
    msim_sweep *w = new (std::nothrow) msim_sweep();
    if (!w) return MSIM_E_INVALID;
    w->m = cfgs[0] ? cfgs[0]->n : 0;
    w->self = false;
    bool any_general = false;
    for (uint32_t i = 0; i < n_points; ++i) any_general = any_general || (cfgs[i] && cfgs[i]->general);
    for (uint32_t i = 0; i < n_points; ++i) {
        // one miner count per sweep; narrow networks with percentages unless the sweep runs on the general
        // engine (the per-lane and entity-engine sweeps share draws and tables between points)
        if (!cfgs[i] || cfgs[i]->n != w->m || (!any_general && (cfgs[i]->wide || cfgs[i]->total_weight != 100))) {
            delete w;
            return MSIM_E_INVALID;
        }
        w->pts.push_back(cfgs[i]->p);
        w->self = w->self || cfgs[i]->selfish || cfgs[i]->p.selfish >= 0;
        w->sel = w->sel || cfgs[i]->sel;
        w->general = w->general || cfgs[i]->general;
        w->gen_full = w->gen_full || cfgs[i]->gen_full;
        w->gens.push_back(cfgs[i]->gh);
        w->max_duration = cfgs[i]->p.duration_ms > w->max_duration ? cfgs[i]->p.duration_ms : w->max_duration;
    }
    if (w->general) {  // a point only the general engine serves: every point on G
        w->sel = false;
    } else if (w->sel) {
        // every point on the entity engine; points grouped by selfish class
        for (uint32_t i = 0; i < n_points; ++i) {
            const msim_config *c = cfgs[i];
            msim::SelParams sp;
            if (c->sel) {
                sp = c->sp;
            } else {
                std::vector<msim_miner> ms(c->n);
                for (uint32_t k = 0; k < c->n; ++k) ms[k] = msim_miner{c->ids[k], c->perc[k], c->prop[k], 0};
                build_sel_params(ms.data(), c->n, c->p.duration_ms, 100, &sp);
            }
            w->sps.push_back(sp);
            w->max_duration = sp.duration_ms > w->max_duration ? sp.duration_ms : w->max_duration;
            const uint32_t nc = msim::sel_ns_class(sp.ns);
            bool placed = false;
            for (auto &g : w->groups)
                if (g.nscls == nc) {
                    g.points.push_back(i);
                    placed = true;
                }
            if (!placed) w->groups.push_back({nc, {i}});
        }
        // A group's workgroups are dispatched in point-list order, and a point's runs cost in proportion to its
        // engine entries: an honest find needs the engine when the next interval is below prop_k (+ prop_s while
        // the selfish miner leads). The costliest points go first, so the launch ends on cheap workgroups
        // (longest-first list scheduling); results are indexed by point, not by list position.
        auto cost = [&](uint32_t p) {
            const msim::SelParams &s = w->sps[p];
            if (!s.macro) return 1e30;  // the engine for every find
            const int64_t ps = s.prop[s.sids[0]];
            double c = 0.0;
            for (uint32_t k = 0; k < s.m; ++k)
                if (k != s.sids[0]) c += (double)(s.cum[k] - (k ? s.cum[k - 1] : 0)) * (double)(s.prop[k] + ps);
            return c / (double)s.W;
        };
        if (!getenv("MSIM_SWEEP_LISTED_ORDER"))  // A/B: the caller's point order
            for (auto &g : w->groups)
                std::stable_sort(g.points.begin(), g.points.end(), [&](uint32_t a, uint32_t b) { return cost(a) > cost(b); });
    }
    *out = w;
    return MSIM_OK;
}

void msim_sweep_destroy(msim_sweep *sw)
{
    if (!sw) return;
    for (const auto &d : sw->dev) (void)hipFree(d.second);
    for (const auto &d : sw->sdev) (void)hipFree(d.second);
    for (const auto &d : sw->gdev) (void)hipFree(d.second);
    delete sw;
}

uint32_t msim_sweep_point_count(const msim_sweep *sw) { return sw ? (uint32_t)sw->pts.size() : 0u; }
uint32_t msim_sweep_miner_count(const msim_sweep *sw) { return sw ? sw->m : 0u; }

size_t msim_sweep_workspace_bytes(const msim_sweep *sw, uint64_t runs_per_point)
{
    if (!sw || runs_per_point == 0 || runs_per_point * sw->pts.size() > MAX_LAUNCH_RUNS) return 0;
    if (sw->general) return gen_only_layout(sw->m, (uint32_t)sw->pts.size(), runs_per_point, sw->max_duration, sw->gen_full).total;
    if (sw->sel) return sel_ws_layout(sw->m, (uint32_t)sw->pts.size(), runs_per_point, sw->max_duration).total;
    return sweep_layout(sw->m, (uint32_t)sw->pts.size(), runs_per_point).total;
}

int msim_sweep_launch(const msim_sweep *sw, uint64_t run_begin, uint64_t runs_per_point, uint32_t seed_base,
                      void *d_sums, void *d_per_run, void *d_best_height, void *d_status, void *d_workspace,
                      size_t workspace_bytes, void *stream)
{
    if (!sw || !d_sums || !d_status || !d_workspace || runs_per_point == 0) return MSIM_E_INVALID;
    const uint32_t np = (uint32_t)sw->pts.size();
    if (runs_per_point * np > MAX_LAUNCH_RUNS) return MSIM_E_INVALID;
    const msim::GenParams *gp = nullptr;
    if (sw->general || sw->sel) {
        msim_sweep *sm = const_cast<msim_sweep *>(sw);
        std::vector<const GenHost *> hs;
        for (const auto &g : sm->gens) hs.push_back(&g);
        const int rc = gen_cached(sm->mu, sm->gdev, hs, &gp);
        if (rc) return rc;
        if (sw->general) {
            const GenOnlyWs w = gen_only_layout(sw->m, np, runs_per_point, sw->max_duration, sw->gen_full);
            if (workspace_bytes < w.total) return MSIM_E_INVALID;
            return gen_launch_impl(sw->m, np, gp, w, (char *)d_workspace, run_begin, runs_per_point, seed_base, d_sums,
                                   d_per_run, d_best_height, d_status, (hipStream_t)stream);
        }
    }
    if (sw->sel) {
        const SelWs w = sel_ws_layout(sw->m, np, runs_per_point, sw->max_duration);
        if (workspace_bytes < w.total) return MSIM_E_INVALID;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return MSIM_E_HIP;
        msim_sweep *sm = const_cast<msim_sweep *>(sw);
        void *d = nullptr;
        const size_t pb = (np * sizeof(msim::SelParams) + 255) / 256 * 256;
        {
            std::lock_guard<std::mutex> g(sm->mu);
            for (const auto &x : sm->sdev)
                if (x.first == dev) d = x.second;
            if (!d) {
                std::vector<char> h(pb + (size_t)np * 4, 0);
                memcpy(h.data(), sm->sps.data(), np * sizeof(msim::SelParams));
                uint32_t *pl = (uint32_t *)(h.data() + pb);
                for (const auto &gr : sm->groups)
                    for (uint32_t p : gr.points) *pl++ = p;
                if (hipMalloc(&d, h.size()) != hipSuccess) return MSIM_E_HIP;
                if (hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice) != hipSuccess) {
                    (void)hipFree(d);
                    return MSIM_E_HIP;
                }
                sm->sdev.push_back({dev, d});
            }
        }
        std::vector<SelGroupDev> groups;
        const uint32_t *pl = (const uint32_t *)((const char *)d + pb);
        for (const auto &gr : sm->groups) {
            uint32_t uni = 1;
            for (uint32_t p : gr.points) uni &= sm->sps[p].uniform_prop != 0 ? 1u : 0u;
            groups.push_back({gr.nscls, (uint32_t)gr.points.size(), pl, uni});
            pl += gr.points.size();
        }
        const msim::LogTab *lt = nullptr;
        int rc = global_log_table(&lt);
        if (rc) return rc;
        return sel_launch_impl(sw->m, np, (const msim::SelParams *)d, gp, groups, lt, w, (char *)d_workspace, run_begin,
                               runs_per_point, seed_base, d_sums, d_per_run, d_best_height, d_status,
                               (hipStream_t)stream, nullptr);
    }
    const SweepLayout l = sweep_layout(sw->m, np, runs_per_point);
    if (workspace_bytes < l.total) return MSIM_E_INVALID;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return MSIM_E_HIP;
    void *pts = nullptr;
    {
        msim_sweep *w = const_cast<msim_sweep *>(sw);
        std::lock_guard<std::mutex> g(w->mu);
        for (const auto &d : w->dev)
            if (d.first == dev) pts = d.second;
        if (!pts) {
            const size_t b = w->pts.size() * sizeof(msim::SimParams);
            if (hipMalloc(&pts, b) != hipSuccess) return MSIM_E_HIP;
            if (hipMemcpy(pts, w->pts.data(), b, hipMemcpyHostToDevice) != hipSuccess) {
                (void)hipFree(pts);
                return MSIM_E_HIP;
            }
            w->dev.push_back({dev, pts});
        }
    }
    char *ws = (char *)d_workspace;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(ws + l.retry_off, 0, l.list_off - l.retry_off, s) != hipSuccess) return MSIM_E_HIP;
    msim::SweepArgs a;
    a.pts = (const msim::SimParams *)pts;
    a.m = sw->m;
    a.self = sw->self;
    a.n_points = np;
    a.rpp = (uint32_t)runs_per_point;
    a.wpp = l.wpp;
    a.run_begin = run_begin;
    a.seed_base = seed_base;
    a.partials = (uint64_t *)(ws + l.partials_off);
    a.retry_sums = (uint64_t *)(ws + l.retry_off);
    a.sums = (uint64_t *)d_sums;
    a.records = (uint32_t *)d_per_run;
    a.best_h = (uint32_t *)d_best_height;
    a.err_count = (uint32_t *)(ws + l.counts_off);
    a.err_list = (uint32_t *)(ws + l.list_off);
    a.err_cap = l.err_cap;
    a.status = (uint32_t *)d_status;
    a.stream = s;
    return msim::launch_sweep(a) == hipSuccess ? MSIM_OK : MSIM_E_HIP;
}

int msim_sweep_run(const msim_sweep *sw, uint64_t run_begin, uint64_t runs_per_point, uint32_t seed_base, int device,
                   msim_stats *out_stats, msim_sums *opt_sums, msim_run_record *opt_per_run, uint32_t *opt_best_height)
{
    if (!sw || !out_stats || runs_per_point == 0) return MSIM_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return MSIM_E_HIP;
    const size_t np = sw->pts.size(), m = sw->m, nr = np * runs_per_point;
    const size_t wsb = msim_sweep_workspace_bytes(sw, runs_per_point);
    if (!wsb) return MSIM_E_INVALID;
    void *ws = nullptr, *sums = nullptr, *status = nullptr, *rec = nullptr, *bh = nullptr;
    std::vector<msim_sums> hs(np * m);
    uint32_t st[2] = {0, 0};
    hipStream_t s = nullptr;
    int rc = MSIM_OK;
    if (sw->general && !workspace_fits(wsb)) return MSIM_E_MINERS;  // as in msim_run
    if (hipMalloc(&ws, wsb) != hipSuccess || hipMalloc(&sums, hs.size() * sizeof(msim_sums)) != hipSuccess ||
        hipMalloc(&status, sizeof(st)) != hipSuccess ||
        (opt_per_run && hipMalloc(&rec, nr * m * sizeof(msim_run_record)) != hipSuccess) ||
        (opt_best_height && hipMalloc(&bh, nr * sizeof(uint32_t)) != hipSuccess) || hipStreamCreate(&s) != hipSuccess) {
        rc = MSIM_E_HIP;
    } else {
        rc = msim_sweep_launch(sw, run_begin, runs_per_point, seed_base, sums, rec, bh, status, ws, wsb, s);
        if (rc == MSIM_OK &&
            (hipMemcpyAsync(hs.data(), sums, hs.size() * sizeof(msim_sums), hipMemcpyDeviceToHost, s) != hipSuccess ||
             hipMemcpyAsync(st, status, sizeof(st), hipMemcpyDeviceToHost, s) != hipSuccess ||
             (opt_per_run && hipMemcpyAsync(opt_per_run, rec, nr * m * sizeof(msim_run_record), hipMemcpyDeviceToHost, s) != hipSuccess) ||
             (opt_best_height && hipMemcpyAsync(opt_best_height, bh, nr * sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess) ||
             hipStreamSynchronize(s) != hipSuccess))
            rc = MSIM_E_HIP;
        if (rc == MSIM_OK && st[1] != 0) rc = MSIM_E_CAPACITY;
    }
    if (rc == MSIM_OK) {
        if (opt_sums) memcpy(opt_sums, hs.data(), hs.size() * sizeof(msim_sums));
        msim_sums_to_stats(hs.data(), (uint32_t)hs.size(), out_stats);
    }
    if (s) (void)hipStreamDestroy(s);
    (void)hipFree(ws);
    (void)hipFree(sums);
    (void)hipFree(status);
    (void)hipFree(rec);
    (void)hipFree(bh);
    return rc;
}

int msim_timing_enable(int on)
{
    Timing &tm = timing();
    std::lock_guard<std::mutex> g(tm.mu);
    destroy_events(tm.k1);
    destroy_events(tm.launch);
    destroy_events(tm.engine);
    tm.launches = 0;
    tm.on = on != 0;
    return MSIM_OK;
}

int msim_timing_read_stages(double *draws_ms, double *engine_ms, double *launch_ms, uint32_t *launches)
{
    if (!draws_ms || !engine_ms || !launch_ms || !launches) return MSIM_E_INVALID;
    Timing &tm = timing();
    std::lock_guard<std::mutex> g(tm.mu);
    double acc[3] = {0, 0, 0};
    int rc = MSIM_OK;
    std::vector<hipEvent_t> *vs[3] = {&tm.k1, &tm.engine, &tm.launch};
    for (int pass = 0; pass < 3; ++pass) {
        std::vector<hipEvent_t> &v = *vs[pass];
        for (size_t i = 0; i + 1 < v.size(); i += 2) {
            float ms = 0;
            if (hipEventSynchronize(v[i + 1]) != hipSuccess || hipEventElapsedTime(&ms, v[i], v[i + 1]) != hipSuccess)
                rc = MSIM_E_HIP;
            acc[pass] += ms;
        }
    }
    *draws_ms = acc[0];
    *engine_ms = acc[1];
    *launch_ms = acc[2];
    *launches = tm.launches;
    destroy_events(tm.k1);
    destroy_events(tm.launch);
    destroy_events(tm.engine);
    tm.launches = 0;
    return rc;
}

// Union length of (begin, end) event pairs. Events are timed against an anchor of their own device: a pair
// whose begin cannot be timed against an existing anchor (hipEventElapsedTime fails across devices) starts a
// new group with its begin as the anchor. Each group's intervals are sorted and merged; the result is the
// largest group's busy time (one device's), so a timed run over several devices reads instead of failing.
static int busy_ms(const std::vector<hipEvent_t> &v, double *out)
{
    *out = 0;
    if (v.size() < 2) return MSIM_OK;
    std::vector<hipEvent_t> anchors;
    std::vector<std::vector<std::pair<double, double>>> groups;
    for (size_t i = 0; i + 1 < v.size(); i += 2) {
        if (hipEventSynchronize(v[i + 1]) != hipSuccess) return MSIM_E_HIP;
        bool placed = false;
        for (size_t g = 0; g < anchors.size() && !placed; ++g) {
            float a = 0, b = 0;
            if (hipEventElapsedTime(&a, anchors[g], v[i]) != hipSuccess) continue;
            if (hipEventElapsedTime(&b, anchors[g], v[i + 1]) != hipSuccess) return MSIM_E_HIP;
            groups[g].emplace_back(a, b);
            placed = true;
        }
        if (!placed) {
            float b = 0;
            if (hipEventElapsedTime(&b, v[i], v[i + 1]) != hipSuccess) return MSIM_E_HIP;
            anchors.push_back(v[i]);
            groups.push_back({{0.0, (double)b}});
        }
    }
    (void)hipGetLastError();  // the failed cross-device queries leave an error behind
    for (auto &iv : groups) {
        std::sort(iv.begin(), iv.end());
        double lo = iv[0].first, hi = iv[0].second, acc = 0;
        for (const auto &p : iv) {
            if (p.first > hi) {
                acc += hi - lo;
                lo = p.first;
                hi = p.second;
            } else if (p.second > hi) {
                hi = p.second;
            }
        }
        acc += hi - lo;
        *out = acc > *out ? acc : *out;
    }
    return MSIM_OK;
}

int msim_timing_read_all(msim_timing *out)
{
    if (!out) return MSIM_E_INVALID;
    memset(out, 0, sizeof(*out));
    int rc = MSIM_OK;
    {
        Timing &tm = timing();
        std::lock_guard<std::mutex> g(tm.mu);
        const std::vector<hipEvent_t> *vs[3] = {&tm.k1, &tm.engine, &tm.launch};
        double *busy[3] = {&out->draws_busy_ms, &out->engine_busy_ms, &out->launch_busy_ms};
        for (int i = 0; i < 3; ++i)
            if (busy_ms(*vs[i], busy[i]) != MSIM_OK) rc = MSIM_E_HIP;
    }
    const int r2 = msim_timing_read_stages(&out->draws_ms, &out->engine_ms, &out->launch_ms, &out->launches);
    return rc ? rc : r2;
}

int msim_timing_read(double *draws_ms, double *launch_ms, uint32_t *launches)
{
    double e = 0;
    return msim_timing_read_stages(draws_ms, &e, launch_ms, launches);
}

int msim_pipeline_info(const msim_config *cfg, uint64_t n_runs, msim_pipeline_layout *out)
{
    if (!cfg || !out || n_runs == 0) return MSIM_E_INVALID;
    memset(out, 0, sizeof(*out));
    out->rho = cfg->rho;
    if (cfg->general) {
        const GenOnlyWs w = gen_only_layout(cfg->n, 1, n_runs, cfg->p.duration_ms, cfg->gen_full);
        out->uses_pipeline = 4;
        out->slice_runs = (uint32_t)w.g.tier[0].lanes;
        out->segment_blocks = w.g.tier[0].cap;
        out->segments = (uint32_t)w.g.nt;
        out->blocks_per_run = w.g.tier[w.g.nt - 1].cap;
        out->workspace_bytes = w.total;
        return MSIM_OK;
    }
    if (cfg->wide) {
        const msim::WideLayout L = wide_layout(cfg, n_runs);
        out->uses_pipeline = 2;
        out->slice_runs = L.nr;
        out->segment_blocks = L.g.S0;
        out->segments = 64;
        out->blocks_per_run = L.g.B0 + 64ull * L.g.ST * L.g.nch;
        out->workspace_bytes = L.total;
        return MSIM_OK;
    }
    if (cfg->sel) {
        const SelCfgWs cw = sel_cfg_layout(cfg, n_runs);
        out->slice_runs = cw.w.nr;
        out->workspace_bytes = cw.total;
        if (cw.seg) {  // the segment-parallel form (msim_selseg.h): SW segments + ST
            out->uses_pipeline = 6;
            out->segment_blocks = cw.L.seg;
            out->segments = cw.L.nseg;
            out->blocks_per_run = cw.L.nseg * cw.L.seg;
            out->rho = cfg->seg_rate;
            return MSIM_OK;
        }
        out->uses_pipeline = 3;  // E1 draws in-lane: no draw segments
        out->segment_blocks = 0;
        out->segments = 0;
        out->blocks_per_run = 0;
        return MSIM_OK;
    }
    if (!cfg->pipe_ok) return MSIM_OK;
    const msim::PipeLayout pl = pipe_layout(cfg, n_runs);
    out->uses_pipeline = 1;
    out->slice_runs = pl.nr;
    out->segment_blocks = pl.seg;
    out->segments = pl.nseg;
    out->blocks_per_run = pl.nb;
    out->workspace_bytes = pl.total;
    return MSIM_OK;
}

// ---------------------------------------------------------------- samplers (test.cpp)
namespace {
int sample_impl(int mode, const msim_config *cfg, uint64_t seed, uint64_t n, int device, unsigned long long *host_out,
                size_t nout)
{
    using namespace msim;
    if (hipSetDevice(device) != hipSuccess) return MSIM_E_HIP;
    const uint64_t target_threads = 131072;
    uint64_t S64 = (n + target_threads - 1) / target_threads;
    if (S64 < 64) S64 = 64;
    if (S64 > 0xFFFFFFFFull) return MSIM_E_INVALID;
    const uint32_t S = (uint32_t)S64;
    // T^(S * 2^b), b = 0..31
    std::vector<uint32_t> jumps(32 * 512);
    {
        Mat128 cur, tmp;
        mat_pow(S, cur);
        for (int b = 0; b < 32; ++b) {
            uint32_t *w = jumps.data() + (size_t)b * 512;
            for (int col = 0; col < 128; ++col) {
                w[4 * col + 0] = (uint32_t)cur.lo[col];
                w[4 * col + 1] = (uint32_t)(cur.lo[col] >> 32);
                w[4 * col + 2] = (uint32_t)cur.hi[col];
                w[4 * col + 3] = (uint32_t)(cur.hi[col] >> 32);
            }
            mat_mul(cur, cur, tmp);
            cur = tmp;
        }
    }
    uint32_t m = 0, W = 100;
    std::vector<uint64_t> cf(1, 0xFFFFFFFFull);
    std::vector<uint16_t> bucket(WB_N, 0);
    if (mode == 0) {
        m = cfg->n;
        W = (uint32_t)cfg->total_weight;
        std::vector<uint64_t> w(m);
        for (uint32_t k = 0; k < m; ++k) w[k] = cfg->wide ? cfg->wperc[k] : cfg->perc[k];
        std::vector<uint32_t> fthr(m, 0);
        cf.assign(m + 1, 0);
        build_wide_pick(w.data(), fthr.data(), m, W, cf.data(), bucket.data());
    }
    LogTab lt;
    build_log_table(&lt);
    const size_t bj = jumps.size() * 4, bc = cf.size() * 8, bb = bucket.size() * 2, bl = sizeof(lt), bo = nout * 8;
    char *d = nullptr;
    int rc = MSIM_OK;
    hipStream_t st = nullptr;
    if (hipMalloc((void **)&d, bj + bc + bb + bl + bo + 64) != hipSuccess || hipStreamCreate(&st) != hipSuccess) {
        (void)hipFree(d);
        return MSIM_E_HIP;
    }
    char *pj = d, *pc = pj + bj, *pb = pc + bc, *pl = pb + ((bb + 7) / 8 * 8), *po = pl + bl;
    if (hipMemcpyAsync(pj, jumps.data(), bj, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(pc, cf.data(), bc, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(pb, bucket.data(), bb, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(pl, &lt, bl, hipMemcpyHostToDevice, st) != hipSuccess || hipMemsetAsync(po, 0, bo, st) != hipSuccess ||
        launch_sample(mode, (const uint32_t *)pj, seed, n, S, (const uint64_t *)pc, (const uint16_t *)pb, m, W,
                      0xFFFFFFFFFFFFFFFFull / W, (const LogTab *)pl, (unsigned long long *)po, st) != hipSuccess ||
        hipMemcpyAsync(host_out, po, bo, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        rc = MSIM_E_HIP;
    (void)hipStreamDestroy(st);
    (void)hipFree(d);
    return rc;
}
}  // namespace

int msim_sample_picks(const msim_config *cfg, uint64_t seed, uint64_t n, uint64_t *out_counts, int device)
{
    if (!cfg || !out_counts) return MSIM_E_INVALID;
    return sample_impl(0, cfg, seed, n, device, (unsigned long long *)out_counts, cfg->n + 1);
}

int msim_sample_intervals(uint64_t seed, uint64_t n, msim_interval_moments *out, int device)
{
    if (!out) return MSIM_E_INVALID;
    unsigned long long o[4] = {0, 0, 0, 0};
    const int rc = sample_impl(1, nullptr, seed, n, device, o, 4);
    if (rc) return rc;
    out->n = n;
    out->sum = o[0];
    out->sumsq_lo = o[1];
    out->sumsq_hi = o[2];
    out->max = o[3];
    return MSIM_OK;
}

const char *msim_strerror(int code)
{
    switch (code) {
    case MSIM_OK: return "ok";
    case MSIM_E_INVALID: return "invalid argument";
    case MSIM_E_WEIGHTS: return "miner weights must be integers adding up to the total weight (100 for percentages)";
    case MSIM_E_SELFISH: return "reserved (not returned: every network with selfish miners runs)";
    case MSIM_E_MINERS: return "network too large for the general engine (one run's explicit chains, miners x blocks per run x 12 B, exceed 96 GiB, or the launch's workspace exceeds the device's free memory)";
    case MSIM_E_HIP: return "HIP runtime error";
    case MSIM_E_CAPACITY: return "a run exceeded the compact state capacity";
    case MSIM_E_PICK: return "PickFinder fell through its table";
    default: return "unknown error";
    }
}

const char *msim_version(void) { return "msim 0.1 (gfx950)"; }

}  // extern "C"
