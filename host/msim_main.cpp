// msim_main.cpp — drop-in replacement for the reference's main.cpp driver on MI355X.
//
// Keeps the reference's configuration surface unchanged — SIM_DURATION (main.cpp:7), SIM_RUNS
// (main.cpp:10), SetupMiners() (main.cpp:44-65) with Miner(id, perc, propagation, selfish) — and its
// report (main.cpp:201, 219-234). The std::async batch loop (main.cpp:205-220) is replaced by
// msim_run_multi through the C ABI (include/msim.h): the runs are sharded over the GPUs, one stream
// per GPU, and combined by one RCCL all-reduce of the integer sums.
//
// Sweeps (BASELINE configs[3]) — the reference edits SetupMiners and rebuilds per network
// (README.md:21-27); here one invocation runs a whole grid or network list in one sweep launch per GPU
// (msim_sweep_run_multi) and prints main.cpp:224-234's report per point, or one JSON line per point:
//   msim_main [n_gpus] [seed_base] [default|c5]
//   msim_main --grid H1,H2,..:P1,P2,.. [--runs R] [--gpus N] [--seed S] [--json]
//        SetupMiners with miner 0 selfish at H% (miner 1 at 59-H%) and every propagation P ms
//   msim_main --sweep FILE.json [--runs R] [--gpus N] [--seed S] [--json]
//        {"runs": R, "seed_base": S, "duration_ms": D, "total_weight": W,
//         "grid": {"selfish_perc": [..], "propagation_ms": [..]}}            or
//         "points": [{"miners": [{"id": 0, "perc": 40, "propagation_ms": 1000, "selfish": true}, ..]}, ..]}
//
// Build: make -C host
// "c5" runs BASELINE configs[4] (2 pools + 1 024 small miners, integer weights summing to
// W = 102 400, msim_config_create_weighted), which the reference's integer percentages cannot express.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../include/msim.h"
#include "json_min.h"

using namespace std::chrono_literals;

//! How long to run each simulation for (main.cpp:7).
static constexpr std::chrono::months SIM_DURATION{12};
//! How many simulations to run (main.cpp:10).
static constexpr int SIM_RUNS{16 * 2'048};

struct Miner {  // simulation.h:57-59 constructor surface
    unsigned id;
    uint64_t perc;
    std::chrono::milliseconds propagation;
    bool is_selfish;
    Miner(unsigned id_, uint64_t perc_, std::chrono::milliseconds prop, bool selfish = false)
        : id{id_}, perc{perc_}, propagation{prop}, is_selfish{selfish} {}
};

/** Set the hashrate distribution for the simulation. Must add up to 100 (main.cpp:43-65). */
std::vector<Miner> SetupMiners()
{
    std::vector<Miner> miners;
    miners.emplace_back(0, 30, 1s);
    miners.emplace_back(1, 29, 1s);
    miners.emplace_back(2, 12, 1s);
    miners.emplace_back(3, 11, 1s);
    miners.emplace_back(4, 8, 1s);
    miners.emplace_back(5, 5, 1s);
    miners.emplace_back(6, 3, 1s);
    miners.emplace_back(7, 1, 1s);
    miners.emplace_back(8, 1, 1s);
    return miners;
}

/** The configs[3] grid network: SetupMiners with miner 0 selfish at h% and miner 1 at (59 - h)%, all at prop. */
std::vector<Miner> SetupSelfishMiners(uint64_t h, std::chrono::milliseconds prop)
{
    auto miners{SetupMiners()};
    miners[0].perc = h;
    miners[0].is_selfish = true;
    miners[1].perc = 59 - h;
    for (auto &m : miners) m.propagation = prop;
    return miners;
}

/** BASELINE configs[4] network: weights out of C5_TOTAL_WEIGHT, all honest, 1 s. */
static constexpr uint64_t C5_TOTAL_WEIGHT{102'400};
std::vector<Miner> SetupLargeNetwork()
{
    std::vector<Miner> miners;
    miners.emplace_back(0, 30'720, 1s);
    miners.emplace_back(1, 29'696, 1s);
    for (unsigned i = 0; i < 1'024; ++i) miners.emplace_back(2 + i, 41, 1s);
    return miners;
}

static int die(const char *what, int rc)
{
    std::fprintf(stderr, "%s: %s (%d)\n", what, msim_strerror(rc), rc);
    return 1;
}

// main.cpp:224-234 for one network.
static void PrintReport(const std::vector<Miner> &miners, const std::vector<msim_stats> &stats_total, uint64_t runs,
                        uint64_t total_weight, long long days)
{
    std::printf("After running %llu simulations for %lldd each, on average:\n", (unsigned long long)runs, days);
    for (size_t i = 0; i < miners.size(); ++i) {
        const auto &miner{miners[i]};
        const auto &stats{stats_total[i]};
        if (total_weight == 100)
            std::printf("  - Miner %u (%llu%% of network hashrate) found %lld blocks i.e. ", miner.id,
                        (unsigned long long)miner.perc, (long long)(stats.blocks_found / (int64_t)runs));
        else
            std::printf("  - Miner %u (%g%% of network hashrate) found %lld blocks i.e. ", miner.id,
                        (double)miner.perc * 100.0 / (double)total_weight, (long long)(stats.blocks_found / (int64_t)runs));
        std::printf("%g%% of blocks. Stale rate: %g%%.", stats.blocks_share * 100 / (double)runs,
                    stats.stale_rate * 100 / (double)runs);
        if (miner.is_selfish) std::printf(" ('selfish mining' strategy)");
        std::printf("\n");
    }
}

// One JSON line for a point: the network and its per-miner averages (the report's numbers).
static void PrintJson(size_t point, const std::vector<Miner> &miners, const std::vector<msim_stats> &st, uint64_t runs,
                      uint64_t total_weight)
{
    std::printf("{\"point\": %zu, \"runs\": %llu, \"total_weight\": %llu, \"miners\": [", point,
                (unsigned long long)runs, (unsigned long long)total_weight);
    for (size_t i = 0; i < miners.size(); ++i)
        std::printf("%s{\"id\": %u, \"perc\": %llu, \"propagation_ms\": %lld, \"selfish\": %s, "
                    "\"blocks_found\": %.17g, \"blocks_share\": %.17g, \"stale_rate\": %.17g}",
                    i ? ", " : "", miners[i].id, (unsigned long long)miners[i].perc,
                    (long long)miners[i].propagation.count(), miners[i].is_selfish ? "true" : "false",
                    (double)st[i].blocks_found / (double)runs, st[i].blocks_share / (double)runs,
                    st[i].stale_rate / (double)runs);
    std::printf("]}\n");
}

// RCCL prints a version banner on stdout when a communicator is created. The report on stdout must keep
// main.cpp's exact format, so library output during the run call goes to stderr instead.
template <class F>
static int WithStdoutOnStderr(F f)
{
    std::fflush(stdout);
    const int saved = dup(1);
    if (saved >= 0) dup2(2, 1);
    const int rc = f();
    std::fflush(stdout);
    if (saved >= 0) {
        dup2(saved, 1);
        close(saved);
    }
    return rc;
}

static std::vector<msim_miner> Describe(const std::vector<Miner> &miners)
{
    std::vector<msim_miner> desc;
    for (const auto &m : miners)
        desc.push_back({m.id, m.perc, (int64_t)m.propagation.count(), (uint8_t)(m.is_selfish ? 1 : 0)});
    return desc;
}

static std::vector<int64_t> ParseList(const std::string &s)
{
    std::vector<int64_t> out;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, ',')) out.push_back(std::stoll(tok));
    return out;
}

struct SweepSpec {
    std::vector<std::vector<Miner>> points;
    uint64_t runs = 2'048;
    uint32_t seed_base = 1000;
    int64_t duration_ms = std::chrono::duration_cast<std::chrono::milliseconds>(SIM_DURATION).count();
    uint64_t total_weight = 100;
    int gpus = 1;
    bool json = false;
};

static void AddGrid(SweepSpec &sp, const std::vector<int64_t> &hs, const std::vector<int64_t> &props)
{
    for (int64_t h : hs)
        for (int64_t p : props) sp.points.push_back(SetupSelfishMiners((uint64_t)h, std::chrono::milliseconds{p}));
}

static SweepSpec LoadSweepFile(const std::string &path)
{
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::stringstream buf;
    buf << f.rdbuf();
    const std::string text = buf.str();
    const jmin::Value root = jmin::Parser(text).parse();
    SweepSpec sp;
    if (const auto *v = root.get("runs")) sp.runs = (uint64_t)v->as_int();
    if (const auto *v = root.get("seed_base")) sp.seed_base = (uint32_t)v->as_int();
    if (const auto *v = root.get("duration_ms")) sp.duration_ms = v->as_int();
    if (const auto *v = root.get("total_weight")) sp.total_weight = (uint64_t)v->as_int();
    if (const auto *v = root.get("gpus")) sp.gpus = (int)v->as_int();
    if (const auto *g = root.get("grid")) {
        std::vector<int64_t> hs, ps;
        for (const auto &x : g->get("selfish_perc")->arr) hs.push_back(x.as_int());
        for (const auto &x : g->get("propagation_ms")->arr) ps.push_back(x.as_int());
        AddGrid(sp, hs, ps);
    }
    if (const auto *pts = root.get("points")) {
        for (const auto &pt : pts->arr) {
            std::vector<Miner> ms;
            for (const auto &m : pt.get("miners")->arr) {
                const auto *sel = m.get("selfish");
                ms.emplace_back((unsigned)m.get("id")->as_int(), (uint64_t)m.get("perc")->as_int(),
                                std::chrono::milliseconds{m.get("propagation_ms")->as_int()}, sel && sel->as_bool());
            }
            sp.points.push_back(std::move(ms));
        }
    }
    if (sp.points.empty()) throw std::runtime_error("no points in " + path);
    return sp;
}

static int RunSweep(const SweepSpec &sp)
{
    std::vector<msim_config *> cfgs;
    int rc = MSIM_OK;
    for (const auto &pt : sp.points) {
        const auto desc{Describe(pt)};
        msim_config *c = nullptr;
        rc = msim_config_create_weighted(desc.data(), (uint32_t)desc.size(), sp.duration_ms, sp.total_weight, &c);
        if (rc) break;
        cfgs.push_back(c);
    }
    msim_sweep *sw = nullptr;
    if (rc == MSIM_OK) rc = msim_sweep_create(cfgs.data(), (uint32_t)cfgs.size(), &sw);
    const uint32_t m = cfgs.empty() ? 0 : msim_config_miner_count(cfgs[0]);
    std::vector<msim_stats> st(sp.points.size() * m);
    if (rc == MSIM_OK)
        rc = WithStdoutOnStderr([&] {
            return msim_sweep_run_multi(sw, 0, sp.runs, sp.seed_base, nullptr, (uint32_t)sp.gpus, st.data(), nullptr);
        });
    if (rc == MSIM_OK) {
        const long long days = sp.duration_ms / 86'400'000;
        for (size_t p = 0; p < sp.points.size(); ++p) {
            const std::vector<msim_stats> ps(st.begin() + p * m, st.begin() + (p + 1) * m);
            if (sp.json) {
                PrintJson(p, sp.points[p], ps, sp.runs, sp.total_weight);
            } else {
                std::printf("Point %zu of %zu:\n", p + 1, sp.points.size());
                PrintReport(sp.points[p], ps, sp.runs, sp.total_weight, days);
            }
        }
    }
    if (sw) msim_sweep_destroy(sw);
    for (auto *c : cfgs) msim_config_destroy(c);
    return rc;
}

int main(int argc, char **argv)
{
    if (argc > 1 && (std::string(argv[1]) == "--grid" || std::string(argv[1]) == "--sweep")) {
        SweepSpec sp;
        try {
            if (argc < 3) throw std::runtime_error("missing argument");
            if (std::string(argv[1]) == "--sweep") {
                sp = LoadSweepFile(argv[2]);
            } else {
                const std::string g = argv[2];
                const size_t colon = g.find(':');
                if (colon == std::string::npos) throw std::runtime_error("--grid H1,H2,..:P1,P2,..");
                AddGrid(sp, ParseList(g.substr(0, colon)), ParseList(g.substr(colon + 1)));
            }
            for (int i = 3; i < argc; ++i) {
                const std::string a = argv[i];
                if (a == "--json") sp.json = true;
                else if (a == "--runs" && i + 1 < argc) sp.runs = std::stoull(argv[++i]);
                else if (a == "--gpus" && i + 1 < argc) sp.gpus = std::stoi(argv[++i]);
                else if (a == "--seed" && i + 1 < argc) sp.seed_base = (uint32_t)std::stoul(argv[++i]);
                else throw std::runtime_error("unknown option " + a);
            }
        } catch (const std::exception &e) {
            std::fprintf(stderr, "msim_main: %s\n", e.what());
            return 2;
        }
        if (int rc = RunSweep(sp)) return die("sweep", rc);
        return 0;
    }
    const bool large = argc > 3 && std::string(argv[3]) == "c5";
    const auto miners{large ? SetupLargeNetwork() : SetupMiners()};
    const uint64_t total_weight = large ? C5_TOTAL_WEIGHT : 100;
    const int n_gpus = argc > 1 ? std::atoi(argv[1]) : 1;
    const int64_t duration_ms = std::chrono::duration_cast<std::chrono::milliseconds>(SIM_DURATION).count();
    const uint32_t seed_base = argc > 2 ? (uint32_t)std::strtoul(argv[2], nullptr, 10) : 1000u;

    const auto desc{Describe(miners)};
    msim_config *cfg = nullptr;
    if (int rc = msim_config_create_weighted(desc.data(), (uint32_t)desc.size(), duration_ms, total_weight, &cfg))
        return die("config", rc);

    // main.cpp:201 (the reference names its thread count; here one stream drives each GPU)
    std::printf("Running %d simulations in parallel using %d threads.\n", SIM_RUNS, n_gpus);
    std::vector<msim_stats> stats_total(miners.size());
    if (int rc = WithStdoutOnStderr([&] {
            return msim_run_multi(cfg, 0, SIM_RUNS, seed_base, nullptr, (uint32_t)n_gpus, stats_total.data(), nullptr);
        }))
        return die("msim_run_multi", rc);
    std::printf("\r100%% progress..\n");  // main.cpp:219-221

    const auto days{std::chrono::duration_cast<std::chrono::days>(SIM_DURATION)};
    PrintReport(miners, stats_total, SIM_RUNS, total_weight, (long long)days.count());
    msim_config_destroy(cfg);
    return 0;
}
