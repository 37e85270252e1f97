// msim_main.cpp — drop-in replacement for the reference's main.cpp driver on MI355X.
//
// Keeps the reference's configuration surface unchanged — SIM_DURATION (main.cpp:7), SIM_RUNS
// (main.cpp:10), SetupMiners() (main.cpp:44-65) with Miner(id, perc, propagation, selfish) — and its
// report (main.cpp:224-234). The std::async batch loop (main.cpp:205-220) is replaced by one msim_run
// call per GPU through the C ABI (include/msim.h); with MSIM_GPUS > 1 the run range is split across
// devices (one host thread per device) and the integer sums are added exactly as an all-reduce would.
//
// Build: make -C host     Run: ./host/msim_main [n_gpus] [seed_base] [default|c5]
// "c5" runs BASELINE configs[4] (2 pools + 1 024 small miners, integer weights summing to
// W = 102 400, msim_config_create_weighted), which the reference's integer percentages cannot express.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../include/msim.h"

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

int main(int argc, char **argv)
{
    const bool large = argc > 3 && std::string(argv[3]) == "c5";
    const auto miners{large ? SetupLargeNetwork() : SetupMiners()};
    const uint64_t total_weight = large ? C5_TOTAL_WEIGHT : 100;
    const int n_gpus = argc > 1 ? std::atoi(argv[1]) : 1;
    const int64_t duration_ms = std::chrono::duration_cast<std::chrono::milliseconds>(SIM_DURATION).count();
    const uint32_t seed_base = argc > 2 ? (uint32_t)std::strtoul(argv[2], nullptr, 10) : 1000u;

    std::vector<msim_miner> desc;
    for (const auto &m : miners)
        desc.push_back({m.id, m.perc, (int64_t)m.propagation.count(), (uint8_t)(m.is_selfish ? 1 : 0)});
    msim_config *cfg = nullptr;
    if (int rc = msim_config_create_weighted(desc.data(), (uint32_t)desc.size(), duration_ms, total_weight, &cfg))
        return die("config", rc);

    std::printf("Running %d simulations in parallel using %d GPU(s).\n", SIM_RUNS, n_gpus);
    std::vector<std::vector<msim_sums>> part(n_gpus, std::vector<msim_sums>(miners.size()));
    std::vector<int> rcs(n_gpus, 0);
    std::vector<std::thread> th;
    for (int g = 0; g < n_gpus; ++g) {
        th.emplace_back([&, g] {
            const uint64_t base = SIM_RUNS / n_gpus, rem = SIM_RUNS % n_gpus;
            const uint64_t begin = g * base + (g < (int)rem ? g : rem), n = base + (g < (int)rem ? 1 : 0);
            std::vector<msim_stats> st(miners.size());
            if (n) rcs[g] = msim_run(cfg, begin, n, seed_base, g, st.data(), part[g].data(), nullptr, nullptr);
        });
    }
    for (auto &t : th) t.join();
    for (int g = 0; g < n_gpus; ++g)
        if (rcs[g]) return die("msim_run", rcs[g]);
    std::vector<msim_sums> total(miners.size());
    for (size_t k = 0; k < miners.size(); ++k)
        for (int g = 0; g < n_gpus; ++g) {  // integer sums: what the RCCL all-reduce computes
            total[k].blocks_found += part[g][k].blocks_found;
            total[k].stale_blocks += part[g][k].stale_blocks;
            total[k].share_hi += part[g][k].share_hi;
            total[k].share_lo += part[g][k].share_lo;
            total[k].rate_hi += part[g][k].rate_hi;
            total[k].rate_lo += part[g][k].rate_lo;
        }
    std::vector<msim_stats> stats_total(miners.size());
    msim_sums_to_stats(total.data(), (uint32_t)total.size(), stats_total.data());
    std::printf("\r100%% progress..\n");

    // main.cpp:224-234
    const auto days{std::chrono::duration_cast<std::chrono::days>(SIM_DURATION)};
    std::printf("After running %d simulations for %lldd each, on average:\n", SIM_RUNS, (long long)days.count());
    for (size_t i = 0; i < miners.size(); ++i) {
        const auto &miner{miners[i]};
        const auto &stats{stats_total[i]};
        if (total_weight == 100)
            std::printf("  - Miner %u (%llu%% of network hashrate) found %lld blocks i.e. ", miner.id,
                        (unsigned long long)miner.perc, (long long)(stats.blocks_found / SIM_RUNS));
        else
            std::printf("  - Miner %u (%g%% of network hashrate) found %lld blocks i.e. ", miner.id,
                        (double)miner.perc * 100.0 / (double)total_weight, (long long)(stats.blocks_found / SIM_RUNS));
        std::printf("%g%% of blocks. Stale rate: %g%%.", stats.blocks_share * 100 / SIM_RUNS,
                    stats.stale_rate * 100 / SIM_RUNS);
        if (miner.is_selfish) std::printf(" ('selfish mining' strategy)");
        std::printf("\n");
    }
    msim_config_destroy(cfg);
    return 0;
}
