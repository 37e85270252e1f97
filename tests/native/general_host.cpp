// general_host.cpp — TEST INFRASTRUCTURE: a host (CPU) build of the product's general engine
// (miningsimulation_amd/csrc/msim_general.h) so its algorithm, including the window fold, can be checked
// against the oracle without a GPU. Never part of the product path (libmsim.so is GPU-only).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../miningsimulation_amd/csrc/msim_general.h"

using namespace msim;

namespace {

struct HostStore {
    uint32_t cap, m;
    std::vector<uint32_t> o, sz, st, pr;
    std::vector<int64_t> a;
    HostStore(uint32_t m_, uint32_t cap_)
        : cap(cap_), m(m_), o((size_t)m_ * cap_), sz(m_), st(m_), pr(m_), a((size_t)m_ * cap_)
    {
    }
    uint32_t own(uint32_t k, uint32_t i) const { return o[(size_t)k * cap + i]; }
    int64_t arr(uint32_t k, uint32_t i) const { return a[(size_t)k * cap + i]; }
    void put(uint32_t k, uint32_t i, uint32_t ow, int64_t ar)
    {
        o[(size_t)k * cap + i] = ow;
        a[(size_t)k * cap + i] = ar;
    }
    void set_arr(uint32_t k, uint32_t i, int64_t ar) { a[(size_t)k * cap + i] = ar; }
    uint32_t size(uint32_t k) const { return sz[k]; }
    void set_size(uint32_t k, uint32_t n) { sz[k] = n; }
    void add_stale(uint32_t k) { ++st[k]; }
    uint32_t stale(uint32_t k) const { return st[k]; }
    void add_pre(uint32_t k, uint32_t v) { pr[k] += v; }
    uint32_t pre(uint32_t k) const { return pr[k]; }
};

}  // namespace

extern "C" {

// One run with seeds (si, sp); weights sum to W. Returns the error bits (GERR_*); on success fills
// found / stale [m] and the best chain height (length - 1).
// ids: Miner::id per miner (NULL: the index); the id classes are built as the library's host code does
// (msim_api.hip gen_id_classes: the lowest index with the same id; the class of id UINT_MAX owns Genesis).
uint32_t gen_run(const uint64_t *weights, const int64_t *props, const uint8_t *selfish, const uint32_t *ids, int m,
                 uint64_t W, int64_t duration, uint32_t si, uint32_t sp, uint32_t cap, uint32_t *found,
                 uint32_t *stale, uint32_t *best_height, uint32_t *base)
{
    std::vector<uint64_t> cum(m);
    std::vector<uint32_t> cls(m);
    uint64_t c = 0;
    uint32_t umax = GEN_GENESIS;
    for (int k = 0; k < m; ++k) {
        cum[k] = (c += weights[k]);
        const uint32_t id = ids ? ids[k] : (uint32_t)k;
        cls[k] = (uint32_t)k;
        for (int j = 0; j < k; ++j)
            if ((ids ? ids[j] : (uint32_t)j) == id) {
                cls[k] = (uint32_t)j;
                break;
            }
        if (id == 0xFFFFFFFFu) umax = cls[k];
    }
    GenParams g;
    memset(&g, 0, sizeof(g));
    g.duration_ms = duration;
    g.mult = 0xFFFFFFFFFFFFFFFFull / W;
    g.m = (uint32_t)m;
    g.umax = umax;
    g.cum = cum.data();
    g.prop = props;
    g.self = selfish;
    g.cls = cls.data();
    HostStore s((uint32_t)m, cap);
    Gen<HostStore> e(s, g);
    GenOut o;
    if (!e.run(rng_seed(si), rng_seed(sp), o)) return o.err;
    for (int k = 0; k < m; ++k) {
        found[k] = e.found((uint32_t)k, o);
        stale[k] = s.stale((uint32_t)k);
    }
    *best_height = Gen<HostStore>::best_height(o);
    *base = o.base;
    return 0;
}

// test.cpp:213-367 TestSelfishStrategy on G's state machine: one selfish miner (miner 0 of the store) with a
// hand-built chain, then FoundBlock (op 0: t, best_chain_size) or NotifyBestChain (op 1: the best chain held
// by miner 1 of the store, t). Owners are the KAT's miner ids (G stores an id class; here the class of the
// selfish miner is its id). Returns the resulting chain length (out arrays of cap entries).
uint32_t gen_kat(uint32_t sid, int64_t prop, int op, int64_t t, uint32_t bcs, const uint32_t *own, const int64_t *arr,
                 uint32_t n, const uint32_t *bown, const int64_t *barr, uint32_t bn, uint32_t *out_own, int64_t *out_arr,
                 uint32_t cap)
{
    const uint32_t wcap = 4096;
    uint64_t cum[2] = {50, 100};
    int64_t props[2] = {prop, prop};
    uint8_t self[2] = {1, 0};
    uint32_t cls[2] = {sid, 0xFFFFFFFEu};
    GenParams g;
    memset(&g, 0, sizeof(g));
    g.duration_ms = 1;
    g.mult = 0xFFFFFFFFFFFFFFFFull / 100;
    g.m = 2;
    g.umax = GEN_GENESIS;
    g.cum = cum;
    g.prop = props;
    g.self = self;
    g.cls = cls;
    HostStore s(2, wcap);
    for (uint32_t i = 0; i < n; ++i) s.put(0, i, own[i], arr[i]);
    s.set_size(0, n);
    for (uint32_t i = 0; i < bn; ++i) s.put(1, i, bown[i], barr[i]);
    s.set_size(1, bn);
    Gen<HostStore> e(s, g);
    e.bcs = (int32_t)bcs;
    e.now = t;
    if (op == 0) {
        e.found_block(0, t);
    } else {
        e.selfish_reveal(0, bn, t);  // simulation.h:177-180: reveal, then reorg
        e.reorg(0, 1, bn);
    }
    const uint32_t m = s.size(0);
    for (uint32_t i = 0; i < m && i < cap; ++i) {
        out_own[i] = s.own(0, i);
        out_arr[i] = s.arr(0, i);
    }
    return m;
}
}
