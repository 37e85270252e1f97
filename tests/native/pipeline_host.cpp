// pipeline_host.cpp — TEST INFRASTRUCTURE: a host (CPU) execution of the event-skipping pipeline
// (miningsimulation_amd/csrc/msim_pipeline.h) built from the SAME lane bodies the gfx950 kernels run
// (draw_segment, episode_entry, combine_run), so the decomposition can be checked against the
// oracle on machines without a GPU. Also checks every jump-ahead state against sequential stepping.
// Never part of the product path (libmsim.so is GPU-only).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../miningsimulation_amd/csrc/msim_dispatch.h"
#include "../../miningsimulation_amd/csrc/msim_jump.h"
#include "../../miningsimulation_amd/csrc/msim_pipeline.h"

using namespace msim;

namespace {

struct HostCtx {
    PipeLayout L;
    uint32_t r, seg, jb, nsl = 0;
    uint32_t cnt[CNT_WORDS] = {0};
    std::vector<uint32_t> *slots, *gsum, *gcum;
    std::vector<uint64_t> *gend;
    std::vector<GroupRec> *grec;
    std::vector<EpEntry> *list;
    void count(uint32_t info)
    {
        const uint32_t k = info_finder(info);
        cnt[k >> 1] += 1u << (16u * (k & 1u));
    }
    bool vote(bool s) const { return s; }
    void quad() {}
    void slow(bool s, uint32_t block, uint64_t offset, uint32_t w0, uint32_t w1, const Rng &ri, const Rng &rp, uint32_t skip)
    {
        if (!s) return;
        const uint32_t idx = (uint32_t)list->size();
        if (idx < L.lcap) list->push_back(EpEntry{r, block, offset, w0, w1, skip, 0, ri, rp});
        if (nsl < L.cap) (*slots)[((size_t)seg * L.cap + nsl) * L.nr + r] = idx;
        ++nsl;
    }
    void group_start(uint32_t g, uint32_t w0, const Rng &ri, const Rng &rp)
    {
        (*grec)[((size_t)jb * L.gps + g) * L.nr + r] = GroupRec{ri, rp, w0, 0};
        for (uint32_t w = 0; w < CNT_WORDS; ++w) (*gcum)[(((size_t)jb * L.gps + g) * CNT_WORDS + w) * L.nr + r] = cnt[w];
    }
    void group(uint32_t g, uint32_t sum, uint64_t end)
    {
        (*gsum)[((size_t)jb * L.gps + g) * L.nr + r] = sum;
        if (g % SGROUP == SGROUP - 1 || g + 1 == L.gps) (*gend)[((size_t)jb * L.nsg + g / SGROUP) * L.nr + r] = end;
    }
};

template <int M>
int run_pipeline(const SimParams &p, const uint64_t *perc, const int64_t *prop, const uint8_t *self, double rho,
                 uint32_t seed_base, uint64_t run_begin, uint32_t n, uint32_t cap_override, uint32_t wave_slots, uint32_t *found,
                 uint32_t *stale, uint8_t *ok, uint32_t *n_episodes)
{
    PipeLayout L = pipe_layout_for(rho, M, p.duration_ms, n, 1e18, wave_slots);
    L.nr = n;  // no padding on the host
    if (cap_override) L.cap = cap_override;
    L.lcap = 0xFFFFFFF0u;
    PickTab pick;
    LogTab logt;
    std::vector<uint32_t> jump((size_t)L.nseg * 128 * 4);
    build_pick_table(perc, prop, self, M, &pick);
    build_log_table(&logt);
    build_jump_table(L.nseg, L.seg, jump.data());
    std::vector<GroupRec> grec((size_t)L.nband * L.gps * n);
    std::vector<uint32_t> segcnt((size_t)L.nseg * CNT_WORDS * n), nslow((size_t)L.nseg * n),
        slots((size_t)L.nseg * L.cap * n, 0xFFFFFFFFu), gsum((size_t)L.nband * L.gps * n),
        gcum((size_t)L.nband * L.gps * CNT_WORDS * n);
    std::vector<uint64_t> segsum((size_t)L.nseg * n), gend((size_t)L.nband * L.nsg * n);
    std::vector<EpEntry> list;
    for (uint32_t r = 0; r < n; ++r) {
        const uint64_t run = run_begin + r;
        Rng si = rng_seed(seed_interval(seed_base, run)), sp = rng_seed(seed_picker(seed_base, run));
        Rng qi = si, qp = sp;  // sequential reference states
        for (uint32_t j = 0; j < L.nseg; ++j) {
            Rng ri, rp;
            Mat128 m;
            for (int c = 0; c < 128; ++c) {
                const uint32_t *w = &jump[((size_t)j * 128 + c) * 4];
                m.lo[c] = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
                m.hi[c] = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
            }
            mat_apply(m, si.s0, si.s1, ri.s0, ri.s1);
            mat_apply(m, sp.s0, sp.s1, rp.s0, rp.s1);
            if (ri.s0 != qi.s0 || ri.s1 != qi.s1 || rp.s0 != qp.s0 || rp.s1 != qp.s1) return -100;  // jump broken
            for (uint32_t i = 0; i < L.seg; ++i) {
                rng_next(qi);
                rng_next(qp);
            }
            HostCtx cx;
            cx.L = L;
            cx.r = r;
            cx.seg = j;
            cx.jb = j - L.band_lo;
            cx.grec = &grec;
            cx.slots = &slots;
            cx.gsum = &gsum;
            cx.gend = &gend;
            cx.gcum = &gcum;
            cx.list = &list;
            segsum[(size_t)j * n + r] = draw_segment(cx, ri, rp, &logt, &pick, j * L.seg, L.seg, j >= L.band_lo);
            for (uint32_t w = 0; w < CNT_WORDS; ++w) segcnt[((size_t)j * CNT_WORDS + w) * n + r] = cx.cnt[w];
            nslow[(size_t)j * n + r] = cx.nsl;
        }
    }
    std::vector<uint32_t> recs(list.size() * L.rec_words + 1);
    uint32_t count = (uint32_t)list.size();
    PipeArgs a;
    a.nr = n;
    a.seg = L.seg;
    a.gps = L.gps;
    a.nseg = L.nseg;
    a.nb = L.nb;
    a.cap = L.cap;
    a.band_lo = L.band_lo;
    a.lcap = L.lcap;
    a.rec_words = L.rec_words;
    a.tab = PipeTables{&pick, &logt, jump.data()};
    a.grec = grec.data();
    a.segsum = segsum.data();
    a.segcnt = segcnt.data();
    a.nslow = nslow.data();
    a.slots = slots.data();
    a.gsum = gsum.data();
    a.gend = gend.data();
    a.gcum = gcum.data();
    a.list = list.data();
    a.list_count = &count;
    a.recs = recs.data();
    for (uint32_t i = 0; i < count; ++i) {
        if (L.k2_kind == 0) episode_entry<M, 0>(p, a, i);
        else if (L.k2_kind == 1) episode_entry<M, 1>(p, a, i);
        else episode_entry<M, 2>(p, a, i);
    }
    for (uint32_t r = 0; r < n; ++r) {
        uint32_t F[M], S[M];
        uint32_t nsw[K3_SCRATCH];
        ok[r] = combine_run<M>(p, a, r, F, S, nsw, 1) ? 1 : 0;
        for (int k = 0; k < M; ++k) {
            found[(size_t)r * M + k] = F[k];
            stale[(size_t)r * M + k] = S[k];
        }
    }
    *n_episodes = count;
    return 0;
}

}  // namespace

extern "C" int pipeline_run(const uint64_t *perc, const int64_t *prop, const uint8_t *selfish, int m,
                            int64_t duration_ms, uint32_t seed_base, uint64_t run_begin, uint32_t n,
                            uint32_t cap_override, uint32_t wave_slots, uint32_t *found, uint32_t *stale, uint8_t *ok,
                            uint32_t *n_episodes)
{
    SimParams p;
    const int rc = make_params(perc, prop, selfish, m, duration_ms, &p);
    if (rc) return rc;
    if (p.selfish >= 0) return -50;  // the pipeline serves honest networks
    double rho = 0;
    for (int k = 0; k < m; ++k) rho += (double)perc[k] / 100.0 * (1.0 - exp(-((double)prop[k] + 1.0) / 599999.5));
#define CASE(MM) \
    case MM:     \
        return run_pipeline<MM>(p, perc, prop, selfish, rho, seed_base, run_begin, n, cap_override, wave_slots, found, stale, ok, n_episodes);
    switch (m) { MSIM_FOR_EACH_M(CASE) default: return -1; }
#undef CASE
}
