// selpipe_host.cpp — TEST INFRASTRUCTURE: a host (CPU) execution of the selfish pipeline
// (miningsimulation_amd/csrc/msim_selpipe.h) from the SAME lane bodies the gfx950 kernels run: K1's
// draw_segment with the nibble context, then per run sp_begin / sp_word / sp_enter / the engine / sp_counts,
// one lane at a time, so the decomposition can be checked run by run against the oracle without a GPU.
// Never part of the product path (libmsim.so is GPU-only).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../miningsimulation_amd/csrc/msim_dispatch.h"
#include "../../miningsimulation_amd/csrc/msim_jump.h"
#include "../../miningsimulation_amd/csrc/msim_selpipe.h"

using namespace msim;

namespace {

struct NibCtx {
    PipeLayout L;
    uint32_t r, seg, jb, ps, nsl = 0, nibw = 0, ma = 0, mb = 0;
    uint32_t cnt[CNT_WORDS] = {0};
    std::vector<uint32_t> *slots, *gcum, *nib;
    std::vector<CMask> *cmask;
    std::vector<uint64_t> *gend;
    std::vector<GroupRec> *grec;
    std::vector<EpEntry> *list;
    void count(uint32_t info)
    {
        const uint32_t k = info_finder(info);
        cnt[k >> 1] += 1u << (16u * (k & 1u));
        nibw = (nibw >> 4) | (k << 28);
    }
    bool vote(bool s) const { return s; }
    void quad() {}
    void quad_done(uint32_t g, uint32_t q4)
    {
        if (q4 & 1u) (*nib)[sp_nib_index(L.nr, r, seg * (L.seg / 8) + g * (GROUP / 8) + (q4 >> 1))] = nibw;
        if (q4 == GROUP / K1_QB - 1) {
            (*cmask)[((size_t)seg * (L.seg / GROUP) + g) * L.nr + r] = CMask{ma, mb};
            ma = mb = 0;
        }
    }
    void slow(bool s, uint32_t block, uint64_t offset, uint32_t w0, uint32_t w1, const Rng &ri, const Rng &rp,
              uint32_t fthr)
    {
        if (!s) return;
        ma |= 1u << (block & (GROUP - 1u));
        if ((w1 >> 5) + ps < fthr) mb |= 1u << (block & (GROUP - 1u));
        const uint32_t idx = (uint32_t)list->size();
        if (idx < L.lcap) list->push_back(EpEntry{r, block, offset, w0, w1, {0, 0}, ri, rp});
        if (nsl < L.cap) (*slots)[((size_t)seg * L.cap + nsl) * L.nr + r] = idx;
        ++nsl;
    }
    void group_start(uint32_t g, uint32_t w0, const Rng &ri, const Rng &rp)
    {
        if (g % SGROUP) return;  // records per super-group (as msim_drawgen.hip DevCtx<true>)
        const size_t gi = (size_t)jb * L.nsg + g / SGROUP;
        (*grec)[gi * L.nr + r] = GroupRec{ri, rp, w0, 0};
        for (uint32_t w = 0; w < CNT_WORDS; ++w) (*gcum)[(gi * CNT_WORDS + w) * L.nr + r] = cnt[w];
    }
    void group(uint32_t g, uint32_t, uint64_t end)
    {
        if (g % SGROUP == SGROUP - 1 || g + 1 == L.gps) (*gend)[((size_t)jb * L.nsg + g / SGROUP) * L.nr + r] = end;
    }
};

struct HostEnv {
    const int64_t *props;
    uint32_t c[4][MAXM];
    ColdAct cs[8];
    int64_t prop(uint32_t k) const { return props[k]; }
    int64_t prop_tab(uint32_t k) const { return props[k]; }
    uint32_t get(int a, uint32_t k) const { return c[a][k]; }
    void add(int a, uint32_t k, uint32_t v) { c[a][k] += v; }
    void set(int a, uint32_t k, uint32_t v) { c[a][k] = v; }
    ColdAct cold(int i) const { return cs[i]; }
    void cold_put(int i, const ColdAct &r) { cs[i] = r; }
    bool fold_vote(bool due) { return due; }
};

// Exact draws (glibc log1p, PickFinder by percentages) behind the device's draw FIFO.
struct HostDraw {
    Rng ri, rp;
    const uint64_t *cum;
    int m;
    void draw(uint32_t &I, uint32_t &k)
    {
        I = (uint32_t)next_interval(ri);
        const uint64_t q = rng_next(rp) / PERC_MULTIPLIER;
        uint32_t f = 0;
        while ((int)f < m && cum[f] <= q) ++f;
        k = f;
    }
};
using Fifo = SelFifo<HostDraw>;
struct EnvRef {  // SpSrc's found-counter access on the host: the lane's one HostEnv
    HostEnv *e;
    void add(uint32_t k, uint32_t v) { e->add(C_F, k, v); }
};

struct Stats {
    uint64_t words, enters, draw_enters, errors, slow;
};
Stats g_st;

template <int M>
int run_sp(const uint64_t *perc, const int64_t *prop, const uint8_t *self, int64_t D, uint32_t seed_base,
           uint64_t run_begin, uint32_t n, uint32_t cap_override, uint32_t wave_slots, uint32_t *found, uint32_t *stale,
           uint32_t *best_h, uint32_t *err)
{
    const double rho = sp_rho(perc, prop, self, M);
    SpLayout SL = sp_layout_for(rho, M, D, n, 1e18, wave_slots);
    PipeLayout &L = SL.L;
    L.nr = n;
    if (cap_override) L.cap = cap_override;
    L.lcap = 0xFFFFFFF0u;
    PickTab pick;
    LogTab logt;
    std::vector<uint32_t> jump((size_t)L.nseg * 128 * 4);
    build_pick_table_sp(perc, prop, self, M, &pick);
    build_log_table(&logt);
    build_jump_table(L.nseg, L.seg, jump.data());
    std::vector<GroupRec> grec((size_t)L.nband * L.nsg * n);
    std::vector<uint32_t> segcnt((size_t)L.nseg * CNT_WORDS * n), nslow((size_t)L.nseg * n),
        slots((size_t)L.nseg * L.cap * n, 0xFFFFFFFFu),
        gcum((size_t)L.nband * L.nsg * CNT_WORDS * n), nib((size_t)L.nb / 8 * n);
    std::vector<CMask> cmask((size_t)L.nb / 32 * n);
    uint32_t ps = 0;
    for (int k = 0; k < M; ++k)
        if (self[k]) ps = (uint32_t)prop[k];
    std::vector<uint64_t> segsum((size_t)L.nseg * n), gend((size_t)L.nband * L.nsg * n);
    std::vector<EpEntry> list;
    for (uint32_t r = 0; r < n; ++r) {
        const uint64_t run = run_begin + r;
        const Rng si = rng_seed(seed_interval(seed_base, run)), sp = rng_seed(seed_picker(seed_base, run));
        for (uint32_t j = 0; j < L.nseg; ++j) {
            Rng ri, rp;
            Mat128 mt;
            for (int c = 0; c < 128; ++c) {
                const uint32_t *w = &jump[((size_t)j * 128 + c) * 4];
                mt.lo[c] = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
                mt.hi[c] = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
            }
            mat_apply(mt, si.s0, si.s1, ri.s0, ri.s1);
            mat_apply(mt, sp.s0, sp.s1, rp.s0, rp.s1);
            NibCtx cx;
            cx.L = L;
            cx.r = r;
            cx.seg = j;
            cx.jb = j - L.band_lo;
            cx.grec = &grec;
            cx.slots = &slots;
            cx.gend = &gend;
            cx.gcum = &gcum;
            cx.list = &list;
            cx.nib = &nib;
            cx.cmask = &cmask;
            cx.ps = ps;
            segsum[(size_t)j * n + r] = draw_segment<NibCtx, true>(cx, ri, rp, &logt, &pick, j * L.seg, L.seg, j >= L.band_lo);
            for (uint32_t w = 0; w < CNT_WORDS; ++w) segcnt[((size_t)j * CNT_WORDS + w) * n + r] = cx.cnt[w];
            nslow[(size_t)j * n + r] = cx.nsl;
        }
    }
    SpArgs a;
    a.nr = n;
    a.seg = L.seg;
    a.nsg = L.nsg;
    a.nseg = L.nseg;
    a.nb = L.nb;
    a.cap = L.cap;
    a.band_lo = L.band_lo;
    a.lcap = (uint32_t)list.size() + 1;
    a.segsum = segsum.data();
    a.segcnt = segcnt.data();
    a.nslow = nslow.data();
    a.slots = slots.data();
    a.gend = gend.data();
    a.gcum = gcum.data();
    a.grec = grec.data();
    a.list = list.data();
    a.nib = nib.data();
    a.cmask = cmask.data();
    std::vector<uint32_t> stalev((size_t)L.nb / 32 * n, 0u);
    a.stale = stalev.data();
    uint32_t lut[SP_LUT];
    for (int i = 0; i < SP_LUT; ++i) lut[i] = sp_lut_entry((uint32_t)i / 16u, (uint32_t)i % 16u);
    auto vote = [](bool b) { return b; };
    uint64_t cum[MAXM];
    uint64_t c = 0;
    uint32_t sids[SEL_MAXS] = {SEL_NONE, SEL_NONE, SEL_NONE, SEL_NONE};
    for (int k = 0; k < M; ++k) {
        cum[k] = (c += perc[k]);
        if (self[k]) sids[0] = (uint32_t)k;
    }
    const uint32_t sid = sids[0];
    int64_t thr = 0;
    for (int k = 0; k < M; ++k)
        if (!self[k]) thr = prop[k] + prop[sid] > thr ? prop[k] + prop[sid] : thr;
    for (uint32_t r = 0; r < n; ++r) {
        HostEnv env;
        env.props = prop;
        memset(env.c, 0, sizeof(env.c));
        memset(env.cs, 0, sizeof(env.cs));
        SpCur cur;
        HostDraw drw;
        drw.cum = cum;
        drw.m = M;
        sp_begin(a, r, D, thr, drw, cur);
        SpSt st;
        st.F = st.h = st.w = st.sst = st.prs = st.pxf = st.smask = st.schunk = st.hbits = 0;
        Sel<M, 1, 1, 4, 1, 4> s;
        SpSrc<Fifo, EnvRef> src;
        src.f.d.cum = cum;
        src.f.d.m = M;
        src.f.n = 0;
        src.cnt = EnvRef{&env};
        src.pidx = SP_NONE;
        src.pk = 0;
        src.B = cur.B;
        SelOut out;
        memset(&out, 0, sizeof(out));
        int mode = cur.err ? 3 : 0;
        uint32_t ring = 0;
        while (mode != 3) {  // as msim_selpipe_kernel, one lane
            if (mode == 0) {
                ++g_st.words;
                // ring slot: table steps since the last refill, mod SP_PF (as the kernel's unrolled steps)
                switch (ring++ % SP_PF) {
                case 0: mode = sp_chunk<M, 0>(a, r, env, vote, lut, cur, st, sid); break;
                case 1: mode = sp_chunk<M, 1 % SP_PF>(a, r, env, vote, lut, cur, st, sid); break;
                case 2: mode = sp_chunk<M, 2 % SP_PF>(a, r, env, vote, lut, cur, st, sid); break;
                default: mode = sp_chunk<M, 3 % SP_PF>(a, r, env, vote, lut, cur, st, sid); break;
                }
            } else if (mode == 9) {
                ++g_st.slow;
                mode = sp_slow_word<M>(a, r, env, cur, st, sid, D);
                if (mode == 0) {
                    sp_refill(a, r, cur);
                    ring = 0;
                }
            } else if (mode == 6) {
                sp_finish<M>(env, st, sid, out);
                mode = 3;
            } else if (mode == 1 || mode == 4) {
                ++(mode == 1 ? g_st.enters : g_st.draw_enters);
                mode = sp_enter<M>(a, r, mode, cur, st, src, s, env, (uint32_t)M, sids);
            } else {  // the engine
                if (!s.step(env, src, D)) {
                    s.finish(env, D, out);
                    mode = 3;
                } else if (src.pidx < src.B) {
                    SelMacro<M> tb;
                    if (tb.take_back(env, s, sid)) {
                        sp_handback<M>(env, tb, st, src.pidx, sid);
                        sp_seek(a, r, cur, src.pidx);
                        mode = (cur.pos & 7u) ? sp_slow_word<M>(a, r, env, cur, st, sid, D) : 0;
                        if (mode == 0) {
                    sp_refill(a, r, cur);
                    ring = 0;
                }
                    }
                }
            }
        }
        uint32_t e = cur.err | out.err;
        if (e) ++g_st.errors;
        uint32_t F[M], X[M];
        if (!e) {
            sp_counts<M>(a, r, cur, F);
            sp_stale_counts<M>(a, r, st, sid, X);
        }
        for (int k = 0; k < M; ++k) {
            found[(size_t)r * M + k] = e ? 0 : out.found[k] + F[k] - X[k];
            stale[(size_t)r * M + k] = e ? 0 : out.stale[k] + X[k];
        }
        best_h[r] = e ? 0 : out.best_height;
        err[r] = e;
    }
    return 0;
}

}  // namespace

extern "C" void selpipe_stats(uint64_t *out)
{
    out[0] = g_st.words;
    out[1] = g_st.enters;
    out[2] = g_st.draw_enters;
    out[3] = g_st.errors;
    out[4] = g_st.slow;
    g_st = Stats{0, 0, 0, 0, 0};
}

// perc (integer percentages summing to 100), prop, selfish (exactly one), m miners. Per run: found/stale [n][m],
// best height, err (nonzero: the device would flag the run for E2).
extern "C" int selpipe_run(const uint64_t *perc, const int64_t *prop, const uint8_t *selfish, int m, int64_t duration_ms,
                           uint32_t seed_base, uint64_t run_begin, uint32_t n, uint32_t cap_override, uint32_t wave_slots,
                           uint32_t *found, uint32_t *stale, uint32_t *best_h, uint32_t *err)
{
    int ns = 0;
    uint64_t tot = 0;
    for (int k = 0; k < m; ++k) {
        ns += selfish[k] ? 1 : 0;
        tot += perc[k];
        if (prop[k] < 1) return -4;
    }
    if (ns != 1) return -3;
    if (tot != 100) return -2;
#define CASE(MM) \
    case MM:     \
        return run_sp<MM>(perc, prop, selfish, duration_ms, seed_base, run_begin, n, cap_override, wave_slots, found, stale, best_h, err);
    switch (m) { MSIM_FOR_EACH_M(CASE) default: return -1; }
#undef CASE
}
