// selseg_host.cpp — TEST INFRASTRUCTURE: a host (CPU) build of the segment-parallel selfish path's lane bodies
// (miningsimulation_amd/csrc/msim_selseg.h: the SW workers and the ST stitch, with the entity engine of
// msim_sel.h inline) so that the decomposition can be checked against the oracle run by run on machines without
// a GPU. Never part of the product path (libmsim.so is GPU-only).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../miningsimulation_amd/csrc/msim_dispatch.h"
#include "../../miningsimulation_amd/csrc/msim_selseg.h"

using namespace msim;

namespace {

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

// The reference's draws (simulation.h:205-221) with integer weights summing to W.
struct HostDraw {
    Rng ri, rp;
    const uint64_t *cum;
    int m;
    uint64_t mult;
    void draw(uint32_t &I, uint32_t &k)
    {
        I = (uint32_t)next_interval(ri);
        const uint64_t q = rng_next(rp) / mult;
        uint32_t f = 0;
        while ((int)f < m && cum[f] <= q) ++f;
        k = f;
    }
};
using Src = SegFifo<HostDraw>;

struct LutInit {
    uint32_t t[SP_LUT];
    LutInit()
    {
        for (int i = 0; i < SP_LUT; ++i) t[i] = sp_lut_entry((uint32_t)i / 16u, (uint32_t)i % 16u);
    }
};
const LutInit g_lut;

template <int M>
struct HostRecs {
    std::vector<std::vector<SegRec<M>>> segs;
    std::vector<std::vector<SegQRec<M>>> qs;
    uint32_t count(uint32_t j) const { return j < segs.size() ? (uint32_t)segs[j].size() : 0u; }
    SegRec<M> rec(uint32_t j, uint32_t q) const { return segs[j][q]; }
    void head(uint32_t j, uint32_t q, uint32_t &b, uint32_t &flags) const
    {
        b = segs[j][q].b;
        flags = segs[j][q].flags;
    }
    uint32_t qcount(uint32_t j) const { return j < qs.size() ? (uint32_t)qs[j].size() : 0u; }
    uint32_t qc(uint32_t j, uint32_t i) const { return qs[j][i].c; }
    uint32_t qspan(uint32_t j, uint32_t i) const { return qs[j][i].span; }
    SegQRec<M> qrec(uint32_t j, uint32_t i) const { return qs[j][i]; }
};

struct Stats {
    uint64_t subs, cuts, quiet, jumps, walk_steps, engine_entries, end_steps;
};
Stats g_st;
int g_true_only = 0;
int g_verify = 0;     // diagnostics: every jump checked against the true state's own walk (stderr)
uint32_t g_qcap = 0;  // checkpoint room per segment (0: cap * SEG_QWIN)  // diagnostics: the true state alone (no jumps)

template <int M>
int run_seg(const int64_t *prop, uint32_t sid, const uint64_t *cum, uint64_t mult, int64_t D, uint32_t seed_i,
            uint32_t seed_p, uint32_t nseg, uint32_t seg, uint32_t cap, SelOut &o)
{
    int64_t thrmax = 0;
    for (int j = 0; j < M; ++j)
        if ((uint32_t)j != sid) thrmax = prop[j] + prop[sid] > thrmax ? prop[j] + prop[sid] : thrmax;
    const uint32_t sids[SEL_MAXS] = {sid, SEL_NONE, SEL_NONE, SEL_NONE};
    auto make_src = [&](uint32_t first) {
        Src s;
        s.d.ri = rng_seed(seed_i);
        s.d.rp = rng_seed(seed_p);
        for (uint32_t i = 0; i < first; ++i) {  // the device jumps (msim_jump.h); the host steps
            rng_next(s.d.ri);
            rng_next(s.d.rp);
        }
        s.d.cum = cum;
        s.d.m = M;
        s.d.mult = mult;
        s.n = 0;
        s.idx = first;
        return s;
    };
    // SW: every segment's worker
    HostRecs<M> R;
    R.segs.resize(nseg);
    R.qs.resize(nseg);
    bool overflow = false;
    for (uint32_t j = 0; j < nseg; ++j) {
        HostEnv ew;
        ew.props = prop;
        memset(ew.c, 0, sizeof(ew.c));
        Src src = make_src(j * seg);
        auto emit = [&](const SegRec<M> &r) {
            if (R.segs[j].size() >= cap) return false;
            R.segs[j].push_back(r);
            ++g_st.subs;
            g_st.cuts += (r.flags & SEG_CUT) ? 1 : 0;
            return true;
        };
        struct EmitQ {
            std::vector<SegQRec<M>> *v;
            size_t cap;
            bool operator()(const SegQRec<M> &r)
            {
                if (v->size() >= cap) return false;
                v->push_back(r);
                ++g_st.quiet;
                return true;
            }
            uint32_t n() const { return (uint32_t)v->size(); }
        } emitq{&R.qs[j], g_qcap ? (size_t)g_qcap : (size_t)cap * SEG_QWIN};
        if (seg_work<M>(ew, src, (j + 1) * seg, sid, prop[sid], thrmax, g_lut.t, emit, emitq)) overflow = true;
    }
    if (overflow) return 1;  // the device flags the run for E2
    // ST: the stitch with the engine inline
    HostEnv et;
    et.props = prop;
    memset(et.c, 0, sizeof(et.c));
    memset(et.cs, 0, sizeof(et.cs));
    Src st = make_src(0);
    SegStitch<M> S;
    S.err = 0;
    S.seg = S.q = S.qi = S.at_rec = 0;
    S.walk_back = 1;
    if (!S.X.begin(st)) return 2;
    if (S.X.T >= D) {
        S.X.finish(et, sid, o);
        return 0;
    }
    S.mode = g_true_only ? ST_END : ST_WALK;
    for (;;) {
        if (S.mode == ST_DONE) {
            if (S.err) {
                o.err = S.err;
                return 3;
            }
            S.X.finish(et, sid, o);
            return 0;
        }
        if (S.mode == ST_ENGINE) {
            ++g_st.engine_entries;
            Sel<M, 1, 1, 4, 1, 4> s;
            S.X.to_exact(et, s, (uint32_t)M, sids);
            for (;;) {
                if (!s.step(et, st, D)) {
                    s.finish(et, D, o);
                    return o.err ? 4 : 0;
                }
                if (S.X.take_back(et, s, sid)) break;
            }
            if (S.X.T >= D) {
                S.X.finish(et, sid, o);
                return 0;
            }
            st.fill();
            S.mode = S.walk_back ? ST_WALK : ST_END;
            continue;
        }
        const uint32_t before = S.mode;
        if (g_verify && S.mode == ST_JUMP) {
            SegStitch<M> S2 = S;
            HostEnv e2 = et;
            Src s2 = st;
            const SegRec<M> r = R.rec(S.seg, S.q);
            int x = 0;
            uint32_t i0 = s2.idx - 1u, qi0 = S.qi;
            while (s2.idx - 1u < r.b && x == 0) {
                x = S2.X.step1(e2, s2, D, sid, prop[sid]);
                s2.fill();
            }
            S2.X.flush_stale(e2, sid);
            seg_stitch_step<M>(S, R, et, st, D, sid, prop[sid], thrmax, g_lut.t);
            if (S.mode != ST_END) {
                bool ok = x == 0 && s2.idx == st.idx && S2.X.F == S.X.F && S2.X.T == S.X.T && S2.X.h == S.X.h && S2.X.w == S.X.w;
                for (int k = 0; k < M; ++k) ok &= e2.c[0][k] == et.c[0][k] && e2.c[1][k] == et.c[1][k];
                if (!ok && g_verify++ < 4) {
                    fprintf(stderr, "JUMP mismatch at_rec %u i0 %u b %u x %d idx %u/%u F %u/%u T %lld/%lld h %u/%u w %u/%u\n",
                            S2.at_rec, i0, r.b, x, s2.idx, st.idx, S2.X.F, S.X.F, (long long)S2.X.T, (long long)S.X.T,
                            S2.X.h, S.X.h, S2.X.w, S.X.w);
                    for (int k = 0; k < M; ++k) fprintf(stderr, " %u/%u:%u/%u", e2.c[0][k], et.c[0][k], e2.c[1][k], et.c[1][k]);
                    fprintf(stderr, "\n");
                    fprintf(stderr, "rec flags %u span %llu dFh %u qn %u; S.qi %u->%u; checkpoints:", r.flags, (unsigned long long)r.span, r.dFh, r.qn, qi0, S.qi);
                    for (uint32_t j = 0; j < R.qcount(S2.seg); ++j)
                        if (R.qc(S2.seg, j) + 80 > i0 && R.qc(S2.seg, j) < r.b + 30) fprintf(stderr, " [%u] c%u s%u f%u", j, R.qc(S2.seg, j), R.qspan(S2.seg, j), R.qrec(S2.seg, j).dFh);
                    fprintf(stderr, "\n");
                }
            }
            ++g_st.jumps;
            continue;
        }
        seg_stitch_step<M>(S, R, et, st, D, sid, prop[sid], thrmax, g_lut.t);
        g_st.jumps += before == ST_JUMP ? 1 : 0;
        g_st.walk_steps += before == ST_WALK ? 1 : 0;
        g_st.end_steps += before == ST_END ? 1 : 0;
    }
}

}  // namespace

extern "C" void selseg_true_only(int on) { g_true_only = on; }
extern "C" void selseg_verify(int on) { g_verify = on; }
extern "C" void selseg_qcap(uint32_t n) { g_qcap = n; }

extern "C" void selseg_stats(uint64_t *out)
{
    out[0] = g_st.subs;
    out[1] = g_st.cuts;
    out[2] = g_st.jumps;
    out[3] = g_st.walk_steps;
    out[4] = g_st.engine_entries;
    out[5] = g_st.end_steps;
    out[6] = g_st.quiet;
    g_st = Stats{0, 0, 0, 0, 0, 0, 0};
}

// One run of a network with ONE selfish miner (weights summing to W, every delay >= 1 ms) through SW + ST with
// nseg segments of seg blocks (cap subs per segment). Returns 0 (results in found/stale/best_height), 1 (a
// segment overflowed its subs: the device hands the run to E2), or an error code.
extern "C" int selseg_run(const uint64_t *weights, const int64_t *prop, const uint8_t *selfish, int m, uint64_t W,
                          int64_t duration_ms, uint32_t seed_i, uint32_t seed_p, uint32_t nseg, uint32_t seg,
                          uint32_t cap, uint32_t *found, uint32_t *stale, uint32_t *best_height, uint32_t *err)
{
    if (m < 1 || m > MAXM || W == 0) return -1;
    uint64_t cum[MAXM];
    uint64_t c = 0;
    int ns = 0;
    uint32_t sid = 0;
    for (int k = 0; k < m; ++k) {
        c += weights[k];
        cum[k] = c;
        if (selfish[k]) {
            ++ns;
            sid = (uint32_t)k;
        }
        if (prop[k] < 1) return -4;
    }
    if (c != W || ns != 1) return -2;
    SelOut o;
    memset(&o, 0, sizeof(o));
    int rc = -1;
#define CASE(MM) \
    case MM:     \
        rc = run_seg<MM>(prop, sid, cum, 0xFFFFFFFFFFFFFFFFull / W, duration_ms, seed_i, seed_p, nseg, seg, cap, o); \
        break;
    switch (m) { MSIM_FOR_EACH_M(CASE) default: return -1; }
#undef CASE
    for (int k = 0; k < m; ++k) {
        found[k] = o.found[k];
        stale[k] = o.stale[k];
    }
    *best_height = o.best_height;
    *err = o.err;
    return rc;
}
