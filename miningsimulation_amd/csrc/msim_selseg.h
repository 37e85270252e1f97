// msim_selseg.h — segment-parallel runs for networks with ONE selfish miner (BASELINE configs[2]): speculative
// settled-form workers per time segment, stitched together per run, exact.
//
// Why. E1 (msim_sel_kernels.hip) runs one lane per run. configs[2] has 131 072 runs per GPU, i.e. 2 048 waves:
// two waves per SIMD whatever the kernel's registers, and every latency of the settled form's dependent chain is
// exposed. More independent work per run needs more lanes per run. The draws are parallel
// (GF(2) jump-ahead, msim_jump.h); the settled form is not, because each find's transition depends on the
// state the previous finds left. It becomes parallel by speculation and coalescence:
//
//   SW  (worker, one lane per (run, segment)): the settled form (msim_selm.h SelMacro, every transition of
//       simulation.h:62-180 that settles before the next find) from the QUIET state (h = w = 0, no honest
//       branch) at the segment's first block, with no end of run (D = infinity). A find that needs the entity
//       engine (simulation.h:124-174 events that overlap the next find) is a CUT: the worker records its state
//       there and restarts from the quiet state at the next block. Between restarts lies a SUB: the worker
//       records, at its end, the settled state, the per-miner counter deltas of the sub, its time span and its
//       draw source (RNG states and held draws), so the sub can be resumed or replayed.
//   ST  (stitch, one lane per run): the run's TRUE state walks the subs in block order. Where the true state
//       equals the worker's state at the same pending block, every later transition of the sub is identical
//       (the settled state (h, w, honest-branch composition) and the draws determine the future; counters are
//       accumulators), so the stitch adds the sub's deltas and jumps to its end (JUMP). At a CUT the true state
//       is the worker's, so it needs the engine there too: ST runs the entity engine (msim_sel.h) until the
//       network is settled again, then replays the worker (from the quiet restart after the cut) beside the
//       true state, one find at a time, until both are settled at the same block in the same state (WALK:
//       any honest find at lead 0 or 2 resolves both branches to quiet, so this takes a few finds); from there
//       the sub's remaining deltas are the true ones. A segment boundary is handled like a cut without the
//       engine: the next segment's worker started quiet there.
//   The end of the run (main.cpp:150, 185-189) is the only absolute-time dependence: a sub is jumped only if
//   the settle threshold of its last find lies before D (its end time + the largest threshold < D); the sub
//   that holds the end is replayed by the true state alone, settled form and engine, with the real D.
//
// Exactness: both the settled form and the engine are exact restatements of the reference's event loop
// (msim_selm.h, msim_sel.h), so the true state's walk is the reference's run; a jump replaces a stretch of
// transitions by the worker's identical ones. tests/native/selseg_host.cpp runs these lane bodies on the host
// against the oracle run by run.
#pragma once
#include "msim_selm.h"

namespace msim {

constexpr uint32_t SEG_CUT = 1u;  // the sub ends at a find that needs the engine
constexpr uint32_t SEG_END = 2u;  // the sub ends at its segment's end (the next segment's first block)
constexpr int64_t SEG_NO_END = 0x3FFFFFFFFFFFFFFFll;  // the workers' D: no end of run

// A held-draw FIFO (msim_selm.h SelFifo) that counts the draws it hands out: idx is the index of the next
// draw a pop returns, so idx - 1 is the index of a SelMacro's pending find.
template <class D>
struct SegFifo : SelFifo<D> {
    uint32_t idx;
    MSIM_HD void pop()
    {
        SelFifo<D>::pop();
        ++idx;
    }
    MSIM_HD void pop_if(bool p)
    {
        SelFifo<D>::pop_if(p);
        idx += p ? 1u : 0u;
    }
    MSIM_HD bool next(uint32_t &I, uint32_t &k)
    {
        this->peek(I, k);
        pop();
        return true;
    }
    MSIM_HD void took4()
    {
        this->n = 0u;
        idx += 4u;
    }
};

// One sub of a worker, recorded at its end (block b pending).
template <int M>
struct SegRec {
    static constexpr int NP = SelMacro<M>::NP;
    uint32_t b;        // index of the pending find at the end
    uint32_t flags;    // SEG_CUT / SEG_END
    uint32_t h, w;     // settled state at b
    uint32_t kb;       // finder of block b
    uint32_t dFh;      // increase of the common prefix F over the sub
    uint32_t n;        // held draws
    uint32_t I[4], k[4];
    uint64_t span;     // time from the sub's first pending find to find b
    uint64_t pend[NP];
    Rng ri, rp;        // the streams after the held draws
    uint32_t dF[M], dS[M];  // counter deltas over the sub (C_F, C_S), stale blocks flushed at b
};

template <int M>
MSIM_HD bool seg_same(const SelMacro<M> &a, const SelMacro<M> &b)
{
    bool eq = (a.h == b.h) & (a.w == b.w);
#pragma unroll
    for (int i = 0; i < SelMacro<M>::NP; ++i) eq &= a.pend[i] == b.pend[i];
    return eq;
}
template <int M>
MSIM_HD bool seg_quiet(const SelMacro<M> &a)
{
    bool q = (a.h == 0u) & (a.w == 0u);
#pragma unroll
    for (int i = 0; i < SelMacro<M>::NP; ++i) q &= a.pend[i] == 0ull;
    return q;
}
// The quiet state with pending find k (time T): what a worker starts from (SelMacro::begin without the draw).
template <int M>
MSIM_HD void seg_set_quiet(SelMacro<M> &a, uint32_t k, int64_t T)
{
    a.T = T;
    a.k = k;
    a.F = a.h = a.w = a.sst = a.Ff = 0u;
#pragma unroll
    for (int i = 0; i < SelMacro<M>::NP; ++i) a.pend[i] = a.stp[i] = 0ull;
}

template <int M, class Src>
MSIM_HD void seg_snapshot(SegRec<M> &r, const Src &src)
{
    r.ri = src.d.ri;
    r.rp = src.d.rp;
    r.n = src.n;
    r.I[0] = src.I0; r.I[1] = src.I1; r.I[2] = src.I2; r.I[3] = src.I3;
    r.k[0] = src.k0; r.k[1] = src.k1; r.k[2] = src.k2; r.k[3] = src.k3;
}
template <int M, class Src>
MSIM_HD void seg_resume(Src &src, const SegRec<M> &r)
{
    src.d.ri = r.ri;
    src.d.rp = r.rp;
    src.n = r.n;
    src.I0 = r.I[0]; src.I1 = r.I[1]; src.I2 = r.I[2]; src.I3 = r.I[3];
    src.k0 = r.k[0]; src.k1 = r.k[1]; src.k2 = r.k[2]; src.k3 = r.k[3];
    src.idx = r.b + 1u;
    src.fill();
}

// SW lane body: the worker of one segment, blocks [first, e) (src positioned at draw `first`, src.idx = first).
// Env: the worker's counter rows C_F / C_S (zero at entry), prop_tab. emit(rec) stores a sub; returns false when
// the caller cannot hold it (the run is then recomputed by E2). Returns 0 or an SERR_* code.
template <int M, class Env, class Src, class Emit>
MSIM_HD uint32_t seg_work(Env &env, Src &src, uint32_t e, uint32_t sid, int64_t ps, int64_t thrmax, const uint32_t *lut,
                          Emit &emit)
{
    SelMacro<M> mc;
    if (!mc.begin(src)) return SERR_DRAWS;
    int64_t T0 = mc.T;
    SegRec<M> r;
    for (;;) {
        const uint32_t i = src.idx - 1u;
        uint32_t fl = 0;
        if (i >= e) {
            fl = SEG_END;
        } else {
            const int x = (i + 4u <= e) ? mc.step4(env, src, SEG_NO_END, sid, ps, thrmax, lut)
                                        : mc.step1(env, src, SEG_NO_END, sid, ps);
            if (x == 1) fl = SEG_CUT;
            src.fill();  // step4 (SelFifo::top4) needs two held draws
        }
        if (fl) {
            mc.flush_stale(env, sid);
            r.b = src.idx - 1u;
            r.flags = fl;
            r.h = mc.h;
            r.w = mc.w;
            r.kb = mc.k;
            r.dFh = mc.F;
            r.span = (uint64_t)(mc.T - T0);
#pragma unroll
            for (int j = 0; j < SegRec<M>::NP; ++j) r.pend[j] = mc.pend[j];
            seg_snapshot<M>(r, src);
#pragma unroll
            for (int kk = 0; kk < M; ++kk) {
                r.dF[kk] = env.get(C_F, (uint32_t)kk);
                r.dS[kk] = env.get(C_S, (uint32_t)kk);
                env.set(C_F, (uint32_t)kk, 0u);
                env.set(C_S, (uint32_t)kk, 0u);
            }
            if (!emit(r)) return SERR_CAP;
            if (fl == SEG_END) return 0;
            mc.begin(src);  // the quiet restart after the cut (pending find b + 1)
            T0 = mc.T;
        }
    }
}

// ST lane state: the run's true settled state X (absolute time, real D) and the worker's replayed trajectory W
// (D = infinity, restarted exactly where the worker restarted), each with its own draw source.
enum : uint32_t { ST_JUMP = 0, ST_WALK = 1, ST_ENGINE = 2, ST_END = 3, ST_DONE = 4 };
template <int M>
struct SegStitch {
    SelMacro<M> X, W;
    int64_t WT0;       // W.T at the start of its sub
    uint32_t seg, q;   // W's sub (in JUMP: the sub to jump)
    uint32_t mode;
    uint32_t wnew;     // after the engine: W restarts from the cut record (seg, q - 1)
    uint32_t walk_back;  // after the engine: back to WALK (1) or END (0)
    uint32_t err;
};

// Rec access: const SegRec<M> &rec(seg, q) (or a copy), uint32_t count(seg), nseg.
// EnvT: the true counters (C_F, C_S, C_A, C_B); EnvW: the replayed worker's (C_F, C_S only).
// One action of a lane that is not in the engine; returns its new mode. ST_ENGINE: X needs the entity engine at
// its pending find (the caller converts X with to_exact, steps the engine, and calls seg_after_engine).
template <int M, class Recs, class EnvT, class EnvW, class Src>
MSIM_HD uint32_t seg_stitch_step(SegStitch<M> &S, const Recs &R, EnvT &et, EnvW &ew, Src &st, Src &sw, int64_t D,
                                 uint32_t sid, int64_t ps, int64_t thrmax, const uint32_t *lut)
{
    if (S.mode == ST_JUMP) {
        if (S.q >= R.count(S.seg)) {  // the worker ran out of records: only past the pre-generated blocks
            S.err |= SERR_DRAWS;
            return S.mode = ST_DONE;
        }
        const SegRec<M> r = R.rec(S.seg, S.q);
        const int64_t Tb = S.X.T + (int64_t)r.span - (S.W.T - S.WT0);
        if (Tb + thrmax >= D) return S.mode = ST_END;  // the run ends in this sub: replay it with the real D
#pragma unroll
        for (int kk = 0; kk < M; ++kk) {
            et.add(C_F, (uint32_t)kk, r.dF[kk] - ew.get(C_F, (uint32_t)kk));
            et.add(C_S, (uint32_t)kk, r.dS[kk] - ew.get(C_S, (uint32_t)kk));
            ew.set(C_F, (uint32_t)kk, 0u);
            ew.set(C_S, (uint32_t)kk, 0u);
        }
        S.X.F += r.dFh - S.W.F;
        S.X.Ff = S.X.F;
        S.X.h = r.h;
        S.X.w = r.w;
        S.X.sst = 0u;
#pragma unroll
        for (int j = 0; j < SegRec<M>::NP; ++j) {
            S.X.pend[j] = r.pend[j];
            S.X.stp[j] = 0ull;
        }
        S.X.T = Tb;
        S.X.k = r.kb;
        seg_resume<M>(st, r);
        if (r.flags & SEG_CUT) {
            S.q += 1u;
            S.wnew = 1u;
            S.walk_back = 1u;
            return S.mode = ST_ENGINE;
        }
        // segment end: the next segment's worker started quiet at b
        S.seg += 1u;
        S.q = 0u;
        seg_set_quiet<M>(S.W, r.kb, 0);
        S.WT0 = 0;
        if (seg_quiet<M>(S.X)) return S.mode = ST_JUMP;
        seg_resume<M>(sw, r);
        return S.mode = ST_WALK;
    }
    if (S.mode == ST_END) {  // the true state alone, to the end of the run
        const int x = S.X.step4(et, st, D, sid, ps, thrmax, lut);
        if (x == 2) return S.mode = ST_DONE;
        if (x == 1) {
            S.walk_back = 0u;
            return S.mode = ST_ENGINE;
        }
        return S.mode;
    }
    // ST_WALK: W catches up with X one find at a time; at the same pending block, equal states coalesce
    const uint32_t it = st.idx - 1u, iw = sw.idx - 1u;
    if (iw < it) {
        if (S.q >= R.count(S.seg)) {
            S.err |= SERR_DRAWS;
            return S.mode = ST_DONE;
        }
        const SegRec<M> r = R.rec(S.seg, S.q);
        if (iw > r.b) {  // cannot happen: the replay left the worker's path
            S.err |= SERR_CAP;
            return S.mode = ST_DONE;
        }
        if ((r.flags & SEG_END) && iw == r.b) {  // W reached its segment's end: the next worker starts quiet
            seg_set_quiet<M>(S.W, S.W.k, S.W.T);
            S.WT0 = S.W.T;
#pragma unroll
            for (int kk = 0; kk < M; ++kk) {
                ew.set(C_F, (uint32_t)kk, 0u);
                ew.set(C_S, (uint32_t)kk, 0u);
            }
            S.seg += 1u;
            S.q = 0u;
            return S.mode;
        }
        const int x = S.W.step1(ew, sw, SEG_NO_END, sid, ps);
        sw.fill();
        if (x == 1) {  // the worker's cut: it restarted quiet at the next block
            if (!(r.flags & SEG_CUT) || r.b != iw) {
                S.err |= SERR_CAP;
                return S.mode = ST_DONE;
            }
            S.q += 1u;
            S.W.begin(sw);
            S.WT0 = S.W.T;
#pragma unroll
            for (int kk = 0; kk < M; ++kk) {
                ew.set(C_F, (uint32_t)kk, 0u);
                ew.set(C_S, (uint32_t)kk, 0u);
            }
        }
        return S.mode;
    }
    if (iw == it && seg_same<M>(S.X, S.W)) {  // coalesced: the sub's remaining deltas are the true ones
        S.X.flush_stale(et, sid);
        S.W.flush_stale(ew, sid);
        return S.mode = ST_JUMP;
    }
    const int x = S.X.step1(et, st, D, sid, ps);
    st.fill();  // a later step4 (END) needs two held draws
    if (x == 2) return S.mode = ST_DONE;
    if (x == 1) {
        S.walk_back = 1u;
        return S.mode = ST_ENGINE;
    }
    return S.mode;
}

// After the engine handed X back settled (take_back succeeded and X.T < D): W restarts from the cut record if
// the episode started at a cut; back to WALK or END.
template <int M, class Recs, class EnvW, class Src>
MSIM_HD void seg_after_engine(SegStitch<M> &S, const Recs &R, EnvW &ew, Src &sw)
{
    if (S.wnew) {
        const SegRec<M> r = R.rec(S.seg, S.q - 1u);
        seg_resume<M>(sw, r);
        S.W.begin(sw);
        S.WT0 = S.W.T;
#pragma unroll
        for (int kk = 0; kk < M; ++kk) {
            ew.set(C_F, (uint32_t)kk, 0u);
            ew.set(C_S, (uint32_t)kk, 0u);
        }
        S.wnew = 0u;
    }
    S.mode = S.walk_back ? ST_WALK : ST_END;
}

}  // namespace msim
