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
    uint32_t dFh;      // increase of the common prefix F since the sub's last checkpoint (or its start)
    uint32_t qn;       // the segment's checkpoints before the next sub
    uint32_t n;        // held draws
    uint32_t I[4], k[4];
    uint64_t span;     // time from the sub's last checkpoint (or its first pending find) to find b
    uint64_t pend[NP];
    Rng ri, rp;        // the streams after the held draws
    uint32_t dF[M], dS[M];  // counter deltas since then (C_F, C_S), stale blocks flushed at b
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

// A worker's quiet checkpoint: its pending find c is quiet (h = w = 0, no honest branch). The true state joins
// the worker at a block where both are quiet. The worker records every quiet block within the first SEG_QWIN
// finds after a (re)start (where the true state usually joins: after an engine episode or at a segment start),
// and after that the first quiet block past every multiple of SEG_QEVERY, so that a late join is never much
// more than SEG_QEVERY blocks away (measured on configs[2] with the window alone: 7 % of the joins walked to the
// next cut, ~600 blocks). A checkpoint holds the counter / F / time deltas since the previous checkpoint of its
// sub (the sub's end record too), so the stitch that joins at a checkpoint adds the later ones and the record's.
// Checkpoints are an optimisation: when the deltas do not fit or the caller has no room, the sub's later
// checkpoints are dropped (its record's deltas then reach back to the last one stored) and ST walks further.
constexpr uint32_t SEG_QWIN = 24, SEG_QEVERY = 64;
template <int M>
struct SegQRec {
    uint32_t c;
    uint32_t span;          // time since the previous checkpoint of the sub (its start for the first)
    uint8_t dFh;            // F since then
    uint8_t dF[M], dS[M];   // counter deltas since then (stale blocks flushed)
};

// SW lane body: the worker of one segment, blocks [first, e) (src positioned at draw `first`, src.idx = first).
// Env: the worker's counter rows C_F / C_S (zero at entry), prop_tab. emit(rec) / emitq(qrec) store a sub's end
// record / a quiet checkpoint and return false when the caller cannot hold it (a record: the run is then
// recomputed by E2; a checkpoint: the sub stores no more);
// emitq.n() is the number of checkpoints stored so far (SegRec::qn). Inside a quiet window, and from a multiple of
// SEG_QEVERY to the next quiet block, the worker steps one find at a time (it must see every pending block);
// elsewhere four. Returns 0 or an SERR_* code.
template <int M, class Env, class Src, class Emit, class EmitQ>
MSIM_HD uint32_t seg_work(Env &env, Src &src, uint32_t e, uint32_t sid, int64_t ps, int64_t thrmax, const uint32_t *lut,
                          Emit &emit, EmitQ &emitq)
{
    SelMacro<M> mc;
    if (!mc.begin(src)) return SERR_DRAWS;
    int64_t Tq = mc.T;  // the time of the last checkpoint (or of the sub's start)
    uint32_t Fq = 0;
    uint32_t qleft = SEG_QWIN, qnext = 0xFFFFFFFFu;
    bool qon = true;
    for (;;) {
        const uint32_t i = src.idx - 1u;
        uint32_t fl = 0;
        if (i >= e) {
            fl = SEG_END;
        } else {
            if (qleft == 0u && qnext == 0xFFFFFFFFu) qnext = (i / SEG_QEVERY + 1u) * SEG_QEVERY;  // window over
            if (qleft != 0u || i >= qnext) {
                qleft -= qleft != 0u ? 1u : 0u;
                if (qon && seg_quiet<M>(mc)) {
                    if (i >= qnext) qnext = (i / SEG_QEVERY + 1u) * SEG_QEVERY;
                    mc.flush_stale(env, sid);
                    SegQRec<M> qr;
                    qr.c = i;
                    const int64_t dt = mc.T - Tq;
                    qr.span = (uint32_t)dt;
                    qr.dFh = (uint8_t)(mc.F - Fq);
                    bool fits = dt >= 0 && dt <= 0xFFFFFFFFll && mc.F - Fq <= 255u;
#pragma unroll
                    for (int kk = 0; kk < M; ++kk) {  // the rows hold the deltas: they restart at every checkpoint
                        const uint32_t f = env.get(C_F, (uint32_t)kk), x = env.get(C_S, (uint32_t)kk);
                        fits &= (f <= 255u) & (x <= 255u);
                        qr.dF[kk] = (uint8_t)f;
                        qr.dS[kk] = (uint8_t)x;
                    }
                    if (fits && emitq(qr)) {
                        Tq = mc.T;
                        Fq = mc.F;
#pragma unroll
                        for (int kk = 0; kk < M; ++kk) {
                            env.set(C_F, (uint32_t)kk, 0u);
                            env.set(C_S, (uint32_t)kk, 0u);
                        }
                    } else {
                        qon = false;  // no more checkpoints in this sub: the record's deltas reach back to the last
                    }
                }
            }
            const bool one = (qon & (qleft != 0u || i >= qnext)) || i + 4u > e;
            const int x = one ? mc.step1(env, src, SEG_NO_END, sid, ps) : mc.step4(env, src, SEG_NO_END, sid, ps, thrmax, lut);
            if (x == 1) fl = SEG_CUT;
            src.fill();  // step4 (SelFifo::top4) needs two held draws
        }
        if (fl) {
            mc.flush_stale(env, sid);
            SegRec<M> r;
            r.b = src.idx - 1u;
            r.flags = fl;
            r.h = mc.h;
            r.w = mc.w;
            r.kb = mc.k;
            r.dFh = mc.F - Fq;  // since the sub's last checkpoint, like the counters and the span
            r.span = (uint64_t)(mc.T - Tq);
            r.qn = emitq.n();
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
            Tq = mc.T;
            Fq = 0;
            qleft = SEG_QWIN;
            qnext = 0xFFFFFFFFu;
            qon = true;
        }
    }
}

// ST lane state: the run's true settled state X (absolute time, real D) and where it stands among the workers'
// records: segment seg, the sub record q that ends X's current stretch (the first with b >= X's pending block),
// the checkpoint cursor qi (the first checkpoint of seg after X's last join test).
enum : uint32_t { ST_JUMP = 0, ST_WALK = 1, ST_ENGINE = 2, ST_END = 3, ST_DONE = 4 };
template <int M>
struct SegStitch {
    SelMacro<M> X;
    uint32_t seg, q, qi;
    uint32_t at_rec;     // JUMP: X joined the worker at sub q's end record (1) or at checkpoint qi - 1 (0)
    uint32_t mode;
    uint32_t walk_back;  // after the engine: back to WALK (1) or END (0)
    uint32_t err;
};

// Recs: uint32_t count(seg); SegRec<M> rec(seg, q); void head(seg, q, b, flags); uint32_t qcount(seg);
// uint32_t qc(seg, i) (a checkpoint's block); uint32_t qspan(seg, i); SegQRec<M> qrec(seg, i).
// One action of a lane that is not in the engine; returns its new mode. ST_ENGINE: X needs the entity engine at
// its pending find (the caller converts X with to_exact, steps the engine, and takes X back; then mode =
// walk_back ? ST_WALK : ST_END). ST_DONE with err == 0: the run ended in the settled form (the caller finishes X).
// A run starts in ST_WALK at its first find (segment 0's worker starts quiet there: the first test joins).
template <int M, class Recs, class EnvT, class Src>
MSIM_HD uint32_t seg_stitch_step(SegStitch<M> &S, const Recs &R, EnvT &et, Src &st, int64_t D, uint32_t sid, int64_t ps,
                                 int64_t thrmax, const uint32_t *lut)
{
    if (S.mode == ST_JUMP) {  // X equals the worker at its pending block: take the rest of sub q from the records
        const SegRec<M> r = R.rec(S.seg, S.q);
        const uint32_t nq = R.qcount(S.seg);
        const bool ar = S.at_rec != 0u;
        int64_t Tb = S.X.T;
        if (!ar) {
            Tb += (int64_t)r.span;
            for (uint32_t j = S.qi; j < nq && R.qc(S.seg, j) <= r.b; ++j) Tb += R.qspan(S.seg, j);
        }
        if (Tb + thrmax >= D) return S.mode = ST_END;  // the run ends in this sub: the true state alone, real D
        if (!ar) {
            for (; S.qi < nq && R.qc(S.seg, S.qi) <= r.b; ++S.qi) {
                const SegQRec<M> qr = R.qrec(S.seg, S.qi);
                S.X.F += qr.dFh;
#pragma unroll
                for (int kk = 0; kk < M; ++kk) {
                    et.add(C_F, (uint32_t)kk, qr.dF[kk]);
                    et.add(C_S, (uint32_t)kk, qr.dS[kk]);
                }
            }
#pragma unroll
            for (int kk = 0; kk < M; ++kk) {
                et.add(C_F, (uint32_t)kk, r.dF[kk]);
                et.add(C_S, (uint32_t)kk, r.dS[kk]);
            }
            S.X.F += r.dFh;
        }
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
        if (r.flags & SEG_CUT) {  // the true state is the worker's: it needs the engine at b too
            S.q += 1u;
            S.qi = r.qn;  // the next sub's checkpoints
            S.walk_back = 1u;
            return S.mode = ST_ENGINE;
        }
        // segment end: the next segment's worker started quiet at b
        S.seg += 1u;
        S.q = 0u;
        S.qi = 0u;
        return S.mode = ST_WALK;
    }
    if (S.mode == ST_END) {  // the true state alone, to the end of the run
        const int x = S.X.step4(et, st, D, sid, ps, thrmax, lut);
        st.fill();
        if (x == 2) return S.mode = ST_DONE;
        if (x == 1) {
            S.walk_back = 0u;
            return S.mode = ST_ENGINE;
        }
        return S.mode;
    }
    // ST_WALK: the true state alone, one find at a time, until it meets the worker in the same state at the same
    // block: at a quiet checkpoint, or at a sub's end record
    const uint32_t i = st.idx - 1u;
    uint32_t b = 0, fl = 0;
    for (;;) {  // the record that ends X's stretch: the first with b >= i
        if (S.q >= R.count(S.seg)) {  // past the pre-generated segments
            S.err |= SERR_DRAWS;
            return S.mode = ST_DONE;
        }
        R.head(S.seg, S.q, b, fl);
        if (b >= i) break;
        if (fl & SEG_END) {  // X passed the segment's end: the next segment
            S.seg += 1u;
            S.q = 0u;
            S.qi = 0u;
        } else {
            S.q += 1u;
        }
    }
    const uint32_t nq = R.qcount(S.seg);
    uint32_t c = 0xFFFFFFFFu;
    while (S.qi < nq && (c = R.qc(S.seg, S.qi)) < i) ++S.qi;
    if (S.qi < nq && c == i && seg_quiet<M>(S.X)) {  // both quiet at block i
        ++S.qi;
        S.X.flush_stale(et, sid);
        S.at_rec = 0u;
        return S.mode = ST_JUMP;
    }
    if (b == i) {
        const SegRec<M> r = R.rec(S.seg, S.q);
        bool eq = (r.h == S.X.h) & (r.w == S.X.w);
#pragma unroll
        for (int j = 0; j < SegRec<M>::NP; ++j) eq &= r.pend[j] == S.X.pend[j];
        if (eq) {
            S.X.flush_stale(et, sid);
            S.at_rec = 1u;
            return S.mode = ST_JUMP;
        }
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

}  // namespace msim
