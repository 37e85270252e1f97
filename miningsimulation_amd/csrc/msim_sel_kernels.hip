// msim_sel_kernels.hip — E1 / E2 of the entity-engine path (msim_sel_launch.h), one translation unit
// per miner count (MSIM_M).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "msim_general_launch.h"
#include "msim_kernels.h"
#include "msim_reduce.h"
#include "msim_sel_launch.h"
#include "msim_selm.h"

namespace msim {

#ifndef SEL_WAVES
#define SEL_WAVES 2  // E1 occupancy target (waves per SIMD): 256 VGPRs, no spills
#endif

// ------------------------------------------------------------------ entity engine (msim_sel.h)
// Per-lane counters of the engine in LDS, [array][miner][lane]: lanes of a wave hit distinct banks for any
// mix of miner indices.
// Counter increments are LDS atomics whose result is unused (ds_add_u32): the lane never waits on them.
// A network whose miners share one propagation delay (every BASELINE config) reads it from a scalar: in the
// engine through a wave-uniform branch (uni), in the settled form at compile time (UNI; measured on MI355X:
// the table read it replaces cost 2.3 % of configs[2], profiles/r03/e1ab/uni_*).
template <int M, bool UNI = false>
struct SelDevEnv {
    uint32_t *c;          // &s_cnt[0][tid]
    const int64_t *pr;    // propagation per miner (LDS or global)
    int64_t uprop;        // the common propagation when `uni`
    bool uni;
    ColdAct *cb;          // this lane's cold slots: cb[c * cstride]
    size_t cstride;
    __device__ __forceinline__ ColdAct cold(int i) const { return cb[(size_t)i * cstride]; }
    __device__ __forceinline__ void cold_put(int i, const ColdAct &r) { cb[(size_t)i * cstride] = r; }
    __device__ __forceinline__ int64_t prop(uint32_t k) const { return uni ? uprop : pr[k]; }
    // the settled form's read: always the table (no branch), issued at the top of a step
    __device__ __forceinline__ int64_t prop_tab(uint32_t k) const { return UNI ? uprop : pr[k]; }
    __device__ __forceinline__ uint32_t get(int a, uint32_t k) const { return c[(a * M + (int)k) * TPB]; }
    __device__ __forceinline__ void add(int a, uint32_t k, uint32_t v) { atomicAdd(&c[(a * M + (int)k) * TPB], v); }
    __device__ __forceinline__ void set(int a, uint32_t k, uint32_t v) { c[(a * M + (int)k) * TPB] = v; }
    // every lane of the wave folds when any lane is due (msim_sel.h step)
    __device__ __forceinline__ bool fold_vote(bool due) const { return __builtin_amdgcn_ballot_w64(due) != 0ull; }
};

__device__ __noinline__ int32_t interval_ms_exact_dev(uint64_t u) { return (int32_t)interval_ms_of(u); }

// The reference's draws made in-lane (SelFifo drawers). PickFinder with integer weights: q = floor(u / MULT)
// is p1 = floor(W u / 2^64) or p1 + 1, and the finder is the first k with cum_k > q (simulation.h:213-221).
template <int M>
__device__ __forceinline__ uint32_t sel_pick_weighted(uint64_t u, const SelParams *P)
{
    const uint64_t p1 = __umul64hi(u, (uint64_t)P->W);
    const uint64_t q = u >= (p1 + 1) * P->mult ? p1 + 1 : p1;
    uint32_t f = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) f += P->cum[j] <= q ? 1u : 0u;  // M = the network's miner count
    return f;
}

// Exact sequence (E2 retries): glibc's log1p for every interval.
template <int M>
struct SelExactDraw {
    Rng ri, rp;
    const SelParams *P;
    __device__ void draw(uint32_t &I, uint32_t &k)
    {
        I = (uint32_t)next_interval(ri);
        k = sel_pick_weighted<M>(rng_next(rp), P);
    }
    uint32_t pI, pk;
    __device__ void draw_spec_a() { draw(pI, pk); }
    __device__ void draw_spec_b(uint32_t &I, uint32_t &k)
    {
        I = pI;
        k = pk;
    }
    __device__ void fix(uint32_t &, uint32_t &) {}
};

// Fast sequence (E1 without a word stream): K1's table interval with its exactness check and exact
// fallback (msim_fastdraw.h), the finder through the LDS code table for percentages (W = 100) or the
// weighted scan otherwise (wave-uniform choice). The settled form's speculative draw is split in two:
// draw_spec() is branch-free (fast interval, fast table pick, the two exactness flags, both uniforms kept)
// so that the compiler can interleave it with the transition it runs beside, and fix() — at the end of
// the step — redoes what the fast forms cannot settle (rare; every pick of a weighted network).
template <int M>
struct SelFastDraw {
    Rng ri, rp;
    const LogTab *lt;     // LDS
    const uint8_t *lut;   // LDS: finder of q = floor(u / PERC_MULTIPLIER)
    const SelParams *P;
    FdConsts kc;
    bool wt;
    // the speculative draw between its parts: both uniforms (until fix()), the interval's reduced argument,
    // exponent and table entries (until draw_spec_b()), the pick's acceptance key and finder
    uint64_t su_i, su_p;
    double sw, sinvc, sA;
    int32_t se;
    uint32_t skp, sk;
    bool sx_i, sx_p;      // the interval / pick need the exact forms
    // part A: both RNG steps, the table indices and the LDS reads (log table, finder table)
    __device__ __forceinline__ void draw_spec_a()
    {
        su_i = rng_next(ri);
        su_p = rng_next(rp);
        const uint32_t lo = (uint32_t)su_i, hi = (uint32_t)(su_i >> 32);
        const double c = __builtin_fma(u32_to_f64(lo >> 11), -0x1.0p-53, 1.0);
        const double v = __builtin_fma(u32_to_f64(hi), -0x1.0p-32, c);  // 1 - (u>>11) 2^-53, exact
        const uint64_t vb = __builtin_bit_cast(uint64_t, v);
        const uint32_t vh = (uint32_t)(vb >> 32);
        se = (int)(vh >> 20) - 1023;
        const uint32_t j = (vh >> (20 - LOG_BITS)) & (LOG_TAB - 1);
        sw = __builtin_bit_cast(double, (vb & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
        uint32_t aoff = j * 8u;
        asm("" : "+v"(aoff));
        sA = *(const double *)((const char *)lt->A + aoff);
        sinvc = lt->invc[j];
        sk = lut[pick_q_fast_key(su_p, skp)];  // q = 100: PickFinder falls through (finder >= m)
    }
    // part B: the interval polynomial (msim_fastdraw.h interval_fast_z, the same operations) and the flags
    __device__ __forceinline__ void draw_spec_b(uint32_t &I, uint32_t &k)
    {
        const double r = __builtin_fma(sw, sinvc, -1.0);
        double p = __builtin_fma(r, kc.c5, kc.c4);
        p = __builtin_fma(r, p, kc.c3);
        p = __builtin_fma(r, p, kc.c2);
        p = __builtin_fma(r, p, kc.c1);
        const double z0 = __builtin_fma(r, p, sA);
        const double z = __builtin_fma((double)se, FD_CE, z0);
        I = (uint32_t)(int32_t)z;
        const double f = __builtin_amdgcn_fract(z);
        const uint32_t ki = (uint32_t)(__builtin_bit_cast(uint64_t, f) >> 32) - FD_OK_LO;
        k = sk;
        sx_i = ki >= FD_OK_RANGE;
        sx_p = skp >= PICK_RARE_LO;
    }
    __device__ __forceinline__ void fix(uint32_t &I, uint32_t &k)
    {
        if (sx_i | sx_p | wt) {
            if (sx_i) I = (uint32_t)interval_ms_exact_dev(su_i);
            if (wt) k = sel_pick_weighted<M>(su_p, P);
            else if (sx_p) k = lut[pick_q_exact(su_p)];
        }
    }
    __device__ __forceinline__ void draw(uint32_t &I, uint32_t &k)
    {
        draw_spec_a();
        draw_spec_b(I, k);
        fix(I, k);
    }
};

template <int M>
__device__ __forceinline__ void sel_terms(const SelOut &o, uint64_t (&v)[6 * M])
{
    const double L = (double)o.best_height;
#pragma unroll
    for (int k = 0; k < M; ++k) {
        const uint32_t f = o.found[k];
        // MinerStats (main.cpp:28-29)
        const double share = f == 0 ? 0.0 : (double)f / L;
        const double rate = f == 0 ? 0.0 : (double)o.stale[k] / (double)f;
        const uint64_t sfx = (uint64_t)(share * 4294967296.0 + 0.5);
        const uint64_t rfx = (uint64_t)(rate * 4294967296.0 + 0.5);
        v[6 * k + 0] = f;
        v[6 * k + 1] = o.stale[k];
        v[6 * k + 2] = sfx >> 32;
        v[6 * k + 3] = sfx & 0xFFFFFFFFull;
        v[6 * k + 4] = rfx >> 32;
        v[6 * k + 5] = rfx & 0xFFFFFFFFull;
    }
}

// The mixed schedule of a network with one selfish miner (msim_selm.h): every lane runs the settled-state
// form until one of its finds needs the entity engine, then waits; when P->xth lanes wait (or no lane is
// left in the settled form) the wave runs an engine phase: the waiting lanes enter the engine, which steps
// every one of them until it hands its run back (episodes are short: 5-6 events on average, 13 at the
// 99th percentile over the configs[3] grid) or finishes it. The engine's state exists only inside a phase,
// so its registers and the settled form's are never live at the same time. Lane modes: 0 settled form,
// 1 waiting for the engine, 2 in the engine, 3 done. The schedule only decides the order in which lanes
// advance: each lane's result is that of its own sequence of transitions (tests/native/sel_host.cpp runs
// one lane alone). A network the settled form does not cover (P->macro == 0) runs one engine phase.
#ifndef SEL_XTH
#define SEL_XTH 16
#endif
#ifndef SEL_PROF
#define SEL_PROF 0
#endif
#ifndef SEL_MSTEPS
#define SEL_MSTEPS 2
#endif
#ifndef SEL_MC_LDS
#define SEL_MC_LDS 1  // the settled-form state waits in LDS during engine phases
#endif
template <int M, class SelT, class Env, class Src>
__device__ __forceinline__ void sel_mixed(Env &env, Src &src, const SelParams *P, int64_t D, SelOut &o, uint32_t *mcs)
{
    SelMacro<M> mc;
    // A lane that finishes parks its counters in its own LDS counter rows (C_F, C_S) so that no result
    // register stays live across the loop of the others.
    uint32_t bh = 0, err = 0;
    auto park = [&](const SelOut &r) {
#pragma unroll
        for (int k = 0; k < M; ++k) {
            env.set(C_F, (uint32_t)k, r.found[k]);
            env.set(C_S, (uint32_t)k, r.stale[k]);
        }
        bh = r.best_height;
        err = r.err;
    };
    const uint32_t sid = P->sids[0];
    const int64_t ps = P->prop[sid];
    const bool mac = P->macro != 0u;  // wave-uniform (one point per workgroup)
    const int xth = (int)__builtin_amdgcn_readfirstlane(P->xth >= 1u && P->xth <= 64u ? P->xth : (uint32_t)SEL_XTH);
    int mode = 0;
    if (!mac) {  // the entity engine for every find
        mode = 1;
    } else if (!mc.begin(src)) {
        err = SERR_DRAWS;
        mode = 3;
    } else if (mc.T >= D) {
        SelOut r;
        mc.finish(env, sid, r);
        park(r);
        mode = 3;
    }
#if SEL_PROF  // per-wave phase timing (diagnostic builds only: scripts/build_sel_variant.sh prof -DSEL_PROF=1)
    uint64_t pt_m = 0, pt_e = 0, pn_m = 0, pn_e = 0, pi_m = 0, pi_e = 0, pl_m = 0, pl_e = 0;
    const uint64_t pt0 = clock64();
#endif
    for (;;) {
        const uint64_t bm = __builtin_amdgcn_ballot_w64(mode == 0);
        const uint64_t be = __builtin_amdgcn_ballot_w64(mode == 1);
        if ((bm | be) == 0ull) break;
#if SEL_PROF
        const uint64_t pc0 = clock64();
        const bool pexact = be != 0ull && (__builtin_popcountll(be) >= xth || bm == 0ull);
#endif
        if (be != 0ull && (__builtin_popcountll(be) >= xth || bm == 0ull)) {
            SelT s;
            if (mode == 1) {
                if (mac) {
                    mc.to_exact(env, s, P->m, P->sids);
                } else {
                    s.init(P->m, P->sids);
                    s.begin(src);
                }
                mode = 2;
            }
#if SEL_MC_LDS
            mc.save(mcs, TPB);  // saved and reloaded for every lane: no settled-form register is live here
#endif
            for (;;) {
                if (mode == 2) {
                    src.prefetch();
                    const bool live = s.step(env, src, D);
                    src.settle();
                    if (!live) {
                        SelOut r;
                        s.finish(env, D, r);
                        park(r);
                        mode = 3;
                    } else if (mac) {
                        SelMacro<M> tb;
                        if (tb.take_back(env, s, sid)) {
                            if (tb.T >= D) {
                                SelOut r;
                                tb.finish(env, sid, r);
                                park(r);
                                mode = 3;
                            } else {
                                src.fill();  // the settled form starts every step with two held draws
#if SEL_MC_LDS
                                tb.save(mcs, TPB);
#else
                                mc = tb;
#endif
                                mode = 0;
                            }
                        }
                    }
                }
#if SEL_PROF
                ++pi_e;
                pl_e += __builtin_popcountll(__builtin_amdgcn_ballot_w64(mode == 2));
#endif
                if (__builtin_amdgcn_ballot_w64(mode == 2) == 0ull) break;
            }
#if SEL_MC_LDS
            mc.load(mcs, TPB);
#endif
        } else {
            for (;;) {
                // SEL_MSTEPS settled-form steps per exit test (a lane that leaves the form skips the rest)
#pragma unroll
                for (int u = 0; u < SEL_MSTEPS; ++u) {
                    if (mode == 0) {
                        src.prefetch();  // consumed at a later refill (peek settles only when it must)
                        const int r = mc.step(env, src, D, sid, ps);
                        if (r == 2) {
                            SelOut q;
                            mc.finish(env, sid, q);
                            park(q);
                            mode = 3;
                        } else if (r == 1) {
                            mode = 1;
                        }
                    }
                }
#if SEL_PROF
                ++pi_m;
                pl_m += __builtin_popcountll(__builtin_amdgcn_ballot_w64(mode == 0));
#endif
                if (__builtin_amdgcn_ballot_w64(mode == 0) == 0ull ||
                    __builtin_popcountll(__builtin_amdgcn_ballot_w64(mode == 1)) >= xth)
                    break;
            }
        }
#if SEL_PROF
        const uint64_t pc1 = clock64();
        if (pexact) {
            pt_e += pc1 - pc0;
            ++pn_e;
        } else {
            pt_m += pc1 - pc0;
            ++pn_m;
        }
#endif
    }
#if SEL_PROF
    if (blockIdx.x < 2 && (threadIdx.x & 63u) == 0u)
        printf("SELPROF blk %u wave %u total %llu | macro phases %llu cyc %llu iters %llu lanes %llu | engine phases %llu cyc %llu iters %llu lanes %llu\n",
               blockIdx.x, threadIdx.x / 64u, (unsigned long long)(clock64() - pt0), (unsigned long long)pn_m,
               (unsigned long long)pt_m, (unsigned long long)pi_m, (unsigned long long)pl_m, (unsigned long long)pn_e,
               (unsigned long long)pt_e, (unsigned long long)pi_e, (unsigned long long)pl_e);
#endif
#pragma unroll
    for (int k = 0; k < M; ++k) {
        o.found[k] = env.get(C_F, (uint32_t)k);
        o.stale[k] = env.get(C_S, (uint32_t)k);
    }
    o.best_height = bh;
    o.err = err;
}

// ------------------------------------------------------------------ E1's workgroup pool
// Why. With one lane per run, every lane of a wave advances its own run in the settled form (msim_selm.h)
// until one of its finds needs the entity engine. Engine episodes are rare (~82 per run-year at configs[2]),
// short (5.6 events on average) and ~9x as costly per step as a settled-form step. Run per wave (the mixed
// schedule above), an engine phase stepped ~16 waiting lanes until the longest episode ended: 7.4 of 64
// lanes active on average, 32 % of E1's cycles (round 3, profiles/r03/e1ab/selprof_c3.txt).
//
// The pool moves a run between lanes instead. A run that needs the engine leaves its home lane: its
// settled state (SelMacro, LDS s_mc) and its draw state (both xoroshiro128++ states and the held draws,
// LDS x) are written to its SLOT (the home lane's index in the workgroup) and the slot is queued in an LDS
// ring shared by the workgroup's four waves; its per-run counters already live in the slot's LDS columns
// (s_cnt) and its cold engine slots in global memory indexed by the slot. Any wave of the workgroup whose
// own lanes have run short of settled-form work, or that sees enough runs queued, becomes an engine worker:
// its lanes claim queued slots, step the entity engine on them, and claim the next queued slot as soon as
// their episode ends (the slot goes back to its home lane with the new settled state, or is finished), so
// engine steps run on (nearly) full waves. Which lane computes which part of a run never changes a result:
// every run performs its own sequence of transitions (tests/native/sel_host.cpp runs one lane alone).
//
// Synchronisation is LDS only (no global memory crosses lanes): a producer writes the slot's state, fences
// (release, workgroup scope) and publishes the slot in the ring (slot + 1; 0 = empty) at a position
// reserved with one atomic on `tail`; a consumer reserves ring positions with a compare-and-swap on `head`,
// waits for the entry to be non-zero, clears it and fences (acquire) before reading the slot. Status words
// tell a home lane that its run is back (PS_BACK) or finished (PS_DONE). Every wait is bounded: a wave that
// waited 2^20 sleeps flags its away runs (SERR_SCHED: E2 recomputes them exactly), so the workgroup always
// drains.
enum : uint32_t { PS_QUEUED = 1u, PS_BACK = 2u, PS_DONE = 3u };
constexpr uint32_t SERR_SCHED = 128u;  // a run whose pool hand-over did not complete (never observed)
constexpr uint32_t POOL_QCAP = 2u * TPB;
constexpr uint32_t POOL_NOSLOT = 0xFFFFFFFFu;
constexpr uint32_t POOL_XW = 12;  // transfer words: RNG states (8), held intervals (3), held finders + count (1)
constexpr uint32_t POOL_SPIN_MAX = 1u << 20;

struct SelPool {
    uint32_t st[TPB];           // slot status (PS_*), written when the slot leaves / returns to its home lane
    uint32_t q[POOL_QCAP];      // ring of queued slots (slot + 1), 0 = empty
    uint32_t head, tail;
    uint32_t x[POOL_XW][TPB];   // the slot's draw state while it is away
};

#ifndef SEL_POOL
#define SEL_POOL 1  // 0: the per-wave mixed schedule for every network (A/B)
#endif
#ifndef SEL_PSTEPS
#define SEL_PSTEPS 2  // settled-form steps between pool checks
#endif

template <int M>
struct SelPoolLds {
    static constexpr int NW = SelMacro<M>::NW;
    // the pool needs two workgroups per CU (two waves per SIMD): s_cnt, s_mc and the pool within 80 KiB
    static constexpr size_t BYTES = (size_t)(4 * M + NW) * TPB * 4 + sizeof(SelPool) + 4096;
    static constexpr bool FITS = SEL_POOL && BYTES <= 80 * 1024;
};

__device__ __forceinline__ uint32_t lds_load(const uint32_t *p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
__device__ __forceinline__ void lds_store(uint32_t *p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_RELAXED); }
__device__ __forceinline__ void fence_rel() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
__device__ __forceinline__ void fence_acq() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); }
__device__ __forceinline__ uint32_t lane_id()
{
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t rank_in(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Queued slots (head first: head never passes a tail read after it).
__device__ __forceinline__ uint32_t pool_queued(const SelPool &pl)
{
    const uint32_t h = lds_load(&pl.head);
    const uint32_t t = lds_load(&pl.tail);
    return (uint32_t)__builtin_amdgcn_readfirstlane(t - h);
}

template <int M>
__device__ __forceinline__ void xfer_save(const SelFifo<SelFastDraw<M>> &f, SelPool &pl, uint32_t slot)
{
    pl.x[0][slot] = (uint32_t)f.d.ri.s0;
    pl.x[1][slot] = (uint32_t)(f.d.ri.s0 >> 32);
    pl.x[2][slot] = (uint32_t)f.d.ri.s1;
    pl.x[3][slot] = (uint32_t)(f.d.ri.s1 >> 32);
    pl.x[4][slot] = (uint32_t)f.d.rp.s0;
    pl.x[5][slot] = (uint32_t)(f.d.rp.s0 >> 32);
    pl.x[6][slot] = (uint32_t)f.d.rp.s1;
    pl.x[7][slot] = (uint32_t)(f.d.rp.s1 >> 32);
    pl.x[8][slot] = f.I0;
    pl.x[9][slot] = f.I1;
    pl.x[10][slot] = f.I2;
    pl.x[11][slot] = (f.k0 & 0xFFu) | ((f.k1 & 0xFFu) << 8) | ((f.k2 & 0xFFu) << 16) | (f.n << 24);
}
template <int M>
__device__ __forceinline__ void xfer_load(SelFifo<SelFastDraw<M>> &f, const SelPool &pl, uint32_t slot)
{
    f.d.ri.s0 = (uint64_t)pl.x[0][slot] | ((uint64_t)pl.x[1][slot] << 32);
    f.d.ri.s1 = (uint64_t)pl.x[2][slot] | ((uint64_t)pl.x[3][slot] << 32);
    f.d.rp.s0 = (uint64_t)pl.x[4][slot] | ((uint64_t)pl.x[5][slot] << 32);
    f.d.rp.s1 = (uint64_t)pl.x[6][slot] | ((uint64_t)pl.x[7][slot] << 32);
    f.I0 = pl.x[8][slot];
    f.I1 = pl.x[9][slot];
    f.I2 = pl.x[10][slot];
    const uint32_t w = pl.x[11][slot];
    f.k0 = w & 0xFFu;
    f.k1 = (w >> 8) & 0xFFu;
    f.k2 = (w >> 16) & 0xFFu;
    f.n = w >> 24;
}

// A slot's final counters (MinerStats inputs) in its LDS columns, best height and error in s_mc words 0-1.
template <int M, class Env>
__device__ __forceinline__ void pool_park(Env &env, const SelOut &r, uint32_t (*s_mc)[TPB], uint32_t slot)
{
#pragma unroll
    for (int k = 0; k < M; ++k) {
        env.set(C_F, (uint32_t)k, r.found[k]);
        env.set(C_S, (uint32_t)k, r.stale[k]);
    }
    s_mc[0][slot] = r.best_height;
    s_mc[1][slot] = r.err;
}

// The pool schedule of one workgroup (one point). Every lane runs it (a lane without a run starts done and
// still serves as an engine worker). On return the lane's own run is finished: counters in its s_cnt
// columns, best height / error in s_mc[0..1][tid].
template <int M, class SelT, bool UNI>
__device__ __forceinline__ void sel_pool(const SelArgs &a, const SelParams *P, SelFifo<SelFastDraw<M>> &src, uint32_t (*s_cnt)[TPB],
                         const int64_t *s_prop, uint32_t (*s_mc)[TPB], SelPool &pl, size_t lane0, bool active)
{
    const uint32_t tid = threadIdx.x;
    const int64_t D = P->duration_ms;
    const uint32_t sid = P->sids[0];
    const int64_t ps = P->prop[sid];
    const uint32_t qe = (uint32_t)__builtin_amdgcn_readfirstlane(P->pool_q >= 1u && P->pool_q <= 64u ? P->pool_q : 32u);
    const uint32_t lmin = (uint32_t)__builtin_amdgcn_readfirstlane(P->pool_lmin <= 64u ? P->pool_lmin : 16u);
    const int iters = (int)__builtin_amdgcn_readfirstlane(P->pool_iters >= 1u ? P->pool_iters : 24u);
    SelDevEnv<M, UNI> env{&s_cnt[0][tid], s_prop, P->prop[0], P->uniform_prop != 0, a.cold + lane0 + tid, a.cold_lanes};
    int mode = 3;  // 0 settled form here, 1 away (queued or in an engine), 3 done
    SelMacro<M> mc;
    if (!active) {
        s_mc[0][tid] = 0;
        s_mc[1][tid] = 0;
    } else if (a.force_retry) {
        s_mc[0][tid] = 0;
        s_mc[1][tid] = SERR_CAP;
    } else if (!mc.begin(src)) {
        s_mc[0][tid] = 0;
        s_mc[1][tid] = SERR_DRAWS;
    } else if (mc.T >= D) {
        SelOut r;
        mc.finish(env, sid, r);
        pool_park<M>(env, r, s_mc, tid);
    } else {
        mode = 0;
    }
#if SEL_PROF
    uint64_t pr_set = 0, pr_setl = 0, pr_eng = 0, pr_engl = 0, pr_ph = 0, pr_spin = 0;
    const uint64_t pr_t0 = clock64();
    uint64_t pr_te = 0;
#endif
    uint32_t spins = 0;
    for (;;) {
        // 1. settled-form steps (an inner loop, so that only the settled form's state is live in it) until
        // this wave has no settled-form work left or enough runs wait for an engine; a run that needs the
        // engine is handed to the pool, a run that comes back is taken up again
        if (__builtin_amdgcn_ballot_w64(mode == 0) != 0ull) {
            for (;;) {
                bool hand = false;
#pragma unroll
                for (int u = 0; u < SEL_PSTEPS; ++u) {
#if SEL_PROF
                    ++pr_set;
                    pr_setl += __builtin_popcountll(__builtin_amdgcn_ballot_w64(mode == 0));
#endif
                    if (mode == 0) {
                        const int r = mc.step(env, src, D, sid, ps);
                        if (r == 2) {
                            SelOut q;
                            mc.finish(env, sid, q);
                            pool_park<M>(env, q, s_mc, tid);
                            mode = 3;
                        } else if (r == 1) {
                            mc.save(&s_mc[0][tid], TPB);
                            xfer_save<M>(src, pl, tid);
                            lds_store(&pl.st[tid], PS_QUEUED);
                            hand = true;
                            mode = 1;
                        }
                    }
                }
                const uint64_t hm = __builtin_amdgcn_ballot_w64(hand);
                if (hm != 0ull) {
                    const uint32_t first = (uint32_t)__builtin_ctzll(hm);
                    uint32_t base = 0;
                    if (lane_id() == first)
                        base = __atomic_fetch_add(&pl.tail, (uint32_t)__builtin_popcountll(hm), __ATOMIC_RELAXED);
                    base = __builtin_amdgcn_readlane(base, first);
                    if (hand) {
                        fence_rel();  // the slot's state before its ring entry
                        lds_store(&pl.q[(base + rank_in(hm)) & (POOL_QCAP - 1u)], tid + 1u);
                    }
                }
                if (__builtin_amdgcn_ballot_w64(mode == 0) == 0ull || pool_queued(pl) >= qe) break;
            }
        }
        // 2. runs that came back from an engine (or finished there)
        if (__builtin_amdgcn_ballot_w64(mode == 1) != 0ull) {
            if (mode == 1) {
                const uint32_t v = lds_load(&pl.st[tid]);
                if (v == PS_BACK) {
                    fence_acq();
                    mc.load(&s_mc[0][tid], TPB);
                    xfer_load<M>(src, pl, tid);
                    mode = 0;
                } else if (v == PS_DONE) {
                    mode = 3;
                }
            }
        }
        // 3. become an engine worker when enough runs wait, or when this wave has no settled-form work left
        const uint32_t nset = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(mode == 0));
        const uint32_t qn = pool_queued(pl);
        if (qn >= qe || (nset == 0u && qn > 0u)) {
            spins = 0;
#if SEL_PROF
            ++pr_ph;
            const uint64_t pc0 = clock64();
#endif
            // this wave's settled runs wait in their slots: no settled-form register is live in the phase
            if (mode == 0) {
                mc.save(&s_mc[0][tid], TPB);
                xfer_save<M>(src, pl, tid);
            }
            {
                uint32_t es = POOL_NOSLOT;
                SelT s;
                SelFifo<SelFastDraw<M>> ex = src;  // the drawer's tables; per-run state comes with each slot
                SelDevEnv<M, UNI> ee = env;
                bool refill = true;
                for (int it = 0;; ++it) {
                    if (refill) {
                        const uint64_t fm = __builtin_amdgcn_ballot_w64(es == POOL_NOSLOT);
                        if (fm != 0ull) {
                            const uint32_t first = (uint32_t)__builtin_ctzll(fm);
                            uint32_t h = 0, c = 0;
                            if (lane_id() == first) {
                                const uint32_t nfree = (uint32_t)__builtin_popcountll(fm);
                                for (int tries = 0; tries < 64; ++tries) {
                                    h = lds_load(&pl.head);
                                    const uint32_t t = lds_load(&pl.tail);
                                    c = t - h < nfree ? t - h : nfree;
                                    if (c == 0u) break;
                                    uint32_t exp = h;
                                    if (__atomic_compare_exchange_n(&pl.head, &exp, h + c, false, __ATOMIC_RELAXED,
                                                                    __ATOMIC_RELAXED))
                                        break;
                                    c = 0;
                                }
                            }
                            h = __builtin_amdgcn_readlane(h, first);
                            c = __builtin_amdgcn_readlane(c, first);
                            const uint32_t rk = rank_in(fm);
                            if (es == POOL_NOSLOT && rk < c) {
                                uint32_t *e = &pl.q[(h + rk) & (POOL_QCAP - 1u)];
                                uint32_t v = lds_load(e);
                                for (uint32_t w = 0; v == 0u && w < POOL_SPIN_MAX; ++w) {
                                    __builtin_amdgcn_s_sleep(1);
                                    v = lds_load(e);
                                }
                                lds_store(e, 0u);
                                fence_acq();
                                if (v != 0u) {
                                    es = v - 1u;
                                    SelMacro<M> t;
                                    t.load(&s_mc[0][es], TPB);
                                    xfer_load<M>(ex, pl, es);
                                    ee.c = &s_cnt[0][es];
                                    ee.cb = a.cold + lane0 + es;
                                    t.to_exact(ee, s, P->m, P->sids);
                                }
                            }
                        }
                    }
                    const uint64_t am = __builtin_amdgcn_ballot_w64(es != POOL_NOSLOT);
                    if (am == 0ull) break;
#if SEL_PROF
                    ++pr_eng;
                    pr_engl += __builtin_popcountll(am);
#endif
                    if (es != POOL_NOSLOT) {
                        const bool live = s.step(ee, ex, D);
                        if (!live) {
                            SelOut r;
                            s.finish(ee, D, r);
                            pool_park<M>(ee, r, s_mc, es);
                            fence_rel();
                            lds_store(&pl.st[es], PS_DONE);
                            es = POOL_NOSLOT;
                        } else {
                            SelMacro<M> tb;
                            if (tb.take_back(ee, s, sid)) {
                                if (tb.T >= D) {
                                    SelOut r;
                                    tb.finish(ee, sid, r);
                                    pool_park<M>(ee, r, s_mc, es);
                                    fence_rel();
                                    lds_store(&pl.st[es], PS_DONE);
                                } else {
                                    ex.fill();  // the settled form starts every step with two held draws
                                    tb.save(&s_mc[0][es], TPB);
                                    xfer_save<M>(ex, pl, es);
                                    fence_rel();
                                    lds_store(&pl.st[es], PS_BACK);
                                }
                                es = POOL_NOSLOT;
                            }
                        }
                    }
                    // keep claiming while the phase is young and full enough; then drain what is in hand
                    const uint32_t act = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(es != POOL_NOSLOT));
                    const uint32_t q2 = pool_queued(pl);
                    refill = refill && it + 1 < iters && act + q2 >= lmin;
                }
            }
            if (mode == 0) {
                mc.load(&s_mc[0][tid], TPB);
                xfer_load<M>(src, pl, tid);
            }
#if SEL_PROF
            pr_te += clock64() - pc0;
#endif
            continue;
        }
        if (nset == 0u) {
            if (__builtin_amdgcn_ballot_w64(mode != 3) == 0ull) break;  // every run of this wave is finished
            // every unfinished run of this wave is in another wave's engine: wait for it
#if SEL_PROF
            ++pr_spin;
#endif
            __builtin_amdgcn_s_sleep(2);
            if (++spins > POOL_SPIN_MAX) {
                if (mode == 1) {
                    s_mc[1][tid] = SERR_SCHED;
                    mode = 3;
                }
            }
        } else {
            spins = 0;
        }
    }
#if SEL_PROF
    if (blockIdx.x < 2 && (tid & 63u) == 0u)
        printf("POOLPROF blk %u wave %u total %llu | settled iters %llu lanes %llu | engine phases %llu cyc %llu iters %llu lanes %llu | spins %llu\n",
               blockIdx.x, tid / 64u, (unsigned long long)(clock64() - pr_t0), (unsigned long long)pr_set,
               (unsigned long long)pr_setl, (unsigned long long)pr_ph, (unsigned long long)pr_te,
               (unsigned long long)pr_eng, (unsigned long long)pr_engl, (unsigned long long)pr_spin);
#endif
}

// E1: one lane per (point, run of the slice); workgroups never straddle points. The lane makes its draws
// itself (SelFastDraw). One selfish miner with the settled form: the workgroup pool (sel_pool) when its LDS
// fits two workgroups per CU, else the per-wave mixed schedule; several selfish miners: the engine alone.
template <int M, int NS, int NA, int NG, int NQ, int NC, bool UNI>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(SEL_WAVES, 8))) void msim_sel_kernel(const SelArgs a)
{
    constexpr bool POOL = NS == 1 && SelPoolLds<M>::FITS;
    __shared__ uint32_t s_cnt[4 * M][TPB];
    __shared__ uint32_t s_mc[NS == 1 ? SelMacro<M>::NW : 1][TPB];
    __shared__ std::conditional_t<POOL, SelPool, uint32_t> s_pool;
    __shared__ int64_t s_prop[MAXM];
    __shared__ uint8_t s_lut[128];
    __shared__ LogTab s_log[1];
    const uint32_t tid = threadIdx.x;
    const uint32_t wps = (a.sn + TPB - 1) / TPB;
    const uint32_t point = a.plist[blockIdx.x / wps], blk = blockIdx.x % wps;
    const SelParams *P = a.pts + point;
    if (tid < MAXM) s_prop[tid] = P->prop[tid];
    if (tid < 128) {
        uint32_t f = 0;
        for (int j = 0; j < MAXM; ++j) f += P->ccum[j] <= tid ? 1u : 0u;
        s_lut[tid] = (uint8_t)f;
    }
    if (tid < LOG_TAB) {
        s_log[0].invc[tid] = a.logt->invc[tid];
        s_log[0].A[tid] = a.logt->A[tid];
    }
#pragma unroll
    for (int i = 0; i < 4 * M; ++i) s_cnt[i][tid] = 0u;
    if constexpr (POOL) {
        s_pool.q[tid] = 0u;
        s_pool.q[tid + TPB] = 0u;
        s_pool.st[tid] = 0u;
        if (tid == 0) s_pool.head = s_pool.tail = 0u;
    }
    __syncthreads();
    const uint32_t lr = blk * TPB + tid;
    const bool active = lr < a.sn;
    const uint32_t rel = a.s0 + lr;
    const size_t lane0 = (size_t)(blockIdx.x / wps) * wps * TPB + (size_t)blk * TPB;  // cold slots: lane0 + slot
    const uint64_t run = a.run_begin + rel;
    SelFifo<SelFastDraw<M>> src;
    src.d.ri = rng_seed(seed_interval(a.seed_base, run));
    src.d.rp = rng_seed(seed_picker(a.seed_base, run));
    src.d.lt = s_log;
    src.d.lut = s_lut;
    src.d.P = P;
    src.d.kc = fd_consts();
    src.d.wt = P->W != 100u;
    src.n = 0;
    SelOut o;
    bool have = false;
    if constexpr (POOL) {
        if (P->macro != 0u) {  // wave-uniform (one point per workgroup)
            sel_pool<M, Sel<M, NS, NA, NG, NQ, NC>, UNI>(a, P, src, s_cnt, s_prop, s_mc, s_pool, lane0, active);
#pragma unroll
            for (int k = 0; k < M; ++k) {
                o.found[k] = s_cnt[C_F * M + k][tid];
                o.stale[k] = s_cnt[C_S * M + k][tid];
            }
            o.best_height = s_mc[0][tid];
            o.err = s_mc[1][tid];
            have = true;
        }
    }
    if (!have && active) {
        SelDevEnv<M, UNI> env{&s_cnt[0][tid], s_prop, P->prop[0], P->uniform_prop != 0, a.cold + lane0 + tid, a.cold_lanes};
        const int64_t D = P->duration_ms;
        if (a.force_retry) {
            o.err = SERR_CAP;
        } else if constexpr (NS == 1 && !POOL) {
            sel_mixed<M, Sel<M, NS, NA, NG, NQ, NC>>(env, src, P, D, o, &s_mc[0][tid]);
        } else {  // several selfish miners, or no settled form (a zero delay): the engine alone
            Sel<M, NS, NA, NG, NQ, NC> s;
            s.init(P->m, P->sids);
            s.begin(src);
            for (;;) {
                const bool live = s.step(env, src, D);
                if (!live) break;
            }
            s.finish(env, D, o);
        }
    }
    uint64_t v[6 * M];
#pragma unroll
    for (int i = 0; i < 6 * M; ++i) v[i] = 0;
    if (active) {
        if (o.err) {
            const uint32_t pos = atomicAdd(a.counts, 1u);
            if (pos < a.err_cap) a.err_list[pos] = point * a.rpp + rel;
        } else {
            sel_terms<M>(o, v);
            const size_t g = (size_t)point * a.rpp + rel;
            if (a.records)
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    a.records[2 * (g * M + k) + 0] = o.found[k];
                    a.records[2 * (g * M + k) + 1] = o.stale[k];
                }
            if (a.best_h) a.best_h[g] = o.best_height;
        }
    }
    block_reduce_store<M>(v, a.partials + ((size_t)point * a.wpp + a.s0 / TPB + blk) * 6 * M);
}

// E2: one lane per flagged (point, run), wide capacities, draws from the seeds.
template <int M, int NS>
__global__ __launch_bounds__(TPB) void msim_sel_retry_kernel(const SelArgs a)
{
    __shared__ uint32_t s_cnt[4 * M][TPB];
    __shared__ uint32_t s_mc[NS == 1 && SEL_MC_LDS ? SelMacro<M>::NW : 1][TPB];
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4 * M; ++i) s_cnt[i][tid] = 0u;
    const uint32_t c = *a.counts, lim = c < a.err_cap ? c : a.err_cap;
    const uint32_t idx = blockIdx.x * TPB + tid;
    if (idx >= lim) return;
    const uint32_t code = a.err_list[idx];
    const uint32_t point = code / a.rpp, rel = code % a.rpp;
    const SelParams *P = a.pts + point;
    const uint64_t run = a.run_begin + rel;
    SelDevEnv<M> env{&s_cnt[0][tid], P->prop, P->prop[0], P->uniform_prop != 0, a.cold + idx, a.cold_lanes};
    SelFifo<SelExactDraw<M>> src;
    src.d.ri = rng_seed(seed_interval(a.seed_base, run));
    src.d.rp = rng_seed(seed_picker(a.seed_base, run));
    src.d.P = P;
    src.n = 0;
    SelOut o;
    if constexpr (NS == 1) {  // the mixed schedule, with the engine's wide capacities
        sel_mixed<M, Sel<M, NS, 4, 16, 4, SEL_NC>>(env, src, P, P->duration_ms, o, &s_mc[0][tid]);
    } else {
        Sel<M, NS, 4, 16, 4, SEL_NC> s;
        s.init(P->m, P->sids);
        s.run(env, src, P->duration_ms, o);
    }
    if (o.err || a.force_gen) {  // G (msim_general.h) takes the run over: its windows have no such limits
        if (a.gen_list) {
            const uint32_t pos = atomicAdd(a.counts + GEN_C_L1, 1u);
            if (pos < a.err_cap) a.gen_list[pos] = code;
            else atomicAdd(a.counts + GEN_C_FAIL, 1u);
        } else {
            atomicAdd(a.counts + GEN_C_FAIL, 1u);
        }
        return;
    }
    uint64_t v[6 * M];
    sel_terms<M>(o, v);
    const size_t g = (size_t)point * a.rpp + rel;
    if (a.records)
#pragma unroll
        for (int k = 0; k < M; ++k) {
            a.records[2 * (g * M + k) + 0] = o.found[k];
            a.records[2 * (g * M + k) + 1] = o.stale[k];
        }
    if (a.best_h) a.best_h[g] = o.best_height;
#pragma unroll
    for (int i = 0; i < 6 * M; ++i)
        if (v[i]) atomicAdd((unsigned long long *)(a.retry_sums + (size_t)point * 6 * M + i), (unsigned long long)v[i]);
}

// Capacity classes (msim_sel_launch.h). Measured on the 360-point configs[3] grid: with one selfish miner the
// (1 hot slot, 2 reveal groups) class flagged ~1 % of the runs (reveal groups) and (1, 4) none; the engine
// alone with a wider register class (3, 8, 3) spilled and ran the sweep 2.1x slower than (2, 4, 2).
template <int M, int NS>
static hipError_t launch_sel_ns(const SelArgs &a, hipStream_t s)
{
    const uint32_t wps = (a.sn + TPB - 1) / TPB;
    const dim3 grid(a.nlist * wps);
    if constexpr (NS == 1) {  // the settled form reads the pending finder's delay: a uniform network's from a scalar
        if (a.uni) hipLaunchKernelGGL((msim_sel_kernel<M, NS, 1, 4, 1, SEL_NC, true>), grid, dim3(TPB), 0, s, a);
        else hipLaunchKernelGGL((msim_sel_kernel<M, NS, 1, 4, 1, SEL_NC, false>), grid, dim3(TPB), 0, s, a);
    } else {  // the engine alone (no settled form)
        hipLaunchKernelGGL((msim_sel_kernel<M, NS, 2, 4, 2, SEL_NC, false>), grid, dim3(TPB), 0, s, a);
    }
    return hipGetLastError();
}

#if defined(MSIM_M)
#define MSIM_CAT2(a, b) a##b
#define MSIM_CAT(a, b) MSIM_CAT2(a, b)
hipError_t MSIM_CAT(launch_sel_m, MSIM_M)(const SelArgs &a, uint32_t ns_class, hipStream_t s)
{
    if (ns_class == 1) return launch_sel_ns<MSIM_M, 1>(a, s);
#if MSIM_M >= 2
    if (ns_class == 2) return launch_sel_ns<MSIM_M, 2>(a, s);
    return launch_sel_ns<MSIM_M, 4>(a, s);
#else
    return hipErrorInvalidValue;
#endif
}
hipError_t MSIM_CAT(launch_sel_retry_m, MSIM_M)(const SelArgs &a, uint32_t ns_class, hipStream_t s)
{
    const dim3 grid((a.err_cap + TPB - 1) / TPB);
    if (ns_class == 1) hipLaunchKernelGGL((msim_sel_retry_kernel<MSIM_M, 1>), grid, dim3(TPB), 0, s, a);
#if MSIM_M >= 2
    else if (ns_class == 2) hipLaunchKernelGGL((msim_sel_retry_kernel<MSIM_M, 2>), grid, dim3(TPB), 0, s, a);
    else hipLaunchKernelGGL((msim_sel_retry_kernel<MSIM_M, 4>), grid, dim3(TPB), 0, s, a);
#endif
    return hipGetLastError();
}
#endif

}  // namespace msim
