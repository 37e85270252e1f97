// msim_sel_kernels.hip — E1 / E2 of the entity-engine path (msim_sel_launch.h), one translation unit
// per miner count (MSIM_M).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "msim_general_launch.h"
#include "msim_jump.h"
#include "msim_kernels.h"
#include "msim_reduce.h"
#include "msim_sel_launch.h"
#include "msim_selm.h"
#include "msim_selseg.h"

namespace msim {

#if SEL_ENGPROF
// per-lane section cycles of the engine step (msim_sel.h SEL_EP), printed by E1 for a few waves
__device__ uint64_t sel_engprof_buf[8][TPB];
__device__ void sel_engprof_acc(int i, uint64_t c)
{
    sel_engprof_buf[i][threadIdx.x] += blockIdx.x == 0 ? c : 0;  // block 0 only (others would race)
}
#endif

#ifndef SEL_SRC_LDS
#define SEL_SRC_LDS 1  // E1's draw source parked in LDS during engine phases (SelLdsSrc); 0: in registers (A/B)
#endif

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
};

// Fast sequence (E1 without a word stream): K1's table interval with its exactness check and exact
// fallback (msim_fastdraw.h), the finder through the LDS code table for percentages (W = 100) or the
// weighted scan otherwise (wave-uniform choice). The fast forms are branch-free (fast interval, fast table
// pick, the two exactness flags) so that the compiler can interleave a draw with the transitions it runs
// beside; the branch at the end redoes what they cannot settle (rare; every pick of a weighted network).
template <int M>
struct SelFastDraw {
    Rng ri, rp;
    const LogTab *lt;     // LDS
    const uint8_t *lut;   // LDS: finder of q = floor(u / PERC_MULTIPLIER)
    const SelParams *P;
    FdConsts kc;
    bool wt;
    __device__ __forceinline__ void draw(uint32_t &I, uint32_t &k)
    {
        // both RNG steps, the table indices and the LDS reads (log table, finder table)
        const uint64_t u_i = rng_next(ri);
        const uint64_t u_p = rng_next(rp);
        const uint32_t lo = (uint32_t)u_i, hi = (uint32_t)(u_i >> 32);
        const double c = __builtin_fma(u32_to_f64(lo >> 11), -0x1.0p-53, 1.0);
        const double v = __builtin_fma(u32_to_f64(hi), -0x1.0p-32, c);  // 1 - (u>>11) 2^-53, exact
        const uint64_t vb = __builtin_bit_cast(uint64_t, v);
        const uint32_t vh = (uint32_t)(vb >> 32);
        const int32_t e = (int)(vh >> 20) - 1023;
        const uint32_t j = (vh >> (20 - LOG_BITS)) & (LOG_TAB - 1);
        const double w = __builtin_bit_cast(double, (vb & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
        uint32_t aoff = j * 8u;
        asm("" : "+v"(aoff));
        const double A = *(const double *)((const char *)lt->A + aoff);
        const double invc = lt->invc[j];
        uint32_t kp;
        k = lut[pick_q_fast_key(u_p, kp)];  // q = 100: PickFinder falls through (finder >= m)
        // the interval polynomial (msim_fastdraw.h interval_fast_z, the same operations) and the flags
        const double r = __builtin_fma(w, invc, -1.0);
        double p = __builtin_fma(r, kc.c5, kc.c4);
        p = __builtin_fma(r, p, kc.c3);
        p = __builtin_fma(r, p, kc.c2);
        p = __builtin_fma(r, p, kc.c1);
        const double z0 = __builtin_fma(r, p, A);
        const double z = __builtin_fma((double)e, FD_CE, z0);
        I = (uint32_t)(int32_t)z;
        const double f = __builtin_amdgcn_fract(z);
        const uint32_t ki = (uint32_t)(__builtin_bit_cast(uint64_t, f) >> 32) - FD_OK_LO;
        const bool x_i = ki >= FD_OK_RANGE;
        const bool x_p = kp >= PICK_RARE_LO;
        if (x_i | x_p | wt) {
            if (x_i) I = (uint32_t)interval_ms_exact_dev(u_i);
            if (wt) k = sel_pick_weighted<M>(u_p, P);
            else if (x_p) k = lut[pick_q_exact(u_p)];
        }
    }
};

// E1's draw source during an engine phase: the lane's held draws and both RNG states wait in its LDS column
// (p[i * TPB], SEL_SRC_WORDS words) instead of registers, so that the engine step, which needs every register
// it can get, does not carry them (measured: its loop spilled 24 scratch instructions per iteration, the bulk of
// E1's 37 GB of HBM traffic per configs[2] launch). The engine takes a draw per find (next); the rest of the
// draw state (tables, constants) is wave-uniform.
constexpr int SEL_SRC_WORDS = 17;  // ri, rp (8), I0..I3, k0..k3 (8), n
template <int M>
struct SelLdsSrc {
    uint32_t *p;        // &s_src[0][tid]
    SelFastDraw<M> d;   // tables and constants (ri / rp are loaded from the column for each fresh draw)
    __device__ __forceinline__ uint32_t &w(int i) { return p[i * TPB]; }
    template <class F>
    __device__ __forceinline__ void park(const F &f)
    {
        w(0) = (uint32_t)f.d.ri.s0; w(1) = (uint32_t)(f.d.ri.s0 >> 32);
        w(2) = (uint32_t)f.d.ri.s1; w(3) = (uint32_t)(f.d.ri.s1 >> 32);
        w(4) = (uint32_t)f.d.rp.s0; w(5) = (uint32_t)(f.d.rp.s0 >> 32);
        w(6) = (uint32_t)f.d.rp.s1; w(7) = (uint32_t)(f.d.rp.s1 >> 32);
        w(8) = f.I0; w(9) = f.I1; w(10) = f.I2; w(11) = f.I3;
        w(12) = f.k0; w(13) = f.k1; w(14) = f.k2; w(15) = f.k3;
        w(16) = f.n;
    }
    template <class F>
    __device__ __forceinline__ void unpark(F &f)
    {
        f.d.ri.s0 = ((uint64_t)w(1) << 32) | w(0);
        f.d.ri.s1 = ((uint64_t)w(3) << 32) | w(2);
        f.d.rp.s0 = ((uint64_t)w(5) << 32) | w(4);
        f.d.rp.s1 = ((uint64_t)w(7) << 32) | w(6);
        f.I0 = w(8); f.I1 = w(9); f.I2 = w(10); f.I3 = w(11);
        f.k0 = w(12); f.k1 = w(13); f.k2 = w(14); f.k3 = w(15);
        f.n = w(16);
    }
    __device__ __forceinline__ bool next(uint32_t &I, uint32_t &k)
    {
        const uint32_t n = w(16);
        if (n == 0u) {  // a fresh draw from the parked streams
            d.ri.s0 = ((uint64_t)w(1) << 32) | w(0);
            d.ri.s1 = ((uint64_t)w(3) << 32) | w(2);
            d.rp.s0 = ((uint64_t)w(5) << 32) | w(4);
            d.rp.s1 = ((uint64_t)w(7) << 32) | w(6);
            d.draw(I, k);
            w(0) = (uint32_t)d.ri.s0; w(1) = (uint32_t)(d.ri.s0 >> 32);
            w(2) = (uint32_t)d.ri.s1; w(3) = (uint32_t)(d.ri.s1 >> 32);
            w(4) = (uint32_t)d.rp.s0; w(5) = (uint32_t)(d.rp.s0 >> 32);
            w(6) = (uint32_t)d.rp.s1; w(7) = (uint32_t)(d.rp.s1 >> 32);
            return true;
        }
        I = w(8);  // the oldest held draw, then the FIFO shifts
        k = w(12);
        w(8) = w(9); w(9) = w(10); w(10) = w(11);
        w(12) = w(13); w(13) = w(14); w(14) = w(15);
        w(16) = n - 1u;
        return true;
    }
    __device__ __forceinline__ void prefetch() {}
    __device__ __forceinline__ void settle() {}
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
#ifndef SEL_ENGPROF
#define SEL_ENGPROF 0
#endif
#ifndef SEL_MSTEPS
#define SEL_MSTEPS 2
#endif
#ifndef SEL_MC_LDS
#define SEL_MC_LDS 1  // the settled-form state waits in LDS during engine phases
#endif
template <int M, class SelT, class Env, class Src>
__device__ __forceinline__ void sel_mixed(Env &env, Src &src, const SelParams *P, int64_t D, SelOut &o, uint32_t *mcs,
                                          const uint32_t *lut, uint32_t *srcs = nullptr)
{
    // E1's draw source waits in LDS during engine phases (SelLdsSrc); E2 keeps it in registers
    constexpr bool lds_src = SEL_SRC_LDS && std::is_same_v<Src, SelFifo<SelFastDraw<M>>>;
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
    int64_t thrmax = 0;  // the largest settle threshold of an honest find (SelMacro::step4)
    for (uint32_t j = 0; j < P->m; ++j)
        if (j != sid) thrmax = P->prop[j] + ps > thrmax ? P->prop[j] + ps : thrmax;
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
#if SEL_PROF  // per-wave phase timing (diagnostic builds only: scripts/build_variant.sh prof msim_sel_kernels.hip -DSEL_PROF=1)
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
            [[maybe_unused]] std::conditional_t<lds_src, SelLdsSrc<M>, char> ls{};
            if constexpr (lds_src) {
                ls.p = srcs;
                ls.d = src.d;
                ls.park(src);
            }
            uint32_t refill = 0;  // lanes back in the settled form: top the FIFO up after the phase
            for (;;) {
                if (mode == 2) {
                    src.prefetch();
                    bool live;
                    if constexpr (lds_src) live = s.step(env, ls, D);
                    else live = s.step(env, src, D);
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
                                if constexpr (lds_src) refill = 1u;
                                else src.fill();  // the settled form starts every step with two held draws
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
            if constexpr (lds_src) {
                ls.unpark(src);
                if (refill) src.fill();  // the settled form starts every step with two held draws
            }
#if SEL_MC_LDS
            mc.load(mcs, TPB);
#endif
        } else {
            for (;;) {
                // SEL_MSTEPS settled-form steps (four finds each when none needs the engine) per exit test (a
                // lane that leaves the form skips the rest)
#pragma unroll
                for (int u = 0; u < SEL_MSTEPS; ++u) {
                    if (mode == 0) {
                        const int r = mc.step4(env, src, D, sid, ps, thrmax, lut);
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

// E1: one lane per (point, run of the slice); workgroups never straddle points. The lane makes its draws
// itself (SelFastDraw). One selfish miner: the mixed schedule (settled form + per-wave engine phases);
// several selfish miners: the engine alone.
//
// Measured and rejected (round 4, profiles/r04/e1pool): a WORKGROUP pool that hands a run needing the engine
// to whichever of the workgroup's four waves is free (the run's settled and draw state through LDS, an LDS
// ring of queued runs), so that engine steps run on fuller waves. Exact, but slower on configs[2]: 80-125 ms
// per 131 072-run launch against 57.5 ms, whatever the queue threshold / refill floor / phase length. An
// engine step costs the same per ACTIVE lane (~1 300 cycles per lane-event at 7 or at 15 active lanes: the
// step is a chain of dependent LDS / cold-slot accesses whose latency grows with the divergent paths taken),
// so fuller engine waves saved nothing, while runs waited longer away from their lanes (32 instead of 57
// lanes active per settled-form step).
template <int M, int NS, int NA, int NG, int NQ, int NC, bool UNI>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(SEL_WAVES, 8))) void msim_sel_kernel(const SelArgs a)
{
    __shared__ uint32_t s_cnt[4 * M][TPB];
    __shared__ uint32_t s_mc[NS == 1 && SEL_MC_LDS ? SelMacro<M>::NW : 1][TPB];
    __shared__ uint32_t s_src[NS == 1 && SEL_SRC_LDS ? SEL_SRC_WORDS : 1][TPB];  // SelLdsSrc columns
    __shared__ uint32_t s_tab[SP_LUT];  // four-find transitions (msim_selm.h sp_lut_entry)
    __shared__ int64_t s_prop[MAXM];
    __shared__ uint8_t s_lut[128];
    __shared__ LogTab s_log[1];
    const uint32_t tid = threadIdx.x;
    if (tid < SP_LUT) s_tab[tid] = sp_lut_entry(tid / 16u, tid % 16u);
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
    __syncthreads();
    const uint32_t lr = blk * TPB + tid;
    const bool active = lr < a.sn;
    const uint32_t rel = a.s0 + lr;
    const size_t lane0 = (size_t)(blockIdx.x / wps) * wps * TPB + (size_t)blk * TPB;  // cold slots: lane0 + tid
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
    if (active) {
        SelDevEnv<M, UNI> env{&s_cnt[0][tid], s_prop, P->prop[0], P->uniform_prop != 0, a.cold + lane0 + tid, a.cold_lanes};
        const int64_t D = P->duration_ms;
        if (a.force_retry) {
            o.err = SERR_CAP;
        } else if constexpr (NS == 1) {
            sel_mixed<M, Sel<M, NS, NA, NG, NQ, NC>>(env, src, P, D, o, &s_mc[0][tid], s_tab, &s_src[0][tid]);
        } else {  // several selfish miners: the engine alone
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
#if SEL_ENGPROF
    if (blockIdx.x == 0 && (tid & 63u) == 0u) {
        unsigned long long t[7];
        for (int i = 0; i < 7; ++i) {
            t[i] = 0;
            for (uint32_t l = tid; l < tid + 64; ++l) t[i] += sel_engprof_buf[i][l];
        }
        printf("ENGPROF wave %u finds %llu publish %llu best %llu notify %llu merge+resolve %llu fold %llu earliest %llu\n",
               tid / 64u, t[0], t[1], t[2], t[3], t[4], t[5], t[6]);
    }
#endif
}


// ------------------------------------------------------------------ segment-parallel form (msim_selseg.h)
// The per-network tables every selfish kernel keeps in LDS (E1's prologue): delays, PickFinder code table,
// interval log table, four-find transition table.
template <int M>
struct SelLds {
    uint32_t tab[SP_LUT];
    int64_t prop[MAXM];
    uint8_t lut[128];
    LogTab log;
    __device__ void load(const SelParams *P, const LogTab *lt, uint32_t tid)
    {
        if (tid < SP_LUT) tab[tid] = sp_lut_entry(tid / 16u, tid % 16u);
        if (tid < MAXM) prop[tid] = P->prop[tid];
        if (tid < 128) {
            uint32_t f = 0;
            for (int j = 0; j < MAXM; ++j) f += P->ccum[j] <= tid ? 1u : 0u;
            lut[tid] = (uint8_t)f;
        }
        if (tid < LOG_TAB) {
            log.invc[tid] = lt->invc[tid];
            log.A[tid] = lt->A[tid];
        }
    }
};

template <int M>
__device__ __forceinline__ void sel_thresholds(const SelParams *P, uint32_t &sid, int64_t &ps, int64_t &thrmax)
{
    sid = P->sids[0];
    ps = P->prop[sid];
    thrmax = 0;
    for (uint32_t j = 0; j < P->m; ++j)
        if (j != sid) thrmax = P->prop[j] + ps > thrmax ? P->prop[j] + ps : thrmax;
}

// SW: one lane per (run of the slice, segment): the settled form from the quiet state at the segment's first
// block, with no end of run; a sub per cut and one at the segment's end (msim_selseg.h seg_work). Grid
// (sn / TPB, nseg): a wave is 64 consecutive runs at one segment, so the jump matrix columns are wave-uniform.
template <int M, bool UNI>
__global__ __launch_bounds__(TPB) void msim_segwork_kernel(const SelArgs a, const SegArgs g)
{
    __shared__ uint32_t s_cnt[2 * M][TPB];
    __shared__ SelLds<M> sl;
    const uint32_t tid = threadIdx.x;
    const SelParams *P = a.pts + a.plist[0];
    sl.load(P, a.logt, tid);
#pragma unroll
    for (int i = 0; i < 2 * M; ++i) s_cnt[i][tid] = 0u;
    __syncthreads();
    const uint32_t lr = blockIdx.x * TPB + tid;  // run of the slice
    const uint32_t j = blockIdx.y;               // segment
    if (lr >= a.sn) return;
    const uint64_t run = a.run_begin + a.s0 + lr;
    SegFifo<SelFastDraw<M>> src;
    src.d.ri = rng_seed(seed_interval(a.seed_base, run));
    src.d.rp = rng_seed(seed_picker(a.seed_base, run));
    if (j) jump2(reinterpret_cast<const uint4 *>(g.jump) + (size_t)j * 128, src.d.ri, src.d.rp);
    src.d.lt = &sl.log;
    src.d.lut = sl.lut;
    src.d.P = P;
    src.d.kc = fd_consts();
    src.d.wt = P->W != 100u;
    src.n = 0;
    src.idx = j * g.seg;
    SelDevEnv<M, UNI> env{&s_cnt[0][tid], sl.prop, P->prop[0], P->uniform_prop != 0, nullptr, 0};
    uint32_t sid;
    int64_t ps, thrmax;
    sel_thresholds<M>(P, sid, ps, thrmax);
    SegRec<M> *out = (SegRec<M> *)g.recs + ((size_t)lr * g.nseg + j) * g.cap;
    SegQRec<M> *qout = (SegQRec<M> *)g.qrecs + ((size_t)lr * g.nseg + j) * g.qcap;
    uint32_t q = 0;
    auto emit = [&](const SegRec<M> &r) {
        if (q >= g.cap) return false;
        out[q++] = r;
        return true;
    };
    struct EmitQ {
        SegQRec<M> *p;
        uint32_t cap, c;
        __device__ bool operator()(const SegQRec<M> &r)
        {
            if (c >= cap) return false;
            p[c++] = r;
            return true;
        }
        __device__ uint32_t n() const { return c; }
    } emitq{qout, g.qcap, 0u};
    const uint32_t err = seg_work<M>(env, src, (j + 1) * g.seg, sid, ps, thrmax, sl.tab, emit, emitq);
    g.cnt[(size_t)j * g.nr + lr] = err ? SEG_OVERFLOW : q;
    g.qcnt[(size_t)j * g.nr + lr] = emitq.c;
}

// The workers' subs and checkpoints of one run, for ST (msim_selseg.h seg_stitch_step's Recs).
template <int M>
struct SegDevRecs {
    const SegRec<M> *recs;    // this run's [nseg][cap]
    const uint32_t *cnt;      // [nseg][nr], offset to this run
    const SegQRec<M> *qrecs;  // this run's [nseg][qcap]
    const uint32_t *qcnt;     // [nseg][nr], offset to this run
    uint32_t nseg, cap, qcap, nr;
    __device__ uint32_t count(uint32_t j) const { return j < nseg ? cnt[(size_t)j * nr] : 0u; }
    __device__ SegRec<M> rec(uint32_t j, uint32_t q) const { return recs[(size_t)j * cap + q]; }
    __device__ void head(uint32_t j, uint32_t q, uint32_t &b, uint32_t &flags) const
    {
        const uint2 v = *(const uint2 *)&recs[(size_t)j * cap + q].b;
        b = v.x;
        flags = v.y;
    }
    __device__ uint32_t qcount(uint32_t j) const { return j < nseg ? qcnt[(size_t)j * nr] : 0u; }
    __device__ uint32_t qc(uint32_t j, uint32_t i) const { return qrecs[(size_t)j * qcap + i].c; }
    __device__ uint32_t qspan(uint32_t j, uint32_t i) const { return qrecs[(size_t)j * qcap + i].span; }
    __device__ SegQRec<M> qrec(uint32_t j, uint32_t i) const { return qrecs[(size_t)j * qcap + i]; }
};

// ST: one lane per run of the slice. Lanes walk their runs through the workers' records (msim_selseg.h
// seg_stitch_step: walks to a join, jumps, the end of the run); a lane whose true state needs the entity engine
// waits, and when g.xth lanes of the wave wait (or nothing else is left) the wave runs an engine phase for them,
// as E1 does, with every lane's settled state parked in LDS. Outputs are E1's: MinerStats terms per workgroup,
// per-run records, flagged runs for E2.
template <int M, bool UNI>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(SEL_WAVES, 8))) void msim_stitch_kernel(const SelArgs a,
                                                                                                           const SegArgs g)
{
    __shared__ uint32_t s_cnt[4 * M][TPB];             // C_F, C_S, C_A, C_B
    __shared__ uint32_t s_x[SelMacro<M>::NW][TPB];     // the settled state during engine phases
    __shared__ SelLds<M> sl;
    const uint32_t tid = threadIdx.x;
    const uint32_t point = a.plist[0];
    const SelParams *P = a.pts + point;
    sl.load(P, a.logt, tid);
#pragma unroll
    for (int i = 0; i < 4 * M; ++i) s_cnt[i][tid] = 0u;
    __syncthreads();
    const uint32_t lr = blockIdx.x * TPB + tid;
    const bool active = lr < a.sn;
    const uint32_t rel = a.s0 + lr;
    const uint64_t run = a.run_begin + rel;
    const int64_t D = P->duration_ms;
    uint32_t sid;
    int64_t ps, thrmax;
    sel_thresholds<M>(P, sid, ps, thrmax);
    SelDevEnv<M, UNI> env{&s_cnt[0][tid], sl.prop, P->prop[0], P->uniform_prop != 0, a.cold + (size_t)blockIdx.x * TPB + tid,
                          a.cold_lanes};
    const uint32_t rr = active ? lr : 0u;
    SegDevRecs<M> R{(const SegRec<M> *)g.recs + (size_t)rr * g.nseg * g.cap, g.cnt + rr,
                    (const SegQRec<M> *)g.qrecs + (size_t)rr * g.nseg * g.qcap, g.qcnt + rr, g.nseg, g.cap, g.qcap, g.nr};
    SegFifo<SelFastDraw<M>> st;
    st.d.ri = rng_seed(seed_interval(a.seed_base, run));
    st.d.rp = rng_seed(seed_picker(a.seed_base, run));
    st.d.lt = &sl.log;
    st.d.lut = sl.lut;
    st.d.P = P;
    st.d.kc = fd_consts();
    st.d.wt = P->W != 100u;
    st.n = 0;
    st.idx = 0;
    SegStitch<M> S;
    S.err = 0;
    S.seg = S.q = S.qi = S.at_rec = 0;
    S.walk_back = 1;
    S.mode = ST_DONE;
    uint32_t bh = 0, fin = 0;  // fin: the result is parked in the C_F / C_S rows
    auto park = [&](const SelOut &r) {
#pragma unroll
        for (int k = 0; k < M; ++k) {
            env.set(C_F, (uint32_t)k, r.found[k]);
            env.set(C_S, (uint32_t)k, r.stale[k]);
        }
        bh = r.best_height;
        S.err |= r.err;
        fin = 1;
    };
    if (active) {
        bool over = a.force_retry != 0;
        for (uint32_t j = 0; j < g.nseg; ++j) over |= R.count(j) == SEG_OVERFLOW;
        if (over) {
            S.err = SERR_CAP;
        } else if (!S.X.begin(st)) {
            S.err = SERR_DRAWS;
        } else if (S.X.T >= D) {
            SelOut r;
            S.X.finish(env, sid, r);
            park(r);
        } else {
            S.mode = ST_WALK;  // segment 0's worker starts quiet at the run's first find
        }
    }
    const int xth = (int)__builtin_amdgcn_readfirstlane(g.xth >= 1u && g.xth <= 64u ? g.xth : 16u);
    for (;;) {
        const uint64_t bm = __builtin_amdgcn_ballot_w64(S.mode <= ST_WALK || S.mode == ST_END);
        const uint64_t be = __builtin_amdgcn_ballot_w64(S.mode == ST_ENGINE);
        if ((bm | be) == 0ull) break;
        if (be != 0ull && (__builtin_popcountll(be) >= xth || bm == 0ull)) {
            // the settled states wait in LDS while the engine runs; an engine lane converts its state first and
            // parks the one it hands back
            Sel<M, 1, 1, 4, 1, SEL_NC> s;
            uint32_t in = S.mode == ST_ENGINE ? 1u : 0u, after = 0u;
            if (in) S.X.to_exact(env, s, P->m, P->sids);
            else S.X.save(&s_x[0][tid], TPB);
            for (;;) {
                if (in) {
                    const bool live = s.step(env, st, D);
                    if (!live) {
                        SelOut r;
                        s.finish(env, D, r);
                        park(r);
                        S.mode = ST_DONE;
                        in = 0;
                    } else {
                        SelMacro<M> tb;
                        if (tb.take_back(env, s, sid)) {
                            in = 0;
                            if (tb.T >= D) {
                                SelOut r;
                                tb.finish(env, sid, r);
                                park(r);
                                S.mode = ST_DONE;
                            } else {
                                tb.save(&s_x[0][tid], TPB);
                                after = 1u;
                            }
                        }
                    }
                }
                if (__builtin_amdgcn_ballot_w64(in != 0u) == 0ull) break;
            }
            S.X.load(&s_x[0][tid], TPB);
            if (after) {
                st.fill();
                S.mode = S.walk_back ? ST_WALK : ST_END;
            }
        } else {
            for (;;) {
                if (S.mode <= ST_WALK || S.mode == ST_END) {
                    seg_stitch_step<M>(S, R, env, st, D, sid, ps, thrmax, sl.tab);
                    if (S.mode == ST_DONE && !S.err) {
                        SelOut r;
                        S.X.finish(env, sid, r);
                        park(r);
                    }
                }
                if (__builtin_amdgcn_ballot_w64(S.mode <= ST_WALK || S.mode == ST_END) == 0ull ||
                    __builtin_popcountll(__builtin_amdgcn_ballot_w64(S.mode == ST_ENGINE)) >= xth)
                    break;
            }
        }
    }
    SelOut o;
    o.err = S.err;
    o.best_height = bh;
    if (active && !S.err) {
#pragma unroll
        for (int k = 0; k < M; ++k) {
            o.found[k] = env.get(C_F, (uint32_t)k);
            o.stale[k] = env.get(C_S, (uint32_t)k);
        }
    }
    uint64_t v[6 * M];
#pragma unroll
    for (int i = 0; i < 6 * M; ++i) v[i] = 0;
    if (active) {
        if (o.err || !fin) {
            const uint32_t pos = atomicAdd(a.counts, 1u);
            if (pos < a.err_cap) a.err_list[pos] = point * a.rpp + rel;
        } else {
            sel_terms<M>(o, v);
            const size_t gi = (size_t)point * a.rpp + rel;
            if (a.records)
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    a.records[2 * (gi * M + k) + 0] = o.found[k];
                    a.records[2 * (gi * M + k) + 1] = o.stale[k];
                }
            if (a.best_h) a.best_h[gi] = o.best_height;
        }
    }
    block_reduce_store<M>(v, a.partials + ((size_t)point * a.wpp + a.s0 / TPB + blockIdx.x) * 6 * M);
}

// E2: one lane per flagged (point, run), wide capacities, draws from the seeds.
template <int M, int NS>
__global__ __launch_bounds__(TPB) void msim_sel_retry_kernel(const SelArgs a)
{
    __shared__ uint32_t s_cnt[4 * M][TPB];
    __shared__ uint32_t s_mc[NS == 1 && SEL_MC_LDS ? SelMacro<M>::NW : 1][TPB];
    __shared__ uint32_t s_tab[SP_LUT];  // four-find transitions (msim_selm.h sp_lut_entry)
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4 * M; ++i) s_cnt[i][tid] = 0u;
    if (tid < SP_LUT) s_tab[tid] = sp_lut_entry(tid / 16u, tid % 16u);
    __syncthreads();
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
        sel_mixed<M, Sel<M, NS, 4, 16, 4, SEL_NC>>(env, src, P, P->duration_ms, o, &s_mc[0][tid], s_tab);
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
hipError_t MSIM_CAT(launch_segwork_m, MSIM_M)(const SelArgs &a, const SegArgs &g, hipStream_t s)
{
    const dim3 grid((a.sn + TPB - 1) / TPB, g.nseg);
    if (a.uni) hipLaunchKernelGGL((msim_segwork_kernel<MSIM_M, true>), grid, dim3(TPB), 0, s, a, g);
    else hipLaunchKernelGGL((msim_segwork_kernel<MSIM_M, false>), grid, dim3(TPB), 0, s, a, g);
    return hipGetLastError();
}
hipError_t MSIM_CAT(launch_stitch_m, MSIM_M)(const SelArgs &a, const SegArgs &g, hipStream_t s)
{
    const dim3 grid((a.sn + TPB - 1) / TPB);
    if (a.uni) hipLaunchKernelGGL((msim_stitch_kernel<MSIM_M, true>), grid, dim3(TPB), 0, s, a, g);
    else hipLaunchKernelGGL((msim_stitch_kernel<MSIM_M, false>), grid, dim3(TPB), 0, s, a, g);
    return hipGetLastError();
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
