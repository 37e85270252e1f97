// msim_wide.hip — gfx950 kernels of the large-network pipeline (msim_wide.h): W1 draws + LDS histogram
// (one wave per run), W2 episodes (one lane per candidate), W3 combine + MinerStats sums (one wave per run).
//
// Roofline: W1 is VALU-issue bound like the narrow K1 (two xoroshiro128++ steps, the FP64 interval and a
// bucketed weighted pick per block, one LDS atomic); W2/W3 are short latency-bound passes over ~rho of
// the blocks and M counters per run. HBM traffic is ~4 KiB of histogram per run plus ~rho * blocks
// candidate records: far below the HBM roofline.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <mutex>
#include <utility>

#include "msim_jump.h"
#include "msim_wide_launch.h"

namespace msim {

__device__ __noinline__ int32_t interval_ms_exact_dev(uint64_t u) { return (int32_t)interval_ms_of(u); }

namespace {

// Both RNG states advanced by one 128x128 GF(2) matrix (msim_jump.h layout). `cols` may differ per lane.
__device__ __forceinline__ void jump_both(const uint4 *__restrict__ cols, Rng &a, Rng &b)
{
    const uint32_t sa[4] = {(uint32_t)a.s0, (uint32_t)(a.s0 >> 32), (uint32_t)a.s1, (uint32_t)(a.s1 >> 32)};
    const uint32_t sb[4] = {(uint32_t)b.s0, (uint32_t)(b.s0 >> 32), (uint32_t)b.s1, (uint32_t)(b.s1 >> 32)};
    uint32_t oa0 = 0, oa1 = 0, oa2 = 0, oa3 = 0, ob0 = 0, ob1 = 0, ob2 = 0, ob3 = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
#pragma unroll 8
        for (int i = 0; i < 32; ++i) {
            const uint4 c = cols[w * 32 + i];
            const uint32_t ma = 0u - ((sa[w] >> i) & 1u), mb = 0u - ((sb[w] >> i) & 1u);
            oa0 ^= c.x & ma;
            oa1 ^= c.y & ma;
            oa2 ^= c.z & ma;
            oa3 ^= c.w & ma;
            ob0 ^= c.x & mb;
            ob1 ^= c.y & mb;
            ob2 ^= c.z & mb;
            ob3 ^= c.w & mb;
        }
    }
    a.s0 = (uint64_t)oa0 | ((uint64_t)oa1 << 32);
    a.s1 = (uint64_t)oa2 | ((uint64_t)oa3 << 32);
    b.s0 = (uint64_t)ob0 | ((uint64_t)ob1 << 32);
    b.s1 = (uint64_t)ob2 | ((uint64_t)ob3 << 32);
}

__device__ __forceinline__ uint64_t wave_excl_scan(uint64_t x, uint32_t lane)
{
    uint64_t v = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up((unsigned long long)v, o, 64);
        if ((int)lane >= o) v += y;
    }
    return v - x;
}

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }

struct W1Lds {
    const uint64_t *cf;
    const uint16_t *bucket;
    uint32_t *hist;  // this wave's run
    uint32_t *cc;    // this wave's candidate counter
};

// Lane segment of nblk blocks starting at block b0 (RNG states positioned at draw b0).
__device__ __forceinline__ uint64_t w1_segment(const WideArgs &a, const W1Lds &s, const LogTab *__restrict__ lt, Rng &ri, Rng &rp,
                               uint32_t nblk, uint32_t b0, uint32_t phase, uint32_t lane, uint32_t r, uint32_t &flast,
                               uint32_t &nc, uint32_t &pick_err_blk, uint32_t &err)
{
    uint32_t Icur = draw_interval(ri, lt), thcur;
    uint32_t fcur = wide_pick(rng_next(rp), s.cf, s.bucket, a.W, a.mult, thcur);
    uint64_t tsum = 0;
    nc = 0;
    for (uint32_t b = 0; b < nblk; ++b) {
        const uint32_t Inext = draw_interval(ri, lt);
        uint32_t thnext;
        const uint32_t fnext = wide_pick(rng_next(rp), s.cf, s.bucket, a.W, a.mult, thnext);
        tsum += Icur;
        bool slow = false;
        if (fcur < a.m) {
            atomicAdd(&s.hist[fcur], 1u);
            slow = Inext <= thcur;
        } else if (pick_err_blk == WIDE_NONE) {
            pick_err_blk = b0 + b;
        }
        if (slow) {
            const uint32_t c = atomicAdd(s.cc, 1u);
            if (c < a.rcap) {
                WideCand e;
                e.block = b0 + b;
                e.f = fcur;
                e.inext = Inext;
                e.fnext = fnext;
                e.phase = phase;
                e.lane_seq = (lane << 16) | nc;
                e.offset = tsum;
                e.ri = ri;
                e.rp = rp;
                a.cand[(size_t)r * a.rcap + c] = e;
            } else {
                err |= WERR_CAND;
            }
            ++nc;
        }
        flast = fcur;
        Icur = Inext;
        fcur = fnext;
        thcur = thnext;
    }
    return tsum;
}

}  // namespace

// ---------------------------------------------------------------- W1
// RUNS runs (waves) per workgroup share one copy of the pick tables in LDS (the host picks RUNS per network
// from the runtime's occupancy, wide_w1_runs); W1_WAVES is the resident waves per SIMD the register budget is
// sized for. The LDS per workgroup ((m+1)*8 + 8 KiB tables + RUNS * 4m histograms) and the VGPRs together set
// the occupancy.
#ifndef W1_WAVES
#define W1_WAVES 1
#endif
template <uint32_t RUNS>
__global__ __launch_bounds__(64 * RUNS) __attribute__((amdgpu_waves_per_eu(W1_WAVES, 8))) void msim_wide_draws_kernel(const WideArgs a)
{
    constexpr uint32_t W1_TPB = 64 * RUNS;
    extern __shared__ uint64_t sh64[];
    __shared__ LogTab s_log;
    __shared__ uint32_t s_cc[RUNS];
    const uint32_t m = a.m, tid = threadIdx.x;
    uint64_t *s_cf = sh64;                                    // [m + 1]
    uint16_t *s_bkt = (uint16_t *)(sh64 + m + 1);             // [WB_N]
    uint32_t *s_hist = (uint32_t *)(s_bkt + WB_N);            // [RUNS][m]
    for (uint32_t i = tid; i <= m; i += W1_TPB) s_cf[i] = a.cf[i];
    for (uint32_t i = tid; i < WB_N; i += W1_TPB) s_bkt[i] = a.bucket[i];
    for (uint32_t i = tid; i < RUNS * m; i += W1_TPB) s_hist[i] = 0;
    for (uint32_t i = tid; i < sizeof(LogTab) / 8; i += W1_TPB) ((double *)&s_log)[i] = ((const double *)a.logt)[i];
    if (tid < RUNS) s_cc[tid] = 0;
    __syncthreads();

    const uint32_t w = tid >> 6, lane = tid & 63u;
    const uint32_t r = blockIdx.x * RUNS + w;  // slice-local run
    if (r >= a.n) return;                   // wave-uniform; no block barrier below
    const W1Lds s{s_cf, s_bkt, s_hist + w * m, s_cc + w};
    const uint64_t run = a.run_begin + r;
    const Rng ri0 = rng_seed(seed_interval(a.seed_base, run));
    const Rng rp0 = rng_seed(seed_picker(a.seed_base, run));
    const int64_t D = a.D;
    WideLane *lanes = a.lanes + (size_t)r * (1 + a.nch) * 64;

    uint32_t err = 0, pick_err_blk = WIDE_NONE, flast = WIDE_NONE;
    uint64_t Tph = 0;                  // T of the last block before the phase (T_{-1} = 0)
    uint32_t fprev = WIDE_NONE;        // finder of that block
    bool done = false;
    uint32_t n_end = 0, lastf = WIDE_NONE, nph_run = 0;
    uint64_t tlast = 0;

    // One phase: lane segments of nblk blocks from draw b0(lane); ri/rp positioned there.
    auto phase = [&](Rng &ri, Rng &rp, uint32_t nblk, uint32_t b0, uint32_t ph) {
        const Rng ris = ri, rps = rp;
        uint32_t nc = 0;
        flast = fprev;
        const uint64_t tsum = w1_segment(a, s, &s_log, ri, rp, nblk, b0, ph, lane, r, flast, nc, pick_err_blk, err);
        const uint64_t excl = wave_excl_scan(tsum, lane);
        const uint64_t t0 = Tph + excl, tend = t0 + tsum;
        lanes[(size_t)ph * 64 + lane] = WideLane{t0, nc, 0u};
        nph_run = ph + 1;
        const uint64_t ge = __ballot(nblk > 0 && (int64_t)tend >= D);
        if (ge) {
            // The run ends in this phase: lane L* holds the first block found at >= D.
            const uint32_t Ls = (uint32_t)__ffsll((unsigned long long)ge) - 1;
            const uint32_t fprev_lane = __shfl(flast, (int)(Ls == 0 ? 0 : Ls - 1), 64);
            uint32_t ne = WIDE_NONE, lf = WIDE_NONE;
            uint64_t tl = 0;
            if (lane > Ls) {  // every block of the segment is past the end: take them out again
                Rng p = rps;
                for (uint32_t b = 0; b < nblk; ++b) {
                    uint32_t th;
                    const uint32_t f = wide_pick(rng_next(p), s.cf, s.bucket, a.W, a.mult, th);
                    if (f < m) atomicSub(&s.hist[f], 1u);
                }
            } else if (lane == Ls) {
                Rng i2 = ris, p2 = rps;
                uint64_t T = t0;
                lf = Ls == 0 ? fprev : fprev_lane;
                tl = t0;
                for (uint32_t b = 0; b < nblk; ++b) {
                    T += (uint32_t)draw_interval(i2, &s_log);
                    uint32_t th;
                    const uint32_t f = wide_pick(rng_next(p2), s.cf, s.bucket, a.W, a.mult, th);
                    if ((int64_t)T >= D) {
                        if (ne == WIDE_NONE) ne = b0 + b;
                        if (f < m) atomicSub(&s.hist[f], 1u);
                    } else {
                        lf = f;
                        tl = T;
                    }
                }
            }
            n_end = __shfl(ne, (int)Ls, 64);
            lastf = __shfl(lf, (int)Ls, 64);
            tlast = __shfl((unsigned long long)tl, (int)Ls, 64);
            done = true;
        } else {
            Tph += __shfl((unsigned long long)(excl + tsum), 63, 64);
            fprev = __shfl(flast, 63, 64);
        }
    };

    if (a.S0 > 0) {
        Rng ri = ri0, rp = rp0;
        jump_both(reinterpret_cast<const uint4 *>(a.jmain) + (size_t)lane * 128, ri, rp);
        phase(ri, rp, a.S0, lane * a.S0, 0u);
    } else {
        lanes[lane] = WideLane{0, 0, 0};
        nph_run = 1;
    }
    if (!done) {
        Rng ri = ri0, rp = rp0;
        jump_both(reinterpret_cast<const uint4 *>(a.jtail) + (size_t)lane * 128, ri, rp);
        for (uint32_t c = 0; c < a.nch && !done; ++c) {
            const uint32_t b0 = (uint32_t)(a.B0 + (uint64_t)c * 64 * a.ST + (uint64_t)lane * a.ST);
            phase(ri, rp, a.ST, b0, 1u + c);
            if (!done && c + 1 < a.nch) jump_both(reinterpret_cast<const uint4 *>(a.jstep), ri, rp);
        }
    }
    if (!done) err |= WERR_DRAWS;
    for (uint32_t ph = nph_run; ph < 1 + a.nch; ++ph) lanes[(size_t)ph * 64 + lane] = WideLane{0, 0, 0};
    // A PickFinder fall-through only matters before the end of the run (the reference never draws later).
    uint32_t pe = pick_err_blk;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(pe, o, 64);
        pe = y < pe ? y : pe;
    }
    if (done && pe != WIDE_NONE && pe < n_end) err |= WERR_PICK;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) err |= __shfl_xor(err, o, 64);
    wave_sync();
    uint32_t *hout = a.hist + (size_t)r * m;
    for (uint32_t k = lane; k < m; k += 64) hout[k] = s.hist[k];
    {  // this run's candidate slots on the dense W2 work list (one atomic per run)
        const uint32_t cc0 = *s.cc, ccn = cc0 < a.rcap ? cc0 : a.rcap;
        uint32_t base = 0;
        if (lane == 0 && ccn) base = atomicAdd(&a.counts[0], ccn);
        base = __shfl(base, 0, 64);
        for (uint32_t c = lane; c < ccn; c += 64) a.work[base + c] = r * a.rcap + c;
    }
    if (lane == 0) {
        const uint32_t cc = *s.cc;
        uint32_t *inf = a.info + (size_t)r * 4;
        inf[0] = n_end;
        inf[1] = lastf;
        inf[2] = cc < a.rcap ? cc : a.rcap;
        inf[3] = err;
        a.tlast[r] = (int64_t)tlast;
    }
}

// ---------------------------------------------------------------- W2
// RETRY = false: every candidate with the small capacities (WE_FAST, WA_FAST); an episode that outgrows them is
// listed for RETRY = true (the record format's WE, WA).
template <bool RETRY>
__device__ __forceinline__ void wide_episode_slot(const WideArgs &a, uint32_t slot)
{
    const size_t idx = slot;
    const uint32_t r = (uint32_t)(idx / a.rcap);
    const uint32_t *inf = a.info + (size_t)r * 4;
    uint32_t *rec = a.recs + idx * WREC_WORDS;
    const WideCand e = a.cand[idx];
    if (inf[3] != 0 || e.block >= inf[0]) {  // failed run, or a block past the end of the run
        rec[0] = e.block + 1;
        rec[1] = WREC_SKIP;
        rec[2] = 0;
        return;
    }
    const WideLane ln = a.lanes[((size_t)r * (1 + a.nch) + e.phase) * 64 + (e.lane_seq >> 16)];
    const int64_t Ts = (int64_t)(ln.t0 + e.offset);
    WideSrc src{e.ri, e.rp, a.logt, a.cf, a.bucket, a.W, a.mult};
    WideEpOut o;
    constexpr int CE = RETRY ? WE : WE_FAST, CA = RETRY ? WA : WA_FAST;
    wide_episode<CE, CA>(a.prop, a.m, a.D, e.block, Ts, e.f, e.inext, e.fnext, src, o);
    if (o.flags & WREC_RETRY) {
        if (RETRY) o.flags = WREC_ERR;
        else a.retry[atomicAdd(&a.counts[1], 1u)] = slot;
    }
    rec[0] = o.end;
    rec[1] = o.flags;
    rec[2] = o.ne;
#pragma unroll
    for (uint32_t i = 0; i < (uint32_t)CA; ++i) {  // static indices: o stays in registers
        if (i >= o.ne) continue;
        rec[4 + 3 * i] = o.gid[i];
        rec[5 + 3 * i] = o.dF[i];
        rec[6 + 3 * i] = o.dS[i];
    }
}

// Grid-stride over the dense lists W1 / the first pass built (every thread of a wave has real work).
template <bool RETRY>
__global__ __launch_bounds__(256) void msim_wide_episode_kernel(const WideArgs a)
{
    const uint32_t total = RETRY ? a.counts[1] : a.counts[0];
    const uint32_t *list = RETRY ? a.retry : a.work;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256)
        wide_episode_slot<RETRY>(a, list[i]);
}

// ---------------------------------------------------------------- W3
// Phase timing (diagnostic builds only, -DW3_PROF=1: scripts/build_variant.sh): clocks at each phase of a run
// for the first wave of a few workgroups, summed over the runs the wave combines.
#if defined(W3_PROF) && W3_PROF
#define W3T(i) w3c[i] += clock64() - w3t0, w3t0 = clock64()
#define W3T_DECL uint64_t w3c[6] = {0, 0, 0, 0, 0, 0}, w3t0 = clock64(); uint32_t w3n = 0
#define W3T_PRINT                                                                                               \
    if (tid == 0 && blockIdx.x % 64 == 0)                                                                       \
        printf("W3PROF blk %u runs %u hist %llu bases %llu sort %llu chain %llu stats %llu\n", blockIdx.x, w3n,  \
               (unsigned long long)w3c[0], (unsigned long long)w3c[1], (unsigned long long)w3c[2],              \
               (unsigned long long)w3c[3], (unsigned long long)w3c[4])
#else
#define W3T(i)
#define W3T_DECL
#define W3T_PRINT
#endif
// LDS: acc[m] x {found, stale, share, rate} u64 (workgroup sums), then per wave: hist F[m], stale S[m],
// sorted candidate keys (block, slot) and their (end, flags), per-(phase, lane) bases.
__global__ __launch_bounds__(256) void msim_wide_combine_kernel(const WideArgs a, const WideOut out)
{
    extern __shared__ uint64_t sh64[];
    const uint32_t m = a.m, tid = threadIdx.x, w = tid >> 6, lane = tid & 63u;
    const uint32_t nph = 1 + a.nch;
    unsigned long long *acc = (unsigned long long *)sh64;  // [m][4]
    uint32_t *wbase = (uint32_t *)(sh64 + (size_t)4 * m);
    const size_t per_wave = (size_t)2 * m + 3 * (size_t)a.rcap + (size_t)nph * 64;
    uint32_t *F = wbase + w * per_wave, *S = F + m, *KB = S + m, *KE = KB + a.rcap, *KF = KE + a.rcap,
             *base = KF + a.rcap;
    for (uint32_t i = tid; i < 4 * m; i += 256) acc[i] = 0;
    __syncthreads();
    const int64_t D = a.D;
    W3T_DECL;
    for (uint32_t r = blockIdx.x * 4 + w; r < a.n; r += gridDim.x * 4) {  // wave-uniform loop
#if defined(W3_PROF) && W3_PROF
        ++w3n;
        w3t0 = clock64();
#endif
        const uint32_t *inf = a.info + (size_t)r * 4;
        const uint32_t n_end = inf[0], lastf = inf[1], cc = inf[2], rerr = inf[3];
        bool ok = rerr == 0;
        {  // the run's histogram, HB loads per lane in flight together (clamped, unconditional), then stored
            constexpr uint32_t HB = 8;
            const uint32_t *h = a.hist + (size_t)r * m;
            for (uint32_t k0 = lane; k0 < m; k0 += 64 * HB) {
                uint32_t v[HB];
#pragma unroll
                for (uint32_t j = 0; j < HB; ++j) v[j] = h[k0 + 64 * j < m ? k0 + 64 * j : m - 1];
#pragma unroll
                for (uint32_t j = 0; j < HB; ++j) {
                    if (k0 + 64 * j < m) {
                        F[k0 + 64 * j] = v[j];
                        S[k0 + 64 * j] = 0;
                    }
                }
            }
        }
        W3T(0);
        // sorted position of every candidate: (phase, lane) base + rank within the lane
        const WideLane *lanes = a.lanes + (size_t)r * nph * 64;
        uint32_t run_total = 0;
        constexpr uint32_t PB = 8;  // phases' counts loaded PB at a time (clamped, unconditional)
        for (uint32_t ph0 = 0; ph0 < nph; ph0 += PB) {
            uint32_t cv[PB];
#pragma unroll
            for (uint32_t j = 0; j < PB; ++j) cv[j] = lanes[(size_t)(ph0 + j < nph ? ph0 + j : nph - 1) * 64 + lane].count;
#pragma unroll
            for (uint32_t j = 0; j < PB; ++j) {
                if (ph0 + j < nph) {  // wave-uniform
                    const uint32_t ex = (uint32_t)wave_excl_scan(cv[j], lane);
                    base[(ph0 + j) * 64 + lane] = run_total + ex;
                    run_total += __shfl(ex + cv[j], 63, 64);
                }
            }
        }
        if (run_total != cc) ok = false;  // overflowed list (also flagged by W1)
        wave_sync();
        W3T(1);
        if (ok) {
            for (uint32_t c = lane; c < cc; c += 64) {
                const WideCand &e = a.cand[(size_t)r * a.rcap + c];
                const uint32_t pos = base[e.phase * 64 + (e.lane_seq >> 16)] + (e.lane_seq & 0xFFFFu);
                const uint32_t *rec = a.recs + ((size_t)r * a.rcap + c) * WREC_WORDS;
                if (pos < cc) {
                    KB[pos] = e.block;
                    KE[pos] = rec[0];
                    KF[pos] = (rec[1] << 16) | c;
                }
            }
        }
        wave_sync();
        W3T(2);
        // chain the episodes whose first block is reached quiet: 64 sorted entries at a time go into the
        // lanes' registers, a wave-uniform walk reads them with v_readlane (no LDS round trip per step) and
        // sets a 64-bit mask of the applied ones, then those lanes apply their sparse deltas (LDS atomics)
        uint32_t cursor = 0;
        bool run_ended = false, stop = !ok;
        for (uint32_t base0 = 0; base0 < cc && !stop; base0 += 64) {
            const uint32_t i = base0 + lane;
            const bool valid = i < cc;
            const uint32_t kb = valid ? KB[i] : 0xFFFFFFFFu, ke = valid ? KE[i] : 0u, kf = valid ? KF[i] : 0u;
            const uint32_t lim = (cc - base0) < 64 ? (cc - base0) : 64;
            uint64_t applied = 0;
            // Fast path (the usual case at small rho): no candidate of the batch starts inside the episode
            // before it, so every candidate before the end of the run applies, up to the first that ended the
            // run: one ballot instead of the walk below.
            const bool in = valid && kb < n_end;  // a prefix of the lanes (the keys are sorted)
            const uint32_t prev_ke = (uint32_t)__shfl_up((int)ke, 1, 64);
            const bool ovl = in && kb < (lane == 0 ? cursor : prev_ke);
            if (__ballot(ovl) == 0ull) {
                const uint64_t inm = __ballot(in);
                const uint32_t fl = kf >> 16;
                const uint64_t endm = __ballot(in && (fl & WREC_ENDED));
                const uint64_t am = endm ? inm & (((endm & (0ull - endm)) << 1) - 1ull) : inm;
                if (__ballot(in && (fl & (WREC_ERR | WREC_SKIP | WREC_RETRY))) & am) {
                    ok = false;
                    stop = true;
                } else {
                    applied = am;
                    if (am) cursor = (uint32_t)__builtin_amdgcn_readlane((int)ke, 63 - __clzll((long long)am));
                    if (endm) {
                        run_ended = true;
                        stop = true;
                    } else if (inm != __ballot(valid)) {
                        stop = true;  // a candidate at or past the end of the run
                    }
                }
            } else {
                for (uint32_t j = 0; j < lim; ++j) {
                    const uint32_t sblk = (uint32_t)__builtin_amdgcn_readlane((int)kb, (int)j);
                    if (sblk >= n_end) {
                        stop = true;
                        break;
                    }
                    if (sblk < cursor) continue;
                    const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)kf, (int)j) >> 16;
                    if (fl & (WREC_ERR | WREC_SKIP | WREC_RETRY)) {
                        ok = false;
                        stop = true;
                        break;
                    }
                    applied |= 1ull << j;
                    cursor = (uint32_t)__builtin_amdgcn_readlane((int)ke, (int)j);
                    if (fl & WREC_ENDED) {
                        run_ended = true;
                        stop = true;
                        break;
                    }
                }
            }
            if (ok && ((applied >> lane) & 1ull)) {
                // the record's first entries are loaded with its count, not after it
                const uint32_t *rec = a.recs + ((size_t)r * a.rcap + (kf & 0xFFFFu)) * WREC_WORDS;
                constexpr uint32_t PRE = 4;
                uint32_t pre[3 * PRE];
#pragma unroll
                for (uint32_t q = 0; q < 3 * PRE; ++q) pre[q] = rec[4 + q];
                const uint32_t ne = rec[2];
#pragma unroll
                for (uint32_t q = 0; q < PRE; ++q) {
                    if (q < ne) {
                        atomicAdd(&F[pre[3 * q]], pre[3 * q + 1]);
                        atomicAdd(&S[pre[3 * q]], pre[3 * q + 2]);
                    }
                }
                for (uint32_t q = PRE; q < ne; ++q) {
                    const uint32_t g = rec[4 + 3 * q];
                    atomicAdd(&F[g], rec[5 + 3 * q]);
                    atomicAdd(&S[g], rec[6 + 3 * q]);
                }
            }
        }
        wave_sync();
        // the run ended quiet and its last block was fast: it counts only if it arrived by D (main.cpp:185)
        if (ok && lane == 0 && !run_ended && n_end > 0 && cursor < n_end && lastf < m) {
            if (a.tlast[r] + a.prop[lastf] > D) F[lastf] -= 1u;
        }
        wave_sync();
        W3T(3);
        if (!ok) {
            if (lane == 0) atomicAdd(out.fail, 1u);
            continue;
        }
        uint32_t Lp = 0;
        for (uint32_t k = lane; k < m; k += 64) Lp += F[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) Lp += __shfl_xor(Lp, o, 64);
        const double Ld = (double)Lp;  // |best chain| - 1 (main.cpp:28)
        const uint32_t rel = out.rel_begin + r;
        for (uint32_t k = lane; k < m; k += 64) {
            const uint32_t f = F[k], st = S[k];
            if (out.records) {
                out.records[2 * ((size_t)rel * m + k) + 0] = f;
                out.records[2 * ((size_t)rel * m + k) + 1] = st;
            }
            if (f == 0 && st == 0) continue;
            // MinerStats (main.cpp:28-29) as Q32.32 fixed point
            const double share = f == 0 ? 0.0 : (double)f / Ld;
            const double rate = f == 0 ? 0.0 : (double)st / (double)f;
            const uint64_t sfx = (uint64_t)(share * 4294967296.0 + 0.5);
            const uint64_t rfx = (uint64_t)(rate * 4294967296.0 + 0.5);
            atomicAdd(&acc[4 * k + 0], (unsigned long long)f);
            atomicAdd(&acc[4 * k + 1], (unsigned long long)st);
            atomicAdd(&acc[4 * k + 2], (unsigned long long)sfx);
            atomicAdd(&acc[4 * k + 3], (unsigned long long)rfx);
        }
        if (out.best_h && lane == 0) out.best_h[rel] = Lp;
        W3T(4);
    }
    W3T_PRINT;
    __syncthreads();
    // flush: msim_sums {found, stale, share_hi, share_lo, rate_hi, rate_lo}; the workgroup's Q32.32 sums
    // are split into 2^32 and 2^0 limbs (the represented value sum(hi) + sum(lo) * 2^-32 is exact).
    for (uint32_t k = tid; k < m; k += 256) {
        const unsigned long long *x = acc + 4 * k;
        unsigned long long *o = (unsigned long long *)out.sums + 6 * k;
        if (x[0]) atomicAdd(o + 0, x[0]);
        if (x[1]) atomicAdd(o + 1, x[1]);
        if (x[2]) {
            atomicAdd(o + 2, x[2] >> 32);
            atomicAdd(o + 3, x[2] & 0xFFFFFFFFull);
        }
        if (x[3]) {
            atomicAdd(o + 4, x[3] >> 32);
            atomicAdd(o + 5, x[3] & 0xFFFFFFFFull);
        }
    }
}

// ---------------------------------------------------------------- weighted pick (test surface)
__global__ void msim_wide_pick_kernel(const uint64_t *__restrict__ cf, const uint16_t *__restrict__ bucket, uint32_t m,
                                      uint32_t W, uint64_t mult, const uint64_t *__restrict__ u, int32_t *__restrict__ out,
                                      uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t th;
    const uint32_t k = wide_pick(u[i], cf, bucket, W, mult, th);
    out[i] = k >= m ? -1 : (int32_t)k;
}

// ---------------------------------------------------------------- host side
size_t wide_w1_lds(uint32_t m, uint32_t runs) { return ((size_t)m + 1) * 8 + (size_t)WB_N * 2 + runs * (size_t)m * 4; }
// Runs per W1 workgroup: the most resident waves per CU (the runtime's occupancy of each instance at its
// LDS, which counts its VGPRs too; ties: fewer runs per workgroup). Measured on configs[4]
// (profiles/r04/w1ab): 4 and 8 runs 9.17 ms, 2 runs 11.2 ms per W1 launch; W1 is issue-bound, so the
// occupancy beyond 4 waves per SIMD gains nothing (a 16-bit packed histogram that allowed 5 was slower).
template <uint32_t R>
static size_t w1_waves_per_cu(uint32_t m)
{
    int blocks = 0;
    const size_t lds = wide_w1_lds(m, R);
    if (lds > 150 * 1024 ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, msim_wide_draws_kernel<R>, 64 * R, lds) != hipSuccess)
        return 0;
    return (size_t)blocks * R;
}
// Depends only on (device, m): cached, since launch_wide asks on every launch (four occupancy queries).
static uint32_t wide_w1_runs_uncached(uint32_t m)
{
    const size_t w[4] = {w1_waves_per_cu<1>(m), w1_waves_per_cu<2>(m), w1_waves_per_cu<4>(m), w1_waves_per_cu<8>(m)};
    uint32_t best = 1;
    size_t bw = 0;
    for (int i = 0; i < 4; ++i)
        if (w[i] > bw) {
            bw = w[i];
            best = 1u << i;
        }
    if (const char *e = getenv("MSIM_W1_RUNS")) {  // A/B override: 1, 2, 4 or 8 runs, when its LDS fits
        const uint32_t r = (uint32_t)atoi(e);
        if ((r == 1 || r == 2 || r == 4 || r == 8) && wide_w1_lds(m, r) <= 150 * 1024) best = r;
    }
    return best;
}
uint32_t wide_w1_runs(uint32_t m)
{
    static std::mutex mu;
    static std::map<std::pair<int, uint32_t>, uint32_t> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    const auto key = std::make_pair(dev, m);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    const uint32_t r = wide_w1_runs_uncached(m);
    cache[key] = r;
    return r;
}
size_t wide_w3_lds(uint32_t m, uint32_t rcap, uint32_t nch)
{
    return (size_t)4 * m * 8 + 4 * ((size_t)2 * m + 3 * (size_t)rcap + (size_t)(1 + nch) * 64) * 4;
}

hipError_t launch_wide(const WideArgs &proto, const WideLayout &L, char *ws, const WideOut &out, hipStream_t s,
                       std::vector<hipEvent_t> *w1_events)
{
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)msim_wide_draws_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        (void)hipFuncSetAttribute((const void *)msim_wide_draws_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        (void)hipFuncSetAttribute((const void *)msim_wide_draws_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        (void)hipFuncSetAttribute((const void *)msim_wide_draws_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        (void)hipFuncSetAttribute((const void *)msim_wide_combine_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_done = true;
    }
    WideArgs a = proto;
    a.hist = (uint32_t *)(ws + L.hist_off);
    a.info = (uint32_t *)(ws + L.info_off);
    a.tlast = (int64_t *)(ws + L.tlast_off);
    a.lanes = (WideLane *)(ws + L.lanes_off);
    a.cand = (WideCand *)(ws + L.cand_off);
    a.recs = (uint32_t *)(ws + L.recs_off);
    a.work = (uint32_t *)(ws + L.work_off);
    a.retry = (uint32_t *)(ws + L.retry_off);
    a.counts = (uint32_t *)(ws + L.counts_off);
    const uint32_t runs = wide_w1_runs(a.m);
    const size_t l1 = wide_w1_lds(a.m, runs), l3 = wide_w3_lds(a.m, a.rcap, a.nch);
    if (l1 > 150 * 1024) return hipErrorInvalidValue;  // WIDE_MAX_M at one run per workgroup: 49 KiB
    if (l3 > 160 * 1024) return hipErrorInvalidValue;
    for (uint64_t off = 0; off < out.n_total; off += L.nr) {
        const uint32_t cn = (uint32_t)((out.n_total - off) < L.nr ? (out.n_total - off) : L.nr);
        a.run_begin = out.run_begin + off;
        a.n = cn;
        hipEvent_t eb = nullptr, ee = nullptr;
        if (w1_events && hipEventCreate(&eb) == hipSuccess && hipEventCreate(&ee) == hipSuccess) {
            w1_events->push_back(eb);
            w1_events->push_back(ee);
            (void)hipEventRecord(eb, s);
        }
        if (hipMemsetAsync(a.counts, 0, 2 * sizeof(uint32_t), s) != hipSuccess) return hipErrorUnknown;
        const dim3 g1((cn + runs - 1) / runs), b1(64 * runs);
        switch (runs) {
        case 1: hipLaunchKernelGGL((msim_wide_draws_kernel<1>), g1, b1, l1, s, a); break;
        case 2: hipLaunchKernelGGL((msim_wide_draws_kernel<2>), g1, b1, l1, s, a); break;
        case 4: hipLaunchKernelGGL((msim_wide_draws_kernel<4>), g1, b1, l1, s, a); break;
        default: hipLaunchKernelGGL((msim_wide_draws_kernel<8>), g1, b1, l1, s, a); break;
        }
        if (ee) (void)hipEventRecord(ee, s);
        // W2 grid: ~rho * blocks candidates per run, grid-stride beyond 16 384 workgroups
        const double est = (double)cn * a.rcap * 0.6;
        const unsigned g2 = (unsigned)(est / 256 < 16384 ? est / 256 + 1 : 16384);
        hipLaunchKernelGGL(msim_wide_episode_kernel<false>, dim3(g2), dim3(256), 0, s, a);
        hipLaunchKernelGGL(msim_wide_episode_kernel<true>, dim3(64), dim3(256), 0, s, a);
        WideOut o = out;
        o.rel_begin = (uint32_t)off;
        uint32_t g3 = (cn + 3) / 4;
        if (g3 > 4096) g3 = 4096;
        hipLaunchKernelGGL(msim_wide_combine_kernel, dim3(g3), dim3(256), l3, s, a, o);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t launch_wide_picks(const WideArgs &a, const uint64_t *u, int32_t *out, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(msim_wide_pick_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a.cf, a.bucket, a.m,
                       a.W, a.mult, u, out, n);
    return hipGetLastError();
}

}  // namespace msim

// ---------------------------------------------------------------- samplers (test.cpp)
// One RNG stream of n draws (test.cpp's MinerPickerSample / BlockIntervalSample loops) split into
// segments of S draws, one per thread: thread j jumps to draw j*S with the wave-uniform matrices
// T^(S*2^b) applied where bit b of j is set, then draws its segment sequentially — the same draws the
// reference's single loop makes, so the integer results are identical to it for any n.
namespace msim {
namespace {

__device__ __forceinline__ void jump_masked(const uint4 *__restrict__ cols, Rng &a, bool apply)
{
    const uint32_t sa[4] = {(uint32_t)a.s0, (uint32_t)(a.s0 >> 32), (uint32_t)a.s1, (uint32_t)(a.s1 >> 32)};
    uint32_t o0 = 0, o1 = 0, o2 = 0, o3 = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
#pragma unroll 8
        for (int i = 0; i < 32; ++i) {
            const uint4 c = cols[w * 32 + i];
            const uint32_t mk = 0u - ((sa[w] >> i) & 1u);
            o0 ^= c.x & mk;
            o1 ^= c.y & mk;
            o2 ^= c.z & mk;
            o3 ^= c.w & mk;
        }
    }
    if (apply) {
        a.s0 = (uint64_t)o0 | ((uint64_t)o1 << 32);
        a.s1 = (uint64_t)o2 | ((uint64_t)o3 << 32);
    }
}

}  // namespace

// MODE 0: pick counts ([m + 1] bins, bin m = fell through); MODE 1: interval moments
// (out[0] = sum, out[1] = sum of squares lo, out[2] = hi, out[3] = max).
template <int MODE>
__global__ __launch_bounds__(256) void msim_sample_kernel(const uint32_t *__restrict__ pow2_jumps, uint64_t seed,
                                                           uint64_t n, uint32_t S, const uint64_t *__restrict__ cf,
                                                           const uint16_t *__restrict__ bucket, uint32_t m, uint32_t W,
                                                           uint64_t mult, const LogTab *__restrict__ logt,
                                                           unsigned long long *__restrict__ out)
{
    extern __shared__ uint32_t s_hist[];  // MODE 0: [m + 1]
    __shared__ LogTab s_log;
    const uint32_t tid = threadIdx.x;
    if (MODE == 0)
        for (uint32_t i = tid; i <= m; i += 256) s_hist[i] = 0;
    for (uint32_t i = tid; i < sizeof(LogTab) / 8; i += 256) ((double *)&s_log)[i] = ((const double *)logt)[i];
    __syncthreads();
    const uint64_t j = (uint64_t)blockIdx.x * 256 + tid;
    const uint64_t b0 = j * S;
    const uint32_t cnt = b0 < n ? (uint32_t)((n - b0) < S ? (n - b0) : S) : 0u;
    Rng r = rng_seed(seed);
    for (int b = 0; b < 32 && ((uint64_t)gridDim.x * 256 >> b) > 0; ++b) {
        const bool bit = (j >> b) & 1u;
        if (__ballot(bit)) jump_masked(reinterpret_cast<const uint4 *>(pow2_jumps) + (size_t)b * 128, r, bit);
    }
    uint64_t sum = 0, sq = 0, mx = 0;
    for (uint32_t i = 0; i < cnt; ++i) {
        if (MODE == 0) {
            uint32_t th;
            const uint32_t k = wide_pick(rng_next(r), cf, bucket, W, mult, th);
            atomicAdd(&s_hist[k < m ? k : m], 1u);
        } else {
            const uint64_t x = (uint64_t)draw_interval(r, &s_log);
            sum += x;
            sq += x * x;
            mx = x > mx ? x : mx;
        }
    }
    if (MODE == 0) {
        __syncthreads();
        for (uint32_t i = tid; i <= m; i += 256)
            if (s_hist[i]) atomicAdd(&out[i], (unsigned long long)s_hist[i]);
    } else if (cnt) {
        atomicAdd(&out[0], (unsigned long long)sum);
        const unsigned long long old = atomicAdd(&out[1], (unsigned long long)sq);
        if (old + sq < old) atomicAdd(&out[2], 1ull);  // carry into the high word
        atomicMax(&out[3], (unsigned long long)mx);
    }
}

// pow2_jumps: 32 matrices T^(S * 2^b) (msim_jump.h layout) in device memory.
hipError_t launch_sample(int mode, const uint32_t *pow2_jumps, uint64_t seed, uint64_t n, uint32_t S, const uint64_t *cf,
                         const uint16_t *bucket, uint32_t m, uint32_t W, uint64_t mult, const LogTab *logt,
                         unsigned long long *out, hipStream_t s)
{
    const uint64_t threads = (n + S - 1) / S;
    const uint32_t grid = (uint32_t)((threads + 255) / 256);
    if (grid == 0) return hipSuccess;
    if (mode == 0)
        hipLaunchKernelGGL(msim_sample_kernel<0>, dim3(grid), dim3(256), (m + 1) * 4, s, pow2_jumps, seed, n, S, cf, bucket,
                           m, W, mult, logt, out);
    else
        hipLaunchKernelGGL(msim_sample_kernel<1>, dim3(grid), dim3(256), 0, s, pow2_jumps, seed, n, S, cf, bucket, m, W,
                           mult, logt, out);
    return hipGetLastError();
}

}  // namespace msim
