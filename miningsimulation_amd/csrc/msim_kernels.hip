// msim_kernels.hip — gfx950 kernels: one simulation run per lane, deterministic integer reductions.
//
//   msim_runs_kernel   replaces the per-run std::async tasks of main() (main.cpp:205-210): lane r
//                      executes RunSimulation (main.cpp:128-192) for run r with the compact state of
//                      msim_model.h held in VGPRs, then contributes its MinerStats to the workgroup's
//                      fixed-point partial sums (main.cpp:211-217, made order-independent).
//   msim_finalize      sums the workgroup partials in a fixed order into msim_sums.
//
// Roofline: VALU issue (no MFMA: nothing is a dense contraction; no HBM stream: each lane reads its
// parameters once and writes ~6*M words per 256 runs). See DESIGN.md §4.
#include <hip/hip_runtime.h>

#include "msim_kernels.h"
#include "msim_reduce.h"
#include "msim_pipeline.h"

namespace msim {

template <int M, bool SELF, bool DEEP, int NX, int NG, bool LIST>
__global__ __launch_bounds__(TPB, 2) void msim_runs_kernel(const SimParams p, const uint64_t run_begin, const uint32_t n,
                                                         const uint32_t seed_base, const uint32_t *__restrict__ list,
                                                         const uint32_t *__restrict__ list_count, const uint32_t list_cap,
                                                         uint64_t *__restrict__ partials, uint32_t *__restrict__ records,
                                                         uint32_t *__restrict__ best_h, uint32_t *__restrict__ err_count,
                                                         uint32_t *__restrict__ err_list, const uint32_t err_cap)
{
    const uint32_t idx = blockIdx.x * TPB + threadIdx.x;
    uint32_t lim = n;
    if (LIST) {
        const uint32_t c = *list_count;
        lim = c < list_cap ? c : list_cap;
    }
    if (LIST && blockIdx.x * TPB >= lim) {  // a retry workgroup with no flagged run (the usual case): zero sums
        for (uint32_t i = threadIdx.x; i < 6 * M; i += TPB) partials[(size_t)blockIdx.x * 6 * M + i] = 0ull;
        return;
    }
    const bool active = idx < lim;
    const uint32_t rel = LIST ? (active ? list[idx] : 0u) : idx;  // run offset from run_begin
    uint64_t v[6 * M];
#pragma unroll
    for (int i = 0; i < 6 * M; ++i) v[i] = 0;
    if (active) {
        const uint64_t run = run_begin + rel;
        RunResult r;
        Sim<M, SELF, DEEP, NX, NG> s;
        s.run(p, rng_seed(seed_interval(seed_base, run)), rng_seed(seed_picker(seed_base, run)), r);
        if (r.err) {
            const uint32_t pos = atomicAdd(err_count, 1u);
            if (!LIST && pos < err_cap) err_list[pos] = rel;
        } else {
            const double L = (double)r.best_height;
#pragma unroll
            for (int k = 0; k < M; ++k) {
                const uint32_t f = r.found[k];
                // MinerStats (main.cpp:28-29)
                const double share = f == 0 ? 0.0 : (double)f / L;
                const double rate = f == 0 ? 0.0 : (double)r.stale[k] / (double)f;
                const uint64_t sfx = (uint64_t)(share * 4294967296.0 + 0.5);
                const uint64_t rfx = (uint64_t)(rate * 4294967296.0 + 0.5);
                v[6 * k + 0] = f;
                v[6 * k + 1] = r.stale[k];
                v[6 * k + 2] = sfx >> 32;
                v[6 * k + 3] = sfx & 0xFFFFFFFFull;
                v[6 * k + 4] = rfx >> 32;
                v[6 * k + 5] = rfx & 0xFFFFFFFFull;
                if (records) {
                    records[2 * ((size_t)rel * M + k) + 0] = f;
                    records[2 * ((size_t)rel * M + k) + 1] = r.stale[k];
                }
            }
            if (best_h) best_h[rel] = r.best_height;
        }
    }
    block_reduce_store<M>(v, partials + (size_t)blockIdx.x * 6 * M);
}

// MinerStats of one finished run (main.cpp:22-30) as the 6*M fixed-point sum terms (msim_sums layout).
template <int M>
__device__ __forceinline__ void stats_terms(const RunResult &r, uint64_t (&v)[6 * M])
{
    const double L = (double)r.best_height;
#pragma unroll
    for (int k = 0; k < M; ++k) {
        const uint32_t f = r.found[k];
        const double share = f == 0 ? 0.0 : (double)f / L;
        const double rate = f == 0 ? 0.0 : (double)r.stale[k] / (double)f;
        const uint64_t sfx = (uint64_t)(share * 4294967296.0 + 0.5);
        const uint64_t rfx = (uint64_t)(rate * 4294967296.0 + 0.5);
        v[6 * k + 0] = f;
        v[6 * k + 1] = r.stale[k];
        v[6 * k + 2] = sfx >> 32;
        v[6 * k + 3] = sfx & 0xFFFFFFFFull;
        v[6 * k + 4] = rfx >> 32;
        v[6 * k + 5] = rfx & 0xFFFFFFFFull;
    }
}

// ------------------------------------------------------------------ parameter sweep (configs[3])
// One lane per (point, run). Workgroups never straddle points, so a wave's parameter block is
// uniform (scalar loads from pts[point]) and its partial sums belong to one point. LIST: the retry
// pass over flagged lanes (codes point * wpp * TPB + rel), wide capacities, atomic per-point sums.
template <int M, bool SELF, bool DEEP, int NX, int NG, bool LIST>
__global__ __launch_bounds__(TPB, 2) void msim_sweep_kernel(const SimParams *__restrict__ pts, const uint64_t run_begin,
                                                          const uint32_t rpp, const uint32_t wpp, const uint32_t seed_base,
                                                          const uint32_t *__restrict__ list, const uint32_t *__restrict__ list_count,
                                                          const uint32_t list_cap, uint64_t *__restrict__ partials,
                                                          uint64_t *__restrict__ retry_sums, uint32_t *__restrict__ records,
                                                          uint32_t *__restrict__ best_h, uint32_t *__restrict__ err_count,
                                                          uint32_t *__restrict__ err_list, const uint32_t err_cap)
{
    uint32_t point, rel;
    bool active;
    if (LIST) {
        const uint32_t c = *list_count, lim = c < list_cap ? c : list_cap;
        const uint32_t idx = blockIdx.x * TPB + threadIdx.x;
        active = idx < lim;
        const uint32_t code = active ? list[idx] : 0u;
        point = code / (wpp * TPB);
        rel = code % (wpp * TPB);
    } else {
        point = blockIdx.x / wpp;
        rel = (blockIdx.x % wpp) * TPB + threadIdx.x;
        active = rel < rpp;
    }
    const SimParams &p = pts[point];
    uint64_t v[6 * M];
#pragma unroll
    for (int i = 0; i < 6 * M; ++i) v[i] = 0;
    if (active) {
        const uint64_t run = run_begin + rel;
        RunResult r;
        Sim<M, SELF, DEEP, NX, NG> s;
        s.run(p, rng_seed(seed_interval(seed_base, run)), rng_seed(seed_picker(seed_base, run)), r);
        if (r.err) {
            const uint32_t pos = atomicAdd(err_count, 1u);
            if (!LIST && pos < err_cap) err_list[pos] = point * wpp * TPB + rel;
        } else {
            stats_terms<M>(r, v);
            const size_t g = (size_t)point * rpp + rel;
            if (records)
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    records[2 * (g * M + k) + 0] = r.found[k];
                    records[2 * (g * M + k) + 1] = r.stale[k];
                }
            if (best_h) best_h[g] = r.best_height;
            if (LIST)
#pragma unroll
                for (int i = 0; i < 6 * M; ++i)
                    if (v[i]) atomicAdd((unsigned long long *)(retry_sums + (size_t)point * 6 * M + i), (unsigned long long)v[i]);
        }
    }
    if (!LIST) block_reduce_store<M>(v, partials + (size_t)blockIdx.x * 6 * M);
}

// ------------------------------------------------------------------ event-skipping pipeline (K2, K3)
// K2 / K3 redraw blocks (msim_pipeline.h draw_word); the exact interval is out of line, as in K1.
__device__ __noinline__ int32_t interval_ms_exact_dev(uint64_t u) { return (int32_t)interval_ms_of(u); }

// K2: one lane per listed non-fast block (msim_pipeline.h episode_entry).
// The lean state machine at three resident waves per SIMD (168 VGPRs; k2_waves below); four waves (128 VGPRs)
// spill and run slower (136.6 vs 79.6 us, profiles/r04/k2v2).
#ifndef MSIM_K2_WAVES
#define MSIM_K2_WAVES 3
#endif
// Workgroup sizes of K2 and K3. K3 has one lane per run, so a 256-lane workgroup put the 32 768 runs of a c2
// slice on 128 workgroups, half the CUs; one-wave workgroups spread them over all 256.
#ifndef MSIM_K2_TPB
#define MSIM_K2_TPB 64  // one-wave workgroups: a finished wave's slot takes new work at once (K2 79.6 -> 76.7 us)
#endif
#ifndef MSIM_K3_TPB
#define MSIM_K3_TPB 64
#endif
constexpr int K2_TPB = MSIM_K2_TPB, K3_TPB = MSIM_K3_TPB;
static_assert(K3_TPB % 64 == 0 && K3_TPB <= TPB && TPB % K3_TPB == 0, "K3 workgroups: whole waves, dividing TPB");
// Resident K2 waves per SIMD by (miner count, kind). The lean machine takes three waves (168 VGPRs) up to 9 miners:
// at 9 it spills 5 VGPRs there and is still faster than at two waves without spills (78.0 vs 86.3 us per c2
// launch, profiles/r05/k2waves); from 10 miners it spills 21-554 at three waves and takes two (one at 15). The mid
// machine needs 259 VGPRs from 14 miners and takes one wave there. Every other instantiation has no VGPR spills.
constexpr int k2_waves(int m, int kind) { return kind == 0 ? (m <= 9 ? MSIM_K2_WAVES : m <= 14 ? 2 : 1) : (m <= 13 ? 2 : 1); }
// The mid and full state machines at two waves per SIMD (256 VGPRs): at three (168) the mid one spilled 31
// VGPRs, the full one 132; a rho > 0.002 network lists ~10x the lean one's blocks, so K2 still fills the chip.
template <int M, int KIND>
__global__ __launch_bounds__(K2_TPB) __attribute__((amdgpu_waves_per_eu(k2_waves(M, KIND), 8))) void msim_episode_kernel(const SimParams p,
                                                                                                    const PipeArgs a)
{
    // the draw tables in LDS: an episode's draws read them in its dependent chain (global: ~600-900 cycles
    // per read, LDS: ~50)
    __shared__ LogTab s_log;
    __shared__ PickTab s_pick;
    for (uint32_t i = threadIdx.x; i < sizeof(LogTab) / 8; i += K2_TPB) ((double *)&s_log)[i] = ((const double *)a.tab.logt)[i];
    for (uint32_t i = threadIdx.x; i < sizeof(PickTab) / 4; i += K2_TPB) ((uint32_t *)&s_pick)[i] = ((const uint32_t *)a.tab.pick)[i];
    __syncthreads();
    PipeArgs la = a;
    la.tab.logt = &s_log;
    la.tab.pick = &s_pick;
    const uint32_t cnt = *a.list_count;
    const uint32_t lim = cnt < a.lcap ? cnt : a.lcap;
    for (uint32_t idx = blockIdx.x * K2_TPB + threadIdx.x; idx < lim; idx += gridDim.x * K2_TPB) episode_entry<M, KIND>(p, la, idx);
}

// K3: one lane per run (msim_pipeline.h combine_run), then the MinerStats reduction.
template <int M>
__global__ __launch_bounds__(K3_TPB) void msim_combine_kernel(const SimParams p, const PipeArgs a, const uint32_t n,
                                                          const uint32_t rel_begin, uint64_t *__restrict__ partials,
                                                          uint32_t *__restrict__ records, uint32_t *__restrict__ best_h,
                                                          uint32_t *__restrict__ err_count, uint32_t *__restrict__ err_list,
                                                          const uint32_t err_cap)
{
    __shared__ uint32_t s_ns[K3_SCRATCH][K3_TPB];  // per-lane scratch of combine_run (segment counts, episodes)
    __shared__ LogTab s_log;                       // the draw tables for the end group's redraw (as K2)
    __shared__ PickTab s_pick;
    for (uint32_t i = threadIdx.x; i < sizeof(LogTab) / 8; i += K3_TPB) ((double *)&s_log)[i] = ((const double *)a.tab.logt)[i];
    for (uint32_t i = threadIdx.x; i < sizeof(PickTab) / 4; i += K3_TPB) ((uint32_t *)&s_pick)[i] = ((const uint32_t *)a.tab.pick)[i];
    __syncthreads();
    PipeArgs la = a;
    la.tab.logt = &s_log;
    la.tab.pick = &s_pick;
    const uint32_t r = blockIdx.x * K3_TPB + threadIdx.x;
    const bool active = r < n;
    uint32_t F[M], S[M];
    const bool ok = active ? combine_run<M>(p, la, r, F, S, &s_ns[0][threadIdx.x], K3_TPB) : false;
    uint64_t v[6 * M];
#pragma unroll
    for (int i = 0; i < 6 * M; ++i) v[i] = 0;
    if (active && !ok) {
        const uint32_t pos = atomicAdd(err_count, 1u);
        if (pos < err_cap) err_list[pos] = rel_begin + r;
    } else if (active) {
        uint32_t L = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) L += F[k];  // sum of found = |best chain| - 1
        const uint32_t rel = rel_begin + r;
        const double Ld = (double)L;
#pragma unroll
        for (int k = 0; k < M; ++k) {
            const uint32_t f = F[k];
            // MinerStats (main.cpp:28-29)
            const double share = f == 0 ? 0.0 : (double)f / Ld;
            const double rate = f == 0 ? 0.0 : (double)S[k] / (double)f;
            const uint64_t sfx = (uint64_t)(share * 4294967296.0 + 0.5);
            const uint64_t rfx = (uint64_t)(rate * 4294967296.0 + 0.5);
            v[6 * k + 0] = f;
            v[6 * k + 1] = S[k];
            v[6 * k + 2] = sfx >> 32;
            v[6 * k + 3] = sfx & 0xFFFFFFFFull;
            v[6 * k + 4] = rfx >> 32;
            v[6 * k + 5] = rfx & 0xFFFFFFFFull;
            if (records) {
                records[2 * ((size_t)rel * M + k) + 0] = f;
                records[2 * ((size_t)rel * M + k) + 1] = S[k];
            }
        }
        if (best_h) best_h[rel] = L;
    }
    block_reduce_store<M, K3_TPB>(v, partials + (size_t)blockIdx.x * 6 * M);
}

// ------------------------------------------------------------------ host-side launch table
template <int M>
static void launch_retry(const LaunchArgs &a, uint64_t *parts_retry, uint32_t nbr)
{
    if (a.p.selfish >= 0)
        hipLaunchKernelGGL((msim_runs_kernel<M, true, true, NX_WIDE, NG_WIDE, true>), dim3(nbr), dim3(TPB), 0, a.stream,
                           a.p, a.run_begin, a.n, a.seed_base, a.err_list, a.err_count, a.err_cap, parts_retry, a.records,
                           a.best_h, a.fail_count, nullptr, 0u);
    else
        hipLaunchKernelGGL((msim_runs_kernel<M, false, true, NX_WIDE, NG_WIDE, true>), dim3(nbr), dim3(TPB), 0, a.stream,
                           a.p, a.run_begin, a.n, a.seed_base, a.err_list, a.err_count, a.err_cap, parts_retry, a.records,
                           a.best_h, a.fail_count, nullptr, 0u);
}

// Event-skipping pipeline (msim_pipeline.h), slice by slice on the caller's stream.
template <int M>
static hipError_t launch_pipeline(const LaunchArgs &a, uint64_t *parts)
{
    const PipeLayout &L = *a.pl;
    char *ws = a.pipe_ws;
    PipeArgs pa;
    pa.nr = L.nr;
    pa.seg = L.seg;
    pa.gps = L.gps;
    pa.nseg = L.nseg;
    pa.nb = L.nb;
    pa.cap = L.cap;
    pa.band_lo = L.band_lo;
    pa.lcap = L.lcap;
    pa.rec_words = L.rec_words;
    pa.tab = a.tab;
    pa.segsum = (const uint64_t *)(ws + L.segsum_off);
    pa.segcnt = (const uint32_t *)(ws + L.segcnt_off);
    pa.nslow = (const uint32_t *)(ws + L.nslow_off);
    pa.slots = (const uint32_t *)(ws + L.slots_off);
    pa.gsum = (const uint32_t *)(ws + L.gsum_off);
    pa.gend = (const uint64_t *)(ws + L.gend_off);
    pa.gcum = (const uint32_t *)(ws + L.gcum_off);
    pa.grec = (const GroupRec *)(ws + L.grec_off);
    pa.list = (const EpEntry *)(ws + L.list_off);
    pa.list_count = (const uint32_t *)(ws + L.count_off);
    pa.recs = (uint32_t *)(ws + L.recs_off);
    DrawArgs da;
    da.tab = a.tab;
    da.seed_base = a.seed_base;
    da.nr = L.nr;
    da.seg = L.seg;
    da.gps = L.gps;
    da.nseg = L.nseg;
    da.cap = L.cap;
    da.band_lo = L.band_lo;
    da.lcap = L.lcap;
    da.lchunk = L.lchunk;
    da.segsum = (uint64_t *)(ws + L.segsum_off);
    da.segcnt = (uint32_t *)(ws + L.segcnt_off);
    da.nslow = (uint32_t *)(ws + L.nslow_off);
    da.slots = (uint32_t *)(ws + L.slots_off);
    da.gsum = (uint32_t *)(ws + L.gsum_off);
    da.gend = (uint64_t *)(ws + L.gend_off);
    da.gcum = (uint32_t *)(ws + L.gcum_off);
    da.grec = (GroupRec *)(ws + L.grec_off);
    da.list = (EpEntry *)(ws + L.list_off);
    da.list_count = (uint32_t *)(ws + L.count_off);
    uint32_t ep_grid = (L.lcap + K2_TPB - 1) / K2_TPB;
    if (ep_grid > 8192u * (TPB / K2_TPB)) ep_grid = 8192u * (TPB / K2_TPB);
    if (ep_grid == 0) ep_grid = 1;
    for (uint32_t off = 0; off < a.n; off += L.nr) {
        const uint32_t cn = (a.n - off) < L.nr ? (a.n - off) : L.nr;
        if (hipMemsetAsync(da.list_count, 0, sizeof(uint32_t), a.stream) != hipSuccess) return hipErrorUnknown;
        da.run_begin = a.run_begin + off;
        da.n = cn;
        hipEvent_t eb = nullptr, ee = nullptr;
        if (a.k1_events && hipEventCreate(&eb) == hipSuccess && hipEventCreate(&ee) == hipSuccess) {
            a.k1_events->push_back(eb);
            a.k1_events->push_back(ee);
            (void)hipEventRecord(eb, a.stream);
        }
        hipError_t e = launch_draws(da, a.stream);
        if (ee) (void)hipEventRecord(ee, a.stream);
        if (e != hipSuccess) return e;
        if (L.k2_kind == 0) hipLaunchKernelGGL((msim_episode_kernel<M, 0>), dim3(ep_grid), dim3(K2_TPB), 0, a.stream, a.p, pa);
        else if (L.k2_kind == 1) hipLaunchKernelGGL((msim_episode_kernel<M, 1>), dim3(ep_grid), dim3(K2_TPB), 0, a.stream, a.p, pa);
        else hipLaunchKernelGGL((msim_episode_kernel<M, 2>), dim3(ep_grid), dim3(K2_TPB), 0, a.stream, a.p, pa);
        hipLaunchKernelGGL((msim_combine_kernel<M>), dim3((cn + K3_TPB - 1) / K3_TPB), dim3(K3_TPB), 0, a.stream, a.p, pa,
                           cn, off, parts + (size_t)(off / K3_TPB) * 6 * M, a.records, a.best_h, a.err_count, a.err_list,
                           a.err_cap);
    }
    return hipGetLastError();
}

template <int M>
static hipError_t launch_m(const LaunchArgs &a)
{
    const uint32_t nb = (a.n + TPB - 1) / TPB;
    const uint32_t nbr = (a.err_cap + TPB - 1) / TPB;
    const uint32_t nrow = a.pl ? (a.n + K3_TPB - 1) / K3_TPB : nb;  // partial rows: one per workgroup
    const bool self = a.p.selfish >= 0;
    uint64_t *parts = a.partials;
    uint64_t *parts_retry = a.partials + (size_t)nrow * 6 * M;
    if (a.pl) {
        const hipError_t e = launch_pipeline<M>(a, parts);
        if (e != hipSuccess) return e;
    } else if (nb) {
        if (self)
            hipLaunchKernelGGL((msim_runs_kernel<M, true, true, NX_FAST, NG_FAST, false>), dim3(nb), dim3(TPB), 0, a.stream,
                               a.p, a.run_begin, a.n, a.seed_base, nullptr, nullptr, 0u, parts, a.records, a.best_h,
                               a.err_count, a.err_list, a.err_cap);
        else
            hipLaunchKernelGGL((msim_runs_kernel<M, false, false, NX_FAST, NG_FAST, false>), dim3(nb), dim3(TPB), 0, a.stream,
                               a.p, a.run_begin, a.n, a.seed_base, nullptr, nullptr, 0u, parts, a.records, a.best_h,
                               a.err_count, a.err_list, a.err_cap);
    }
    // Retry kernel: wider capacities and deep branches for every run flagged above. Its grid is fixed
    // (err_cap lanes); lanes beyond the device-side count exit at once.
    launch_retry<M>(a, parts_retry, nbr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_finalize(a.partials, nrow + nbr, (uint32_t)(6 * M), a.sums, a.err_count, a.fail_count, a.err_cap,
                           a.status, a.stream);
}

template <int M>
static hipError_t launch_sweep_impl(const SweepArgs &a)
{
    const uint32_t nb = a.n_points * a.wpp, nbr = (a.err_cap + TPB - 1) / TPB;
    if (a.self) {
        hipLaunchKernelGGL((msim_sweep_kernel<M, true, true, NX_FAST, NG_FAST, false>), dim3(nb), dim3(TPB), 0, a.stream,
                           a.pts, a.run_begin, a.rpp, a.wpp, a.seed_base, nullptr, nullptr, 0u, a.partials, a.retry_sums,
                           a.records, a.best_h, a.err_count, a.err_list, a.err_cap);
        hipLaunchKernelGGL((msim_sweep_kernel<M, true, true, NX_WIDE, NG_WIDE, true>), dim3(nbr), dim3(TPB), 0, a.stream,
                           a.pts, a.run_begin, a.rpp, a.wpp, a.seed_base, a.err_list, a.err_count, a.err_cap, a.partials,
                           a.retry_sums, a.records, a.best_h, a.err_count + 1, nullptr, 0u);
    } else {
        hipLaunchKernelGGL((msim_sweep_kernel<M, false, false, NX_FAST, NG_FAST, false>), dim3(nb), dim3(TPB), 0, a.stream,
                           a.pts, a.run_begin, a.rpp, a.wpp, a.seed_base, nullptr, nullptr, 0u, a.partials, a.retry_sums,
                           a.records, a.best_h, a.err_count, a.err_list, a.err_cap);
        hipLaunchKernelGGL((msim_sweep_kernel<M, false, true, NX_WIDE, NG_WIDE, true>), dim3(nbr), dim3(TPB), 0, a.stream,
                           a.pts, a.run_begin, a.rpp, a.wpp, a.seed_base, a.err_list, a.err_count, a.err_cap, a.partials,
                           a.retry_sums, a.records, a.best_h, a.err_count + 1, nullptr, 0u);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_sweep_finalize(a);
}

#if defined(MSIM_M)
// One translation unit per miner count (built in parallel): explicit entry point for M = MSIM_M.
#define MSIM_CAT2(a, b) a##b
#define MSIM_CAT(a, b) MSIM_CAT2(a, b)
hipError_t MSIM_CAT(launch_runs_m, MSIM_M)(const LaunchArgs &a) { return launch_m<MSIM_M>(a); }
hipError_t MSIM_CAT(launch_sweep_m, MSIM_M)(const SweepArgs &a) { return launch_sweep_impl<MSIM_M>(a); }
#endif

}  // namespace msim
