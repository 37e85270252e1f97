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

namespace msim {

// Wave-level (DPP/bpermute) reduction of 6*M 64-bit sums, then the workgroup's 4 waves through LDS.
template <int M>
__device__ __forceinline__ void block_reduce_store(const uint64_t (&v)[6 * M], uint64_t *__restrict__ out)
{
    __shared__ uint64_t red[TPB / 64][6 * M];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 6 * M; ++i) {
        unsigned long long x = v[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if (lane == 0) red[wv][i] = x;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 6 * M; i += TPB) out[i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

template <int M, bool SELF, bool DEEP, int NX, int NG, bool LIST>
__global__ __launch_bounds__(TPB) void msim_runs_kernel(const SimParams p, const uint64_t run_begin, const uint32_t n,
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

// ------------------------------------------------------------------ host-side launch table
template <int M>
static hipError_t launch_m(const LaunchArgs &a)
{
    const uint32_t nb = (a.n + TPB - 1) / TPB;
    const uint32_t nbr = (a.err_cap + TPB - 1) / TPB;
    const bool self = a.p.selfish >= 0;
    uint64_t *parts = a.partials;
    uint64_t *parts_retry = a.partials + (size_t)nb * 6 * M;
    if (nb) {
        if (self)
            hipLaunchKernelGGL((msim_runs_kernel<M, true, true, NX_FAST, NG_FAST, false>), dim3(nb), dim3(TPB), 0, a.stream,
                               a.p, a.run_begin, a.n, a.seed_base, nullptr, nullptr, 0u, parts, a.records, a.best_h,
                               a.err_count, a.err_list, a.err_cap);
        else
            hipLaunchKernelGGL((msim_runs_kernel<M, false, false, NX_FAST, NG_FAST, false>), dim3(nb), dim3(TPB), 0, a.stream,
                               a.p, a.run_begin, a.n, a.seed_base, nullptr, nullptr, 0u, parts, a.records, a.best_h,
                               a.err_count, a.err_list, a.err_cap);
    }
    // Retry kernel: wider capacities and deep branches for every run the fast kernel flagged. Its
    // grid is fixed (err_cap lanes); lanes beyond the device-side count exit at once.
    if (self)
        hipLaunchKernelGGL((msim_runs_kernel<M, true, true, NX_WIDE, NG_WIDE, true>), dim3(nbr), dim3(TPB), 0, a.stream,
                           a.p, a.run_begin, a.n, a.seed_base, a.err_list, a.err_count, a.err_cap, parts_retry, a.records,
                           a.best_h, a.fail_count, nullptr, 0u);
    else
        hipLaunchKernelGGL((msim_runs_kernel<M, false, true, NX_WIDE, NG_WIDE, true>), dim3(nbr), dim3(TPB), 0, a.stream,
                           a.p, a.run_begin, a.n, a.seed_base, a.err_list, a.err_count, a.err_cap, parts_retry, a.records,
                           a.best_h, a.fail_count, nullptr, 0u);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_finalize(a.partials, nb + nbr, (uint32_t)(6 * M), a.sums, a.err_count, a.fail_count, a.err_cap,
                           a.status, a.stream);
}

#if defined(MSIM_M)
// One translation unit per miner count (built in parallel): explicit entry point for M = MSIM_M.
#define MSIM_CAT2(a, b) a##b
#define MSIM_CAT(a, b) MSIM_CAT2(a, b)
hipError_t MSIM_CAT(launch_runs_m, MSIM_M)(const LaunchArgs &a) { return launch_m<MSIM_M>(a); }
#endif

}  // namespace msim
