// msim_general.hip — G, the general engine (msim_general.h) on the device: one lane per run, the run's
// chains in a window of global memory, runs taken from a list (the runs a fast engine could not finish) or
// from an index range (networks only G serves), in tiers of growing windows.
//
// Per lane: chains [M][CAP] (owner u32, arrival i64; contiguous per lane, so a lane's walks over one chain
// stay inside its own lines) and the per-miner counters size / stale / folded prefix as [M][lanes] (the
// loops over miners are wave-uniform, so these loads are coalesced). Results: MinerStats terms (the same
// Q32.32 fixed point as every other path) added atomically to per-point sums, optional per-run records.
// A run that outgrows the window goes to the next tier's list; the last tier's window holds every block a
// run can have (msim_gen_caps), so a failure there is only a run longer than its pre-sized draws.
#include <hip/hip_runtime.h>

#include "msim_general.h"
#include "msim_general_launch.h"
#include "msim_model.h"

namespace msim {

struct GenDevStore {
    uint32_t *o;          // this lane's owners [M][cap]
    int64_t *a;           // this lane's arrivals [M][cap]
    uint32_t *sz, *st, *pr;  // &array[lane]; miner k at [k * L]
    size_t L;
    uint32_t cap;
    __device__ __forceinline__ uint32_t own(uint32_t k, uint32_t i) const { return o[(size_t)k * cap + i]; }
    __device__ __forceinline__ int64_t arr(uint32_t k, uint32_t i) const { return a[(size_t)k * cap + i]; }
    __device__ __forceinline__ void put(uint32_t k, uint32_t i, uint32_t ow, int64_t ar)
    {
        o[(size_t)k * cap + i] = ow;
        a[(size_t)k * cap + i] = ar;
    }
    __device__ __forceinline__ void set_arr(uint32_t k, uint32_t i, int64_t ar) { a[(size_t)k * cap + i] = ar; }
    __device__ __forceinline__ uint32_t size(uint32_t k) const { return sz[k * L]; }
    __device__ __forceinline__ void set_size(uint32_t k, uint32_t n) { sz[k * L] = n; }
    __device__ __forceinline__ void add_stale(uint32_t k) { st[k * L] += 1u; }
    __device__ __forceinline__ uint32_t stale(uint32_t k) const { return st[k * L]; }
    __device__ __forceinline__ void add_pre(uint32_t k, uint32_t v) { pr[k * L] += v; }
    __device__ __forceinline__ uint32_t pre(uint32_t k) const { return pr[k * L]; }
};

__global__ __launch_bounds__(256) void msim_gen_kernel(const GenArgs a)
{
    const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= a.lanes) return;
    const uint32_t n_items = a.list ? *a.list_count : a.n_items;
    const uint32_t items = a.list ? (n_items < a.list_cap ? n_items : a.list_cap) : n_items;
    if (a.list && n_items > a.list_cap && lane == 0) atomicAdd(a.counts + GEN_C_FAIL, n_items - a.list_cap);
    GenDevStore s;
    s.cap = a.cap;
    s.L = a.lanes;
    s.sz = a.sizes + lane;
    s.st = a.sizes + (size_t)a.max_m * a.lanes + lane;
    s.pr = a.sizes + 2 * (size_t)a.max_m * a.lanes + lane;
    for (uint32_t it = (uint32_t)lane; it < items; it += (uint32_t)a.lanes) {
        const uint32_t code = a.list ? a.list[it] : it;
        const uint32_t point = code / a.rpp, rel = code % a.rpp;
        const GenParams &g = a.pts[point];
        s.o = a.owners + lane * (size_t)g.m * a.cap;
        s.a = a.arrivals + lane * (size_t)g.m * a.cap;
        for (uint32_t k = 0; k < g.m; ++k) {
            s.st[k * s.L] = 0;
            s.pr[k * s.L] = 0;
        }
        const uint64_t run = a.run_begin + rel;
        Gen<GenDevStore> e(s, g);
        GenOut o;
        if (!e.run(rng_seed(seed_interval(a.seed_base, run)), rng_seed(seed_picker(a.seed_base, run)), o)) {
            if ((o.err & GERR_CAP) && a.next) {
                const uint32_t pos = atomicAdd(a.next_count, 1u);
                if (pos < a.list_cap) a.next[pos] = code;
                else atomicAdd(a.counts + GEN_C_FAIL, 1u);
            } else {
                atomicAdd(a.counts + GEN_C_FAIL, 1u);
            }
            continue;
        }
        e.count_best(o);
        const uint32_t L = Gen<GenDevStore>::best_height(o);
        const size_t gi = (size_t)point * a.rpp + rel;
        unsigned long long *sums = (unsigned long long *)(a.sums + (size_t)point * 6 * a.max_m);
        for (uint32_t k = 0; k < g.m; ++k) {
            const uint32_t f = e.found_after_count(k), st = s.stale(k);
            if (a.records) {
                a.records[2 * (gi * g.m + k) + 0] = f;
                a.records[2 * (gi * g.m + k) + 1] = st;
            }
            if (st) atomicAdd(sums + 6 * k + 1, (unsigned long long)st);
            if (f == 0) continue;  // share and rate are 0 (main.cpp:28-29)
            // MinerStats (main.cpp:22-30) as Q32.32 fixed point, as every other path sums them
            const uint64_t sfx = (uint64_t)((double)f / (double)L * 4294967296.0 + 0.5);
            const uint64_t rfx = (uint64_t)((double)st / (double)f * 4294967296.0 + 0.5);
            atomicAdd(sums + 6 * k + 0, (unsigned long long)f);
            atomicAdd(sums + 6 * k + 2, (unsigned long long)(sfx >> 32));
            atomicAdd(sums + 6 * k + 3, (unsigned long long)(sfx & 0xFFFFFFFFull));
            if (rfx) {
                atomicAdd(sums + 6 * k + 4, (unsigned long long)(rfx >> 32));
                atomicAdd(sums + 6 * k + 5, (unsigned long long)(rfx & 0xFFFFFFFFull));
            }
        }
        if (a.best_h) a.best_h[gi] = L;
    }
}

// Status of a general-network launch: [0] runs that needed a wider window, [1] runs that failed.
__global__ void msim_gen_status(const uint32_t *counts, uint32_t *status)
{
    if (threadIdx.x == 0 && status) {
        status[0] = counts[GEN_C_L2] + counts[GEN_C_L3];
        status[1] = counts[GEN_C_FAIL];
    }
}

hipError_t launch_gen(const GenArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL(msim_gen_kernel, dim3((unsigned)((a.lanes + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_gen_status(const uint32_t *counts, uint32_t *status, hipStream_t s)
{
    hipLaunchKernelGGL(msim_gen_status, dim3(1), dim3(64), 0, s, counts, status);
    return hipGetLastError();
}

}  // namespace msim
