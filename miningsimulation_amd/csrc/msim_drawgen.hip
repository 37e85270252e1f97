// msim_drawgen.hip — K1 of the event-skipping pipeline (msim_pipeline.h): every block's draws.
//
// One lane = (run, segment): both of the run's xoroshiro128++ streams (main.cpp:134) are jumped to
// draw j*SEG (msim_jump.h), then the lane produces SEG blocks exactly as the reference's sequential
// loop would draw them (simulation.h:205-221): interval I_i (ms), finder k_i, and the "fast" bit
// I_{i+1} > prop_{k_i} (honest finders only). A wave = 64 consecutive runs at one segment, so the
// jump matrix columns are wave-uniform scalar loads. Nothing is stored per block: a non-fast block is
// listed with both RNG states (K2 redraws its episode), and each group of the band where a run can end
// keeps its first word and RNG states (K3 redraws the last group). Roofline: VALU issue (FP64 log +
// 64-bit integer RNG).
#include <hip/hip_runtime.h>

#include "msim_jump.h"
#include "msim_kernels.h"
#include "msim_pipeline.h"

namespace msim {

__device__ __noinline__ int32_t interval_ms_exact_dev(uint64_t u) { return (int32_t)interval_ms_of(u); }


// Side effects of one K1 lane (msim_pipeline.h draw_segment): LDS per-owner counters (one u32 per owner
// and lane, [owner][lane]: conflict-free, and the increment is one ds_add_u32 of a constant), wave-
// aggregated appends to the dense episode list, the band's group records.
constexpr uint32_t K1_OWNERS = 2 * CNT_WORDS;  // 15 miners + PickFinder's fall-through (index 15)
constexpr uint32_t K1_NSL = K1_OWNERS;         // LDS row after the owners: the lane's slow-block count
constexpr uint32_t K1_ROWS = K1_NSL + 1;

// The slow path keeps no per-lane register across the draw loop: its lane-dependent values are rebuilt from
// the ballot mask (mbcnt), wave-uniform SGPRs and LDS (the per-lane list count), so the loop's register
// budget (K1_WAVES below) goes to the draws. Measured on MI355X (profiles/r03/INDEX.md): with the lane id,
// its bit, the list count and the counter address held across the loop, the compiler reloaded them from
// scratch once per quad (six scratch loads and two vmcnt(0) waits per quad).
struct DevCtx {
    const DrawArgs &a;
    uint32_t (*cnt)[256];
    uint64_t amask;  // active lanes of the wave (runs < n)
    uint32_t tid, r0, seg, jb;  // r0: the wave's first run (wave-uniform)
    uint32_t cbase;             // tid * 4, rebuilt every quad (quad())
    uint32_t wbase;             // 4 x the wave's first thread (SGPR)
    __device__ __forceinline__ void quad()
    {
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\tv_lshl_add_u32 %0, %0, 2, %1"
                     : "=&v"(cbase) : "s"(wbase));
    }
    // owner row k = info_finder(info) sits at byte offset k << 10 = info & (15 << INFO_K_SHIFT)
    __device__ __forceinline__ void count(uint32_t info)
    {
        // the array's base is a constant the compiler folds into the instruction's offset field
        const uint32_t ad = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)&cnt[0][0] +
                            ((info & (15u << INFO_K_SHIFT)) | cbase);
        __atomic_fetch_add((__attribute__((address_space(3))) uint32_t *)(uintptr_t)ad, 1u, __ATOMIC_RELAXED);
    }
    __device__ __forceinline__ bool vote(bool s) const { return (__builtin_amdgcn_ballot_w64(s) & amask) != 0ull; }
    // the owner counters packed as the u16 pairs of the workspace layout (msim_pipeline.h CNT_WORDS)
    __device__ __forceinline__ uint32_t packed(uint32_t w) const { return cnt[2 * w][tid] | (cnt[2 * w + 1][tid] << 16); }
    // The wave's reserved chunk of the episode list, [lend - lleft, lend) still free (wave-uniform).
    uint32_t lend, lleft;
    // Mark the unused tail of the wave's chunk (K2 skips EP_HOLE slots; no run's slots point there). A chunk
    // holds up to max(lchunk, 64) slots, so the tail can be longer than the wave: every slot of it is marked,
    // 64 per pass (K2 reads every slot below the list count, and the workspace is not cleared between launches).
    __device__ void holes()
    {
        uint32_t lane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=&v"(lane));
        const uint32_t lo = lend - lleft;
        for (uint32_t i = lane; i < lleft; i += 64u)
            if (lo + i < a.lcap) a.list[lo + i].run = EP_HOLE;
    }
    __device__ void slow(bool s, uint32_t block, uint64_t offset, uint32_t w0, uint32_t w1, const Rng &ri, const Rng &rp,
                         uint32_t skip)
    {
        const uint64_t mask = __builtin_amdgcn_ballot_w64(s) & amask;
        // rank of this lane among the slow ones (asm volatile: computed here, not hoisted out of the loop)
        uint32_t below;
        asm volatile("v_mbcnt_lo_u32_b32 %0, %1, 0\n\tv_mbcnt_hi_u32_b32 %0, %2, %0"
                     : "=&v"(below) : "s"((uint32_t)mask), "s"((uint32_t)(mask >> 32)));
        const uint32_t nsel = (uint32_t)__popcll(mask);
        if (nsel > lleft) {  // wave-uniform: a new chunk (the old one's tail becomes holes)
            holes();
            const uint32_t need = nsel > a.lchunk ? nsel : a.lchunk;
            uint32_t base = 0;
            if (s & (below == 0u)) base = atomicAdd(a.list_count, need);
            base = __builtin_amdgcn_readlane(base, (uint32_t)(__ffsll((unsigned long long)mask) - 1));
            lend = base + need;
            lleft = need;
        }
        const uint32_t base = lend - lleft;
        lleft -= nsel;
        if (!s) return;
        uint32_t lane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=&v"(lane));
        if (!((amask >> lane) & 1ull)) return;
        const uint32_t r = r0 + lane;
        const uint32_t idx = base + below;
        if (idx < a.lcap) {
            EpEntry e;
            e.run = r;
            e.block = block;
            e.offset = offset;
            e.w0 = w0;
            e.w1 = w1;
            e.skip = skip;
            e.pad = 0;
            e.ri = ri;
            e.rp = rp;
            a.list[idx] = e;
        }
        uint32_t *nsl = &cnt[K1_NSL][r & 255u];
        const uint32_t c = *nsl;
        if (c < a.cap) a.slots[((size_t)seg * a.cap + c) * a.nr + r] = idx;
        *nsl = c + 1u;
    }
    __device__ __forceinline__ uint32_t run() const { return r0 + (tid & 63u); }
    __device__ void group_start(uint32_t g, uint32_t w0, const Rng &ri, const Rng &rp)
    {
        const uint32_t r = run();
        const size_t gi = (size_t)jb * a.gps + g;
        GroupRec gr;
        gr.ri = ri;
        gr.rp = rp;
        gr.w0 = w0;
        gr.pad = 0;
        a.grec[gi * a.nr + r] = gr;
#pragma unroll
        for (uint32_t w = 0; w < CNT_WORDS; ++w) a.gcum[(gi * CNT_WORDS + w) * a.nr + r] = packed(w);
    }
    __device__ void group(uint32_t g, uint32_t sum, uint64_t end)
    {
        a.gsum[((size_t)jb * a.gps + g) * a.nr + run()] = sum;
        if (g % SGROUP == SGROUP - 1 || g + 1 == a.gps) {
            const uint32_t nsg = (a.gps + SGROUP - 1) / SGROUP;
            a.gend[((size_t)jb * nsg + g / SGROUP) * a.nr + run()] = end;
        }
    }
};

// Resident K1 waves per SIMD the register budget is sized for (VGPRs <= 512 / waves). Measured on MI355X
// (c2, profiles/r03/INDEX.md): 4 waves (113 VGPRs) 4.17 ms, 5 (96) 4.02 ms, 6 (80) 3.75 ms, 7 (72) 7.3 ms and
// 8 (64) 13.7 ms, where the spills reach the draw loop's hot values. Re-measured on round 5's K1 (chunked list
// reservation; profiles/r05/k1waves): 4 waves (104 VGPRs) 3.27 ms, 5 (96, 10 spills) 3.17-3.21 ms, 6 (80, 23
// spills) 3.27 ms serial, same box, alternating.
#ifndef MSIM_K1_WAVES
#define MSIM_K1_WAVES 5
#endif
#if MSIM_K1_WAVES
__global__ __launch_bounds__(256, MSIM_K1_WAVES) void msim_draws_kernel(const DrawArgs a)
#else
__global__ __launch_bounds__(256) void msim_draws_kernel(const DrawArgs a)
#endif
{
    // one LDS block: pick table, log table, owner counters
    __shared__ struct {
        PickTab pick;
        LogTab log;
        uint32_t cnt[K1_ROWS][256];
    } sm;
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < sizeof(PickTab) / 4; i += 256) ((uint32_t *)&sm.pick)[i] = ((const uint32_t *)a.tab.pick)[i];
    for (uint32_t i = tid; i < sizeof(LogTab) / 8; i += 256) ((double *)&sm.log)[i] = ((const double *)a.tab.logt)[i];
    auto s_cnt = sm.cnt;
#pragma unroll
    for (uint32_t w = 0; w < K1_ROWS; ++w) s_cnt[w][tid] = 0;
    __syncthreads();

    const uint32_t r = blockIdx.x * 256 + tid;  // slice-local run (< nr)
    const uint32_t seg = blockIdx.y;
    const uint64_t run = a.run_begin + r;
    Rng ri = rng_seed(seed_interval(a.seed_base, run));
    Rng rp = rng_seed(seed_picker(a.seed_base, run));
    if (seg) jump2(reinterpret_cast<const uint4 *>(a.tab.jump) + (size_t)seg * 128, ri, rp);

    const uint32_t b0 = seg * a.seg;
    DevCtx cx{a, s_cnt, __builtin_amdgcn_ballot_w64(r < a.n), tid, (uint32_t)__builtin_amdgcn_readfirstlane(r & ~63u), seg,
              seg - a.band_lo, 0u,
              (uint32_t)__builtin_amdgcn_readfirstlane((tid & ~63u) * 4u), 0u, 0u};
    const uint64_t tsum = draw_segment<DevCtx>(cx, ri, rp, &sm.log, &sm.pick, b0, a.seg, seg >= a.band_lo);
    cx.holes();
    a.segsum[(size_t)seg * a.nr + r] = tsum;
#pragma unroll
    for (uint32_t w = 0; w < CNT_WORDS; ++w) a.segcnt[((size_t)seg * CNT_WORDS + w) * a.nr + r] = cx.packed(w);
    a.nslow[(size_t)seg * a.nr + r] = s_cnt[K1_NSL][tid];
}

__global__ void msim_interval_kernel(const LogTab *__restrict__ lt, const uint64_t *__restrict__ u,
                                     int64_t *__restrict__ out, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bool ok;
    const int32_t q = interval_ms_fast(u[i], lt, ok);
    out[i] = ok ? q : interval_ms_exact_dev(u[i]);
}

__global__ void msim_pick_kernel(const PickTab *__restrict__ pt, const uint64_t *__restrict__ u,
                                 int32_t *__restrict__ out, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = info_finder(pick_info(u[i], pt));
    out[i] = k == 15u ? -1 : (int32_t)k;
}

hipError_t launch_intervals(const LogTab *lt, const uint64_t *u, int64_t *out, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(msim_interval_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, lt, u, out, n);
    return hipGetLastError();
}

hipError_t launch_picks(const PickTab *pt, const uint64_t *u, int32_t *out, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(msim_pick_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, pt, u, out, n);
    return hipGetLastError();
}

hipError_t draws_blocks_per_cu(int *blocks)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, msim_draws_kernel, 256, 0);
}

hipError_t launch_draws(const DrawArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL(msim_draws_kernel, dim3(a.nr / 256, a.nseg), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace msim
