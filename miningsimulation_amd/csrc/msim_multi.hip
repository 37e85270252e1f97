// msim_multi.hip — msim_run_multi / msim_sweep_run_multi: the reference's run loop (main.cpp:205-220) spread over several GPUs
// of one node, combined with RCCL.
//
// The reference runs SIM_RUNS independent runs as std::async tasks and adds their MinerStats on the main
// thread (main.cpp:209-217). Runs are independent and their seeds are a pure function of the run index,
// so here the run range is cut into contiguous shards, one per device; each device runs its shard
// through msim_launch (device-resident, asynchronous on its own stream), and the per-miner msim_sums (integers)
// with the two status words packed behind them are combined by ONE ncclAllReduce per job over a single-process
// communicator (ncclCommInitAll: RCCL over xGMI on MI355X), cached per device list. Integer sums make the result bit-identical to msim_run for every
// device count.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <mutex>
#include <vector>

#include "../../include/msim.h"
#include "msim_commcache.h"

namespace {

// runs per msim_launch on one device (as msim_run: keeps every launch's workspace bounded)
constexpr uint64_t MULTI_CHUNK = 1ull << 22;
constexpr uint64_t MAX_LAUNCH_RUNS = 1ull << 26;  // msim_launch / msim_sweep_launch limit (runs x points)

__global__ void add_sums_kernel(uint64_t *acc, const uint64_t *part, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) acc[i] += part[i];
}

// the launch's two status words, added as u64 behind the sums (one all-reduce operand)
__global__ void add_status_kernel(uint64_t *acc, const uint32_t *part)
{
    if (threadIdx.x < 2) acc[threadIdx.x] += part[threadIdx.x];
}

// One device's shard and everything it needs, allocated before any launch or collective.
struct Shard {
    int device;
    uint64_t begin, n, chunk;
    size_t wsb = 0;
    int rc = MSIM_OK;
    hipStream_t s = nullptr;
    void *ws = nullptr;
    uint64_t *d_acc = nullptr;   // [nv + 2] sums of every chunk, then their status words (the all-reduce operand)
    uint64_t *d_part = nullptr;  // [nv] one chunk's sums
    uint32_t *d_pst = nullptr;   // [2] one chunk's status
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};  // timing: shard start, shard done, all-reduce done
};

// What one device launches for a chunk of runs: a config (msim_launch) or a sweep (msim_sweep_launch).
struct Job {
    const msim_config *cfg;
    const msim_sweep *sweep;
    uint32_t nv;  // int64 values of the sums: 6 * M (config) or 6 * M * points (sweep)
    // runs per launch: a sweep launch covers every point, so its limit is MAX_LAUNCH_RUNS / points
    uint64_t max_chunk() const
    {
        if (cfg) return MULTI_CHUNK;
        const uint64_t np = msim_sweep_point_count(sweep), c = np ? MAX_LAUNCH_RUNS / np : 1;
        return c < 1 ? 1 : (c < MULTI_CHUNK ? c : MULTI_CHUNK);
    }
    size_t ws_bytes(uint64_t n) const
    {
        return cfg ? msim_workspace_bytes(cfg, n) : msim_sweep_workspace_bytes(sweep, n);
    }
    int launch(uint64_t begin, uint64_t n, uint32_t seed_base, void *sums, void *status, void *ws, size_t wsb,
               hipStream_t s) const
    {
        return cfg ? msim_launch(cfg, begin, n, seed_base, sums, nullptr, nullptr, status, ws, wsb, s)
                   : msim_sweep_launch(sweep, begin, n, seed_base, sums, nullptr, nullptr, status, ws, wsb, s);
    }
};

int alloc_shard(const Job &job, Shard &sh, bool timed)
{
    const uint32_t nv = job.nv;
    const uint64_t mc = job.max_chunk();
    sh.chunk = sh.n < mc ? sh.n : mc;
    sh.wsb = sh.chunk ? job.ws_bytes(sh.chunk) : 0;
    if (sh.chunk && sh.wsb == 0) return MSIM_E_INVALID;
    if (hipSetDevice(sh.device) != hipSuccess || hipStreamCreate(&sh.s) != hipSuccess ||
        hipMalloc(&sh.d_acc, (nv + 2) * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&sh.d_part, nv * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&sh.d_pst, 2 * sizeof(uint32_t)) != hipSuccess || (sh.wsb && hipMalloc(&sh.ws, sh.wsb) != hipSuccess) ||
        hipMemsetAsync(sh.d_acc, 0, (nv + 2) * sizeof(uint64_t), sh.s) != hipSuccess)
        return MSIM_E_HIP;
    if (timed)
        for (hipEvent_t &e : sh.ev)
            if (hipEventCreate(&e) != hipSuccess) return MSIM_E_HIP;
    return MSIM_OK;
}

void free_shard(Shard &sh)
{
    (void)hipSetDevice(sh.device);
    (void)hipFree(sh.ws);
    (void)hipFree(sh.d_part);
    (void)hipFree(sh.d_pst);
    (void)hipFree(sh.d_acc);
    for (hipEvent_t &e : sh.ev)
        if (e) (void)hipEventDestroy(e);
    if (sh.s) (void)hipStreamDestroy(sh.s);
}

// Enqueue one device's shard (asynchronous: every device runs its chunks concurrently on its stream).
void enqueue_shard(const Job &job, uint32_t seed_base, Shard &sh)
{
    if (hipSetDevice(sh.device) != hipSuccess) {
        sh.rc = MSIM_E_HIP;
        return;
    }
    if (sh.ev[0]) (void)hipEventRecord(sh.ev[0], sh.s);
    for (uint64_t off = 0; sh.rc == MSIM_OK && off < sh.n; off += sh.chunk) {
        const uint64_t cn = (sh.n - off) < sh.chunk ? (sh.n - off) : sh.chunk;
        sh.rc = job.launch(sh.begin + off, cn, seed_base, sh.d_part, sh.d_pst, sh.ws, sh.wsb, sh.s);
        if (sh.rc) break;
        hipLaunchKernelGGL(add_sums_kernel, dim3((job.nv + 255) / 256), dim3(256), 0, sh.s, sh.d_acc, sh.d_part, job.nv);
        hipLaunchKernelGGL(add_status_kernel, dim3(1), dim3(64), 0, sh.s, sh.d_acc + job.nv, sh.d_pst);
        if (hipGetLastError() != hipSuccess) sh.rc = MSIM_E_HIP;
    }
    if (sh.ev[1]) (void)hipEventRecord(sh.ev[1], sh.s);
}

// Communicator cache (msim_commcache.h) over RCCL: one single-process communicator set per device list.
struct RcclBackend {
    using Comm = ncclComm_t;
    static bool init(Comm *comms, int n, const int *devs) { return ncclCommInitAll(comms, n, devs) == ncclSuccess; }
    static void destroy(Comm c) { (void)ncclCommDestroy(c); }
};
using Cache = msim::CommCache<RcclBackend>;
Cache &comm_cache()
{
    static Cache c;
    return c;
}

// Test hook: MSIM_MULTI_FAIL_COLLECTIVE=1 makes every grouped collective report failure, so the retire path
// runs on a real communicator set (the race itself is covered on the host: tests/native/commcache_host.cpp).
bool forced_collective_failure()
{
    const char *e = getenv("MSIM_MULTI_FAIL_COLLECTIVE");
    return e && e[0] == '1';
}

// Shards [run_begin, run_begin + n_runs) over the devices, runs them, all-reduces; acc = reduced sums.
// Every buffer of every device is allocated before anything is enqueued, and the collectives are issued
// for all devices by this one thread inside one ncclGroupStart / ncclGroupEnd (the single-process
// multi-device form), so no device can be left waiting in a collective that another never joins: a
// device whose launches failed contributes its (zero-initialised) buffers and the call returns its error.
int run_job(const Job &job, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base, const int *devices,
            uint32_t n_devices, std::vector<uint64_t> &acc, double *opt_shard_ms)
{
    std::vector<int> devs(n_devices);
    for (uint32_t g = 0; g < n_devices; ++g) devs[g] = devices ? devices[g] : (int)g;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return MSIM_E_HIP;
    for (int d : devs)
        if (d < 0 || d >= count) return MSIM_E_INVALID;
    // contiguous shards, as distributed.shard: the first n_runs % n_devices shards take one run more
    std::vector<Shard> sh(n_devices);
    const uint64_t base = n_runs / n_devices, rem = n_runs % n_devices;
    int rc = MSIM_OK;
    for (uint32_t g = 0; g < n_devices; ++g) {
        sh[g].device = devs[g];
        sh[g].begin = run_begin + g * base + (g < rem ? g : rem);
        sh[g].n = base + (g < rem ? 1 : 0);
        if (rc == MSIM_OK) rc = alloc_shard(job, sh[g], opt_shard_ms != nullptr);
    }
    // one device: its sums are the result (no collective)
    Cache::Lease ce;
    if (rc == MSIM_OK && n_devices > 1) {
        ce = comm_cache().acquire(devs);
        if (!ce.ok) rc = MSIM_E_HIP;
    }
    if (rc == MSIM_OK) {
        for (auto &x : sh) enqueue_shard(job, seed_base, x);
        bool coll_failed = false;
        if (ce.ok && (forced_collective_failure() || ncclGroupStart() != ncclSuccess)) {
            rc = MSIM_E_HIP;
            coll_failed = true;
        } else if (ce.ok) {
            for (uint32_t g = 0; g < n_devices; ++g)  // sums and status: one collective per device
                if (ncclAllReduce(sh[g].d_acc, sh[g].d_acc, job.nv + 2, ncclUint64, ncclSum, ce.e->comms[g], sh[g].s) !=
                    ncclSuccess)
                    rc = MSIM_E_HIP;
            if (ncclGroupEnd() != ncclSuccess) rc = MSIM_E_HIP;
            coll_failed = rc != MSIM_OK;
        }
        for (auto &x : sh)
            if (x.ev[2]) (void)hipEventRecord(x.ev[2], x.s);
        for (auto &x : sh)
            if (hipSetDevice(x.device) != hipSuccess || hipStreamSynchronize(x.s) != hipSuccess) rc = rc ? rc : MSIM_E_HIP;
        for (const auto &x : sh)
            if (x.rc) rc = rc ? rc : x.rc;
        if (coll_failed) comm_cache().retire(ce);  // under the entry's lock (msim_commcache.h)
    }
    if (ce.lock.owns_lock()) ce.lock.unlock();
    if (opt_shard_ms) {  // per device: its launches, and the all-reduce after them
        for (uint32_t g = 0; g < n_devices; ++g) {
            float a = 0, b = 0;
            if (rc == MSIM_OK && (hipSetDevice(sh[g].device) != hipSuccess ||
                                  hipEventElapsedTime(&a, sh[g].ev[0], sh[g].ev[1]) != hipSuccess ||
                                  hipEventElapsedTime(&b, sh[g].ev[1], sh[g].ev[2]) != hipSuccess))
                rc = MSIM_E_HIP;
            opt_shard_ms[2 * g] = a;
            opt_shard_ms[2 * g + 1] = b;
        }
    }
    acc.assign(job.nv + 2, 0);
    if (rc == MSIM_OK) {  // every device holds the reduced sums and status: read the first one's
        if (hipSetDevice(sh[0].device) != hipSuccess ||
            hipMemcpy(acc.data(), sh[0].d_acc, acc.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
            rc = MSIM_E_HIP;
        else if (acc[job.nv + 1] != 0)
            rc = MSIM_E_CAPACITY;
    }
    acc.resize(job.nv);
    for (uint32_t g = 0; g < n_devices; ++g) free_shard(sh[g]);
    return rc;
}

}  // namespace

extern "C" int msim_run_multi_timed(const msim_config *cfg, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base,
                                    const int *devices, uint32_t n_devices, msim_stats *out_sums, msim_sums *opt_sums,
                                    double *opt_shard_ms)
{
    if (!cfg || !out_sums || n_runs == 0 || n_devices == 0 || n_devices > 64) return MSIM_E_INVALID;
    const uint32_t m = msim_config_miner_count(cfg);
    std::vector<uint64_t> acc;
    const int rc = run_job(Job{cfg, nullptr, 6 * m}, run_begin, n_runs, seed_base, devices, n_devices, acc, opt_shard_ms);
    if (rc) return rc;
    const msim_sums *fs = (const msim_sums *)acc.data();
    if (opt_sums) memcpy(opt_sums, fs, sizeof(msim_sums) * m);
    msim_sums_to_stats(fs, m, out_sums);
    return MSIM_OK;
}

extern "C" int msim_run_multi(const msim_config *cfg, uint64_t run_begin, uint64_t n_runs, uint32_t seed_base,
                              const int *devices, uint32_t n_devices, msim_stats *out_sums, msim_sums *opt_sums)
{
    return msim_run_multi_timed(cfg, run_begin, n_runs, seed_base, devices, n_devices, out_sums, opt_sums, nullptr);
}

extern "C" int msim_sweep_run_multi(const msim_sweep *sweep, uint64_t run_begin, uint64_t runs_per_point,
                                    uint32_t seed_base, const int *devices, uint32_t n_devices, msim_stats *out_stats,
                                    msim_sums *opt_sums)
{
    if (!sweep || !out_stats || runs_per_point == 0 || n_devices == 0 || n_devices > 64) return MSIM_E_INVALID;
    const uint32_t nv = 6 * msim_sweep_miner_count(sweep) * msim_sweep_point_count(sweep);
    std::vector<uint64_t> acc;
    const int rc =
        run_job(Job{nullptr, sweep, nv}, run_begin, runs_per_point, seed_base, devices, n_devices, acc, nullptr);
    if (rc) return rc;
    const msim_sums *fs = (const msim_sums *)acc.data();
    if (opt_sums) memcpy(opt_sums, fs, sizeof(uint64_t) * nv);
    msim_sums_to_stats(fs, nv / 6, out_stats);
    return MSIM_OK;
}

extern "C" int msim_multi_release(void) { return comm_cache().release(); }
