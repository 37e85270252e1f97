// wide_host.cpp — TEST INFRASTRUCTURE: a sequential host (CPU) execution of the large-network pipeline
// (miningsimulation_amd/csrc/msim_wide.h) built from the SAME lane bodies the gfx950 kernels run
// (wide_pick, draw_interval, wide_episode), composed the way W1-W3 compose them: every block before the
// end of the run counted for its finder, every non-fast block a candidate episode from a quiet state,
// episodes chained in block order from the first one reached quiet, the last fast block's arrival
// correction. Checked run by run against the oracle (tests/test_wide_host.py) on machines without a GPU.
// Never part of the product path (libmsim.so is GPU-only).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../miningsimulation_amd/csrc/msim_wide.h"

using namespace msim;

extern "C" int wide_host_pick(const uint64_t *w, uint32_t m, uint64_t W, const uint64_t *u, int32_t *out, uint64_t n)
{
    std::vector<uint64_t> cf(m + 1);
    std::vector<uint16_t> bucket(WB_N);
    std::vector<uint32_t> fthr(m, 0);
    build_wide_pick(w, fthr.data(), m, (uint32_t)W, cf.data(), bucket.data());
    const uint64_t mult = 0xFFFFFFFFFFFFFFFFull / W;
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t th;
        const uint32_t k = wide_pick(u[i], cf.data(), bucket.data(), (uint32_t)W, mult, th);
        out[i] = k >= m ? -1 : (int32_t)k;
    }
    return 0;
}

// Runs [run_begin, run_begin + n) with the SURVEY seed convention; found/stale [n][m]; err [n].
extern "C" int wide_host_run(const uint64_t *w, const int64_t *prop, uint32_t m, uint64_t W, int64_t D,
                             uint32_t seed_base, uint64_t run_begin, uint32_t n, uint32_t *found, uint32_t *stale,
                             uint32_t *err_out, uint32_t *n_episodes)
{
    std::vector<uint64_t> cf(m + 1);
    std::vector<uint16_t> bucket(WB_N);
    std::vector<uint32_t> fthr(m);
    for (uint32_t k = 0; k < m; ++k) fthr[k] = prop[k] < (int64_t)FTHR_NEVER ? (uint32_t)prop[k] : FTHR_NEVER;
    build_wide_pick(w, fthr.data(), m, (uint32_t)W, cf.data(), bucket.data());
    LogTab lt;
    build_log_table(&lt);
    const uint64_t mult = 0xFFFFFFFFFFFFFFFFull / W;
    uint32_t neps = 0, n_retry = 0;
    for (uint32_t r = 0; r < n; ++r) {
        const uint64_t run = run_begin + r;
        Rng ri = rng_seed(seed_interval(seed_base, run)), rp = rng_seed(seed_picker(seed_base, run));
        std::vector<uint32_t> I, F;
        std::vector<int64_t> T;
        std::vector<Rng> SI, SP;  // states after drawing block i
        int64_t t = 0;
        // draw until the first block at >= D, plus one more (its successor decides fast/slow)
        for (;;) {
            const uint32_t x = draw_interval(ri, &lt);
            uint32_t th;
            const uint32_t f = wide_pick(rng_next(rp), cf.data(), bucket.data(), (uint32_t)W, mult, th);
            t += x;
            I.push_back(x);
            F.push_back(f);
            T.push_back(t);
            SI.push_back(ri);
            SP.push_back(rp);
            if (T.size() >= 2 && T[T.size() - 2] >= D) break;
        }
        uint32_t n_end = 0;
        while (n_end < T.size() && T[n_end] < D) ++n_end;
        uint32_t *Fo = found + (size_t)r * m, *So = stale + (size_t)r * m;
        memset(Fo, 0, 4 * m);
        memset(So, 0, 4 * m);
        uint32_t err = 0;
        for (uint32_t i = 0; i < n_end; ++i) {
            if (F[i] >= m) err |= WERR_PICK;
            else Fo[F[i]]++;
        }
        uint32_t cursor = 0;
        bool ended = false;
        for (uint32_t s = 0; s < n_end && !err; ++s) {
            if (s < cursor) continue;
            if (!(I[s + 1] <= fthr[F[s]])) continue;  // fast block
            WideSrc src{SI[s + 1], SP[s + 1], &lt, cf.data(), bucket.data(), (uint32_t)W, mult};
            WideEpOut o;
            wide_episode<WE_FAST, WA_FAST>(prop, m, D, s, T[s], F[s], I[s + 1], F[s + 1], src, o);
            if (o.flags & WREC_RETRY) {  // the device's retry pass: same episode, larger capacities
                WideSrc src2{SI[s + 1], SP[s + 1], &lt, cf.data(), bucket.data(), (uint32_t)W, mult};
                wide_episode<WE, WA>(prop, m, D, s, T[s], F[s], I[s + 1], F[s + 1], src2, o);
                ++n_retry;
            }
            ++neps;
            if (o.flags & WREC_ERR) {
                err |= WERR_EP;
                break;
            }
            for (uint32_t e = 0; e < o.ne; ++e) {
                Fo[o.gid[e]] += o.dF[e];
                So[o.gid[e]] += o.dS[e];
            }
            cursor = o.end;
            if (o.flags & WREC_ENDED) {
                ended = true;
                break;
            }
        }
        if (!err && !ended && n_end > 0 && cursor < n_end) {
            const uint32_t f = F[n_end - 1];
            if (T[n_end - 1] + prop[f] > D) Fo[f] -= 1;
        }
        err_out[r] = err;
    }
    if (n_episodes) *n_episodes = neps | (n_retry << 24);
    return 0;
}
