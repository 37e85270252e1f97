// Host test of msim_commcache.h (the communicator cache of msim_run_multi, csrc/msim_multi.hip) with
// stand-in communicators: several threads share one device list, every call "runs a collective" on the
// set it holds, and some calls fail and retire the set (a retire that released the lock before
// destroying let a waiting caller use a destroyed communicator). Every stand-in communicator records whether
// it was destroyed; using a destroyed one, destroying one twice, or two holders at once fails the test.
// Prints "OK <calls> <inits> <destroys>" on success; exits non-zero otherwise.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../miningsimulation_amd/csrc/msim_commcache.h"

namespace {

struct Fake {
    std::atomic<int> destroyed{0};
    std::atomic<int> users{0};
};
std::atomic<long> g_inits{0}, g_destroys{0}, g_bad{0};

struct FakeBackend {
    using Comm = Fake *;
    static bool init(Comm *comms, int n, const int *)
    {
        for (int i = 0; i < n; ++i) comms[i] = new Fake;  // leaked on purpose: a later use must still be detectable
        g_inits += n;
        return true;
    }
    static void destroy(Comm c)
    {
        if (c->destroyed.exchange(1)) ++g_bad;  // destroyed twice
        ++g_destroys;
    }
};

}  // namespace

int main(int argc, char **argv)
{
    const int threads = argc > 1 ? atoi(argv[1]) : 4;
    const int calls = argc > 2 ? atoi(argv[2]) : 2000;
    msim::CommCache<FakeBackend> cache;
    std::atomic<long> done{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
            unsigned x = 12345u + 977u * (unsigned)t;
            for (int i = 0; i < calls; ++i) {
                auto lease = cache.acquire({0, 1});
                if (!lease.ok) {
                    ++g_bad;
                    continue;
                }
                for (Fake *c : lease.e->comms) {  // "the collective": every communicator must be alive and unshared
                    if (c == nullptr || c->destroyed.load()) ++g_bad;
                    if (c && c->users.fetch_add(1) != 0) ++g_bad;
                }
                std::this_thread::yield();
                for (Fake *c : lease.e->comms)
                    if (c) c->users.fetch_sub(1);
                x = x * 1103515245u + 12345u;
                if ((x >> 16) % 5 == 0) cache.retire(lease);  // a failed collective
                ++done;
            }
        });
    for (auto &t : ts) t.join();
    const int released = cache.release();
    if (cache.size() != 0 || released > 1) ++g_bad;
    if (g_bad.load()) {
        fprintf(stderr, "FAIL bad=%ld\n", g_bad.load());
        return 1;
    }
    printf("OK %ld %ld %ld\n", done.load(), g_inits.load(), g_destroys.load());
    return 0;
}
