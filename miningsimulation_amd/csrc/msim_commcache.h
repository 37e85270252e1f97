// msim_commcache.h — the communicator cache behind msim_run_multi / msim_sweep_run_multi (msim_multi.hip).
//
// ncclCommInitAll costs milliseconds to seconds, so a communicator set is created once per device list and
// kept until release(). A set is used by one call at a time: acquire() returns it with its `use` lock held
// from the first enqueue to the last synchronisation. A set whose collectives failed is retired WHILE that
// lock is held (communicators destroyed, `dead` set, removed from the cache), so a caller that was blocked on
// the same entry finds it dead once it gets the lock and fetches a fresh one; it never touches a destroyed
// communicator. Lock order is `use`, then the cache mutex; lookups take only the cache mutex, so the order
// cannot invert. Templated over the backend so that the host test (tests/native/commcache_host.cpp) drives
// the same code with counting stand-in communicators and two racing threads.
#pragma once
#include <memory>
#include <mutex>
#include <vector>

namespace msim {

template <class B>
class CommCache {
public:
    using Comm = typename B::Comm;
    struct Entry {
        std::vector<int> devs;
        std::vector<Comm> comms;
        std::mutex use;
        bool dead = false;  // guarded by `use`
        ~Entry()
        {
            for (Comm c : comms)
                if (c) B::destroy(c);
        }
    };
    // The live entry for `devs`, locked for this caller (ok == false: creating it failed).
    struct Lease {
        std::shared_ptr<Entry> e;
        std::unique_lock<std::mutex> lock;
        bool ok = false;
    };

    // Each pass that finds its entry dead follows another caller's retire (one per failed call), so the loop
    // ends: it either gets a live entry or fails to create one.
    Lease acquire(const std::vector<int> &devs)
    {
        Lease l;
        for (;;) {
            l.e = lookup(devs);
            if (!l.e) return l;
            l.lock = std::unique_lock<std::mutex>(l.e->use);
            if (!l.e->dead) {
                l.ok = true;
                return l;
            }
            l.lock.unlock();  // retired by the previous holder: look again (its replacement or a new set)
        }
    }

    // The holder of `l` saw its collectives fail: destroy the set now, under its lock.
    void retire(Lease &l)
    {
        Entry &e = *l.e;
        for (Comm &c : e.comms) {
            if (c) B::destroy(c);
            c = Comm{};
        }
        e.dead = true;
        std::lock_guard<std::mutex> g(mu_);
        for (size_t i = 0; i < cache_.size(); ++i)
            if (cache_[i].get() == &e) {
                cache_.erase(cache_.begin() + (long)i);
                break;
            }
    }

    // Drop every cached set that no call holds (msim_multi_release); returns how many were released.
    int release()
    {
        std::vector<std::shared_ptr<Entry>> keep, drop;
        {
            std::lock_guard<std::mutex> g(mu_);
            for (auto &e : cache_) (e.use_count() > 1 ? keep : drop).push_back(e);
            cache_.swap(keep);
        }
        return (int)drop.size();  // destroyed here, outside the cache mutex (~Entry)
    }

    size_t size()
    {
        std::lock_guard<std::mutex> g(mu_);
        return cache_.size();
    }

private:
    std::shared_ptr<Entry> lookup(const std::vector<int> &devs)
    {
        std::lock_guard<std::mutex> g(mu_);
        for (const auto &e : cache_)
            if (e->devs == devs) return e;
        auto e = std::make_shared<Entry>();
        e->devs = devs;
        e->comms.assign(devs.size(), Comm{});
        if (!B::init(e->comms.data(), (int)devs.size(), devs.data())) {
            e->comms.assign(devs.size(), Comm{});
            return nullptr;
        }
        cache_.push_back(e);
        return e;
    }

    std::mutex mu_;
    std::vector<std::shared_ptr<Entry>> cache_;
};

}  // namespace msim
