// sm_host_pool.h — persistent host worker threads of a context (the NL tree builds, sm_capi.cpp).
// Item b of a job always runs on worker b % size, so a pair's host data (its tree and scratch)
// stays with one thread across calls instead of moving with freshly spawned threads.
#pragma once
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sm {

class HostPool {
public:
    explicit HostPool(int nth) : nth_(nth) {
        for (int t = 0; t < nth; t++) th_.emplace_back([this, t] { worker(t); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& x : th_) x.join();
    }
    int size() const { return nth_; }
    // runs f(0 .. n-1) on the workers and returns when every item is done; false if any item
    // threw (e.g. std::bad_alloc from a resize): the exception stays on its worker, which goes on
    // with its next item, and the caller reports a status instead of the process terminating
    bool run(int n, const std::function<void(int)>& f) {
        std::unique_lock<std::mutex> g(m_);
        job_ = &f;
        n_ = n;
        pending_ = nth_;
        failed_ = false;
        gen_++;
        cv_.notify_all();
        done_.wait(g, [this] { return pending_ == 0; });
        job_ = nullptr;
        return !failed_;
    }

private:
    void worker(int t) {
        long seen = 0;
        for (;;) {
            const std::function<void(int)>* f;
            int n;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                f = job_;
                n = n_;
            }
            bool bad = false;
            for (int b = t; b < n; b += nth_) {
                try {
                    (*f)(b);
                } catch (...) {
                    bad = true;
                }
            }
            {
                std::lock_guard<std::mutex> g(m_);
                failed_ = failed_ || bad;
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    const int nth_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int n_ = 0, pending_ = 0;
    long gen_ = 0;
    bool stop_ = false;
    bool failed_ = false;
};

}  // namespace sm
