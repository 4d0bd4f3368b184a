// A context's persistent host worker threads: run(T, f) calls f(0 .. T-1), the
// caller itself running f(0), and returns when all have finished.  Replaces a
// thread spawn per call on the per-batch host paths (store submit, host
// encoders), where spawning 16 threads costs as much as the work it splits.
#pragma once
#include <stdint.h>

#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace gd {

class WorkerPool {
   public:
    explicit WorkerPool(uint32_t n) {
        for (uint32_t t = 1; t < n; t++) th_.emplace_back([this, t] { loop(t); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& x : th_) x.join();
    }
    uint32_t size() const { return (uint32_t)th_.size() + 1; }
    // f(t) for t in [0, T); T is clamped to size()
    void run(uint32_t T, const std::function<void(uint32_t)>& f) {
        T = T < 1 ? 1 : (T > size() ? size() : T);
        if (T == 1) {
            f(0);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &f;
            T_ = T;
            left_ = T - 1;
            gen_++;
            worker_ex_ = nullptr;
        }
        cv_.notify_all();
        std::exception_ptr ex;
        try {
            f(0);
        } catch (...) {
            ex = std::current_exception();  // the workers still read f: wait for them first
        }
        {
            std::unique_lock<std::mutex> g(m_);
            done_.wait(g, [&] { return left_ == 0; });
            job_ = nullptr;
            if (!ex) ex = worker_ex_;  // a worker's exception (e.g. std::bad_alloc) reaches the caller too
            worker_ex_ = nullptr;
        }
        if (ex) std::rethrow_exception(ex);
    }

   private:
    void loop(uint32_t t) {
        uint64_t seen = 0;
        while (true) {
            const std::function<void(uint32_t)>* job;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (t >= T_) continue;  // not part of this run
                job = job_;
            }
            std::exception_ptr ex;
            try {
                (*job)(t);
            } catch (...) {
                ex = std::current_exception();  // never leaves the thread (std::terminate): run() rethrows it
            }
            std::lock_guard<std::mutex> g(m_);
            if (ex && !worker_ex_) worker_ex_ = ex;
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(uint32_t)>* job_ = nullptr;
    uint32_t T_ = 0, left_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
    std::exception_ptr worker_ex_;  // the first exception a worker thread threw in the current run
};

}  // namespace gd
