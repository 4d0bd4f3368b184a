// Timed multi-thread sweeps for the oracle's CPU baselines (TEST
// INFRASTRUCTURE / CPU BASELINE ONLY).  The n items are cut into T slices
// [n s / T, n (s + 1) / T); threads are spawned once and sweep until
// min_seconds have passed (at least once), thread t taking slice (t + i) % T
// in its i-th sweep -- so a thread never re-walks the slice its own caches
// hold from the previous sweep (a small sample would otherwise be timed from
// L1/L2).  body(s, begin, end) gets the slice index.  Returns the items
// processed / n (fractional sweeps); *seconds = wall time until the last
// thread finished.
#pragma once
#include <stddef.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

namespace oracle {

template <class F>
double timed_sweeps(size_t n, int threads, double min_seconds, double* seconds, F&& body) {
    if (threads < 1) threads = 1;
    if (n == 0) {
        if (seconds) *seconds = 0;
        return 0;
    }
    std::vector<size_t> done(threads, 0);
    const auto t0 = std::chrono::steady_clock::now();
    auto run = [&](int t) {
        size_t i = 0;
        do {
            const int sl = (int)((t + i++) % (size_t)threads);
            const size_t b = n * sl / threads, e = n * (sl + 1) / threads;
            body(sl, b, e);
            done[t] += e - b;
        } while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < min_seconds);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; t++) th.emplace_back(run, t);
    run(0);
    for (auto& x : th) x.join();
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    size_t tot = 0;
    for (size_t d : done) tot += d;
    return (double)tot / (double)n;
}

}  // namespace oracle
