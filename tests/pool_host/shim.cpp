// tests/pool_host/shim.cpp -- TEST INFRASTRUCTURE ONLY: quicknet_amd/csrc/qfec_pool.cpp (the host
// thread pool of the module/rs.h host paths and of qfec_zfec's session machines) driven from
// tests/test_host_pool.py on CPU.  Never shipped.
#include <atomic>
#include <chrono>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../../quicknet_amd/csrc/qfec_pool.hpp"

extern "C" {
int pool_usable_cpus(void) { return qfec::usable_cpus(); }

// a pool of `threads`; `jobs` runs of fn(t, nt) over `parts` parts from `callers` threads at once;
// counts[t] += 1 per part index seen, and each run's nt must be min(threads, max(1, parts)).
// Returns the number of runs whose parts were not each seen exactly once (0 = all good).
int pool_check(int threads, int parts, int jobs, int callers, long long* calls_out) {
    qfec::HostPool pool(threads);
    std::atomic<int> bad{0};
    std::atomic<long long> calls{0};
    auto caller = [&]() {
        for (int j = 0; j < jobs; ++j) {
            const int want = std::min(pool.threads(), std::max(1, parts));
            std::vector<std::atomic<int>> seen(want);
            for (auto& s : seen) s = 0;
            std::atomic<int> wrong_nt{0};
            pool.run(
                [&](int t, int nt) {
                    if (nt != want || t < 0 || t >= nt) {
                        wrong_nt++;
                        return;
                    }
                    seen[t]++;
                    calls++;
                },
                parts);
            int ok = wrong_nt == 0;
            for (auto& s : seen) ok &= s == 1;
            if (!ok) bad++;
        }
    };
    std::vector<std::thread> th;
    for (int c = 0; c < callers; ++c) th.emplace_back(caller);
    for (auto& t : th) t.join();
    *calls_out = calls.load();
    return bad.load();
}

// part `thrower` of each job throws; run() must rethrow it only after every other part has returned
// (a part sleeps first, so a run() that returned early would be seen).  Returns the number of jobs
// that did not rethrow, or rethrew before all parts were done; then checks the pool still works.
int pool_throw_check(int threads, int thrower, int jobs) {
    qfec::HostPool pool(threads);
    int bad = 0;
    for (int j = 0; j < jobs; ++j) {
        std::atomic<int> done{0};
        int nt_seen = 0;
        bool threw = false;
        try {
            pool.run([&](int t, int nt) {
                if (t == 0) nt_seen = nt;
                if (t == thrower % nt) throw std::runtime_error("part failed");
                std::this_thread::sleep_for(std::chrono::milliseconds(2));
                done++;
            });
        } catch (const std::runtime_error&) {
            threw = true;
        }
        if (!threw || done.load() != nt_seen - 1) bad++;
    }
    std::atomic<int> after{0};
    pool.run([&](int, int) { after++; });
    if (after.load() != pool.threads()) bad++;
    return bad;
}
}
