// qfec_pool.hpp -- a small fixed pool of host threads for the byte copies around the device
// (gathering caller rows into pinned staging and scattering results back, module/rs.h on host
// pointer arrays).  One job at a time: run(fn) calls fn(t, nt) for t = 0 .. nt-1 on the pool's
// threads and the caller (t = 0) and returns when every part is done.
#pragma once

#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace qfec {

class HostPool {
public:
    explicit HostPool(int nthreads);
    ~HostPool();
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;

    int threads() const { return (int)workers_.size() + 1; }
    // fn(t, nt) for t in [0, nt); nt = min(threads(), max(1, parts)).  Serialised between callers:
    // concurrent module/rs.h calls, on one device or several, run their copy phases one after
    // another (each phase already uses every thread of the process's CPU share).  An exception
    // thrown by any part is rethrown here once every part has finished, so no worker is left
    // holding `fn`.
    void run(const std::function<void(int, int)>& fn, int parts = 1 << 30);

private:
    void loop(int id);
    std::vector<std::thread> workers_;
    std::mutex run_mu_;  // one job at a time
    std::mutex mu_;
    std::condition_variable cv_job_, cv_done_;
    const std::function<void(int, int)>* job_ = nullptr;
    int nt_ = 0;
    unsigned long long gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
    std::exception_ptr err_;  // the first exception a part of the current job threw
};

// CPUs this process may actually use: the affinity mask, capped by a cgroup CPU quota
// (cgroup v2 cpu.max or v1 cpu.cfs_quota_us / cpu.cfs_period_us)
int usable_cpus();

// the process-wide pool of libqfec's module/rs.h host paths (defined in qfec_runtime.cpp), created
// on first use with tuning "host_threads" threads (0: usable_cpus(), at most 32) and re-created
// when that knob changes; callers keep the returned reference while they use it
std::shared_ptr<HostPool> host_pool();

}  // namespace qfec
