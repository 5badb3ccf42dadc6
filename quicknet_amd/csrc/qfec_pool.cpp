// qfec_pool.cpp -- host thread pool for the copies around the device (qfec_pool.hpp).
#include "qfec_pool.hpp"

#include <sched.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

namespace qfec {

HostPool::HostPool(int nthreads) {
    for (int i = 1; i < nthreads; ++i) workers_.emplace_back([this, i] { loop(i); });
}

HostPool::~HostPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_job_.notify_all();
    for (auto& t : workers_) t.join();
}

void HostPool::loop(int id) {
    unsigned long long seen = 0;
    for (;;) {
        const std::function<void(int, int)>* job;
        int nt;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_job_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            job = job_;
            nt = nt_;
        }
        std::exception_ptr e;
        if (id < nt) {
            try {
                (*job)(id, nt);
            } catch (...) {
                e = std::current_exception();
            }
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (e && !err_) err_ = e;
            if (--pending_ == 0) cv_done_.notify_one();
        }
    }
}

void HostPool::run(const std::function<void(int, int)>& fn, int parts) {
    const int nt = std::max(1, std::min(threads(), parts));
    if (nt == 1 || workers_.empty()) {
        fn(0, 1);
        return;
    }
    std::lock_guard<std::mutex> one(run_mu_);
    {
        std::lock_guard<std::mutex> lk(mu_);
        job_ = &fn;
        nt_ = nt;
        pending_ = (int)workers_.size();
        err_ = nullptr;
        ++gen_;
    }
    cv_job_.notify_all();
    std::exception_ptr mine;
    try {
        fn(0, nt);
    } catch (...) {
        mine = std::current_exception();
    }
    std::unique_lock<std::mutex> lk(mu_);
    cv_done_.wait(lk, [&] { return pending_ == 0; });  // every worker is done with fn
    job_ = nullptr;
    std::exception_ptr e = mine ? mine : err_;
    err_ = nullptr;
    lk.unlock();
    if (e) std::rethrow_exception(e);
}

static int read_int_file(const char* path, long long* a, long long* b) {
    FILE* f = fopen(path, "r");
    if (!f) return 0;
    char buf[128] = {0};
    const bool ok = fgets(buf, sizeof buf, f) != nullptr;
    fclose(f);
    if (!ok) return 0;
    if (!strncmp(buf, "max", 3)) return -1;  // cgroup v2: no quota
    return sscanf(buf, "%lld %lld", a, b);
}

int usable_cpus() {
    int n = 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = std::max(1, CPU_COUNT(&set));
    long long q = 0, p = 0;
    if (read_int_file("/sys/fs/cgroup/cpu.max", &q, &p) == 2 && q > 0 && p > 0) {
        n = std::min<long long>(n, std::max<long long>(1, (q + p - 1) / p));
    } else {
        long long q1 = 0, p1 = 0, d = 0;
        if (read_int_file("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", &q1, &d) >= 1 && q1 > 0 &&
            read_int_file("/sys/fs/cgroup/cpu/cpu.cfs_period_us", &p1, &d) >= 1 && p1 > 0)
            n = std::min<long long>(n, std::max<long long>(1, (q1 + p1 - 1) / p1));
    }
    return n;
}

}  // namespace qfec
