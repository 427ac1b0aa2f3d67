// pool.cpp -- WorkerPool (pool.h).
#include "pool.h"

namespace opk {

WorkerPool::WorkerPool(int workers)
{
    for (int w = 1; w < workers; ++w) threads_.emplace_back([this, w] { loop(w); });
}

WorkerPool::~WorkerPool()
{
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    start_.notify_all();
    for (auto& t : threads_) t.join();
}

void WorkerPool::work(int worker)
{
    for (int t = next_.fetch_add(1); t < tasks_; t = next_.fetch_add(1)) {
        try {
            (*fn_)(t, worker);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu_);
            if (!error_) error_ = std::current_exception();
        }
    }
}

void WorkerPool::loop(int worker)
{
    unsigned seen = 0;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu_);
            start_.wait(lk, [&] { return stop_ || generation_ != seen; });
            if (stop_) return;
            seen = generation_;
        }
        work(worker);
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (--busy_ == 0) done_.notify_one();
        }
    }
}

void WorkerPool::run(int tasks, const std::function<void(int, int)>& fn)
{
    if (tasks <= 0) return;
    if (threads_.empty() || tasks == 1) {
        for (int t = 0; t < tasks; ++t) fn(t, 0);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(mu_);
        fn_ = &fn;
        tasks_ = tasks;
        next_.store(0);
        error_ = nullptr;
        busy_ = (int)threads_.size();
        ++generation_;
    }
    start_.notify_all();
    work(0);
    std::exception_ptr err;
    {
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return busy_ == 0; });
        err = error_;
        fn_ = nullptr;
    }
    if (err) std::rethrow_exception(err);
}

}  // namespace opk
