// pool.h -- a fixed set of host worker threads for the per-frame people assembly (product code).
//
// The reference assembles each frame's people on the thread that runs its pose extractor
// (connectBodyPartsGpu, one frame at a time per GPU worker, wrapper/wrapperAuxiliary.hpp); here a
// batch's frames are independent tasks spread over the pool's threads, which live as long as the
// PoseHip that owns them (no thread start-up per batch).
#pragma once
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace opk {

class WorkerPool {
public:
    // `workers` threads of work in total: the caller of run() is worker 0, workers - 1 are started
    explicit WorkerPool(int workers);
    ~WorkerPool();
    WorkerPool(const WorkerPool&) = delete;
    WorkerPool& operator=(const WorkerPool&) = delete;

    int workers() const { return (int)threads_.size() + 1; }
    // fn(task, worker) for every task in [0, tasks), each exactly once, tasks handed out in order
    // to whichever worker is free; returns when all are done and rethrows the first exception
    // (the other tasks still run).  One run() at a time per pool.
    void run(int tasks, const std::function<void(int, int)>& fn);

private:
    void loop(int worker);
    void work(int worker);

    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable start_, done_;
    const std::function<void(int, int)>* fn_ = nullptr;
    int tasks_ = 0;
    unsigned generation_ = 0;
    int busy_ = 0;            // started workers still inside the current generation
    bool stop_ = false;
    std::atomic<int> next_{0};
    std::exception_ptr error_;
};

}  // namespace opk
