// Persistent fork-join pool: see workpool.hpp.
#include "workpool.hpp"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace nodexa {

namespace {

thread_local bool t_in_worker = false;

// One fork-join call: the workers that wake for it keep a reference, so a worker that is slow to
// claim cannot take a part of the next call with this call's function and step.
struct Job {
    const std::function<void(size_t, size_t)>* fn;
    size_t n, step, parts;
    std::atomic<size_t> next{1};     // part 0 is the caller's
    std::atomic<size_t> pending{0};  // parts not finished yet
    std::mutex mu;
    std::condition_variable done;
    std::exception_ptr error;  // the first exception a part threw (rethrown on the caller)

    void fail(std::exception_ptr e) {
        std::lock_guard<std::mutex> g(mu);
        if (!error) error = e;
    }

    void work() {
        for (size_t p; (p = next.fetch_add(1, std::memory_order_relaxed)) < parts;) {
            try {
                (*fn)(p * step, std::min(n, (p + 1) * step));
            } catch (...) {
                fail(std::current_exception());  // the part still counts as finished
            }
            if (pending.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> g(mu);
                done.notify_all();
            }
        }
    }
};

class Pool {
public:
    Pool() : size_(std::min<size_t>(16, std::max(1u, std::thread::hardware_concurrency()))) {}
    size_t size() const { return size_; }

    void run(size_t n, const std::function<void(size_t, size_t)>& fn, size_t min_chunk, size_t max_threads) {
        size_t parts = std::min(max_threads ? std::min(max_threads, size_) : size_,
                                (n + std::max<size_t>(1, min_chunk) - 1) / std::max<size_t>(1, min_chunk));
        if (parts <= 1 || t_in_worker) {
            if (n) fn(0, n);
            return;
        }
        std::lock_guard<std::mutex> one(call_mu_);  // one fork-join at a time
        start_workers();
        auto job = std::make_shared<Job>();
        job->fn = &fn;
        job->n = n;
        job->step = (n + parts - 1) / parts;
        job->parts = (n + job->step - 1) / job->step;
        job->pending.store(job->parts - 1, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = job;
            ++gen_;
        }
        cv_.notify_all();
        try {
            fn(0, std::min(n, job->step));
        } catch (...) {
            job->fail(std::current_exception());
        }
        job->work();  // the caller helps with the parts no worker has claimed yet
        {
            // every part has returned before `fn` (the caller's) can go out of scope
            std::unique_lock<std::mutex> g(job->mu);
            job->done.wait(g, [&] { return job->pending.load(std::memory_order_acquire) == 0; });
        }
        {
            std::lock_guard<std::mutex> g2(mu_);
            job_.reset();
        }
        if (job->error) std::rethrow_exception(job->error);
    }

private:
    void start_workers() {
        if (!threads_.empty()) return;
        for (size_t i = 1; i < size_; ++i) threads_.emplace_back([this] { loop(); });
        for (auto& t : threads_) t.detach();  // parked forever; the process exits around them
    }

    void loop() {
        t_in_worker = true;
        size_t seen = 0;
        for (;;) {
            std::shared_ptr<Job> job;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen && job_ != nullptr; });
                seen = gen_;
                job = job_;
            }
            job->work();
        }
    }

    const size_t size_;
    std::vector<std::thread> threads_;
    std::mutex call_mu_, mu_;
    std::condition_variable cv_;
    std::shared_ptr<Job> job_;
    size_t gen_ = 0;
};

Pool& pool() {
    static Pool* p = new Pool();  // never destroyed: workers may outlive static destruction order
    return *p;
}

}  // namespace

void parallel_for_range(size_t n, const std::function<void(size_t, size_t)>& fn, size_t min_chunk,
                        size_t max_threads) {
    pool().run(n, fn, min_chunk, max_threads);
}

size_t workpool_size() { return pool().size(); }

}  // namespace nodexa
