// pcx_sync.h -- the host-side concurrency of libpcx, in plain C++17 (no HIP, no RCCL), so
// that the same code runs in the library and in the sanitizer builds of the CPU suite
// (tests/c/host_selftest.cpp under -fsanitize=thread and -fsanitize=address,undefined):
//
//   * pcx_group         the barrier + abort of virtual ranks exchanging through host memory
//                       (pcx_comm.cpp GroupComm, pcx_create_grouped / pcx_create_devices);
//   * AbortOnce         a communicator handle many threads use and any may abort (RcclComm);
//   * run_workers       one thread per rank, the first failure releases the others
//                       (pcx_api.cpp run_devices);
//   * schedule_rounds   the round scheduler's hand-out / ENOMEM hand-back (pcx_rounds.cpp).
//
// The self-tests that drive them with fake work live in pcx_selftest.cpp.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

struct pcx_group {
    int world = 1;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t generation = 0;
    std::vector<std::vector<char>> slot;  // per rank host staging
    std::vector<char> result;             // reduced data (written by the last arriver)

    bool aborted = false;                 // a rank failed: every waiting and later exchange fails

    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return false;
        const int64_t g = generation;
        if (++arrived == world) {
            arrived = 0;
            generation++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != g || aborted; });
        }
        // a barrier every rank reached counts as passed even when an abort follows before this
        // rank wakes (it saw the others' data); only a barrier left incomplete fails
        return generation != g;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
    // clear an abort once no rank is inside an exchange (the caller has joined every rank)
    void reset() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = false;
        arrived = 0;
    }
};

namespace pcx {

// A communicator handle that many threads use and any of them may abort: `use` loads the
// handle and runs the enqueue under `mu`; `abort` marks the handle dead (later uses fail),
// waits up to `wait_ms` for a use in progress, then swaps the handle out and frees it exactly
// once, whatever the number of callers.
//
// When the wait succeeds, no handle is freed between another thread's load and its enqueue.
// When it times out -- a use blocked inside RCCL on a peer that failed (lazy connection
// set-up), which is exactly what ncclCommAbort exists to interrupt -- the free DOES overlap
// that use: the blocked thread is still inside the library call on the handle being aborted.
// RCCL's abort is designed to interrupt such a call, but the overlap is real and deliberate;
// the alternative (waiting for the use) can hang forever.  `dead` still fails every use that
// had not taken `mu` yet, and `overlaps` counts the timed-out frees (pcx_selftest_abort_once's
// slow-holder mode checks both).
template <class H>
struct AbortOnce {
    std::atomic<H> h{H{}};
    std::atomic<bool> dead{false};
    std::atomic<int> overlaps{0};
    // `busy` (under `mu`) marks a use in progress; uses run one at a time, as the enqueues of one
    // communicator must.  (A condition variable with a system_clock deadline rather than a timed
    // mutex or a steady_clock wait: libstdc++ maps those to pthread_mutex_clocklock /
    // pthread_cond_clockwait, which GCC 11's ThreadSanitizer does not intercept, so the sanitizer
    // build could not check this code.  A wall-clock jump only stretches or shortens the wait.)
    std::mutex mu;
    std::condition_variable cv;
    bool busy = false;
    template <class F>
    int use(F&& f, int gone_rc) {
        H c;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return !busy; });
            c = h.load();
            if (c == H{} || dead) return gone_rc;
            busy = true;
        }
        const int rc = f(c);
        {
            std::lock_guard<std::mutex> lk(mu);
            busy = false;
        }
        cv.notify_all();
        return rc;
    }
    template <class F>
    void abort(F&& free_fn, int wait_ms) {
        std::unique_lock<std::mutex> lk(mu);
        dead = true;  // uses that have not started yet fail from here on
        const auto deadline = std::chrono::system_clock::now() + std::chrono::milliseconds(wait_ms);
        const bool idle = cv.wait_until(lk, deadline, [&] { return !busy; });
        if (H c = h.exchange(H{})) {
            if (!idle) overlaps++;
            free_fn(c);
        }
    }
};

// One thread per rank k running work(k) -> status (0 = ok).  The first rank that fails calls
// release(k) once -- it aborts every other rank's exchange, so ranks blocked waiting on the
// failed one return instead of hanging -- and later failures do nothing.  Every thread is
// joined before this returns; rcs[k] holds each rank's status.
template <class Work, class Release>
void run_workers(int n, Work&& work, Release&& release, std::vector<int>& rcs) {
    rcs.assign(n, 0);
    std::atomic<bool> aborting{false};
    std::vector<std::thread> th;
    th.reserve(n);
    for (int k = 0; k < n; k++)
        th.emplace_back([&, k] {
            rcs[k] = work(k);
            if (rcs[k] && !aborting.exchange(true)) release(k);
        });
    for (auto& t : th) t.join();
}

// Rounds [0, B) handed to K worker threads by an atomic counter; run(k, b, err) -> status.
// A worker whose round returns `enomem` while another worker is still alive calls
// release(k) (frees its workspace), hands the round back and leaves: fewer rounds run in
// flight instead of the batch failing.  Any other failure stops the hand-out; the first failing
// worker's status and message are returned.  On success `retry` holds the handed-back rounds
// (the caller runs them afterwards on a worker whose workspace is resident).
template <class Run, class Release>
int schedule_rounds(int K, int64_t B, int enomem, Run&& run, Release&& release, std::vector<int64_t>& retry,
                    std::string& err) {
    std::atomic<int64_t> next{0};
    std::atomic<int> failed{0};
    std::atomic<int> alive{K};
    std::vector<std::string> errs(K);
    std::vector<int> rcs(K, 0);
    std::mutex retry_mu;
    auto worker = [&](int k) {
        for (;;) {
            const int64_t b = next.fetch_add(1);
            if (b >= B || failed.load()) return;
            const int rc = run(k, b, errs[k]);
            if (rc == enomem && alive.fetch_sub(1) > 1) {
                release(k);
                std::lock_guard<std::mutex> lk(retry_mu);
                retry.push_back(b);
                errs[k].clear();
                return;
            }
            if (rc) {
                rcs[k] = rc;
                errs[k] = "round " + std::to_string(b) + ": " + errs[k];
                failed.store(1);
                return;
            }
        }
    };
    std::vector<std::thread> th;
    th.reserve(K);
    for (int k = 0; k < K; k++) th.emplace_back(worker, k);
    for (auto& t : th) t.join();
    for (int k = 0; k < K; k++)
        if (rcs[k]) {
            err = errs[k];
            return rcs[k];
        }
    return 0;
}

// A large copy through `nslots` staging slots: the main thread issues chunk k's transfer into slot
// k % nslots (issue(k, slot), e.g. a DMA into pinned memory) as soon as that slot's previous chunk
// has been moved out; T worker threads wait for the chunk (wait(slot)) and each move their share
// out of the slot (part(k, slot, t, T), e.g. a memcpy into pageable memory, whose first-touch page
// faults then spread over T threads).  Returns 0, or the first non-zero status of issue / wait
// (the copy then stops; every thread is joined before the return).
template <class Issue, class Wait, class Part>
int chunked_copy(int64_t nchunks, int nslots, int T, Issue&& issue, Wait&& wait, Part&& part) {
    std::mutex mu;
    std::condition_variable cv;
    int64_t issued = -1;                        // last chunk issued (under mu)
    std::vector<int64_t> consumed(nslots, -1);  // last chunk moved out of each slot (under mu)
    std::vector<int> left(nslots, 0);           // workers still moving the slot's chunk (under mu)
    std::atomic<int> rc{0};
    std::vector<std::thread> th;
    th.reserve(T);
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            for (int64_t k = 0; k < nchunks; k++) {
                const int slot = (int)(k % nslots);
                {
                    std::unique_lock<std::mutex> lk(mu);
                    // (every chunk is marked issued, also after a failure -- a worker must not run
                    // ahead of that: its count on the slot would precede the slot's reset)
                    cv.wait(lk, [&] { return issued >= k; });
                }
                if (rc.load() == 0) {
                    const int w = wait(slot);
                    if (w) {
                        int z = 0;
                        rc.compare_exchange_strong(z, w);
                    } else {
                        part(k, slot, t, T);
                    }
                }
                std::lock_guard<std::mutex> lk(mu);
                if (--left[slot] == 0) {
                    consumed[slot] = k;
                    cv.notify_all();
                }
            }
        });
    for (int64_t k = 0; k < nchunks; k++) {
        const int slot = (int)(k % nslots);
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return consumed[slot] >= k - nslots; });
        }
        const int r = rc.load() == 0 ? issue(k, slot) : 1;
        std::lock_guard<std::mutex> lk(mu);
        if (r) {
            int z = 0;
            rc.compare_exchange_strong(z, r);
        }
        left[slot] = T;
        issued = k;
        cv.notify_all();
    }
    for (auto& t : th) t.join();
    return rc.load();
}

// CPU self-tests (pcx_selftest.cpp); each returns the number of violations, -1 on bad arguments.
// mode 0: users race aborters on a fast handle; mode 1: one user holds the handle longer than
// the abort's wait (the timed-out path)
int selftest_abort_once(int users, int aborters, int iters, int mode = 0);
// `world` ranks run `steps` group barriers; rank `fail_rank` fails at step `fail_step` (-1: none)
// and releases the others through run_workers + pcx_group::abort; then reset, and a clean run
int selftest_group_abort(int world, int steps, int fail_rank, int fail_step);
// K workers, B rounds; worker `enomem_worker` reports ENOMEM on its first round (-1: none),
// round `fail_round` fails hard (-1: none)
int selftest_rounds_sched(int K, int64_t B, int enomem_worker, int64_t fail_round);
// chunked_copy of `bytes` through `nslots` slots of `chunk` bytes by T threads (memcpy as the
// transfer, a slow `issue` every 3rd chunk); chunk `fail_chunk`'s issue fails (-1: none)
int selftest_chunked_copy(int64_t bytes, int64_t chunk, int nslots, int T, int64_t fail_chunk);

}  // namespace pcx
