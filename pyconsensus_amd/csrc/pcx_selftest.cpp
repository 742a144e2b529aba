// pcx_selftest.cpp -- CPU self-tests of libpcx's host concurrency (pcx_sync.h) with fake work:
// no HIP, no RCCL.  Compiled into libpcx (exported as pcx_selftest_*, run by tests/test_abi.py)
// and, with the same sources, into tests/c/host_selftest.cpp's sanitizer builds
// (tests/test_sanitizers.py: -fsanitize=thread and -fsanitize=address,undefined).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pcx.h"
#include "pcx_sync.h"

namespace pcx {

namespace {
constexpr int ABORT_SELFTEST_WAIT_MS = 100;

struct FakeHandle {
    std::atomic<int> freed{0}, frees{0}, bad{0};
};

// mode 0: `users` threads exchange in a loop while `aborters` threads abort; a use that sees
// a freed handle, a use that succeeds after abort() returned, or a free count other than one
// is a violation.
int abort_race(int users, int aborters, int iters) {
    AbortOnce<FakeHandle*> a;
    FakeHandle f;
    a.h = &f;
    std::atomic<bool> go{false}, aborted_done{false};
    std::atomic<int> ok_after{0};
    std::vector<std::thread> th;
    for (int u = 0; u < users; u++)
        th.emplace_back([&] {
            while (!go) std::this_thread::yield();
            for (int i = 0; i < iters; i++) {
                const bool after = aborted_done;
                const int rc = a.use(
                    [&](FakeHandle* p) {
                        if (p->freed) p->bad++;  // the handle was freed while in use
                        return 0;
                    },
                    1);
                if (rc == 0 && after) ok_after++;  // a use that started after abort() returned succeeded
            }
        });
    for (int k = 0; k < aborters; k++)
        th.emplace_back([&, k] {
            while (!go) std::this_thread::yield();
            for (int i = 0; i < iters / 4 + k; i++) std::this_thread::yield();
            a.abort(
                [](FakeHandle* p) {
                    p->frees++;
                    p->freed = 1;
                },
                ABORT_SELFTEST_WAIT_MS);
            aborted_done = true;
        });
    go = true;
    for (auto& t : th) t.join();
    return (f.frees != 1) + f.bad + ok_after + a.overlaps;
}

// mode 1: one holder sits inside `use` for twice the abort's wait (an enqueue blocked in RCCL);
// `aborters` threads abort meanwhile.  Expected: every abort returns after about the wait (not
// after the holder), the handle is freed exactly once while the holder is still inside (one
// counted overlap -- the documented window), and every use attempted after that fails.
int abort_slow_holder(int users, int aborters) {
    AbortOnce<FakeHandle*> a;
    FakeHandle f;
    a.h = &f;
    std::atomic<bool> inside{false}, holder_done{false};
    std::atomic<int> ok_after{0}, violations{0};
    std::thread holder([&] {
        a.use(
            [&](FakeHandle*) {
                inside = true;
                std::this_thread::sleep_for(std::chrono::milliseconds(2 * ABORT_SELFTEST_WAIT_MS));
                return 0;
            },
            1);
        holder_done = true;
    });
    while (!inside) std::this_thread::yield();
    std::vector<std::thread> th;
    std::atomic<int> aborts_back{0};
    for (int k = 0; k < aborters; k++)
        th.emplace_back([&] {
            const auto t0 = std::chrono::steady_clock::now();
            a.abort(
                [](FakeHandle* p) {
                    p->frees++;
                    p->freed = 1;
                },
                ABORT_SELFTEST_WAIT_MS);
            const double ms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            // bounded: an abort must not wait for the blocked holder (2x the wait), only the wait itself
            if (ms > 1.8 * ABORT_SELFTEST_WAIT_MS) violations++;
            aborts_back++;
        });
    for (auto& t : th) t.join();
    // every abort has returned: later uses (users threads) must all fail, even while the holder is inside
    std::vector<std::thread> us;
    for (int u = 0; u < users; u++)
        us.emplace_back([&] {
            for (int i = 0; i < 100; i++)
                if (a.use([](FakeHandle*) { return 0; }, 1) == 0) ok_after++;
        });
    for (auto& t : us) t.join();
    holder.join();
    if (!holder_done) violations++;
    return (f.frees != 1) + (a.overlaps != 1) + ok_after + violations + (aborts_back != aborters);
}
}  // namespace

int selftest_abort_once(int users, int aborters, int iters, int mode) {
    if (users < 1 || aborters < 1 || iters < 1 || users + aborters > 256 || mode < 0 || mode > 1) return -1;
    return mode == 0 ? abort_race(users, aborters, iters) : abort_slow_holder(users, aborters);
}

int selftest_group_abort(int world, int steps, int fail_rank, int fail_step) {
    if (world < 1 || world > 256 || steps < 1 || fail_rank >= world || (fail_rank >= 0 && fail_step >= steps))
        return -1;
    pcx_group g;
    g.world = world;
    g.slot.resize(world);
    int violations = 0;
    // each rank writes its slot, meets the others, reads every slot (as GroupComm::allgather does)
    auto exchange_run = [&](int fr, int fs, std::vector<int>& passed) {
        passed.assign(world, 0);
        std::vector<std::atomic<int>> bad(world);
        std::vector<int> rcs;
        run_workers(
            world,
            [&](int k) -> int {
                for (int s = 0; s < steps; s++) {
                    if (k == fr && s == fs) return PCX_ENOMEM;  // this rank fails before the exchange
                    g.slot[k].assign(64, (char)(k + s));
                    if (!g.barrier()) return PCX_ECOMM;
                    for (int w = 0; w < world; w++)
                        if (g.slot[w].size() != 64 || g.slot[w][7] != (char)(w + s)) bad[k]++;
                    if (!g.barrier()) return PCX_ECOMM;
                    passed[k]++;
                }
                return 0;
            },
            [&](int) { g.abort(); }, rcs);
        int b = 0;
        for (int k = 0; k < world; k++) b += bad[k];
        return std::make_pair(rcs, b);
    };
    std::vector<int> passed;
    if (fail_rank >= 0) {
        auto r = exchange_run(fail_rank, fail_step, passed);
        violations += r.second;
        for (int k = 0; k < world; k++) {
            if (k == fail_rank) {
                violations += r.first[k] != PCX_ENOMEM;
            } else {
                // the others got through the steps before the failure and were then released
                violations += r.first[k] != (world > 1 ? PCX_ECOMM : 0);
                violations += passed[k] != fail_step;
            }
        }
        g.reset();  // every rank has been joined
    }
    auto r = exchange_run(-1, -1, passed);  // a clean run after the reset
    violations += r.second;
    for (int k = 0; k < world; k++) violations += (r.first[k] != 0) + (passed[k] != steps);
    return violations;
}

int selftest_rounds_sched(int K, int64_t B, int enomem_worker, int64_t fail_round) {
    if (K < 1 || K > 256 || B < 0 || B > (1 << 24) || enomem_worker >= K) return -1;
    std::vector<std::atomic<int>> ran(B);
    std::vector<std::atomic<int>> released(K);
    std::vector<char> faulted(K, 0);
    std::vector<int64_t> retry;
    std::string err;
    const int rc = schedule_rounds(
        K, B, PCX_ENOMEM,
        [&](int k, int64_t b, std::string& e) -> int {
            if (k == enomem_worker && !faulted[k]) {
                faulted[k] = 1;
                e = "fake ENOMEM";
                return PCX_ENOMEM;  // not run: handed back
            }
            if (b == fail_round) {
                e = "fake failure";
                return PCX_EHIP;
            }
            ran[b]++;
            if ((b * 7 + k) % 5 == 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
            return 0;
        },
        [&](int k) { released[k]++; }, retry, err);
    int violations = 0;
    // the faulting worker may have found no round left to take (the others were faster)
    const bool faulted_any = enomem_worker >= 0 && faulted[enomem_worker];
    if (faulted_any && K == 1) return violations + (rc != PCX_ENOMEM);  // no other worker: the batch fails
    const bool fail_handed_back = retry.size() == 1 && retry[0] == fail_round;  // faulted on that very round
    if (fail_round >= 0 && fail_round < B && !fail_handed_back) {
        violations += rc != PCX_EHIP;
        violations += err.find("round " + std::to_string(fail_round)) == std::string::npos;
        for (int64_t b = 0; b < B; b++) violations += ran[b] > 1;  // nothing runs twice
        return violations;
    }
    violations += rc != 0;
    for (int64_t b : retry) ran[b]++;  // the caller runs the handed-back rounds afterwards
    for (int64_t b = 0; b < B; b++) violations += ran[b] != 1;
    const bool expect_handback = faulted_any;
    for (int k = 0; k < K; k++) violations += released[k] != (expect_handback && k == enomem_worker ? 1 : 0);
    violations += (int64_t)retry.size() != (expect_handback ? 1 : 0);
    return violations;
}

int selftest_chunked_copy(int64_t bytes, int64_t chunk, int nslots, int T, int64_t fail_chunk) {
    if (bytes < 0 || bytes > (1ll << 30) || chunk < 1 || nslots < 1 || nslots > 8 || T < 1 || T > 64) return -1;
    std::vector<unsigned char> src((size_t)bytes), dst((size_t)bytes, 0), slots((size_t)(nslots * chunk));
    for (int64_t i = 0; i < bytes; i++) src[(size_t)i] = (unsigned char)(i * 131 + 7);
    const int64_t nchunks = (bytes + chunk - 1) / chunk;
    std::vector<std::atomic<int>> moved((size_t)nchunks);
    const int rc = chunked_copy(
        nchunks, nslots, T,
        [&](int64_t k, int slot) -> int {
            if (k == fail_chunk) return PCX_EHIP;
            if (k % 3 == 1) std::this_thread::sleep_for(std::chrono::microseconds(200));
            const int64_t len = std::min(chunk, bytes - k * chunk);
            std::memcpy(&slots[(size_t)(slot * chunk)], &src[(size_t)(k * chunk)], (size_t)len);
            return 0;
        },
        [&](int) { return 0; },
        [&](int64_t k, int slot, int t, int nt) {
            const int64_t len = std::min(chunk, bytes - k * chunk);
            const int64_t a = len * t / nt, b = len * (t + 1) / nt;
            if (b > a) std::memcpy(&dst[(size_t)(k * chunk + a)], &slots[(size_t)(slot * chunk + a)], (size_t)(b - a));
            moved[(size_t)k]++;
        });
    int violations = 0;
    if (fail_chunk >= 0 && fail_chunk < nchunks) {
        violations += rc != PCX_EHIP;
        for (int64_t k = fail_chunk; k < nchunks; k++) violations += moved[(size_t)k] != 0;  // nothing after the failure
        return violations;
    }
    violations += rc != 0;
    for (int64_t k = 0; k < nchunks; k++) violations += moved[(size_t)k] != T;
    violations += std::memcmp(src.data(), dst.data(), (size_t)bytes) != 0;
    return violations;
}

}  // namespace pcx
