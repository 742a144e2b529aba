// host_selftest.cpp -- libpcx's host concurrency (csrc/pcx_sync.h: the virtual-rank group
// barrier and abort, the RCCL handle's abort-once, the per-device worker release and the round
// scheduler) driven by csrc/pcx_selftest.cpp, built from the same sources WITHOUT HIP or RCCL so
// that it runs under ThreadSanitizer and AddressSanitizer + UBSan on the CPU
// (tests/test_sanitizers.py).  Exit status 0 = every self-test reported no violation.
#include <cstdio>
#include <cstdlib>

#include "../../pyconsensus_amd/csrc/pcx_sync.h"

namespace {
int failures = 0;

void expect(const char* what, int violations) {
    if (violations != 0) {
        std::printf("FAIL %s: %d violation(s)\n", what, violations);
        failures++;
    } else {
        std::printf("ok   %s\n", what);
    }
}
}  // namespace

int main(int argc, char** argv) {
    std::setvbuf(stdout, nullptr, _IOLBF, 0);  // (a hang shows its last self-test)
    const int scale = argc > 1 ? std::atoi(argv[1]) : 1;  // iterations multiplier
    char name[128];
    // AbortOnce: users racing aborters, then one holder blocked past the abort's wait
    for (int users : {1, 4, 8})
        for (int aborters : {1, 3}) {
            std::snprintf(name, sizeof name, "abort_once race users=%d aborters=%d", users, aborters);
            expect(name, pcx::selftest_abort_once(users, aborters, 2000 * scale, 0));
        }
    expect("abort_once slow holder users=4 aborters=3", pcx::selftest_abort_once(4, 3, 1, 1));
    // group barrier / abort / reset through run_workers, every failing rank and step
    for (int world : {1, 2, 3, 8})
        for (int fr = -1; fr < world; fr++)
            for (int fs : {0, 3}) {
                std::snprintf(name, sizeof name, "group world=%d fail_rank=%d fail_step=%d", world, fr, fs);
                expect(name, pcx::selftest_group_abort(world, 5 * scale, fr, fr < 0 ? -1 : fs));
            }
    // round scheduler: plain, ENOMEM hand-back by several workers, a hard failure
    for (int K : {1, 3, 16})
        for (int enw : {-1, 0, 2}) {
            if (enw >= K) continue;
            for (long fail : {-1L, 5L}) {
                std::snprintf(name, sizeof name, "rounds K=%d B=%d enomem_worker=%d fail_round=%ld", K, 64 * scale, enw,
                              fail);
                expect(name, pcx::selftest_rounds_sched(K, 64 * scale, enw, fail));
            }
        }
    // the staged large copy of the host-memory path (chunked_copy): slots, threads, ragged tail, failure
    for (int slots : {1, 2, 3})
        for (int T : {1, 4, 16}) {
            std::snprintf(name, sizeof name, "chunked_copy slots=%d T=%d", slots, T);
            expect(name, pcx::selftest_chunked_copy(1000003 * scale, 65536, slots, T, -1));
        }
    expect("chunked_copy failure at chunk 5", pcx::selftest_chunked_copy(1 << 20, 65536, 2, 8, 5));
    expect("chunked_copy failure at chunk 0", pcx::selftest_chunked_copy(1 << 20, 65536, 2, 8, 0));
    std::printf("%s (%d failure(s))\n", failures ? "FAILED" : "PASSED", failures);
    return failures ? 1 : 0;
}
