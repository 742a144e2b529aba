"""Throughput of batched_round_kernel against resident rounds per CU (diagnostic).

Pads the kernel's dynamic LDS (PCX_BATCHED_LDS_PAD, read once per process) so that
at most k rounds fit one CU's 160 KiB, for k = 10 (unpadded) down to 6, and times the
C3 launch (65,536 50x20 rounds) with HIP events.  If time scales like 1/k the kernel is
latency bound and more resident rounds (less LDS / fewer VGPRs per round) pay off.

    gpurun -- 'python tools/occupancy_batched.py'
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LDS_CU = 160 * 1024


def child():
    sys.path.insert(0, ROOT)
    import torch

    from pyconsensus_amd import synthetic
    from pyconsensus_amd.batched import consensus_batched

    dev = torch.device("cuda:0")
    R, sc, lo, hi, rep = synthetic.rounds(65536, 50, 20, seed=20261015)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt).to(dev)
    args = (t(R), t(rep), t(sc, torch.uint8), t(lo), t(hi))
    for _ in range(2):
        consensus_batched(*args, device=dev)
    torch.cuda.synchronize(dev)
    s = torch.cuda.current_stream(dev)
    ms = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        consensus_batched(*args, device=dev)
        e1.record(s)
        torch.cuda.synchronize(dev)
        ms.append(e0.elapsed_time(e1))
    print("%.4f" % min(ms))


def main():
    # batched_lds_bytes(50, 20, PCA): smem_doubles() in pcx_batched.hip -- F [50][21], packed C
    # (210), M (the median scratch, 239), rep, five event vectors
    base = 8 * (50 * 21 + 210 + 239 + 50 + 5 * 20)
    for k in (12, 10, 9, 8, 6):
        pad = max(0, LDS_CU // k - base - 256) if k < LDS_CU // base else 0
        env = dict(os.environ, PCX_BATCHED_LDS_PAD=str(pad))
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                           timeout=300)
        if r.returncode != 0:
            print("k=%d failed rc=%d\n%s" % (k, r.returncode, r.stderr[-2000:]))
            return 1
        ms = float(r.stdout.strip().splitlines()[-1])
        print("rounds/CU<=%d  lds/round=%6d B  kernel %.3f ms  %.2fM rounds/s" % (k, base + pad, ms,
                                                                             65536 / ms / 1e3), flush=True)
    return 0


if __name__ == "__main__":
    if "--child" in sys.argv:
        child()
    else:
        sys.exit(main())
