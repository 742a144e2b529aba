"""Where a single-matrix consensus spends its wall time between kernels: from a rocprofv3
kernel trace (kt_kernel_trace.csv), split the trace into consensus calls (each starts with
k_rep_* -- the M_REPUTATION stage), and for the chosen call report the span, the summed kernel
time, the idle gaps above a threshold with the kernels around them, and the short launches.

usage: python tools/trace_gaps.py TRACE.csv [call_index=-1] [gap_us=15]
"""
import csv
import sys


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("pcx::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0][:60]))
    rows.sort()
    return rows


def calls(rows):
    out, cur = [], []
    for r in rows:
        if r[2].startswith("k_rep_") and cur and not cur[-1][2].startswith("k_rep_"):
            out.append(cur)
            cur = []
        cur.append(r)
    if cur:
        out.append(cur)
    return [c for c in out if any(k[2].startswith("k_rep_") for k in c)]


def main():
    path = sys.argv[1]
    idx = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    thr = float(sys.argv[3]) if len(sys.argv) > 3 else 15.0
    cs = calls(load(path))
    c = cs[idx]
    t0, t1 = c[0][0], max(r[1] for r in c)
    busy = sum(r[1] - r[0] for r in c)
    print("calls in trace: %d; call %d: %d launches, span %.3f ms, kernel time %.3f ms, idle %.3f ms"
          % (len(cs), idx, len(c), (t1 - t0) / 1e6, busy / 1e6, (t1 - t0 - busy) / 1e6))
    gaps = []
    end = c[0][1]
    for i in range(1, len(c)):
        g = (c[i][0] - end) / 1e3
        if g > thr:
            gaps.append((g, c[i - 1][2], c[i][2]))
        end = max(end, c[i][1])
    print("gaps > %.0f us: %d, %.3f ms" % (thr, len(gaps), sum(g for g, _, _ in gaps) / 1e3))
    for g, a, b in gaps:
        print("  %7.1f us  %s -> %s" % (g, a, b))
    short = [r for r in c if r[1] - r[0] < 50_000]
    print("launches < 50 us: %d, %.3f ms" % (len(short), sum(r[1] - r[0] for r in short) / 1e6))
    agg = {}
    for r in c:
        a = agg.setdefault(r[2], [0, 0.0])
        a[0] += 1
        a[1] += (r[1] - r[0]) / 1e6
    print("per kernel (count, ms):")
    for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("  %-28s %4d %8.3f" % (k, n, ms))


if __name__ == "__main__":
    main()
