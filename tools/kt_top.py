"""Per-kernel device time of one single-matrix consensus call from a rocprofv3 kernel trace
(kt_kernel_trace.csv; calls split as in tools/trace_gaps.py): launches, total and mean ms per kernel,
largest first.

usage: python tools/kt_top.py TRACE.csv [call_index=-1] [top=15] [name_prefix]
(with name_prefix: also every launch of the kernels whose name starts with it, in order)
"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_gaps import calls, load  # noqa: E402


def main():
    path = sys.argv[1]
    idx = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    c = calls(load(path))[idx]
    agg = {}
    for t0, t1, name in c:
        n, s = agg.get(name, (0, 0))
        agg[name] = (n + 1, s + (t1 - t0))
    span = (max(r[1] for r in c) - c[0][0]) / 1e6
    print("call %d: span %.3f ms, kernels %.3f ms" % (idx, span, sum(s for _, s in agg.values()) / 1e6))
    for name, (n, s) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print("  %-48s %4d x  %8.3f ms  (mean %.3f)" % (name, n, s / 1e6, s / 1e6 / n))
    if len(sys.argv) > 4:
        print("  launches of %s*: %s" % (sys.argv[4], " ".join("%.3f" % ((t1 - t0) / 1e6) for t0, t1, name in c
                                                             if name.startswith(sys.argv[4]))))


if __name__ == "__main__":
    main()
