"""Summarise rocprofv3 CSV output into profiles/ (kernel stats + per-launch HBM traffic).

    python tools/pmc_summary.py --stats DIR/kt_kernel_stats.csv --fetch DIR/pmc_counter_collection.csv \
        --write DIR2/pmc_counter_collection.csv --out profiles/pmc_traffic.json

SQ_INSTS_VALU (optional, its own pass) is the launch's wave-level VALU instruction count.
HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a coalesced streaming read, so
bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.  Each counter comes from its own
--pmc pass (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2).

    python tools/pmc_summary.py --per-kernel DIR

prints every counter of every pass under DIR/p*/ per kernel (median over launches), the int8
GEMM's launches split into the grid x grid and the mixed block (they alternate).
"""
import glob
import re
import argparse
import csv
import json
import statistics


def kname(full):
    """Short kernel name: drop namespaces, template arguments and the parameter list."""
    s = full.replace("(anonymous namespace)::", "")
    return s.split("(")[0].split("<")[0].split("::")[-1].split(" ")[-1]


def ours(full):
    """Only libpcx kernels (torch's own fill/copy kernels of the bench setup are left out)."""
    return "pcx::" in full


class GemmSplit:
    """The int8 GEMM's launches alternate: the grid x grid block, then the mixed block."""

    def __init__(self):
        self.n = {}

    def __call__(self, name, key=None):
        if name != "k_gemm_i8":
            return name
        self.n[key] = self.n.get(key, -1) + 1
        return name + ("_grid" if self.n[key] % 2 == 0 else "_mixed")


def per_kernel(path, counter):
    out, split = {}, GemmSplit()
    rows = [r for r in csv.DictReader(open(path)) if r.get("Counter_Name") == counter and ours(r["Kernel_Name"])]
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        name = split(kname(r["Kernel_Name"]))
        out.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def per_kernel_times(path):
    """Average duration (ns) and launch count per kernel from a kernel_trace.csv."""
    out, split = {}, GemmSplit()
    rows = [r for r in csv.DictReader(open(path)) if ours(r["Kernel_Name"])]
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        name = split(kname(r["Kernel_Name"]))
        out.setdefault(name, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in out.items()}


def per_kernel_passes(d, pattern="p*"):
    vals, seen = {}, {}
    for f in sorted(glob.glob(d + "/" + pattern + "/**/pmc_counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if not ours(n):
                continue
            m = re.search(r"(k_[a-z0-9_]+(<[^>]*>)?)", n)
            k = m.group(1) if m else kname(n)
            if k.startswith("k_gemm_i8<") and pattern == "p*":  # launches alternate: grid x grid, then the mixed block
                key = (f, r["Counter_Name"])
                seen[key] = seen.get(key, -1) + 1
                k += "_grid" if seen[key] % 2 == 0 else "_mixed"
            vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k in sorted(vals):
        med = {c: statistics.median(v) for c, v in vals[k].items()}
        if med.get("SQ_WAVE_CYCLES", 0) == 0 and med.get("FETCH_SIZE", 0) < 1e5:
            continue
        gb = (2 * med.get("FETCH_SIZE", 0) * 1024 + med.get("WRITE_SIZE", 0) * 1024) / 1e9
        print("%-22s hbm_GB=%.2f " % (k, gb) + " ".join("%s=%.4g" % (c, v) for c, v in sorted(med.items())))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-kernel", help="directory of --pmc passes p1, p2, ...: print per-kernel medians")
    ap.add_argument("--glob", default="p*", help="--per-kernel: the pass directories' pattern")
    ap.add_argument("--stats")
    ap.add_argument("--trace", help="kernel_trace.csv: per-launch durations (the int8 GEMM split grid / mixed)")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--valu", help="pmc_counter_collection.csv of an SQ_INSTS_VALU pass")
    ap.add_argument("--out")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    if a.per_kernel:
        per_kernel_passes(a.per_kernel, a.glob)
        return
    if not (a.fetch and a.write and a.out):
        ap.error("--fetch, --write and --out are required without --per-kernel")
    f = per_kernel(a.fetch, "FETCH_SIZE")
    w = per_kernel(a.write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fk, wk = f.get(k), w.get(k)
        res[k] = {"fetch_size_kib": fk, "write_size_kib": wk,
                  "bytes_per_launch": (2 * fk * 1024 if fk is not None else 0) + (wk * 1024 if wk is not None else 0),
                  "correction": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halves wide reads)"}
    if a.valu:
        for k, v in per_kernel(a.valu, "SQ_INSTS_VALU").items():
            res.setdefault(k, {})["insts_valu_per_launch"] = v
    if a.trace:
        for k, (avg, n) in per_kernel_times(a.trace).items():
            res.setdefault(k, {})["avg_ns"] = avg
            res[k]["calls"] = n
    elif a.stats:
        for r in csv.DictReader(open(a.stats)):
            if not ours(r["Name"]):
                continue
            k = kname(r["Name"])
            res.setdefault(k, {})["avg_ns"] = float(r["AverageNs"])
            res[k]["calls"] = int(r["Calls"])
    if a.note:
        res["_note"] = a.note
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
