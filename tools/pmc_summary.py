"""Summarise rocprofv3 CSV output into profiles/ (kernel stats + per-launch HBM traffic).

    python tools/pmc_summary.py --stats DIR/kt_kernel_stats.csv --fetch DIR/pmc_counter_collection.csv \
        --write DIR2/pmc_counter_collection.csv --out profiles/pmc_traffic.json

SQ_INSTS_VALU (optional, its own pass) is the launch's wave-level VALU instruction count.
HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a coalesced streaming read, so
bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.  Each counter comes from its own
--pmc pass (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2).
"""
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


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter or not ours(r["Kernel_Name"]):
            continue
        name = kname(r["Kernel_Name"])
        out.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--valu", help="pmc_counter_collection.csv of an SQ_INSTS_VALU pass")
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
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
    if a.stats:
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
