"""rocprofv3 --pmc (+ --kernel-trace) CSVs -> one markdown table per kernel: dispatches, mean
duration and the mean of every collected counter per dispatch, for the kernels that take most
of the time. Several passes (one counter group each) can be given; their kernels are matched
by name.

    python scripts/pmc_summary.py <title> <pass_dir> [<pass_dir> ...] > out.md

Derived columns when the counters are present (GRBM_GUI_ACTIVE is summed over the 8 XCDs: 8 x
the dispatch's GPU clocks; SQ_VALU_MFMA_BUSY_CYCLES over the 1024 SIMDs): MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024), HBM GB/s from
(FETCH_SIZE + WRITE_SIZE) KiB over the kernel's duration (FETCH_SIZE can read half the bytes of a
wide coalesced stream on gfx950: a lower bound, CDNA4 guide §9).
"""
import csv
import glob
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
XCDS = 8


def _load(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    vals = defaultdict(lambda: defaultdict(list))
    for f in cc:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("KernelName")
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(list)
    for f in kt:
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, dur


def short(n):
    return n.replace("tdp::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]


def main():
    title, dirs = sys.argv[1], sys.argv[2:]
    vals, dur = defaultdict(dict), defaultdict(list)
    for d in dirs:
        v, t = _load(d)
        for k, cs in v.items():
            for c, xs in cs.items():
                vals[k][c] = sum(xs) / len(xs)
        for k, xs in t.items():
            dur[k] += xs
    total = {k: sum(xs) for k, xs in dur.items()}
    top = sorted(total, key=lambda k: -total[k])[:8]
    counters = sorted({c for k in top for c in vals.get(k, {})})
    print(f"# {title}\n")
    print("Passes: " + ", ".join(f"`{d}`" for d in dirs) + ". Mean per dispatch.\n")
    head = ["kernel", "dispatches", "avg us"] + counters + ["MFMA busy", "HBM GB/s (>=)"]
    print("| " + " | ".join(head) + " |")
    print("|" + "---|" * len(head))
    for k in top:
        n = len(dur[k])
        us = total[k] / n / 1e3
        v = vals.get(k, {})
        row = [f"`{short(k)}`", str(n), f"{us:.1f}"]
        row += [f"{v[c]:.3g}" if c in v else "" for c in counters]
        busy = ""
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v and v.get("GRBM_GUI_ACTIVE"):
            clocks = v["GRBM_GUI_ACTIVE"] / XCDS
            busy = f"{100 * v['SQ_VALU_MFMA_BUSY_CYCLES'] / (clocks * SIMDS):.0f} %"
        bw = ""
        if "FETCH_SIZE" in v or "WRITE_SIZE" in v:
            kib = v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0)
            bw = f"{kib * 1024 / (us * 1e-6) / 1e9:.0f}"
        row += [busy, bw]
        print("| " + " | ".join(row) + " |")


if __name__ == "__main__":
    main()
