"""rocprofv3 kernel trace (CSV) -> the kernels of ONE steady-state step in launch order, with each
kernel's median duration and the median idle gap before it (end of the previous kernel to its
start) over the last `last_steps` steps.

python scripts/step_timeline.py <kernel_trace.csv> [marker_substring] [last_steps] > timeline.md
Complements step_kernels.py: where the per-kernel table hides launch gaps, this shows them."""
import csv
import statistics
import sys

from step_kernels import short


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "ce_fwd"
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    steps = [rows[idx[k]: idx[k + 1]] for k in range(len(idx) - last - 1, len(idx) - 1)]
    n = min(len(s) for s in steps)
    steps = [s for s in steps if len(s) == n]
    print(f"One step of `{path}` (marker `{marker}`, median over {len(steps)} steps with {n} "
          f"kernels each)\n")
    print("| # | kernel | us | gap before (us) |")
    print("|---|---|---|---|")
    tot_k = tot_g = 0.0
    for j in range(n):
        d = statistics.median((int(s[j]["End_Timestamp"]) - int(s[j]["Start_Timestamp"])) / 1e3
                              for s in steps)
        if j == 0:
            prev = [rows[rows.index(s[0]) - 1] for s in steps]
            g = statistics.median((int(s[0]["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3
                                  for s, p in zip(steps, prev))
        else:
            g = statistics.median((int(s[j]["Start_Timestamp"]) -
                                   int(s[j - 1]["End_Timestamp"])) / 1e3 for s in steps)
        tot_k += d
        tot_g += g
        print(f"| {j} | `{short(steps[0][j]['Kernel_Name'])[:70]}` | {d:.1f} | {g:.1f} |")
    print(f"\nkernels {tot_k:.1f} us + gaps {tot_g:.1f} us = {tot_k + tot_g:.1f} us per step")


if __name__ == "__main__":
    main()
