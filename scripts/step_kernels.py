"""rocprofv3 kernel trace (CSV) -> per-step kernel table of the steady state.

python scripts/step_kernels.py <kernel_trace.csv> [marker_substring] [last_steps] > table.md
Steps are delimited by the marker kernel (default: the cross-entropy forward, once per training
step); the table covers the last `last_steps` complete steps before the final one."""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    n = re.sub(r"tdp::\(anonymous namespace\)::", "", name)
    n = n.replace("void ", "")
    return n[:110].replace("|", "/")


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "ce_fwd"
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[-last - 1], idx[-1]
    seg = rows[a:b]
    tot, cnt = collections.defaultdict(float), collections.Counter()
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        tot[short(r["Kernel_Name"])] += d
        cnt[short(r["Kernel_Name"])] += 1
    span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1000.0 / last
    ksum = sum(tot.values()) / last
    print(f"Steady state: last {last} steps of `{path}` (step marker `{marker}`): kernel time "
          f"{ksum:.1f} us/step, {len(seg) / last:.1f} kernels/step, step-to-step span "
          f"{span:.1f} us (profiled).\n")
    print("| kernel | calls/step | avg us | us/step | % |")
    print("|---|---|---|---|---|")
    for n, t in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"| `{n}` | {cnt[n] / last:.1f} | {t / cnt[n]:.1f} | {t / last:.1f} | "
              f"{100 * t / last / ksum:.1f} |")


if __name__ == "__main__":
    main()
