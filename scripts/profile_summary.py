"""rocprofv3 --kernel-trace --stats CSV -> markdown table for profiles/.

python scripts/profile_summary.py <kernel_stats.csv> <steps_in_run> <title> [notes_file] > out.md
Per kernel: calls per step, average us, ms per step, share of kernel time (top 30)."""
import csv
import sys


def main():
    path, steps, title = sys.argv[1], float(sys.argv[2]), sys.argv[3]
    notes = open(sys.argv[4]).read().strip() if len(sys.argv) > 4 else ""
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print(f"Source: `{path}` ({steps:g} steps incl. warm-up); total kernel time "
          f"{tot / 1e6:.2f} ms = {tot / 1e6 / steps:.3f} ms/step.\n")
    if notes:
        print(notes + "\n")
    print("| kernel | calls/step | avg us | ms/step | % |")
    print("|---|---|---|---|---|")
    for r in rows[:30]:
        name = r["Name"].replace("tdp::(anonymous namespace)::", "").replace("|", "/")
        name = name[:95]
        t = float(r["TotalDurationNs"])
        print(f"| `{name}` | {int(r['Calls']) / steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{t / 1e6 / steps:.3f} | {100 * t / tot:.1f} |")


if __name__ == "__main__":
    main()
