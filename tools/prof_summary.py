"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel ms/step table.

usage: python tools/prof_summary.py <prefix>_kernel_stats.csv <steps> [out.md]
"""
import csv
import sys


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"| kernel | calls/step | avg us | ms/step | % |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]
        lines.append(f"| `{name}` | {int(r['Calls']) / steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['TotalDurationNs']) / 1e6 / steps:.3f} | {float(r['Percentage']):.1f} |")
    lines.append(f"| **total** | | | {tot / 1e6 / steps:.3f} | 100 |")
    text = "\n".join(lines)
    print(text)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text + "\n")


if __name__ == "__main__":
    main()
