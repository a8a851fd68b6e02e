"""Merged timeline of every queue over one train step from a rocprofv3 kernel trace: one line per
kernel, time-sorted, with its queue column, so the side / comm streams' kernels can be read against
the main stream's.  Steps are delimited by adam_prep_kernel as in step_breakdown.py.

  python tools/queues.py <run_kernel_trace.csv> [min_us] [t_from_us] [t_to_us]
"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n)
    n = n.replace("(anonymous namespace)::", "").replace("avcg::", "")
    return n[:44]


def main():
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]))
                   for r in csv.DictReader(open(sys.argv[1]))), key=lambda r: r[1])
    ad = [i for i, r in enumerate(rows) if "adam_prep_kernel" in r[0]]
    seg = rows[ad[-3] + 1:ad[-2] + 1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    lo = float(sys.argv[3]) if len(sys.argv) > 3 else -1e9
    hi = float(sys.argv[4]) if len(sys.argv) > 4 else 1e9
    t0 = seg[0][1]
    qs = sorted({r[3] for r in seg})
    col = {q: i for i, q in enumerate(qs)}
    print("   start     end    dur  " + "  ".join(f"queue {q}".ljust(44) for q in qs))
    for n, s, e, q in seg:
        a, b = (s - t0) / 1e3, (e - t0) / 1e3
        if (e - s) / 1e3 < min_us or b < lo or a > hi:
            continue
        pad = " " * (46 * col[q])
        print(f"{a:8.1f} {b:7.1f} {b - a:6.1f}  {pad}{short(n)}")


if __name__ == "__main__":
    main()
