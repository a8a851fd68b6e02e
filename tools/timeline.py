"""Main-stream timeline of one train step from a rocprofv3 kernel trace: every main-queue kernel
with its start offset, duration and the other queues' kernels running beside it (the contention a
main-stream kernel sees).  Steps are delimited by adam_prep_kernel as in step_breakdown.py.

  python tools/timeline.py <run_kernel_trace.csv> [main_queue] [min_us]
"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n)
    return n[:46]


def main():
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]))
                   for r in csv.DictReader(open(sys.argv[1]))), key=lambda r: r[1])
    ad = [i for i, r in enumerate(rows) if "adam_prep_kernel" in r[0]]
    seg = rows[ad[-3] + 1:ad[-2] + 1]
    qmain = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    t0 = seg[0][1]
    others = [r for r in seg if r[3] != qmain]
    for n, s, e, q in seg:
        if q != qmain or (e - s) / 1e3 < min_us:
            continue
        beside = [short(o[0]) for o in others if o[1] < e and o[2] > s]
        side = ", ".join(sorted(set(beside)))[:110]
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {short(n):46s} | {side}")


if __name__ == "__main__":
    main()
