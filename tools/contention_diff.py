"""Pair the main-queue kernels of one step in two rocprofv3 kernel traces (the normal recorded step and
the AVC_ABLATE_WGRAD=1 one, tools/contention_trace.py) instance by instance and print each kernel's
inflation, with the other queues' kernels that ran beside it in the normal trace.

  python tools/contention_diff.py <normal trace.csv> <ablated trace.csv> [min_delta_us]
"""
import csv
import re
import sys
from collections import Counter, defaultdict


def short(n):
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n)
    return n.replace("(anonymous namespace)::", "").replace("avcg::", "")[:40]


def step_rows(path):
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]))
                   for r in csv.DictReader(open(path))), key=lambda r: r[1])
    # main queue = the one running lstm2_persist_bwd; steps delimited by that queue's adam_prep_kernel
    qmain = next(q for n, s, e, q in rows if "lstm2_persist_bwd" in n)
    ad = [i for i, r in enumerate(rows) if "adam_prep_kernel" in r[0]]
    seg = rows[ad[-3] + 1:ad[-2] + 1]
    return [r for r in seg if r[3] == qmain], [r for r in seg if r[3] != qmain]


def main():
    a_main, a_other = step_rows(sys.argv[1])
    b_main, _ = step_rows(sys.argv[2])
    lim = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
    # match the k-th instance of each kernel name
    idx = defaultdict(list)
    for r in b_main:
        idx[r[0]].append(r)
    seen = Counter()
    tot = defaultdict(float)
    t0 = a_main[0][1]
    tsum_a = tsum_b = 0.0
    print(f"{'start':>8} {'step':>7} {'alone':>7} {'delta':>7}  kernel / beside it")
    for n, s, e, q in a_main:
        k = seen[n]
        seen[n] += 1
        if k >= len(idx[n]):
            continue
        bn, bs, be, _ = idx[n][k]
        da, db = (e - s) / 1e3, (be - bs) / 1e3
        tsum_a += da
        tsum_b += db
        tot[short(n)] += da - db
        if da - db >= lim:
            beside = sorted({short(o[0]) for o in a_other if o[1] < e and o[2] > s})
            print(f"{(s - t0) / 1e3:8.1f} {da:7.1f} {db:7.1f} {da - db:7.1f}  {short(n)} | {', '.join(beside)[:120]}")
    print(f"\nmain-queue kernel time: {tsum_a:.1f} us with the side stream, {tsum_b:.1f} us without "
          f"(+{tsum_a - tsum_b:.1f})")
    print("inflation by kernel:")
    for n, d in sorted(tot.items(), key=lambda kv: -kv[1])[:20]:
        print(f"  {d:8.1f} us  {n}")


if __name__ == "__main__":
    main()
