"""Per-stream kernel-time breakdown of one train step from a rocprofv3 kernel trace
(CSV run_kernel_trace.csv or rocpd run_results.db).  Steps are delimited by adam_kernel.

  python tools/step_breakdown.py <trace.csv|results.db> [top]
"""
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(n, s, e, q) for n, s, e, q in c.execute("select name,start,end,queue_id from kernels order by start")]
    rows = list(csv.DictReader(open(path)))
    out = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"])) for r in rows]
    return sorted(out, key=lambda r: r[1])


def main():
    rows = load(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    # one adam_prep_kernel per step (Adam may run as several slices)
    ad = [i for i, r in enumerate(rows) if "adam_prep_kernel" in r[0]]
    seg = rows[ad[-3] + 1:ad[-2] + 1]
    t0, t1 = seg[0][1], max(r[2] for r in seg)
    print(f"step span {(t1 - t0) / 1e6:.3f} ms, {len(seg)} kernels")
    # union of busy intervals over all queues: the time no kernel at all runs is host / launch bound
    iv = sorted((s, e) for _, s, e, _ in seg)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"some kernel running {busy / 1e6:.3f} ms; no kernel running {(t1 - t0 - busy) / 1e6:.3f} ms")
    for q in sorted(set(r[3] for r in seg)):
        d = defaultdict(lambda: [0, 0])
        for n, s, e, qq in seg:
            if qq != q:
                continue
            n = re.sub(r"\(anonymous namespace\)::", "", n).split("(")[0][:72]
            d[n][0] += e - s
            d[n][1] += 1
        tot = sum(v[0] for v in d.values())
        print(f"queue {q}: {tot / 1e3:.1f} us busy")
        for k, v in sorted(d.items(), key=lambda kv: -kv[1][0])[:top]:
            print(f"  {v[0] / 1e3:8.1f} us {v[1]:4d}  {k}")


if __name__ == "__main__":
    main()
