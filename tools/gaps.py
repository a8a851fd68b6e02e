"""Largest idle gaps on the main queue within one step (kernel -> next kernel)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]))
               for r in rows), key=lambda r: r[1])
ad = [i for i, r in enumerate(rows) if "adam_prep_kernel" in r[0]]  # one per step
seg = [r for r in rows[ad[-3] + 1:ad[-2] + 1] if r[3] == int(sys.argv[2] if len(sys.argv) > 2 else 1)]


def nm(n):
    n = re.sub(r"\(anonymous namespace\)::|avcg::|void ", "", n)
    return n.split("(")[0][:50]


gaps = [(b[1] - a[2], nm(a[0]), nm(b[0]), i) for i, (a, b) in enumerate(zip(seg, seg[1:]))]
print("total gap us", sum(g[0] for g in gaps) / 1e3, "kernels", len(seg))
for g in sorted(gaps, reverse=True)[:25]:
    print("%7.1f us  #%3d %s -> %s" % (g[0] / 1e3, g[3], g[1], g[2]))
