"""HBM bytes per launch, per kernel, from two rocprofv3 PMC passes (separate runs, CSV output):
FETCH_SIZE and WRITE_SIZE.  gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE
counts wide reads at half size, so bytes = 2*FETCH_SIZE_KB*1024 + WRITE_SIZE_KB*1024.

  python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {"correction": "bytes = 2*FETCH_SIZE_KB*1024 + WRITE_SIZE_KB*1024 (gfx950 FETCH_SIZE halves wide reads)",
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        f, w = fetch.get(name, []), write.get(name, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        out["kernels"][name] = {"FETCH_SIZE_KB": fk, "WRITE_SIZE_KB": wk,
                                "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
                                "launches_FETCH_SIZE": len(f), "launches_WRITE_SIZE": len(w)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print("wrote", sys.argv[3], len(out["kernels"]), "kernels")


if __name__ == "__main__":
    main()
