"""MFMA-busy / wait / LDS counters per kernel from one rocprofv3 --pmc pass (CSV output).

  python tools/pmc_mfma.py <counter_collection.csv> <out.json> [top]

Per kernel (averaged over its dispatches):
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs): the fraction of
                the launch's SIMD-cycles the matrix pipes were busy (SQ_VALU_MFMA_BUSY_CYCLES counts
                MFMA cycles, MI355X_MICROARCH.md 'Per-instruction cycle constants');
  wait / issue-stall / active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
                (disjoint, they sum to ~1: MI355X_MICROARCH.md 'rocprofv3 PMC slots');
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles per LDS-array cycle);
  bf16 MFMA TFLOP/s from SQ_INSTS_VALU_MFMA_MOPS_BF16 (x512 flop per MOP) over the dispatch time.
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    # one dispatch = one (Dispatch_Id); counters spread over rows
    disp = defaultdict(dict)
    name = {}
    dur = {}
    for r in rows:
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
        if "Start_Timestamp" in r and r.get("End_Timestamp"):
            dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(list)
    for d, c in disp.items():
        per[name[d]].append((c, dur.get(d)))
    out = {}
    for k, lst in per.items():
        n = len(lst)
        avg = defaultdict(float)
        for c, _ in lst:
            for cn, v in c.items():
                avg[cn] += v / n
        durs = [t for _, t in lst if t]
        e = {"dispatches": n}
        g = avg.get("GRBM_GUI_ACTIVE", 0.0)
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            e["mfma_util"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024)
        wc = avg.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            for cn, key in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "issue_stall"), ("SQ_ACTIVE_INST_ANY", "active")):
                if cn in avg:
                    e[key] = avg[cn] / wc
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict"] = avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_LDS_IDX_ACTIVE"]
        if durs and "SQ_INSTS_VALU_MFMA_MOPS_BF16" in avg:
            e["bf16_tflops"] = avg["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / (sum(durs) / len(durs)) / 1e12
        if durs:
            e["avg_us"] = sum(durs) / len(durs) * 1e6
        if g:
            e["clock_ghz"] = g / 8 / (sum(durs) / len(durs)) / 1e9 if durs else None
        e["counters"] = dict(avg)
        out[k] = e
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    rank = sorted(out.items(), key=lambda kv: -(kv[1].get("avg_us", 0) * kv[1]["dispatches"]))
    for k, e in rank[:top]:
        short = k.replace("(anonymous namespace)::", "").split("(")[0][:60]
        print(f"{short:60s} n={e['dispatches']:3d} avg={e.get('avg_us', 0):8.1f}us mfma={e.get('mfma_util', 0):.3f} "
              f"wait={e.get('wait', 0):.2f} stall={e.get('issue_stall', 0):.2f} act={e.get('active', 0):.2f} "
              f"ldsc={e.get('lds_conflict', 0):.3f} tf={e.get('bf16_tflops', 0):7.1f} clk={e.get('clock_ghz') or 0:.2f}")


if __name__ == "__main__":
    main()
