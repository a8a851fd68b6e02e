"""From a rocprofv3 kernel_trace.csv: how much kernel time overlaps between queues/streams."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(rows[0].keys())
ev = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r.get('Queue_Id', r.get('Stream_Id', '?')), r['Kernel_Name'][:40]) for r in rows]
ev.sort()
qs = {}
for s, e, q, n in ev:
    qs.setdefault(q, 0)
    qs[q] += e - s
print({q: v / 1e6 for q, v in qs.items()})
# overlap: sweep
pts = []
for s, e, q, n in ev:
    pts.append((s, 1)); pts.append((e, -1))
pts.sort()
cur = 0; last = pts[0][0]; busy = 0; multi = 0
for t, d in pts:
    if cur > 0: busy += t - last
    if cur > 1: multi += t - last
    cur += d; last = t
print(f"busy {busy/1e6:.2f} ms, >1 kernel concurrently {multi/1e6:.2f} ms, span {(ev[-1][1]-ev[0][0])/1e6:.2f} ms")
