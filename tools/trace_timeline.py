#!/usr/bin/env python3
"""Print a per-dispatch timeline (start offset, duration, gap) from a rocprofv3 kernel trace csv."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = None
last_end = {}
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("svx::", "")[:28]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if not any(k in name for k in ("stage", "offsets", "fill", "resident", "keep_table")):
        continue
    if t0 is None:
        t0 = s
    q = r.get("Queue_Id", "?")
    print(f"q{q:>2} {name:28s} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us  grid {r['Grid_Size_X']}")
