#!/usr/bin/env python3
"""Print the last N events of a rocprofv3 kernel + memory-copy trace (csv) as one timeline (ms from the first
printed event): start, end, duration, stream, name.  usage: trace_timeline.py TRACE_DIR [N]"""
import csv
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 120
ev = []
mc = os.path.join(d, "run_memory_copy_trace.csv")
if os.path.exists(mc):
    for r in csv.DictReader(open(mc)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r["Direction"].replace("MEMORY_COPY_", ""),
                   r["Stream_Id"]))
for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48], r["Stream_Id"]))
ev.sort()
sel = ev[-n:]
base = sel[0][0]
for s, e, name, st in sel:
    print("%9.3f %9.3f %7.3f  st%-3s %s" % ((s - base) / 1e6, (e - base) / 1e6, (e - s) / 1e6, st, name))
