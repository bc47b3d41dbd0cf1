"""Kernel-by-kernel timeline of the last TD batch in a rocprofv3 kernel trace
of tools/diag/td_trace.py (diagnostic): each kernel's duration and the idle
gap before it, from the last replay kernel on."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
i0 = [i for i, r in enumerate(rows) if "replay" in r["Kernel_Name"]][-1]
prev, busy, gaps = None, 0.0, 0.0
for r in rows[i0:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = max(0.0, (s - prev) / 1e3) if prev else 0.0
    busy += (e - s) / 1e3
    gaps += gap
    print("%8.1f gap %8.1f us  %s" % (gap, (e - s) / 1e3, r["Kernel_Name"][:80]))
    prev = e
print("kernels %.1f us, gaps %.1f us, span %.1f us" % (busy, gaps, (prev - int(rows[i0]["Start_Timestamp"])) / 1e3))
