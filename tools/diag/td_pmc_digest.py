"""Digest of tools/diag/td_pmc.sh (diagnostic): per TD kernel of the last of
three 262,144-game batches, the kernel-trace duration and the FETCH_SIZE /
WRITE_SIZE counters (KiB; FETCH x2 as MI355X_MICROARCH.md's gfx950
correction for wide loads, an upper bound), and the HBM rate they imply.
    python tools/diag/td_pmc_digest.py gpurun_out/tdpmc > profiles/r05_td_pmc.md"""
import csv
import glob
import os
import sys

d = sys.argv[1]


def last_per_kernel(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    by = {}
    for r in rows:  # the last dispatch of each kernel name (batch 3)
        by[r["Kernel_Name"]] = float(r["Counter_Value"])
    return by


fetch = last_per_kernel(glob.glob(os.path.join(d, "fetch", "**", "*counter_collection.csv"), recursive=True)[0],
                        "FETCH_SIZE")
write = last_per_kernel(glob.glob(os.path.join(d, "write", "**", "*counter_collection.csv"), recursive=True)[0],
                        "WRITE_SIZE")
tr = glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True)
dur = {}
if tr:
    for r in csv.DictReader(open(tr[0])):
        dur[r["Kernel_Name"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("| kernel | us | fetch MB (x2) | write MB | HBM GB/s |")
print("|---|---|---|---|---|")
for k in sorted(fetch, key=lambda k: -(fetch[k] + write.get(k, 0))):
    if not any(s in k for s in ("td_", "replay", "rocprim", "sort")):
        continue
    f, w = 2 * fetch[k] * 1024 / 1e6, write.get(k, 0) * 1024 / 1e6
    us = dur.get(k)
    rate = "%.0f" % ((f + w) / us * 1e3) if us else "-"  # MB per us = TB/s
    name = k.replace("(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0] if not name.startswith("rocprim") else "rocprim " + name.split("<")[2][:40]
    print("| `%s` | %s | %.0f | %.0f | %s |" % (name[:70], "%.1f" % us if us else "-", f, w, rate))
