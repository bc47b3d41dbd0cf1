#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output per kernel (mean over dispatches)."""
import collections
import csv
import sys


def summarise(path, match=None):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if match and match not in name:
            continue
        agg[(name[:70], r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {}
    for (k, c), v in sorted(agg.items()):
        out.setdefault(k, {})[c] = sum(v) / len(v)
    return out


if __name__ == "__main__":
    match = "rollout"
    paths = sys.argv[1:]
    if paths and paths[0].startswith("--match="):
        match, paths = paths[0][8:], paths[1:]
    for p in paths:
        for k, cs in summarise(p, match).items():
            print(k)
            for c, v in cs.items():
                print(f"   {c:28s} {v:16.1f}")
