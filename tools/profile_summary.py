#!/usr/bin/env python3
"""Per-kernel, per-launch summary of a tools/profile_round.sh output directory.

Corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
  * FETCH_SIZE / WRITE_SIZE are in KiB per dispatch;
  * on gfx950 FETCH_SIZE reads half the bytes of a wide (16 B/lane) coalesced
    streaming read: fetch_bytes_corrected = 2 * FETCH_SIZE * 1024 (an upper
    estimate for narrower accesses, which the guide leaves uncalibrated);
  * valu_issue_frac = 2 * SQ_INSTS_VALU / (1024 SIMDs * gpu_cycles_pmc): the
    fraction of the hardware's issue peak (one wave64 VALU instruction per SIMD
    every 2 cycles, MI355X_MICROARCH.md) the dispatch used, which cannot pass
    1.  (Rounds 1-4 published valu_busy = 4 * SQ_ACTIVE_INST_VALU / SIMD
    cycles, which priced every instruction at 4 cycles and passed 1 for mixes
    with fast logic; it is no longer reported.)
"""
import collections
import csv
import glob
import json
import os
import sys

N_SE = 32
N_SIMD = 1024


def short(name):
    """Stable short names: rollout_kernel<POLICY, RECORD> (the GameRunner
    instances as rollout_runner<POLICY, RECORD>), replay_kernel (strided) and
    replay_rows_kernel (packed rows, round 3)."""
    import re
    m = re.search(r"rollout_kernel<(\d), (true|false)(?:, (true|false))?>", name)
    if m:
        return "rollout_%s<%s, %s>" % ("runner" if m.group(3) == "true" else "kernel", m.group(1), m.group(2))
    m = re.search(r"replay_kernel<(true|false)>", name)
    if m:
        return "replay_rows_kernel" if m.group(1) == "true" else "replay_kernel"
    for k in ("step_kernel", "legal_kernel", "result_kernel", "reset_kernel", "sample_midgame_kernel",
              "replay_kernel", "book_text_kernel", "book_parse_kernel", "features_kernel", "eval_kernel",
              "td_updates_kernel", "td_records_kernel", "td_ema_spec_kernel", "td_ema_long_kernel", "td_ema_kernel",
              "td_merge_kernel", "td_lookup_kernel", "td_splits_kernel"):
        if k in name:
            return k
    return None


def pmc(d, durs=None):
    """Counter values per (kernel, grid); with `durs`, also each dispatch's
    duration in this pass (PMC passes serialize the dispatches, so this is a
    launch alone on the chip), once per dispatch."""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    seen = set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k is None:
                continue
            # key by grid size too: step_kernel runs at two batch sizes
            key = (k, int(r["Grid_Size"]))
            out[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if durs is not None and (f, r["Dispatch_Id"]) not in seen and r.get("End_Timestamp"):
                seen.add((f, r["Dispatch_Id"]))
                durs[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


PASSES = {
    "avg_ns": "kernel-trace pass (rocprofv3 --kernel-trace --stats) of the bench command: launches as the bench "
              "issues them, so the headline rollout shares the chip with the launch on the other stream "
              "(two in flight)",
    "avg_ns_serialized": "the GRBM PMC pass of the same command: counter collection serializes dispatches, so each "
                         "launch runs alone on the chip",
    "fetch_bytes_raw/fetch_bytes_corrected": "FETCH_SIZE pass (x2 gfx950 correction)",
    "write_bytes": "WRITE_SIZE pass",
    "SQ_*": "SQ pass (serialized dispatches)",
    "GRBM_GUI_ACTIVE/gpu_cycles_pmc": "GRBM pass (serialized dispatches); gpu_cycles_pmc = GRBM_GUI_ACTIVE / 8 XCDs",
    "clock_ghz_pmc": "gpu_cycles_pmc / avg_ns_serialized, both from the GRBM pass (one dispatch, one pass); "
                     "meaningful for launches of >> 10 us only (a few-us launch's GRBM count includes the "
                     "dispatch's fixed overhead outside its timestamps)",
    "valu_issue_frac": "2 x SQ_INSTS_VALU (SQ pass) / (1024 SIMDs x gpu_cycles_pmc (GRBM pass)): both serialized; "
                       "not comparable with avg_ns, which overlaps a neighbouring launch",
}


def main(d):
    stats = {}
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            if k:
                stats[k] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                            "max_ns": float(r["MaxNs"])}
    trace = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                trace[(k, int(r.get("Grid_Size") or r["Grid_Size_X"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    counters = {}
    serialized = collections.defaultdict(list)
    for sub in ("fetch", "write", "sq", "grbm"):
        for key, cs in pmc(os.path.join(d, sub), serialized if sub == "grbm" else None).items():
            for c, v in cs.items():
                counters.setdefault(key, {})[c] = sum(v) / len(v)
    # the build every figure below was measured on (bench.py compares it with
    # the library it runs, and marks PMC figures of another build as stale)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from subproc_amd._lib import library_sha16
    out = {"library_sha16": library_sha16(), "passes": PASSES, "kernels": {}}
    for (k, grid), cs in sorted(counters.items()):
        e = {"grid_threads": grid}
        durs = trace.get((k, grid))
        if durs:
            e["launches"] = len(durs)
            e["avg_ns"] = sum(durs) / len(durs)
        sd = serialized.get((k, grid))
        if sd:
            e["avg_ns_serialized"] = sum(sd) / len(sd)
        if "FETCH_SIZE" in cs:
            e["fetch_bytes_raw"] = cs["FETCH_SIZE"] * 1024
            e["fetch_bytes_corrected"] = 2 * cs["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in cs:
            e["write_bytes"] = cs["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            e["hbm_bytes"] = e["fetch_bytes_corrected"] + e["write_bytes"]
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "GRBM_GUI_ACTIVE"):
            if c in cs:
                e[c] = cs[c]
        if "GRBM_GUI_ACTIVE" in cs:
            # GPU cycles of the (serialized) PMC dispatch; not divided by the kernel-trace
            # duration, which overlaps a neighbouring launch in the two-stream bench
            e["gpu_cycles_pmc"] = cs["GRBM_GUI_ACTIVE"] / 8
            if e.get("avg_ns_serialized"):
                e["clock_ghz_pmc"] = e["gpu_cycles_pmc"] / e["avg_ns_serialized"]
            if "SQ_INSTS_VALU" in cs and e["gpu_cycles_pmc"] > 0:
                e["valu_issue_frac"] = 2 * cs["SQ_INSTS_VALU"] / (N_SIMD * e["gpu_cycles_pmc"])
        out["kernels"][f"{k}@{grid}"] = e
    out["kernel_stats"] = stats
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
