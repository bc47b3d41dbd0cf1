#!/usr/bin/env python3
"""Per-launch start/end times of the bench's two-stream rollout steps inside one
timed region (HIP events on each launch's own stream, relative to the region's
first event): where a short timed region (the driver's --steps 20) loses time
against a long one -- the first launches, the last one's drain, or the gaps.
    python tools/diag/timeline.py [--steps 20] [--streams 2] [--games 1048576]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--streams", type=int, default=2)
    p.add_argument("--games", type=int, default=1 << 20)
    p.add_argument("--regions", type=int, default=3)
    a = p.parse_args()
    import torch

    from subproc_amd import _lib
    from subproc_amd._lib import HIST_BINS

    lib = _lib.load()
    dev = torch.device("cuda", 0)
    n = a.games
    main_st = torch.cuda.current_stream()
    streams = [main_st] + [torch.cuda.Stream(dev) for _ in range(a.streams - 1)]
    bufs = [(torch.empty((n, 2), dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int8, device=dev),
             torch.empty(n, dtype=torch.uint8, device=dev)) for _ in streams]
    works = torch.zeros(len(streams), dtype=torch.int64, device=dev)
    hist = torch.zeros(HIST_BINS, dtype=torch.int64, device=dev)

    def launch(s, st_i):
        fb, df, pl = bufs[st_i]
        _lib.check(lib.oth_rollout(None, None, 0x5EED, s * n, 0, 10, fb.data_ptr(), df.data_ptr(), pl.data_ptr(),
                                   None, hist.data_ptr(), works[st_i:st_i + 1].data_ptr(), n,
                                   streams[st_i].cuda_stream), "rollout")

    t_w = time.perf_counter()
    while time.perf_counter() - t_w < 0.3:
        launch(0, 0)
        torch.cuda.synchronize()
    out = []
    s = 1
    for r in range(a.regions):
        for _ in range(a.warmup):
            launch(s, s % a.streams)
            s += 1
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(main_st)
        fork = torch.cuda.Event()
        fork.record(main_st)
        for st in streams[1:]:
            st.wait_event(fork)
        evs = []
        for k in range(a.steps):
            i = k % a.streams
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(streams[i])
            launch(s, i)
            e1.record(streams[i])
            evs.append((i, e0, e1))
            s += 1
        for st in streams[1:]:
            e = torch.cuda.Event()
            e.record(st)
            main_st.wait_event(e)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record(main_st)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        rows = [(i, round(ev0.elapsed_time(e0), 4), round(ev0.elapsed_time(e1), 4)) for i, e0, e1 in evs]
        out.append({"region": r, "wall_ms": round(wall, 4), "event_ms": round(ev0.elapsed_time(ev1), 4),
                    "per_step_ms": round(ev0.elapsed_time(ev1) / a.steps, 5), "launches": rows})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
