#!/usr/bin/env python3
"""Benchmark: env-steps/s of batched self-play on MI355X (BASELINE.json metric).

Default workload = config 3: 1,048,576 random-policy games from the opening to
terminal per GPU, one ``oth_rollout`` launch per bench step (each step plays a
fresh range of global game ids); at N>1 the int64[133] win/score histogram of
the run is all-reduced over RCCL once, inside the timed region (config 4, weak
scaling).  Measured at world size 1 under torchrun: one
all-reduce per run costs 1.3% vs no RCCL, one per step 2-3%, one per step
overlapped with the next rollout 5.5% (RCCL's kernel contends for CUs).  value = env-steps (plies summed from the kernel's own
histogram, passes included) of ALL ranks / max-over-ranks wall time.

Also reported on rank 0 (secondary, same JSON line):
  * step_65536 : config 2, one oth_step launch over 65,536 reachable mid-game
    positions (52 algorithmic HBM bytes per step), repeated launches;
  * step_65536_graph: the same 65,536-board launches captured in a HIP graph;
  * step_steady: the same kernel over 16,777,216 positions (HBM roofline);
  * rollout_16M: the config-3 kernel on 16,777,216 games per launch (the
    per-launch tail amortised: the kernel's steady-state rate);
  * greedy     : config 5, 1,048,576 1-ply greedy-mobility games;
  * eval       : 1,048,576 games of the 1-ply linear-eval policy with the
    learner's default weights;
  * td_state_map: the learner's TD state-map update for 262,144 GPU games;
  * book_emitter: replay and serialize_str text of 262,144 games (§8f row 1),
    and the text parsed back by the reader's kernel (oth_book_parse);
  * cpu_baseline: the C oracle (mailbox restatement of board.py) on a bounded
    sample of the same workload on the host cores.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload rollout|greedy|step]
Multi-GPU: python bench.py --gpus N ... (starts N rank processes itself), or
           python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, MI355X_MICROARCH.md
# VALU issue peak: a wave64 instruction can issue every 2 cycles on a SIMD-32
# (MI355X_MICROARCH.md), 1024 SIMDs at the 2.4 GHz max clock = 1.229e12
# wave-instructions/s.  valu.frac is the fraction of THIS hardware figure.
# Measured on the box (tools/diag/valu_rate*.cpp) only plain logic streams at
# ~2.2 cycles; 64-bit shifts, bfrev, bcnt ... take ~4, so these kernels cannot
# reach it: the ceilings priced from each hot loop's own instruction mix
# (tools/valu_mix.py -> profiles/valu_mix.json) are reported beside it under
# valu.model, as model statements, not as the roofline.
VALU_PEAK_HW = 1024 * 2.4e9 / 2


def valu_entry(kernel, achieved, **extra):
    """VALU roofline of `kernel` at `achieved` wave-instructions/s: the fraction
    of the hardware issue peak, with the mix-model ceilings under 'model'."""
    e = {"achieved": achieved, "peak": VALU_PEAK_HW, "unit": "wave-instr/s", "frac": achieved / VALU_PEAK_HW,
         "peak_basis": "2 cycles per wave64 VALU instruction per SIMD, 1024 SIMDs, 2.4 GHz (MI355X_MICROARCH.md)"}
    mix = None
    try:
        with open(os.path.join(ROOT, "profiles", "valu_mix.json")) as f:
            mix = json.load(f)["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        pass
    if mix:
        # the model's ceilings as figures only: an issue-cost model the kernel
        # can beat is no ceiling, so no fraction of it is published (only
        # valu.frac, of the hardware's 2-cycle issue peak, which it cannot pass)
        m = {"basis": "ceilings fitted to the hot loop's static instruction mix with per-opcode costs measured "
                      "on the box (tools/valu_mix.py); a model, not a hardware peak",
             "mean_cycles": mix["mean_cycles"], "peak": mix["peak_winstr_s"]}
        if "peak_winstr_s_mixed" in mix:
            m.update(mean_cycles_mixed=mix.get("mean_cycles_mixed"), peak_mixed=mix["peak_winstr_s_mixed"])
        e["model"] = m
    e.update(extra)
    return e


STEP_BYTES = 52  # algorithmic bytes per oth_step: in 16+1+1, out 16+1+8+8+1
LAUNCH_EVENTS = os.environ.get("BENCH_LAUNCH_EVENTS", "1") == "1"
PREWARM_SYNC = os.environ.get("BENCH_PREWARM_SYNC") == "1"  # diag: the round-2 pre-warm (a sync per launch)
# tests only: BENCH_DIST_BACKEND=gloo runs the N>1 line's collectives over gloo on
# host copies, so two ranks can share one GPU (RCCL needs one GPU per rank)
DIST_BACKEND = os.environ.get("BENCH_DIST_BACKEND", "nccl")
ROLLOUT_BYTES_PER_GAME = 18  # final board 16 + diff 1 + plies 1 written; opening generated in-kernel


def load_profile():
    """Per-launch PMC figures of the newest committed round profile
    (profiles/rNN_profile_summary.json, made by tools/profile_round.sh), if it
    was measured on the library this run loads: returns (file, kernels, stale)
    where stale describes a profile of another build (its PMC figures are then
    not used: no line mixes the counters of one build with the clock of another)."""
    import glob

    from subproc_amd._lib import library_sha16

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_profile_summary.json")))
    if not files:
        return None, {}, None
    with open(files[-1]) as f:
        d = json.load(f)
    name, have = os.path.basename(files[-1]), library_sha16()
    if d.get("library_sha16") != have:
        return name, {}, {"profile": name, "profile_library_sha16": d.get("library_sha16"),
                          "library_sha16": have, "note": "profile of another build: PMC figures omitted"}
    return name, d.get("kernels", {}), None


def profile_entry(kernels, name, grid=None, largest=False):
    """The profile entry of kernel `name` (at `grid` threads, or at its largest grid)."""
    best = None
    for k, e in kernels.items():
        kn, g = k.rsplit("@", 1)
        if kn == name and (grid is None or int(g) == grid):
            if not largest:
                return e
            if best is None or int(g) > best[0]:
                best = (int(g), e)
    return best[1] if best else None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--prewarm-ms", type=float, default=300.0,
                   help="untimed rollout launches before the warmup steps, so the GPU clock has ramped")
    p.add_argument("--workload", choices=["rollout", "greedy", "step"], default="rollout")
    p.add_argument("--games", type=int, default=1 << 20, help="games per GPU per bench step (rollout workloads)")
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--no-secondary", action="store_true", help="skip the secondary step/greedy/cpu measurements")
    p.add_argument("--cpu-games", type=int, default=250000,
                   help="bounded cpu_baseline sample (games): ~20 s of CPU work on 16 host threads")
    p.add_argument("--allreduce", choices=["async", "sync", "end"], default="end",
                   help="histogram all-reduce at N>1: per step overlapped with the next step (async), "
                        "per step blocking (sync), or once over all timed steps (end)")
    p.add_argument("--streams", type=int, default=2,
                   help="HIP streams the rollout steps are issued on round-robin (1 = serialized)")
    p.add_argument("--lib", default=None, help="diagnostic A/B only: load this build of the library instead of "
                                               "subproc_amd/lib/libsubproc_amd_hip.so")
    return p.parse_args()


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, cmd, env=None, port=None, poll_s=0.2):
    """Start `n` ranks of `cmd` as child processes (one per GPU, the layout
    torch.distributed.run gives) with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT set, and wait for them.  The children inherit
    stdout, so rank 0's JSON line is the line this process prints.  Returns 0
    if every rank exits 0; otherwise the first failing rank's code (a signal
    death maps to 128 + signal), after ending the remaining ranks, whose
    collectives could no longer complete.  The caller must not have touched
    the GPU: the children are fresh processes, never an exec.  This is the
    fan-out the reference does with replearn.py:78-86 -> eljem_worker.py:10."""
    import signal
    import subprocess

    base = dict(os.environ if env is None else env)
    port = port or free_port()
    procs = []

    def end_all(sig):  # the exact children this call started, never a pattern
        for q in procs:
            if q.poll() is None:
                q.send_signal(sig)

    # the children stay in this process's group, so a timeout that kills the
    # group ends them too; a SIGTERM to this process alone is passed on
    prev = signal.signal(signal.SIGTERM, lambda *_: (end_all(signal.SIGTERM), sys.exit(128 + signal.SIGTERM)))
    rc = 0
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                     MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen(cmd, env=e))
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    end_all(signal.SIGTERM)  # their collectives can no longer complete
            if live:
                time.sleep(poll_s)
    finally:
        end_all(signal.SIGKILL)
        for p in procs:
            p.wait()
        signal.signal(signal.SIGTERM, prev)
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without torchrun: this process stays off the
        # GPU and runs N ranks of the same command line as child processes
        raise SystemExit(spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__), *sys.argv[1:]]))
    if args.lib:
        from subproc_amd import _lib
        _lib.LIB_PATH = os.path.abspath(args.lib)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    # one rank per GPU; a box with fewer GPUs than ranks (the test that runs
    # two ranks on one GPU over gloo) puts ranks on GPU local % count
    ngpu = torch.cuda.device_count()
    local = local % ngpu if ngpu else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # BENCH_FORCE_DIST=1 runs the RCCL path (barrier, per-step histogram
    # all-reduce, max-over-ranks timing) even at world size 1
    use_dist = world > 1 or os.environ.get("BENCH_FORCE_DIST") == "1"
    if use_dist:
        if DIST_BACKEND == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from subproc_amd import ops

    stream = torch.cuda.current_stream()

    def barrier():
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if not use_dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if DIST_BACKEND != "gloo" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    policy = "greedy" if args.workload == "greedy" else "random"
    out = {}

    if args.workload in ("rollout", "greedy"):
        out.update(_bench_rollout(torch, dist, dev, stream, args, policy, world, rank, use_dist, barrier,
                                  max_over_ranks, args.streams))
    else:
        out.update(_bench_step(ops, torch, dev, stream, args, 65536, world, barrier, max_over_ranks,
                               index0=rank * 65536))

    # secondary + cpu_baseline: rank 0 at N=1 only (BENCH_FORCE_DIST=1 at N=1
    # takes the N>1 branch below instead, so one GPU exercises it)
    if world == 1 and not use_dist and not args.no_secondary:
        sec = {}

        def guarded(name, fn):
            # a failing secondary measurement is recorded, never costs the headline line
            try:
                sec[name] = fn()
            except Exception as e:  # noqa: BLE001
                sec[name] = {"error": repr(e)}

        if args.workload != "step":
            guarded("step_65536", lambda: _bench_step(ops, torch, dev, stream, args, 65536, 1, torch.cuda.synchronize,
                                                      lambda x: x, launches=200))
            guarded("step_65536_graph", lambda: _bench_step_graph(ops, torch, dev, args))
            guarded("step_steady_16M", lambda: _bench_step(ops, torch, dev, stream, args, 1 << 24, 1,
                                                           torch.cuda.synchronize, lambda x: x, launches=10))
        # BENCH_SKIP (comma list) drops secondary lines; tools/profile_round.sh skips
        # rollout_16M, which runs the headline kernel at the headline grid and would
        # otherwise be averaged into the headline's per-launch profile figures
        skip = set(filter(None, os.environ.get("BENCH_SKIP", "").split(",")))
        if args.workload in ("rollout", "greedy") and args.streams != 1 and "rollout_1stream" not in skip:
            def serial():
                r = _bench_rollout(torch, dist, dev, stream, args, policy, 1, 0, False, torch.cuda.synchronize,
                                   lambda x: x, 1)
                return {"metric": r["metric"] + ", one stream (launches serialized)", "value": r["value"],
                        "unit": r["unit"], "ms_per_step": r["ms_per_step"], "launch_ms": r["roofline"]["launch_ms"],
                        "valu_frac": r.get("valu", {}).get("frac")}
            guarded("rollout_1stream", serial)
        if args.workload in ("rollout", "greedy") and "rollout_sharded" not in skip:
            guarded("rollout_sharded_steps10", lambda: _bench_sharded(torch, args, policy))
        if args.workload == "rollout" and "rollout_16M" not in skip:
            guarded("rollout_16M", lambda: _bench_rollout_big(ops, torch, dev, args))
        def policy_line(pol):
            a = argparse.Namespace(**vars(args))
            a.steps, a.warmup, a.prewarm_ms = 10, 2, 0.0  # the GPU is warm by now
            r = _bench_rollout(torch, dist, dev, stream, a, pol, 1, 0, False, torch.cuda.synchronize, lambda x: x,
                               args.streams)
            what = "greedy-mobility" if pol == "greedy" else "linear-eval (learner default weights)"
            return {"metric": f"env-steps/sec ({what} self-play)", "value": r["value"], "unit": r["unit"],
                    "games": args.games, "steps": a.steps, "streams": args.streams, "ms_per_step": r["ms_per_step"],
                    "launch_ms": r["roofline"]["launch_ms"], "valu": r.get("valu"),
                    "grid_blocks": r["config"]["grid_blocks"], "cus": r["config"]["cus"]}

        if args.workload != "greedy":
            guarded("greedy_1M", lambda: policy_line("greedy"))
        guarded("eval_1M", lambda: policy_line("eval"))
        guarded("td_state_map", lambda: _bench_td(ops, torch, dev, args))
        guarded("book_emitter", lambda: _bench_books(ops, torch, dev, args))
        out["secondary"] = sec
        try:
            out["cpu_baseline"] = _cpu_baseline(args, policy if args.workload != "step" else "step")
        except Exception as e:  # noqa: BLE001
            out["cpu_baseline"] = {"error": repr(e)}
    elif use_dist and not args.no_secondary and args.workload != "step":
        # N>1: config 2's step over synthetic mid-game positions on every rank
        # (disjoint positions per rank, barrier + max-over-ranks timing), so the
        # step's env-steps/s and HBM roofline are reported at 2/4/8 GPUs too.
        # Not guarded: every rank must reach the same collectives.
        out["secondary"] = {
            "step_steady_16M": _bench_step(ops, torch, dev, stream, args, 1 << 24, world, barrier, max_over_ranks,
                                           launches=10, index0=rank << 24),
            "step_65536": _bench_step(ops, torch, dev, stream, args, 65536, world, barrier, max_over_ranks,
                                      launches=200, index0=rank * 65536)}
    if rank == 0:
        from subproc_amd._lib import library_sha16

        out["library_sha16"] = library_sha16()  # the build measured (profiles/ digests carry theirs)
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


def _bench_rollout(torch, dist, dev, stream, args, policy, world, rank, use_dist, barrier, max_over_ranks,
                   nstreams):
    """Configs 3/4/5: K bench steps, each one oth_rollout launch over `games`
    fresh games per GPU (+ the histogram all-reduce at N>1).  Steps are issued
    round-robin on `nstreams` HIP streams, each with its own output buffers:
    a launch's last batches (the per-launch tail) then share
    the CUs with the next step's first batches instead of idling them.  Every
    step still plays all of its games; nstreams=1 is the serialized figure."""
    from subproc_amd import _lib
    from subproc_amd._lib import HIST_BINS
    from subproc_amd.dist import bench_game_id0

    n = args.games
    hists = torch.zeros((args.warmup + args.steps, HIST_BINS), dtype=torch.int64, device=dev)
    # side streams from the process's one pool (ops._side_streams, which
    # rollout_batches uses too): every bench line reuses the same few streams
    # instead of creating its own, so the HIP runtime's hardware queues
    # (GPU_MAX_HW_QUEUES, 4 per process) are not spread over ever more streams
    from subproc_amd.ops import _side_streams

    streams = [stream] + _side_streams(dev, nstreams - 1)
    bufs = [(torch.empty((n, 2), dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int8, device=dev),
             torch.empty(n, dtype=torch.uint8, device=dev)) for _ in streams]
    # one work word per stream (include/othello.h: 0 before and after each launch)
    works = torch.zeros(len(streams), dtype=torch.int64, device=dev)
    lib = _lib.load()
    pid = {"random": 0, "greedy": 1, "eval": 2}[policy]
    wptr = None
    if policy == "eval":
        from subproc_amd.ops import _weights_ptr
        from subproc_amd.params import DEFAULT_WEIGHTS

        wptr = _weights_ptr(DEFAULT_WEIGHTS)  # the learner's default table

    def launch(gid, fb, df, pl, h, w, st):
        if policy == "eval":
            return lib.oth_rollout_eval(None, None, args.seed, gid, 10, wptr, fb.data_ptr(), df.data_ptr(),
                                        pl.data_ptr(), None, h.data_ptr(), w.data_ptr(), n, st.cuda_stream)
        return lib.oth_rollout(None, None, args.seed, gid, pid, 10, fb.data_ptr(), df.data_ptr(), pl.data_ptr(), None,
                               h.data_ptr(), w.data_ptr(), n, st.cuda_stream)

    pending = []
    # per-launch events on the launch's own stream (the roofline's launch duration)
    l0 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    l1 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    def one_step(s, k=None):
        # bench step s plays global game ids [(s*world + rank)*n, +n): fresh games every step
        st = streams[s % nstreams]
        fb, df, pl = bufs[s % nstreams]
        h = hists[s]
        if k is not None and LAUNCH_EVENTS:
            l0[k].record(st)
        w = works[s % nstreams:s % nstreams + 1]
        _lib.check(launch(bench_game_id0(s, rank, world, n), fb, df, pl, h, w, st), "rollout")
        if k is not None and LAUNCH_EVENTS:
            l1[k].record(st)
        if use_dist and args.allreduce != "end":
            if DIST_BACKEND == "gloo":
                raise SystemExit("bench: BENCH_DIST_BACKEND=gloo supports --allreduce end only")
            # config 4: the one collective, ordered after this step's rollout on its stream.
            # Async on RCCL's stream, so it overlaps the next steps (each step owns its
            # histogram row); all are waited for inside the timed region.
            with torch.cuda.stream(st):
                work = dist.all_reduce(h, op=dist.ReduceOp.SUM, async_op=args.allreduce == "async")
            if work is not None:
                pending.append(work)

    def drain():
        while pending:
            pending.pop().wait()

    def fork():  # side streams start after everything issued so far on the main stream
        e = torch.cuda.Event()
        e.record(stream)
        for st in streams[1:]:
            st.wait_event(e)

    def join():  # the main stream waits for the side streams
        for st in streams[1:]:
            e = torch.cuda.Event()
            e.record(st)
            stream.wait_event(e)

    # clock pre-warm (untimed, local, no collective): the GPU ramps its clock
    # over the first ~100 ms of work, longer than a few warmup steps take.  The
    # launches go round-robin on the bench's streams with no host sync between
    # them (a sync every 16 bounds the queue), the load the timed steps put on
    # the chip: with a sync after every launch the first timed region still
    # ran ~3% slower than the next ones (tools/diag/timeline.py)
    scratch = torch.zeros(HIST_BINS, dtype=torch.int64, device=dev)
    t_w = time.perf_counter()
    k = 0
    fork()
    while (time.perf_counter() - t_w) * 1e3 < args.prewarm_ms:
        i = k % nstreams
        fb, df, pl = bufs[i]
        _lib.check(launch(1 << 52, fb, df, pl, scratch, works[i:i + 1], streams[i]), "rollout")
        k += 1
        if PREWARM_SYNC or k % 16 == 0:
            torch.cuda.synchronize()
    join()
    torch.cuda.synchronize()
    fork()
    for s in range(args.warmup):
        one_step(s)
    join()
    drain()
    barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    fork()  # host-side set-up of the side streams' start, before the clock starts
    t0 = time.perf_counter()
    for k, s in enumerate(range(args.warmup, args.warmup + args.steps)):
        one_step(s, k)
    join()
    if use_dist and args.allreduce == "end":
        total = hists[args.warmup:].sum(0)
        if DIST_BACKEND == "gloo":  # tests only: gloo reduces host memory
            host = total.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM)
            total.copy_(host)
        else:
            dist.all_reduce(total, op=dist.ReduceOp.SUM)
        hists[args.warmup].copy_(total)
        hists[args.warmup + 1:].zero_()
    ev1.record(stream)
    drain()
    barrier()
    t1 = time.perf_counter()
    elapsed = max_over_ranks(t1 - t0)
    step_ms = ev0.elapsed_time(ev1) / args.steps  # stream time per step (+ the all-reduce at N>1)
    launch = sorted(l0[k].elapsed_time(l1[k]) for k in range(args.steps)) if LAUNCH_EVENTS else [step_ms]
    launch_ms = sum(launch) / len(launch)
    median_ms = launch[len(launch) // 2] if len(launch) % 2 else \
        0.5 * (launch[len(launch) // 2 - 1] + launch[len(launch) // 2])
    timed = hists[args.warmup:].sum(0).cpu()  # already global (all-reduced) when distributed
    env_steps = int(timed[132])
    games = n * world * args.steps
    # self-check of the sharding: every game of every rank is in the reduced
    # histogram exactly once (its 129 diff bins and its W/L/D bins)
    counted = int(timed[:129].sum())
    if counted != games or int(timed[129:132].sum()) != games:
        raise SystemExit(f"bench: the reduced histogram counts {counted} games, expected {games}")
    out = dict(metric="env-steps/sec (batched self-play)", value=env_steps / elapsed, unit="env-steps/s",
               n_gpus=world, steps=args.steps, warmup=args.warmup, ms_per_step=elapsed / args.steps * 1e3,
               higher_is_better=True, scaling="weak", vs_baseline=None, dtype="u64",
               data="synthetic (games from the opening, counter-based RNG seed %#x)" % args.seed,
               prewarm_ms=args.prewarm_ms,
               config={"workload": "config%s: %s-policy self-play rollouts to terminal" %
                       ({"random": "3" if world == 1 else "4", "greedy": "5", "eval": " §8f"}[policy], policy),
                       "games_per_gpu": n, "global_batch": n * world, "parallelism": "dp%d" % world,
                       "streams": nstreams, "env_steps_per_game": env_steps / games, "world_size": world,
                       "grid_blocks": lib.oth_rollout_grid(pid, n),
                       "cus": torch.cuda.get_device_properties(dev).multi_processor_count,
                       "game_ids": _game_id_ranges(n, world, args.warmup, args.steps),
                       "games_counted": counted, "env_steps": env_steps,
                       "black_white_draw": [int(v) for v in timed[129:132]]})
    # roofline: algorithmic bytes of one launch / that launch's duration (events on its stream)
    achieved = n * ROLLOUT_BYTES_PER_GAME / (launch_ms * 1e-3) / 1e9
    kname = "rollout_kernel<%d, false>" % pid
    pfile, kernels, stale = load_profile()
    prof = profile_entry(kernels, kname, largest=True) if n == 1 << 20 else None
    # "bound" prices the launch's algorithmic HBM bytes (the contract's roofline);
    # the resource that binds this kernel is VALU issue ("binding", and "valu")
    out["roofline"] = {"bound": "hbm", "binding": "valu", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": achieved / HBM_PEAK_GBS,
                       "traffic": prof.get("hbm_bytes") if prof else None,
                       "kernel": kname, "launch_ms": launch_ms, "launch_ms_median": median_ms,
                       "step_ms": step_ms, "profile": pfile if prof else None, "profile_stale": stale,
                       "note": "%d algorithmic B/game written (final board, diff, plies); the kernel is "
                               "integer-VALU-bound, see 'valu'. launch_ms: one launch's duration; step_ms: "
                               "stream time per step with %d launches in flight" % (ROLLOUT_BYTES_PER_GAME,
                                                                                     nstreams)}
    if prof and "SQ_INSTS_VALU" in prof:
        # device-wide issue rate: a launch's instructions per step of stream time
        va = prof["SQ_INSTS_VALU"] / (step_ms * 1e-3)
        out["valu"] = valu_entry(kname, va, instr_per_launch=prof["SQ_INSTS_VALU"])
    return out


def _game_id_ranges(n, world, warmup, steps):
    """The global game ids each rank plays in the timed steps (dist.bench_game_id0):
    step s on rank r plays [(s*world + r)*n, +n); listed per rank as its first
    and last timed range, with the rule, so an N-GPU line is self-describing."""
    from subproc_amd.dist import bench_game_id0

    first, last = warmup, warmup + steps - 1
    return {"rule": "step s on rank r: [(s*%d + r)*%d, +%d), timed steps s = %d..%d" % (world, n, n, first, last),
            "per_rank": {str(r): [[bench_game_id0(first, r, world, n), bench_game_id0(first, r, world, n) + n],
                                  [bench_game_id0(last, r, world, n), bench_game_id0(last, r, world, n) + n]]
                         for r in range(world)}}


def _bench_step(ops, torch, dev, stream, args, n, world, barrier, max_over_ranks, launches=None, index0=0):
    """config 2: oth_step over n reachable mid-game positions (inputs resident in
    HBM); at N>1 each rank steps its own positions [index0, index0 + n)."""
    from subproc_amd import _lib

    lib = _lib.load()
    pos = ops.sample_midgame(n, args.seed, index0=index0, device=dev)
    bo = torch.empty_like(pos.boards)
    to = torch.empty_like(pos.turn)
    fl = torch.empty(n, dtype=torch.int64, device=dev)
    ln = torch.empty(n, dtype=torch.int64, device=dev)
    rt = torch.empty(n, dtype=torch.int8, device=dev)
    K = launches if launches is not None else args.steps
    ptrs = (pos.boards.data_ptr(), pos.turn.data_ptr(), pos.move.data_ptr(), bo.data_ptr(), to.data_ptr(),
            fl.data_ptr(), ln.data_ptr(), rt.data_ptr(), None, n, stream.cuda_stream)
    for _ in range(max(3, args.warmup)):
        _lib.check(lib.oth_step(*ptrs), "oth_step")
    if n >= 1 << 20:
        # the steady-state line: ~200 ms more of untimed launches, so the clock
        # has ramped back up after the launch-bound lines before it (10
        # warmup launches of 16M boards are 2 ms; timed that way the step ran
        # 10-13% slower than after a ramp, tools/diag/step_ab.py)
        torch.cuda.synchronize()
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < 0.2:
            for _ in range(20):
                _lib.check(lib.oth_step(*ptrs), "oth_step")
            torch.cuda.synchronize()
    barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(K):
        _lib.check(lib.oth_step(*ptrs), "oth_step")
    ev1.record(stream)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    kern_ms = ev0.elapsed_time(ev1) / K
    steps = n * K * world
    achieved = n * STEP_BYTES / (kern_ms * 1e-3) / 1e9
    pfile, kernels, stale = load_profile()
    prof = profile_entry(kernels, "step_kernel", n)
    r = {"metric": "env-steps/sec (batched step)", "value": steps / elapsed, "unit": "env-steps/s",
         "n_gpus": world, "batch": n, "launches": K, "us_per_launch": kern_ms * 1e3, "dtype": "u64",
         "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": achieved / HBM_PEAK_GBS, "traffic": prof.get("hbm_bytes") if prof else None,
                      "kernel": "step_kernel", "profile": pfile if prof else None, "profile_stale": stale}}
    if prof and "SQ_INSTS_VALU" in prof:
        va = prof["SQ_INSTS_VALU"] / (kern_ms * 1e-3)
        r["valu"] = valu_entry("step_kernel", va)
    return r


def _bench_step_graph(ops, torch, dev, args, n=65536, launches=200):
    """config 2 with the launch-bound loop captured in a HIP graph (one replay =
    `launches` oth_step launches; the C-ABI launches on the capturing stream)."""
    from subproc_amd import _lib

    lib = _lib.load()
    pos = ops.sample_midgame(n, args.seed, index0=0, device=dev)
    bo, to = torch.empty_like(pos.boards), torch.empty_like(pos.turn)
    fl, ln = torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int64, device=dev)
    rt = torch.empty(n, dtype=torch.int8, device=dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(launches):
            _lib.check(lib.oth_step(pos.boards.data_ptr(), pos.turn.data_ptr(), pos.move.data_ptr(), bo.data_ptr(),
                                    to.data_ptr(), fl.data_ptr(), ln.data_ptr(), rt.data_ptr(), None, n, st),
                       "oth_step")
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"metric": "env-steps/sec (batched step, HIP graph of %d launches)" % launches,
            "value": n * launches / dt, "unit": "env-steps/s", "batch": n, "launches": launches,
            "us_per_launch": dt / launches * 1e6}


def _bench_sharded(torch, args, policy, steps=10, reps=5):
    """The product's multi-GPU entry as a single-process caller uses it:
    dist.rollout_sharded(steps * games, steps=steps) -- `steps` batches of
    `games` games (ops.rollout_batches: merged into launches of up to
    ops.ROLLOUT_MERGE_GAMES, round-robin on the streams) -- timed by the host
    clock around the call and a device sync (median of `reps`, after ~0.3 s
    of the same calls so that the clock has ramped, as for the headline)."""
    from subproc_amd.dist import rollout_sharded
    from subproc_amd.ops import ROLLOUT_MERGE_GAMES

    n = args.games
    t_end = time.perf_counter() + args.prewarm_ms * 1e-3
    while True:  # first use, then the clock ramp
        rollout_sharded(steps * n, args.seed, policy, steps=steps, game_id_base=1 << 45)
        torch.cuda.synchronize()
        if time.perf_counter() >= t_end:
            break
    out = {"metric": "env-steps/sec (dist.rollout_sharded, %d batches of %d games, one process)" % (steps, n),
           "unit": "env-steps/s", "policy": policy, "merge_games": ROLLOUT_MERGE_GAMES}
    for streams in (2,):
        rates, gpu_rates = [], []
        for r in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            hist, _ = rollout_sharded(steps * n, args.seed, policy, steps=steps, streams=streams,
                                      game_id_base=(1 << 45) + (r + 1) * steps * n)
            e1.record()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            env = int(hist[132])
            rates.append(env / dt)  # the caller's clock: Python set-up and the last launch's tail included
            gpu_rates.append(env / (e0.elapsed_time(e1) * 1e-3))  # the stream's clock, call entry to last launch end
        rates.sort()
        gpu_rates.sort()
        key = "" if streams == 2 else "_3streams"
        out["value" + key] = rates[len(rates) // 2]
        out["gpu_clock_value" + key] = gpu_rates[len(gpu_rates) // 2]
        out["reps" + key] = rates
    return out


def _bench_rollout_big(ops, torch, dev, args, games=1 << 24, reps=3):
    """The config-3 kernel on 16,777,216 games per launch: the per-launch tail
    (the last batches of 64 games start late and run ~60 plies) amortises, so
    this shows the kernel's steady-state rate next to config 3's 1M batch."""
    hist = torch.zeros(133, dtype=torch.int64, device=dev)
    ops.rollout(games, args.seed, 1 << 42, "random", hist=hist, device=dev, want_boards=False, want_diff=False,
                want_plies=False)
    torch.cuda.synchronize()
    hist.zero_()
    t0 = time.perf_counter()
    for k in range(reps):
        ops.rollout(games, args.seed, (1 << 42) + (k + 1) * games, "random", hist=hist, device=dev,
                    want_boards=False, want_diff=False, want_plies=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"metric": "env-steps/sec (random self-play, 16M games per launch)", "value": int(hist[132]) / dt,
            "unit": "env-steps/s", "games": games, "launches": reps, "ms_per_launch": dt / reps * 1e3}


def _bench_books(ops, torch, dev, args, games=1 << 18, reps=10):
    """§8f row 1: the book emitter over 262,144 games -- the packed-rows replay
    (oth_replay_rows: each game's plies + 1 recorded positions, turn and
    is_game_over) and oth_book_text of exactly those rows, as GameBooks runs
    them; the strided replay (oth_replay, all 129 rows per game) beside it.
    HIP events, after 3 untimed launches each."""
    r = ops.rollout(games, args.seed, 1 << 40, "random", record_moves=True, device=dev)
    out = {}

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    from subproc_amd import _lib
    lib = _lib.load()
    row_off, rows = ops.row_offsets(r.plies)
    pk = ops.replay_rows(r.moves, r.plies)
    st = torch.cuda.current_stream().cuda_stream
    args_rows = (None, None, r.moves.data_ptr(), r.plies.data_ptr(), row_off.data_ptr(), pk.boards.data_ptr(),
                 pk.turn.data_ptr(), pk.end.data_ptr(), games, st)
    us = timed(lambda: _lib.check(lib.oth_replay_rows(*args_rows), "oth_replay_rows"))
    # algorithmic bytes: 128-B move record + plies + row offset read; 18 B per recorded row written
    rb = games * (128 + 1 + 8) + rows * 18
    out["replay_rows"] = {"games": games, "rows": rows, "us": us, "achieved_gbs": rb / us / 1e3,
                          "frac_hbm": rb / us / 1e3 / HBM_PEAK_GBS, "algorithmic_bytes": rb}
    us = timed(lambda: ops.book_text(pk.boards, pk.turn))
    tb = rows * (16 + 1 + 67)
    out["book_text"] = {"lines": rows, "us": us, "achieved_gbs": tb / us / 1e3, "frac_hbm": tb / us / 1e3 / HBM_PEAK_GBS}
    # the reader's side: the same text parsed back in place (oth_book_parse,
    # stride 67 with the side to move) -- checked against the rows it came from
    text = ops.book_text(pk.boards, pk.turn)
    pb, pt = ops.book_parse(text, rows, stride=67, want_turn=True)
    if not (torch.equal(pb, pk.boards) and torch.equal(pt, pk.turn)):
        raise SystemExit("bench: oth_book_parse did not give back the replayed rows")
    us = timed(lambda: ops.book_parse(text, rows, stride=67, want_turn=True))
    pbytes = rows * (67 + 16 + 1)
    out["book_parse"] = {"lines": rows, "us": us, "achieved_gbs": pbytes / us / 1e3,
                         "frac_hbm": pbytes / us / 1e3 / HBM_PEAK_GBS}
    del text, pb, pt
    packed = torch.empty(rows * 64, dtype=torch.uint8, device=dev).view(rows, 64)
    packed.copy_(ops.book_text(pk.boards, pk.turn).view(rows, 67)[:, :64])
    packed = packed.view(-1)
    us = timed(lambda: ops.book_parse(packed, rows, stride=64))
    pbytes = rows * (64 + 16)
    out["book_parse_packed"] = {"lines": rows, "us": us, "achieved_gbs": pbytes / us / 1e3,
                                "frac_hbm": pbytes / us / 1e3 / HBM_PEAK_GBS}
    del packed
    us = timed(lambda: ops.replay(r.moves, r.plies))
    sb = games * (128 + 1 + 129 * 18)  # the strided table: all 129 rows per game written
    out["replay_strided"] = {"games": games, "us": us, "achieved_gbs": sb / us / 1e3,
                             "useful_gbs": rb / us / 1e3, "frac_hbm": sb / us / 1e3 / HBM_PEAK_GBS}
    out["metric"] = ("book emitter (packed replay + serialize_str text) per 262,144 games; book_parse: the text "
                     "parsed back (flat-file lines, and packed 64-byte strings)")
    return out


def _bench_td(ops, torch, dev, args, games=1 << 18, reps=7):
    """§8f row 2: the learner's TD state-map update for a batch of GPU self-play
    books (packed replay + ordered update stream + stable sort + per-key EMA +
    merge into a table that already holds two batches).  The third batch is
    applied `reps` times, each time to a fresh copy of the two-batch table (the
    copy outside the timed region), and the median is reported (round 5: the
    round-4 line timed one application once)."""
    import statistics

    from subproc_amd.td import StateMap

    rs = [ops.rollout(games, args.seed, (1 << 41) + k * games, "random", record_moves=True, device=dev)
          for k in range(3)]
    sm = StateMap(dev)
    for r in rs[:2]:  # the empty-table path, then the merge path (first-use kernel loading)
        sm.update_rows(ops.replay_rows(r.moves, r.plies), r.plies)
    base_k, base_v = sm.keys.clone(), sm.values.clone()
    r2 = rs[2]
    times, n_upd = [], 0
    for _ in range(reps + 1):  # the first application warms the merge path at this size
        sm.keys, sm.values = base_k.clone(), base_v.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # the books as GameBooks holds them: the packed replay (each game's
        # recorded rows only), then the update over those rows
        n_upd = sm.update_rows(ops.replay_rows(r2.moves, r2.plies), r2.plies)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    times = times[1:]
    dt = statistics.median(times)
    return {"metric": "TD state-map updates/sec (position x side, learner order)", "value": n_upd / dt,
            "unit": "updates/s", "games": games, "updates": n_upd, "keys": len(sm), "ms": dt * 1e3,
            "ms_min": min(times) * 1e3, "ms_max": max(times) * 1e3, "reps": reps, "stat": "median"}


def _cpu_baseline(args, workload):
    """The C oracle (board.py restated as an 8x8 mailbox ray scan) on host cores."""
    import oracle

    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    # every core of the affinity mask, capped by OMP_NUM_THREADS where the
    # environment sets it (the GPU box sets 16: its CPU share per GPU)
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = max(1, min(affinity, int(omp))) if omp and omp.isdigit() else affinity
    host = {"nproc": os.cpu_count(), "affinity_cores": affinity, "omp_num_threads": omp,
            "cores_note": "threads = min(affinity cores, OMP_NUM_THREADS): the GPU box's affinity mask shows the "
                          "whole host (%d cores) but its CPU share per GPU is OMP_NUM_THREADS=%s, which the pool "
                          "sets and asks jobs to stay within; the one_thread figure scales the port per core"
                          % (affinity, omp)}
    if workload == "step":
        pos = oracle.sample_midgame(65536, args.seed)
        t0 = time.perf_counter()
        reps = 20
        for _ in range(reps):
            oracle.step(pos["boards"], pos["turn"], pos["move"])
        dt = time.perf_counter() - t0
        return {"value": 65536 * reps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port", **host,
                "sample": "%d x oracle_step over 65,536 mid-game positions" % reps}
    games = args.cpu_games
    pid = 0 if workload == "random" else 1
    if pid == 1:
        games = max(1000, games // 10)

    def timed_rollout(n_games, n_threads, game_id0):
        t0 = time.perf_counter()
        r = oracle.rollout(n_games, args.seed, game_id0, pid, 10, n_threads=n_threads)
        dt = time.perf_counter() - t0
        return int(r["hist"][132]), dt

    steps, dt = timed_rollout(games, threads, 0)
    # the same restatement on one thread: 1/16 of the sample, other game ids
    g1 = max(100, games // 16)
    steps1, dt1 = timed_rollout(g1, 1, 1 << 40)
    return {"value": steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port", **host,
            "sample": "%d %s games from the opening (%d env-steps), C mailbox restatement of board.py "
                      "(oracle/othello_oracle.c: board.py's 8x8 ray scan from every cell), OpenMP %d threads, "
                      "%.2f s wall" % (games, workload, steps, threads, dt),
            "one_thread": {"value": steps1 / dt1, "unit": "env-steps/s", "cores": 1,
                           "sample": "%d %s games (%d env-steps), 1 thread, %.2f s" % (g1, workload, steps1, dt1)},
            "board_py_note": "board.py itself (Python) measured at ~2.9e3 env-steps/s/core in the build container "
                             "(BASELINE.md); it cannot run on the GPU box"}


if __name__ == "__main__":
    main()
