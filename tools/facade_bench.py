"""Cost of the drop-in facade per GameRunner ply (SURVEY.md §8b layer 1), on the GPU box.

A GameRunner ply through a `board` module is go_for's puttables(turn)
(game_runner.py:137-152), put_s (157) and is_game_over (158): this plays random
games that way through subproc_amd.board.Board and reports microseconds per ply,
next to board.py's own per-ply cost measured in the build container (BASELINE.md
§2: ~2,900 env-steps/s on one core = ~345 us per ply).  Also times the greedy
and eval engines' move choice (subproc_amd.engine), one call per position.
"""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import board as gboard  # noqa: E402
from subproc_amd import engine  # noqa: E402
from subproc_amd.codec import handstr_from_coord  # noqa: E402


def play(n_games, seed):
    rng = random.Random(seed)
    plies = 0
    for _ in range(n_games):
        b = gboard.Board()
        while True:
            puts = b.puttables(b.turn)
            mv = handstr_from_coord(*puts[rng.randrange(len(puts))]) if puts else "PS"
            b.put_s(mv)
            plies += 1
            if b.is_game_over():
                break
    return plies


def engine_choice(policy, n_games, seed):
    eng = engine.Engine(policy=policy, seed=seed)
    calls = 0
    t = 0.0
    for _ in range(n_games):
        eng.board = gboard.Board()
        while not eng.board.is_game_over():
            t0 = time.perf_counter()
            mv = eng.choose()
            t += time.perf_counter() - t0
            calls += 1
            eng.board.put_s(mv.lower() if mv != "PS" else "PS")
    return calls, t


def main():
    torch.cuda.init()
    play(2, 1)  # warm-up: library load, first launches
    t0 = time.perf_counter()
    plies = play(int(os.environ.get("FACADE_GAMES", "40")), 7)
    dt = time.perf_counter() - t0
    out = {"facade_ply_us": dt / plies * 1e6, "plies": plies, "facade_env_steps_per_s": plies / dt,
           "board_py_ply_us_build_container": 1e6 / 2.9e3}
    for pol in ("greedy", "eval"):
        engine_choice(pol, 1, 0)
        calls, t = engine_choice(pol, 10, 3)
        out[f"engine_{pol}_choose_us"] = t / calls * 1e6
    print(json.dumps(out))


if __name__ == "__main__":
    main()
