"""Loaders for the committed golden fixtures (tests/golden/, made by gen_golden.py
from the real reference board.py).  Pure data: JSON and allow_pickle=False npz."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def h(x):
    return np.uint64(int(x, 16))


ROLLOUT_FIXTURES = ["rollout_random", "rollout_random_offset", "rollout_random_from_mid", "rollout_greedy",
                    "rollout_greedy_from_mid", "rollout_eval", "rollout_eval_rand_from_mid", "rollout_match"]

RUNNER_FIXTURES = ["rollout_runner_eval", "rollout_runner_greedy", "rollout_runner_eval_mid"]
