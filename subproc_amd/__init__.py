"""subproc_amd — MI355X-native batched Othello environment (the board.py step
path of ysnrkdm/subproc, re-designed for gfx950).

Modules:
  ops     tensor-level batched kernels (reset / legal / step / result / rollout)
  env     VecEnv: reset / legal_moves / step / result over N games in HBM
  board   drop-in ``board`` module: the reference Board class API
  codec   Edax move strings and book text (host side)
  dist    one-process-per-GPU sharded rollouts + histogram all-reduce
The compute lives in lib/libsubproc_amd_hip.so (C-ABI: include/othello.h).
"""
__version__ = "0.1.0"

from ._lib import (BLACK, HIST_BINS, PASS, WHITE, OthelloCallError, OthelloLibraryError, load as load_library,
                   version as library_version)

__all__ = ["BLACK", "WHITE", "PASS", "HIST_BINS", "OthelloLibraryError", "OthelloCallError", "load_library",
           "library_version", "__version__"]
