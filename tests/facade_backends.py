"""Backends for the drop-in Board facade in the tests.

The facade (subproc_amd/board.py) sends every rule question to a device object
(``board._TLS.dev``, this thread's) with four calls: legal, result, step, hands.  On the GPU box
that is the HIP library.  For the CPU suite, :class:`CpuAbiDevice` answers the
same four calls from libothello_cpu.so -- include/othello.h built for the host
over the oracle (test infrastructure) -- so the facade's own host logic
(index wrapping, the live board view, other-valued cells, put's direction
order) is checked against board.py's fixtures without a GPU.
"""
import ctypes

import numpy as np
import pytest

import oracle

P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


def _i64(x):
    return x - (1 << 64) if x >= 1 << 63 else x


class CpuAbiDevice:
    def __init__(self):
        self.L = oracle.cpu_abi()

    def legal(self, black, white, code):
        b = np.array([[black, white]], np.uint64)
        out = np.zeros(1, np.uint64)
        assert self.L.oth_legal(P(b), P(np.array([code], np.uint8)), P(out), 1, None) == 0
        return int(out[0])

    def result(self, black, white):
        b = np.array([[black, white]], np.uint64)
        nb, nw, te = np.zeros(1, np.uint8), np.zeros(1, np.uint8), np.zeros(1, np.uint8)
        assert self.L.oth_result(P(b), P(nb), P(nw), None, P(te), 1, None) == 0
        return int(nb[0]), int(nw[0]), bool(te[0])

    def step(self, black, white, code, move):
        b = np.array([[black, white]], np.uint64)
        bo, fl = np.zeros((1, 2), np.uint64), np.zeros(1, np.uint64)
        to, ret = np.zeros(1, np.uint8), np.zeros(1, np.int8)
        assert self.L.oth_step(P(b), P(np.array([code], np.uint8)), P(np.array([move], np.uint8)), P(bo), P(to),
                               P(fl), None, P(ret), None, 1, None) == 0
        return int(bo[0, 0]), int(bo[0, 1]), int(fl[0]), int(ret[0])

    def hands(self, own, hostile, rows):
        n = len(rows)
        a = np.array(rows, np.int64).reshape(n, 4)
        cols = [np.ascontiguousarray(a[:, k]) for k in range(4)]
        ow = np.full(n, own, np.uint64)
        ho = np.full(n, hostile, np.uint64)
        out = np.zeros(n, np.uint8)
        assert self.L.oth_hands(P(ow), P(ho), *[P(c) for c in cols], P(out), n, None) == 0
        return out.tolist()


BACKENDS = ["cpu_abi", pytest.param("gpu", marks=pytest.mark.gpu)]


@pytest.fixture(params=BACKENDS)
def facade(request):
    """subproc_amd.board with its device calls served by `request.param`."""
    from subproc_amd import board as gboard
    saved = getattr(gboard._TLS, "dev", None)
    gboard._TLS.dev = CpuAbiDevice() if request.param == "cpu_abi" else gboard._Device()
    try:
        yield gboard
    finally:
        gboard._TLS.dev = saved
