"""numpy front-end of the CPU oracle (liboracle.so built from pcr_oracle.c).

TEST INFRASTRUCTURE ONLY -- used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker.  Nothing in the product imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def nnd_forward(xyz1, xyz2):
    """Restatement of my_lib.cpp:28-60: returns dist1, dist2, idx1, idx2."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, n, m = xyz1.shape[0], xyz1.shape[1], xyz2.shape[1]
    d1 = np.zeros((b, n), np.float32)
    d2 = np.zeros((b, m), np.float32)
    i1 = np.zeros((b, n), np.int32)
    i2 = np.zeros((b, m), np.int32)
    lib().oracle_nnd_forward(_p(xyz1), _p(xyz2), b, n, m, _p(d1), _p(d2), _p(i1), _p(i2))
    return d1, d2, i1, i2


def nnd_backward(xyz1, xyz2, gd1, gd2, idx1, idx2):
    """Restatement of my_lib.cpp:64-133: returns gradxyz1, gradxyz2."""
    xyz1, xyz2, gd1, gd2 = _f32(xyz1), _f32(xyz2), _f32(gd1), _f32(gd2)
    idx1, idx2 = _i32(idx1), _i32(idx2)
    b, n, m = xyz1.shape[0], xyz1.shape[1], xyz2.shape[1]
    g1 = np.zeros((b, n, 3), np.float32)
    g2 = np.zeros((b, m, 3), np.float32)
    lib().oracle_nnd_backward(_p(xyz1), _p(xyz2), _p(gd1), _p(gd2), _p(idx1), _p(idx2),
                              b, n, m, _p(g1), _p(g2))
    return g1, g2
