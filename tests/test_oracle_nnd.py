"""CPU: the nnd oracle (oracle/pcr_oracle.c) is bit-exact with the reference's
compiled my_lib.cpp on every committed golden case (tests/golden/nnd_golden.npz)."""
import hashlib

import numpy as np
import pytest

from nnd_cases import CASES, make_inputs


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference_golden(oracle, golden_nnd, name):
    x1, x2, gd1, gd2 = make_inputs(CASES[name])
    d1, d2, i1, i2 = oracle.nnd_forward(x1, x2)
    h = hashlib.sha256()
    for a in (d1, d2, i1, i2):
        h.update(a.tobytes())
    assert h.digest() == bytes(golden_nnd[f"{name}/sha_fwd"])
    g1, g2 = oracle.nnd_backward(x1, x2, gd1, gd2, i1, i2)
    h = hashlib.sha256()
    h.update(g1.tobytes())
    h.update(g2.tobytes())
    assert h.digest() == bytes(golden_nnd[f"{name}/sha_bwd"])


def test_oracle_first_index_tie_rule(oracle):
    # two identical candidates: the lower index must win (my_lib.cpp:16 strict '<')
    x1 = np.array([[[0.5, 0.5, 0.5]]], np.float32)
    x2 = np.array([[[1, 1, 1], [0.5, 0.5, 0.75], [0.5, 0.5, 0.75], [0.5, 0.5, 0.25]]], np.float32)
    d1, d2, i1, i2 = oracle.nnd_forward(x1, x2)
    assert i1[0, 0] == 1
    assert np.all(i2 == 0)


def test_oracle_empty_candidates(oracle):
    x1 = np.random.default_rng(0).random((2, 5, 3), dtype=np.float32)
    x2 = np.zeros((2, 0, 3), np.float32)
    d1, d2, i1, i2 = oracle.nnd_forward(x1, x2)
    assert np.all(d1 == 0) and np.all(i1 == 0) and d2.size == 0
