"""Input specs of the nndistance golden cases (shared by the generator and tests).

Inputs are regenerated bit-identically from numpy's PCG64 seeds, so the committed
nnd_golden.npz only holds the reference's outputs.
"""
import numpy as np

CASES = {
    # config 2: B=1, N=M=4096, U[0,1)^3
    "c2_4096": dict(b=1, n=4096, m=4096, seed=0),
    # the reference's own smoke shape (dip/torch-nndistance/test.py:8-9)
    "testpy_16x2048x1024": dict(b=16, n=2048, m=1024, seed=1),
    "small_1024": dict(b=1, n=1024, m=1024, seed=2),
    # N != M, ragged small sizes, B > 32 (the CUDA grid.x of 32 wraps)
    "ragged_37": dict(b=3, n=1000, m=37, seed=3),
    "ragged_1": dict(b=2, n=5, m=1, seed=4),
    "batch40": dict(b=40, n=64, m=80, seed=5),
    # 1/16-quantised cloud: massive exact ties -> first-index rule
    "quantised_ties": dict(b=2, n=1500, m=1700, seed=6, quant=16),
    # duplicated candidate points (identical rows) -> first index wins
    "duplicates": dict(b=1, n=700, m=600, seed=7, dup=True),
    # NaN coordinates, including candidate 0 (the k == 0 seed rule)
    "nan_inputs": dict(b=2, n=50, m=60, seed=8, nan=True),
    # large-magnitude coords (catastrophic cancellation exercised bit-exactly)
    "offset_1e4": dict(b=1, n=900, m=800, seed=9, offset=1.0e4),
}


def make_inputs(spec):
    rng = np.random.default_rng(spec["seed"])
    b, n, m = spec["b"], spec["n"], spec["m"]
    x1 = rng.random((b, n, 3), dtype=np.float32)
    x2 = rng.random((b, m, 3), dtype=np.float32)
    if spec.get("quant"):
        q = spec["quant"]
        x1 = (np.floor(x1 * q) / q).astype(np.float32)
        x2 = (np.floor(x2 * q) / q).astype(np.float32)
    if spec.get("dup"):
        src = rng.integers(0, m // 4, size=m)
        x2 = x2[:, src, :].copy()
    if spec.get("offset"):
        x1 = (x1 + np.float32(spec["offset"])).astype(np.float32)
        x2 = (x2 + np.float32(spec["offset"])).astype(np.float32)
    if spec.get("nan"):
        x2[0, 0, 1] = np.nan          # candidate 0 of batch 0 is NaN (seed rule)
        x2[1, 7, 0] = np.nan          # an interior NaN candidate (skipped)
        x1[1, 3, 2] = np.nan          # a NaN query
    gd1 = rng.standard_normal((b, n)).astype(np.float32)
    gd2 = rng.standard_normal((b, m)).astype(np.float32)
    return x1, x2, gd1, gd2
