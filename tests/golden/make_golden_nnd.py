"""Generate tests/golden/nnd_golden.npz from the REFERENCE's compiled CPU nndistance.

Runs in the build container only (needs /root/reference + oracle/_ref, built by
oracle/build_ref.sh from dip/torch-nndistance/src/my_lib.cpp).  The committed
.npz is data: inputs are regenerated from the recorded numpy seeds, outputs are
the reference's nnd_forward / nnd_backward results (full arrays for small cases,
SHA-256 + sampled rows for large ones).

    python tests/golden/make_golden_nnd.py
"""
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle", "_ref"))
import torch_nndistance_ref as ref  # noqa: E402

sys.path.insert(0, HERE)
from nnd_cases import CASES, make_inputs  # noqa: E402


def sha(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def run_ref(x1, x2, gd1, gd2):
    b, n, m = x1.shape[0], x1.shape[1], x2.shape[1]
    t1, t2 = torch.from_numpy(x1), torch.from_numpy(x2)
    d1, d2 = torch.zeros(b, n), torch.zeros(b, m)
    i1 = torch.zeros(b, n, dtype=torch.int32)
    i2 = torch.zeros(b, m, dtype=torch.int32)
    assert ref.nnd_forward(t1, t2, d1, d2, i1, i2) == 1
    g1, g2 = torch.zeros(b, n, 3), torch.zeros(b, m, 3)
    assert ref.nnd_backward(t1, t2, g1, g2, torch.from_numpy(gd1), torch.from_numpy(gd2),
                            i1, i2) == 1
    return d1.numpy(), d2.numpy(), i1.numpy(), i2.numpy(), g1.numpy(), g2.numpy()


def main():
    out = {}
    for name, spec in CASES.items():
        x1, x2, gd1, gd2 = make_inputs(spec)
        d1, d2, i1, i2, g1, g2 = run_ref(x1, x2, gd1, gd2)
        out[f"{name}/sha_fwd"] = np.frombuffer(bytes.fromhex(sha(d1, d2, i1, i2)), np.uint8)
        out[f"{name}/sha_bwd"] = np.frombuffer(bytes.fromhex(sha(g1, g2)), np.uint8)
        if d1.size + d2.size <= 20000:
            for k, v in dict(d1=d1, d2=d2, i1=i1, i2=i2, g1=g1, g2=g2).items():
                out[f"{name}/{k}"] = v
        else:  # sampled rows of the large cases
            rs = np.random.default_rng(123)
            r1 = rs.choice(d1.size, 512, replace=False)
            r2 = rs.choice(d2.size, 512, replace=False)
            out[f"{name}/rows1"] = r1.astype(np.int64)
            out[f"{name}/rows2"] = r2.astype(np.int64)
            out[f"{name}/d1s"] = d1.reshape(-1)[r1]
            out[f"{name}/i1s"] = i1.reshape(-1)[r1]
            out[f"{name}/d2s"] = d2.reshape(-1)[r2]
            out[f"{name}/i2s"] = i2.reshape(-1)[r2]
        print(f"{name}: b={x1.shape[0]} n={x1.shape[1]} m={x2.shape[1]} ok")
    np.savez_compressed(os.path.join(HERE, "nnd_golden.npz"), **out)


if __name__ == "__main__":
    main()
