"""Generate tests/golden/kpconv_golden.npz from the REFERENCE's compiled KPConv
helpers (oracle/_ref/libref_kpconv.so, built by oracle/build_ref.sh from
c2p-net/ngenet/cpp_wrappers/{cpp_subsampling,cpp_neighbors,cpp_utils} sources
in place).  The inputs are regenerated from kpconv_cases.py; the file holds the
reference's outputs only.

    python tests/golden/make_golden_kpconv.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)
import ref_kpconv as R  # noqa: E402
from kpconv_cases import NB_CASES, SUB_CASES, nb_case, sub_case  # noqa: E402


def main():
    out = {}
    for name in SUB_CASES:
        c = sub_case(name)
        res = R.subsample_batch(c["points"], c["batches"], features=c["features"],
                                sampleDl=c["dl"], max_p=c["max_p"])
        out[f"{name}/points"], out[f"{name}/lengths"] = res[0], res[1]
        if c["features"] is not None:
            out[f"{name}/features"] = res[2]
    for name in NB_CASES:
        c = nb_case(name)
        out[f"{name}/neighbors"] = R.batch_query(c["queries"], c["supports"], c["q_batches"],
                                                 c["s_batches"], radius=c["radius"])
    np.savez_compressed(os.path.join(HERE, "kpconv_golden.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
