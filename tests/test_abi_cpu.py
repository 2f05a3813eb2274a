"""CPU: the ctypes mirrors of the C ABI's structs have the layout gcc gives the
declarations in include/pcr_api.h (size and every field offset), so a field
added or reordered on one side only fails here instead of as a device fault."""
import ctypes
import os
import subprocess
import tempfile

import pytest

from pointcloudregistration_amd import _lib, ndp, ndp_opt, pipeline

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MIRRORS = {
    "pcr_ransac_params": _lib.RansacParams,
    "pcr_icp_params": _lib.IcpParams,
    "pcr_ndp_level": ndp._Level,
    "pcr_adam_tensor": ndp_opt._AdamTensor,
    "pcr_ndp_train": ndp_opt._TrainC,
    "pcr_ndp_chamfer": ndp_opt._ChamferC,
    "pcr_pipeline_io": pipeline._PipelineIO,
}


def _c_layout():
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "pcr_api.h"', "int main(void) {"]
    for cname, py in MIRRORS.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "abi.c"), os.path.join(d, "abi")
        with open(src, "w") as fh:
            fh.write("\n".join(lines))
        try:
            subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True,
                           capture_output=True)
        except (OSError, subprocess.CalledProcessError) as e:  # pragma: no cover
            pytest.skip(f"gcc unavailable: {e}")
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    return {tuple(ln.split()[:2]): int(ln.split()[2]) for ln in out.splitlines()}


def test_ctypes_mirrors_match_c_layout():
    lay = _c_layout()
    for cname, py in MIRRORS.items():
        assert lay[(cname, "sizeof")] == ctypes.sizeof(py), cname
        for f in py._fields_:
            assert lay[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])
