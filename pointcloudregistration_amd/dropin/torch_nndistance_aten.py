"""Drop-in for the reference extension module ``torch_nndistance_aten``
(built by dip/torch-nndistance/build.py:48-60 from my_lib_cuda.cpp + nnd_cuda.cu).

Exports the same pybind names (my_lib_cuda.cpp:74-77); they bind libpcr's C ABI.
"""
from pointcloudregistration_amd.nndistance import (  # noqa: F401
    nnd_backward, nnd_backward_cuda, nnd_forward, nnd_forward_cuda)
