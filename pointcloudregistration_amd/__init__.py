"""pointcloudregistration_amd -- MI355X-native (gfx950) registration core.

Hot path of VatsalPandey0202/PointCloudRegistration rebuilt as HIP kernels behind
the C ABI in include/pcr_api.h (libpcr.so), with host-side mirrors of the
reference's operator interfaces:

  nndistance     torch_nndistance.nnd / NNDFunction / torch_nndistance_aten
"""
from ._lib import PcrError, load as load_library  # noqa: F401

__all__ = ["PcrError", "load_library"]
