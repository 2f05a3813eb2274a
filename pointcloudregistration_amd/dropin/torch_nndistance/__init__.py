"""Drop-in replacement for the reference package ``torch_nndistance``
(dip/torch-nndistance/torch_nndistance/__init__.py).

Put ``pointcloudregistration_amd/dropin`` on ``sys.path`` (or PYTHONPATH) and the
reference's ``import torch_nndistance as NND; NND.nnd(p1, p2)`` runs unchanged on
libpcr (HIP, gfx950).  See INTEGRATION.md.
"""
__version__ = "1.0.0"

import torch_nndistance_aten as my_lib  # noqa: F401  (same import as the reference)
from pointcloudregistration_amd.nndistance import NNDFunction, nnd  # noqa: F401
