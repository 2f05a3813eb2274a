"""Exit-time fault probe under rocprofv3: the smallest programs that
do or do not end in the SIGSEGV seen after the profiler's finalisation.
usage: python3 tools/exit_probe.py torch|load|nnd|coop|plain
coop / plain: torch, libpcr loaded, and ONE trivial launch from libpcr
(pcr_coop_probe: 64 blocks, cooperative or plain) -- no other library work.
The standalone counterpart without torch is tools/coop_probe.hip."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1] if len(sys.argv) > 1 else "torch"
x = torch.ones(1024, device="cuda")
print("sum", float(x.sum()))
if mode in ("load", "nnd", "coop", "plain"):
    from pointcloudregistration_amd import _lib
    lib = _lib.load()
    print("loaded", lib is not None)
if mode == "nnd":
    from pointcloudregistration_amd import nndistance
    a = torch.rand(2, 4096, 3, device="cuda")
    b = torch.rand(2, 4096, 3, device="cuda")
    nndistance.nnd(a, b)
    torch.cuda.synchronize()
    print("nnd ok")
if mode in ("coop", "plain"):
    out = torch.zeros(64, dtype=torch.int32, device="cuda")
    _lib.call("pcr_coop_probe", _lib.ptr(out), 64, 1 if mode == "coop" else 0, _lib.stream_handle())
    torch.cuda.synchronize()
    print(mode, "probe ok", int(out[63]))
