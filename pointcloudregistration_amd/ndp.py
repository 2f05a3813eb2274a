"""a10: NDP deformation-pyramid warp on the GPU.

`warp_pyramid(pyramid, x, max_level, min_level)` is Deformation_Pyramid.warp
(c2p-net/deformationpyramid/model/nets.py:36-48) for a reference pyramid
object (its `.pyramid` list of NDPLayer modules); `warp(levels, x, ...)`
takes the layers' modules or state dicts directly.  Both return
(x, data) with data[i] = (x after level i, nonrigidity of level i or None),
as the reference.  Every level runs in one libpcr launch (pcr_ndp_warp);
the NDP optimisation loop itself (forward + backward per iteration) stays in
torch.  Supported: motion "SE3" with rotation
"axis_angle" (config/NDP.yaml), width in {32, 64, 96, 128}.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

_PTRS = ("w_in", "b_in", "w_hid", "b_hid", "w_rot", "b_rot", "w_trn", "b_trn", "w_nr", "b_nr")


class _Level(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in _PTRS] + [("m", ctypes.c_int32),
                                                        ("reserved", ctypes.c_int32)]


def _state(layer):
    if hasattr(layer, "state_dict"):
        if getattr(layer, "motion", "SE3") != "SE3" or \
                getattr(layer, "rotation_format", "axis_angle") != "axis_angle":
            raise NotImplementedError("pcr_ndp_warp implements motion SE3 + axis_angle (C5)")
        return layer.state_dict(), getattr(layer, "m", None), getattr(layer, "k0", None)
    return layer, None, None


def warp(levels, x, k0=-8, max_level=None, min_level=0, ms=None):
    """levels: NDPLayer modules or their state dicts (level i has m = i + 1
    unless the module says otherwise or `ms` is given)."""
    xt = torch.as_tensor(x)
    dev = xt.device if xt.is_cuda else torch.device("cuda")
    xt = xt.to(device=dev, dtype=torch.float32).contiguous().reshape(-1, 3)
    if max_level is None:
        max_level = len(levels) - 1
    sel = list(range(min_level, max_level + 1))
    keep, structs = [], []
    width = depth = None
    for i in sel:
        sd, m_mod, k0_mod = _state(levels[i])
        k0 = k0_mod if k0_mod is not None else k0
        m = ms[i] if ms is not None else (m_mod if m_mod is not None else i + 1)

        def dv(key):
            t = torch.as_tensor(np.asarray(sd[key].detach().cpu() if hasattr(sd[key], "detach")
                                           else sd[key]), dtype=torch.float32, device=dev)
            t = t.contiguous()
            keep.append(t)
            return t
        w_in = dv("input.0.weight")
        W = w_in.shape[0]
        hid = []
        while f"mlp.pts_linears.{len(hid)}.weight" in sd:
            hid.append(len(hid))
        d = len(hid) + 1
        if width is None:
            width, depth = W, d
        elif (W, d) != (width, depth):
            raise ValueError("all levels must share width and depth")
        st = _Level()
        st.w_in, st.b_in = w_in.data_ptr(), dv("input.0.bias").data_ptr()
        if hid:
            wh = torch.stack([dv(f"mlp.pts_linears.{k}.weight") for k in hid]).contiguous()
            bh = torch.stack([dv(f"mlp.pts_linears.{k}.bias") for k in hid]).contiguous()
            keep += [wh, bh]
            st.w_hid, st.b_hid = wh.data_ptr(), bh.data_ptr()
        st.w_rot, st.b_rot = dv("rot_brach.weight").data_ptr(), dv("rot_brach.bias").data_ptr()
        st.w_trn, st.b_trn = dv("trn_branch.weight").data_ptr(), dv("trn_branch.bias").data_ptr()
        if "nr_branch.weight" in sd:
            st.w_nr, st.b_nr = dv("nr_branch.weight").data_ptr(), dv("nr_branch.bias").data_ptr()
        st.m = int(m)
        structs.append(st)
    n = xt.shape[0]
    L = len(structs)
    out = torch.empty_like(xt)
    xl = torch.empty(L, n, 3, dtype=torch.float32, device=dev)
    nr = torch.full((L, n), float("nan"), dtype=torch.float32, device=dev)
    arr = (_Level * max(L, 1))(*structs)
    with torch.cuda.device(dev):
        _lib.call("pcr_ndp_warp", _lib.ptr(xt), n, ctypes.cast(arr, ctypes.c_void_p), L,
                  int(width or 32), int(depth or 1), int(k0), _lib.ptr(out), _lib.ptr(xl),
                  _lib.ptr(nr), _lib.stream_handle(dev))
    data = {}
    for k, i in enumerate(sel):
        has_nr = structs[k].w_nr is not None
        data[i] = (xl[k], nr[k] if has_nr else None)
    return out, data


def warp_pyramid(pyramid, x, max_level=None, min_level=0):
    """Deformation_Pyramid.warp for a reference pyramid object."""
    layers = pyramid.pyramid if hasattr(pyramid, "pyramid") else pyramid
    return warp(layers, x, max_level=max_level, min_level=min_level)
