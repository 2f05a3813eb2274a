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


class PreparedPyramid:
    """Device-resident weights + level descriptors, built once (no per-call
    host copies); `warp` then costs one launch."""

    def __init__(self, levels, k0=-8, ms=None, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda")
        self.device, self.k0 = dev, k0
        self._keep, self.structs, self.width, self.depth = [], [], None, None
        for i, layer in enumerate(levels):
            sd, m_mod, k0_mod = _state(layer)
            if k0_mod is not None:
                self.k0 = k0_mod
            m = ms[i] if ms is not None else (m_mod if m_mod is not None else i + 1)
            st = self._level(sd, int(m))
            self.structs.append(st)

    def _as_dev(self, v):
        t = v.detach() if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
        return t.to(device=self.device, dtype=torch.float32)

    def _dev(self, v):
        t = self._as_dev(v).contiguous()
        self._keep.append(t)
        return t

    def _level(self, sd, m):
        w_in = self._dev(sd["input.0.weight"])
        W = w_in.shape[0]
        hid = []
        while f"mlp.pts_linears.{len(hid)}.weight" in sd:
            hid.append(len(hid))
        d = len(hid) + 1
        if self.width is None:
            self.width, self.depth = W, d
        elif (W, d) != (self.width, self.depth):
            raise ValueError("all levels must share width and depth")
        st = _Level()
        st.w_in, st.b_in = w_in.data_ptr(), self._dev(sd["input.0.bias"]).data_ptr()
        if hid:  # the depth-1 MLP layers, contiguous (pcr_ndp_level.w_hid)
            wh = self._dev(torch.stack([self._as_dev(sd[f"mlp.pts_linears.{k}.weight"]) for k in hid]))
            bh = self._dev(torch.stack([self._as_dev(sd[f"mlp.pts_linears.{k}.bias"]) for k in hid]))
            st.w_hid, st.b_hid = wh.data_ptr(), bh.data_ptr()
        st.w_rot, st.b_rot = self._dev(sd["rot_brach.weight"]).data_ptr(), self._dev(sd["rot_brach.bias"]).data_ptr()
        st.w_trn, st.b_trn = self._dev(sd["trn_branch.weight"]).data_ptr(), self._dev(sd["trn_branch.bias"]).data_ptr()
        if "nr_branch.weight" in sd:
            st.w_nr = self._dev(sd["nr_branch.weight"]).data_ptr()
            st.b_nr = self._dev(sd["nr_branch.bias"]).data_ptr()
        st.m = m
        return st

    def warp(self, x, max_level=None, min_level=0, per_level=True):
        dev = self.device
        xt = torch.as_tensor(x)
        xt = xt.to(device=dev, dtype=torch.float32).contiguous().reshape(-1, 3)
        if max_level is None:
            max_level = len(self.structs) - 1
        sel = list(range(min_level, max_level + 1))
        structs = [self.structs[i] for i in sel]
        n, L = xt.shape[0], len(structs)
        out = torch.empty_like(xt)
        xl = torch.empty(L, n, 3, dtype=torch.float32, device=dev) if per_level else None
        nr = torch.full((L, n), float("nan"), dtype=torch.float32, device=dev) if per_level else None
        arr = (_Level * max(L, 1))(*structs)
        with torch.cuda.device(dev):
            _lib.call("pcr_ndp_warp", _lib.ptr(xt), n, ctypes.cast(arr, ctypes.c_void_p), L,
                      int(self.width or 32), int(self.depth or 1), int(self.k0), _lib.ptr(out),
                      _lib.ptr(xl), _lib.ptr(nr), _lib.stream_handle(dev))
        data = {}
        if per_level:
            for k, i in enumerate(sel):
                data[i] = (xl[k], nr[k] if structs[k].w_nr is not None else None)
        return out, data


def warp(levels, x, k0=-8, max_level=None, min_level=0, ms=None):
    """levels: NDPLayer modules or their state dicts (level i has m = i + 1
    unless the module says otherwise or `ms` is given).  For repeated warps
    with the same weights build a PreparedPyramid once."""
    xt = torch.as_tensor(x)
    dev = xt.device if xt.is_cuda else None
    return PreparedPyramid(levels, k0=k0, ms=ms, device=dev).warp(x, max_level, min_level)


def warp_pyramid(pyramid, x, max_level=None, min_level=0):
    """Deformation_Pyramid.warp for a reference pyramid object."""
    layers = pyramid.pyramid if hasattr(pyramid, "pyramid") else pyramid
    return warp(layers, x, max_level=max_level, min_level=min_level)
