"""f4: the NDP level optimisation as one captured HIP graph per level.

``optimize_deformation_pyramid(src_pcd, tgt_pcd, inds, config)`` is
Registration.optimize_deformation_pyramid (c2p-net/deformationpyramid/model/
registration.py:149-289, the no-landmark path the C2P pipeline runs):

  * centre both clouds (:171-174);
  * for each level: Adam(lr) on that level's parameters only, up to ``iters``
    iterations of  warp(level) -> truncated Chamfer of the ``inds`` subset
    (trunc 1e9, :236) [+ w_reg * BCE(nonrigidity, 0) for level > 0, :241-245] ->
    early-stop rule (:246-256) -> backward -> step; the warped sample feeds the
    next level (:268-270);
  * final warp of the whole source through every level (:280-285).

MI355X mapping: one iteration = the layer's MLP forward/backward (hipBLASLt via
torch autograd), the truncated Chamfer on libpcr's nnd kernels (a1/a2/a3), and
two libpcr kernels -- ``pcr_ndp_control`` (the early-stop rule evaluated on the
device) and ``pcr_adam_masked`` (Adam for all tensors of the level, skipped once
the rule fired) -- captured once per level with torch.cuda.graph and replayed
``iters`` times with no host round trip (the reference synchronises on
``loss.item()`` every iteration).  The final all-level warp is libpcr's
pcr_ndp_warp (a10).  Supported: motion "SE3", rotation "axis_angle" (the C5
configuration, config/NDP.yaml).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as Fn

from . import _lib
from .chamfer import compute_truncated_chamfer_distance
from .ndp import warp_pyramid


@dataclass
class NDPConfig:
    """config/NDP.yaml:8-32 (the fields optimize_deformation_pyramid reads)."""
    iters: int = 40
    lr: float = 0.01
    max_break_count: int = 15
    break_threshold_ratio: float = 0.001
    w_reg: float = 0.05
    m: int = 9
    k0: int = -8
    depth: int = 3
    width: int = 128
    motion_type: str = "SE3"
    rotation_format: str = "axis_angle"

    @classmethod
    def from_any(cls, cfg):
        if isinstance(cfg, cls):
            return cfg
        get = (lambda k, d: cfg.get(k, d)) if isinstance(cfg, dict) else \
            (lambda k, d: getattr(cfg, k, d))
        out = cls()
        for k in out.__dataclass_fields__:
            setattr(out, k, type(getattr(out, k))(get(k, getattr(out, k))))
        return out


# --------------------------------------------------------------------------
# mirror of the reference modules (same parameter names: state dicts load
# into either), nets.py:111-177 and rigid_body.py:89-119
# --------------------------------------------------------------------------


class _MLP(nn.Module):
    def __init__(self, depth, width):
        super().__init__()
        self.pts_linears = nn.ModuleList([nn.Linear(width, width) for _ in range(depth - 1)])

    def forward(self, x):
        for lin in self.pts_linears:
            x = Fn.relu(lin(x))
        return x


def _skew(w):
    z = torch.zeros_like(w[..., 0])
    return torch.stack([z, -w[..., 2], w[..., 1], w[..., 2], z, -w[..., 0],
                        -w[..., 1], w[..., 0], z], dim=-1).reshape((-1, 3, 3))


class NDPLayer(nn.Module):
    """NDPLayer(depth, width, k0, m, 'axis_angle', nonrigidity_est, 'SE3')."""

    def __init__(self, depth, width, k0, m, nonrigidity_est=False):
        super().__init__()
        self.k0, self.m = k0, m
        self.motion, self.rotation_format = "SE3", "axis_angle"
        self.nonrigidity_est = nonrigidity_est
        self.input = nn.Sequential(nn.Linear(6, width), nn.ReLU())
        self.mlp = _MLP(depth, width)
        self.rot_brach = nn.Linear(width, 3)
        self.trn_branch = nn.Linear(width, 3)
        if nonrigidity_est:
            self.nr_branch = nn.Linear(width, 1)
        self.mlp_scale = 0.001
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    def posenc(self, pos):
        mul = 2 ** (self.m + self.k0)
        x, y, z = pos[..., 0:1], pos[..., 1:2], pos[..., 2:3]
        return torch.cat([torch.sin(x * mul), torch.cos(x * mul), torch.sin(y * mul),
                          torch.cos(y * mul), torch.sin(z * mul), torch.cos(z * mul)], dim=-1)

    def forward(self, x):
        fea = self.mlp(self.input(self.posenc(x)))
        t = self.mlp_scale * self.trn_branch(fea)
        r = self.mlp_scale * self.rot_brach(fea)
        theta = torch.norm(r, dim=-1, keepdim=True)
        W = _skew(r / theta)
        th = theta[..., None]
        R = torch.eye(3, device=x.device)[None] + torch.sin(th) * W + (1 - torch.cos(th)) * W @ W
        x_ = (R @ x[..., None]).squeeze() + t
        if self.nonrigidity_est:
            nr = torch.sigmoid(self.mlp_scale * self.nr_branch(fea))
            x_ = x + nr * (x_ - x)
            nr = nr.squeeze()
        else:
            nr = None
        return x_.squeeze(), nr


class DeformationPyramid:
    """Deformation_Pyramid(depth, width, device, k0, m, 'axis_angle',
    nonrigidity_est, 'SE3') (nets.py:10-65)."""

    def __init__(self, depth, width, device, k0, m, nonrigidity_est=False):
        self.pyramid = [NDPLayer(depth, width, k0, i + 1, nonrigidity_est and i != 0).to(device)
                        for i in range(m)]
        self.n_hierarchy = m

    def warp(self, x, max_level=None, min_level=0):
        max_level = self.n_hierarchy - 1 if max_level is None else max_level
        data = {}
        for i in range(min_level, max_level + 1):
            x, nr = self.pyramid[i](x)
            data[i] = (x, nr)
        return x, data

    def gradient_setup(self, optimized_level):
        for i, net in enumerate(self.pyramid):
            for p in net.parameters():
                p.requires_grad = i == optimized_level


# --------------------------------------------------------------------------
# one level
# --------------------------------------------------------------------------


class _AdamTensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_int32), ("reserved", ctypes.c_int32)]


def _bce_to_zero(p):
    """nn.BCELoss()(p, zeros): mean(-max(log(1 - p), -100))."""
    return torch.mean(-torch.clamp(torch.log(1 - p), min=-100.0))


class _Level:
    def __init__(self, layer, s_sample, t_sample, inds, level, cfg: NDPConfig):
        dev = s_sample.device
        self.layer, self.level, self.cfg = layer, level, cfg
        self.s, self.t, self.inds = s_sample, t_sample, inds
        self.params = [p for p in layer.parameters()]
        self.grads = [torch.zeros_like(p) for p in self.params]
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        self.warped = torch.zeros_like(s_sample)
        self.state = torch.zeros(8, dtype=torch.float64, device=dev)
        # loss of every replay (the first state[6] are the evaluated iterations)
        self.log = torch.zeros(cfg.iters + 1, dtype=torch.float32, device=dev)
        self.ctr = torch.zeros(1, dtype=torch.long, device=dev)
        tab = (_AdamTensor * len(self.params))()
        for k, (p, g, m, v) in enumerate(zip(self.params, self.grads, self.m, self.v)):
            tab[k] = _AdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), 0)
        raw = np.frombuffer(bytes(tab), dtype=np.uint8).copy()
        self.table = torch.from_numpy(raw).to(dev)
        self.max_numel = max(p.numel() for p in self.params)
        self.reset()

    def reset(self):
        """Fresh optimizer + early-stop state (registration.py:202-206)."""
        self.state.copy_(torch.tensor([1.0, 0.0, 1e6, 0.0, 0.0, 0.0, 0.0, 0.0], dtype=torch.float64))
        for t in self.m + self.v:
            t.zero_()
        self.ctr.zero_()

    def step(self):
        cfg = self.cfg
        warped, nr = self.layer(self.s)
        loss = compute_truncated_chamfer_distance(warped[None, self.inds], self.t[None], trunc=1e9)
        if self.level > 0 and cfg.w_reg > 0:
            loss = loss + cfg.w_reg * _bce_to_zero(nr)
        grads = torch.autograd.grad(loss, self.params)
        for gs, g in zip(self.grads, grads):
            gs.copy_(g)
        self.loss.copy_(loss.detach())
        self.log.index_copy_(0, torch.clamp(self.ctr, max=self.cfg.iters), self.loss.reshape(1))
        self.ctr += 1
        self.warped.copy_(warped.detach())
        st = _lib.stream_handle(self.s.device)
        _lib.call("pcr_ndp_control", _lib.ptr(self.loss), _lib.ptr(self.state),
                  float(cfg.break_threshold_ratio), int(cfg.max_break_count), 1e-4, st)
        _lib.call("pcr_adam_masked", _lib.ptr(self.table), len(self.params), self.max_numel,
                  _lib.ptr(self.state), float(cfg.lr), 0.9, 0.999, 1e-8, st)

    def run(self, use_graph=True):
        iters = self.cfg.iters
        if not use_graph or iters <= 1:
            for _ in range(iters):
                self.step()
            return
        # warm-up on a side stream (allocator pools, library handles, libpcr
        # workspaces) then restore parameters and optimizer state
        keep = [p.detach().clone() for p in self.params]
        side = torch.cuda.Stream(device=self.s.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self.step()
        torch.cuda.current_stream().wait_stream(side)
        with torch.no_grad():
            for p, k in zip(self.params, keep):
                p.copy_(k)
        self.reset()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.step()
        for _ in range(iters):
            g.replay()


def optimize_deformation_pyramid(src_pcd, tgt_pcd, inds, config=None, NDP=None, use_graph=True):
    """Returns (warped_pcd (N, 3) cuda f32, hist (levels + 1, N_s, 3) numpy, iter_cnt) like
    the reference, plus ``info`` per level {steps, evaluated, last_loss}.  ``NDP`` may be
    the reference's Deformation_Pyramid (SE3 / axis_angle) or this module's mirror;
    by default a fresh mirror is built from the config, as the reference does."""
    cfg = NDPConfig.from_any(config or {})
    if cfg.motion_type != "SE3" or cfg.rotation_format != "axis_angle":
        raise NotImplementedError("f4 implements motion SE3 + axis_angle (config/NDP.yaml)")
    dev = torch.device("cuda", torch.cuda.current_device())
    src = torch.as_tensor(src_pcd, dtype=torch.float32).to(dev)
    tgt = torch.as_tensor(tgt_pcd, dtype=torch.float32).to(dev)
    if NDP is None:
        NDP = DeformationPyramid(cfg.depth, cfg.width, dev, cfg.k0, cfg.m, cfg.w_reg > 0)
    src_mean = src.mean(dim=0, keepdim=True)
    tgt_mean = tgt.mean(dim=0, keepdim=True)
    src_c = (src - src_mean).contiguous()
    s_sample = src_c.clone()
    t_sample = (tgt - tgt_mean).contiguous()
    ind = torch.as_tensor(np.asarray(inds), dtype=torch.long, device=dev)
    hist, info = [], []
    for level in range(NDP.n_hierarchy):
        NDP.gradient_setup(optimized_level=level)
        lv = _Level(NDP.pyramid[level], s_sample, t_sample, ind, level, cfg)
        lv.run(use_graph)
        st = lv.state.cpu().numpy()
        info.append({"steps": int(st[3]), "evaluated": int(st[6]), "last_loss": float(st[4]),
                     "losses": lv.log[:int(st[6])].cpu().numpy()})
        hist.append((lv.warped + tgt_mean).cpu().numpy())
        s_sample = lv.warped.clone()
    NDP.gradient_setup(optimized_level=-1)
    warped, _ = warp_pyramid(NDP, src_c)
    warped = warped + tgt_mean
    hist.append(warped.cpu().numpy())
    return warped, np.array(hist), {}, info


__all__ = ["NDPConfig", "NDPLayer", "DeformationPyramid", "optimize_deformation_pyramid"]
