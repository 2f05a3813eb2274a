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
import os
import time
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
    CHECK = 8  # iterations between the host's looks at the early-stop flag
    # iterations per captured graph (PCR_NDP_GRAPH_STEPS): each graph launch costs
    # a gap of ~8 us on the device; more steps per graph cost capture time
    GRAPH_STEPS = int(os.environ.get("PCR_NDP_GRAPH_STEPS", "2"))

    def __init__(self, layer, s_sample, t_sample, inds, level, cfg: NDPConfig, shared=None):
        dev = s_sample.device
        # buffers that do not depend on the level (same N, K, M on every level of a
        # pyramid) are allocated once per optimize_deformation_pyramid call
        self.shared = {} if shared is None else shared
        self.layer, self.level, self.cfg = layer, level, cfg
        self.s, self.t, self.inds = s_sample, t_sample, inds
        self.params = [p for p in layer.parameters()]
        # gradients and Adam moments: views of one buffer (one fill per reset)
        sizes = [p.numel() for p in self.params]
        self._gmv = torch.zeros(3, sum(sizes), dtype=self.params[0].dtype, device=dev)
        self.grads, self.m, self.v = ([t.view_as(p) for t, p in zip(self._gmv[r].split(sizes), self.params)]
                                      for r in range(3))
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
        st0 = self.shared.get("state0")
        if st0 is None:  # one host -> device copy per pyramid, not per level
            st0 = torch.tensor([1.0, 0.0, 1e6, 0.0, 0.0, 0.0, 0.0, 0.0], dtype=torch.float64,
                               device=self.state.device)
            self.shared["state0"] = st0
        self.state.copy_(st0)
        self._gmv[1:].zero_()
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

    def needs_warmup(self):
        return True  # torch autograd: its allocations must precede the capture

    def run(self, use_graph=True):
        iters = self.cfg.iters
        if not use_graph or iters <= 1:
            for _ in range(iters):
                self.step()
            return
        side = torch.cuda.Stream(device=self.s.device)
        side.wait_stream(torch.cuda.current_stream())
        if self.needs_warmup():
            # warm-up on a side stream (allocator pools, library handles, libpcr
            # workspaces) then restore parameters and optimizer state
            keep = [p.detach().clone() for p in self.params]
            with torch.cuda.stream(side):
                self.step()
            torch.cuda.current_stream().wait_stream(side)
            with torch.no_grad():
                for p, k in zip(self.params, keep):
                    p.copy_(k)
            self.reset()
            side.wait_stream(torch.cuda.current_stream())
        # capture on the side stream (torch.cuda.graph would also synchronise the
        # device and run the garbage collector, ~1 ms per level)
        # a graph of `spg` iterations (the iterations are gated on the rule, so a
        # graph that runs past the stop is a no-op from there on), and one of
        # the remainder
        spg = max(1, min(self.GRAPH_STEPS, iters))
        graphs = {}
        for n in {spg, iters % spg} - {0}:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                g.capture_begin()
                try:
                    for _ in range(n):
                        self.step()
                finally:
                    g.capture_end()
            graphs[n] = g
        torch.cuda.current_stream().wait_stream(side)
        self.capture_done = time.perf_counter()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        done, seen = 0, 0
        while done < iters:
            n = spg if iters - done >= spg else iters - done
            graphs[n].replay()
            done += n
            # the replays after the rule fired are no-ops (gated kernels); every
            # CHECK iterations the host looks whether the level has stopped and
            # skips the rest (one 8-byte read; the results do not depend on it)
            if done - seen >= self.CHECK and done < iters:
                seen = done
                if self.state[0].item() == 0.0:
                    break
        ev[1].record()
        self.replay_events = ev


class _NdpLevelC(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("w_in", "b_in", "w_hid", "b_hid", "w_rot", "b_rot",
                                               "w_trn", "b_trn", "w_nr", "b_nr")] + \
        [("m", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class _TrainC(ctypes.Structure):
    """pcr_ndp_train (include/pcr_api.h)."""
    _fields_ = [("x", ctypes.c_void_p), ("N", ctypes.c_int32), ("width", ctypes.c_int32),
                ("depth", ctypes.c_int32), ("k0", ctypes.c_int32), ("level", _NdpLevelC),
                ("w_hid", ctypes.c_void_p * 4), ("b_hid", ctypes.c_void_p * 4),
                ("pe", ctypes.c_void_p), ("H", ctypes.c_void_p), ("aux", ctypes.c_void_p),
                ("x_out", ctypes.c_void_p), ("g", ctypes.c_void_p), ("bce_scale", ctypes.c_double),
                ("dO", ctypes.c_void_p), ("D", ctypes.c_void_p),
                ("inv", ctypes.c_void_p), ("xs", ctypes.c_void_p), ("gsub", ctypes.c_void_p),
                ("gacc", ctypes.c_void_p), ("gacc_k", ctypes.c_int32), ("reserved", ctypes.c_int32)]

GACC_REPLICAS = 16  # PCR_NDP_GACC_REPLICAS (include/pcr_api.h)


class _ChamferC(ctypes.Structure):
    """pcr_ndp_chamfer (include/pcr_api.h)."""
    _fields_ = [("xs", ctypes.c_void_p), ("tgt", ctypes.c_void_p), ("K", ctypes.c_int32),
                ("M", ctypes.c_int32), ("trunc", ctypes.c_double), ("d1", ctypes.c_void_p),
                ("d2", ctypes.c_void_p), ("i1", ctypes.c_void_p), ("i2", ctypes.c_void_p),
                ("gacc", ctypes.c_void_p), ("scratch", ctypes.c_void_p)]


class _LevelFused(_Level):
    """One level with the warp forward/backward and the weight gradients on libpcr
    kernels (csrc/ndp_train.hip) instead of torch autograd; same loss, same
    early-stop rule and Adam (pcr_ndp_control / pcr_adam_masked)."""

    # points per weight-gradient partial (split-K chunk; PCR_NDP_CHUNK: a tuning hook)
    CHUNK = int(os.environ.get("PCR_NDP_CHUNK", "128"))

    def __init__(self, layer, s_sample, t_sample, inds, level, cfg: NDPConfig, shared=None):
        sd = dict(layer.named_parameters())
        self.W = sd["input.0.weight"].shape[0]
        self.nhid = sum(1 for k in sd if k.startswith("mlp.pts_linears.") and k.endswith(".weight"))
        if self.W != 128 or self.nhid > 4:
            raise NotImplementedError("fused NDP training: width 128, depth <= 5")
        super().__init__(layer, s_sample, t_sample, inds, level, cfg, shared)
        dev, N, W, d = s_sample.device, s_sample.shape[0], self.W, self.nhid + 1
        f32 = dict(dtype=torch.float32, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        # the scratch of the kernels depends on (N, W, depth, K, M) only: shared by
        # the levels of one pyramid (keyed by those sizes)
        key = (N, W, d, inds.shape[0], t_sample.shape[0], t_sample.data_ptr(), inds.data_ptr())

        def buf(name, make):
            k = (name,) + key
            b = self.shared.get(k)
            if b is None:
                b = make()
                self.shared[k] = b
            return b
        self._buf = buf
        self.N = N
        self.pe = buf("pe", lambda: torch.zeros(6, N, **f32))
        self.H = buf("H", lambda: torch.zeros(d, W, N, **f32))
        self.aux = buf("aux", lambda: torch.zeros(8, N, **f32))
        self.dO = buf("dO", lambda: torch.zeros(8, N, **f32))
        self.D = buf("D", lambda: torch.zeros(d, W, N, **f32))
        self.gx = buf("gx", lambda: torch.zeros(N, 3, **f32))
        self.xo = self.warped  # the forward writes the level output in place
        nparts = _lib.load().pcr_ndp_train_partial_floats(N, W, d, self.CHUNK)
        self.part = buf("part", lambda: torch.zeros(max(int(nparts), 1), **f32))
        # gradient buffers in the kernel's order; the Adam table must see the same
        # storage, so the branch parameters' grads are row views of one buffer
        self.gw_b = buf("gw_b", lambda: torch.zeros(7, W, **f32))
        self.gb_b = buf("gb_b", lambda: torch.zeros(7, **f32))
        names = [n for n, _ in layer.named_parameters()]
        view = {"rot_brach.weight": self.gw_b[0:3], "rot_brach.bias": self.gb_b[0:3],
                "trn_branch.weight": self.gw_b[3:6], "trn_branch.bias": self.gb_b[3:6],
                "nr_branch.weight": self.gw_b[6:7], "nr_branch.bias": self.gb_b[6:7]}
        own = {n: buf("g:" + n, lambda p=p: torch.zeros_like(p)) for n, p in layer.named_parameters() if n not in view}
        order = ["input.0.weight", "input.0.bias"]
        for k in range(self.nhid):
            order += [f"mlp.pts_linears.{k}.weight", f"mlp.pts_linears.{k}.bias"]
        kernel_grads = [own[n] for n in order] + [self.gw_b, self.gb_b]
        self.grad_ptrs = (ctypes.c_void_p * len(kernel_grads))(*[g.data_ptr() for g in kernel_grads])
        self._keep = kernel_grads
        self.grads = [view[n] if n in view else own[n] for n in names]
        self._rebuild_table()
        t = _TrainC()
        t.x, t.N, t.width, t.depth, t.k0 = s_sample.data_ptr(), N, W, d, int(layer.k0)
        lv = _NdpLevelC()
        lv.w_in, lv.b_in = sd["input.0.weight"].data_ptr(), sd["input.0.bias"].data_ptr()
        lv.w_rot, lv.b_rot = sd["rot_brach.weight"].data_ptr(), sd["rot_brach.bias"].data_ptr()
        lv.w_trn, lv.b_trn = sd["trn_branch.weight"].data_ptr(), sd["trn_branch.bias"].data_ptr()
        self.has_nr = "nr_branch.weight" in sd
        if self.has_nr:
            lv.w_nr, lv.b_nr = sd["nr_branch.weight"].data_ptr(), sd["nr_branch.bias"].data_ptr()
        lv.m = int(layer.m)
        t.level = lv
        for k in range(self.nhid):
            t.w_hid[k] = sd[f"mlp.pts_linears.{k}.weight"].data_ptr()
            t.b_hid[k] = sd[f"mlp.pts_linears.{k}.bias"].data_ptr()
        t.pe, t.H, t.aux, t.x_out = (self.pe.data_ptr(), self.H.data_ptr(), self.aux.data_ptr(),
                                     self.xo.data_ptr())
        t.g = self.gx.data_ptr()
        self.bce_on = level > 0 and cfg.w_reg > 0 and self.has_nr
        t.bce_scale = (cfg.w_reg / N) if self.bce_on else 0.0
        t.dO, t.D = self.dO.data_ptr(), self.D.data_ptr()
        K, M = inds.shape[0], t_sample.shape[0]
        self.K, self.M = K, M
        self.d1 = buf("d1", lambda: torch.zeros(1, K, **f32))
        self.d2 = buf("d2", lambda: torch.zeros(1, M, **f32))
        self.gd1 = buf("gd1", lambda: torch.zeros(1, K, **f32))
        self.gd2 = buf("gd2", lambda: torch.zeros(1, M, **f32))
        # the level Chamfer's answers: shared by the levels, so each level's
        # searches start from the previous level's answers (box path, ndp_chamfer.hip)
        self.i1 = buf("i1", lambda: torch.zeros(1, K, **i32))
        self.i2 = buf("i2", lambda: torch.zeros(1, M, **i32))
        self.gsub = buf("gsub", lambda: torch.zeros(1, K, 3, **f32))
        self.gt = buf("gt", lambda: torch.zeros(1, M, 3, **f32))
        self.t3 = buf("t3", lambda: t_sample[None].contiguous())
        # duplicate-free subset: the forward writes x'[inds] and the backward reads
        # dL/dx' of the subset through inv (no gather / index_add launches)
        self.use_inv = buf("use_inv", lambda: int(torch.unique(inds).numel()) == K)
        if self.use_inv:
            def make_inv():
                inv = torch.full((N,), -1, **i32)
                inv[inds] = torch.arange(K, **i32)
                return inv
            self.inv = buf("inv", make_inv)
            self.xs = buf("xs", lambda: torch.zeros(1, K, 3, **f32))
            t.inv, t.xs, t.gsub = self.inv.data_ptr(), self.xs.data_ptr(), self.gsub.data_ptr()
        # the level's Chamfer with its gradient in one pass (csrc/ndp_chamfer.hip):
        # the target grid built once here, the subset grid rebuilt per iteration
        # the fused pass holds each cloud's grid starts in one workgroup's LDS
        # (K, M <= pcr_ndp_chamfer_max_points()); larger clouds -- an unsampled
        # target above 32K points (c2p.register_c2p passes tgt whole, as the
        # reference's t_sample = tgt_pcd does) -- take the nnd drop-in path
        lim = int(_lib.load().pcr_ndp_chamfer_max_points())
        self.use_nc = (self.use_inv and 1 <= K <= lim and 1 <= M <= lim
                       and os.environ.get("PCR_NDP_CHAMFER", "1") != "0")
        if self.use_nc:
            lib = _lib.load()
            nbytes = int(lib.pcr_ndp_chamfer_scratch_bytes(K, M))
            self.nc_raw = buf("nc_raw", lambda: torch.empty(nbytes + 256, dtype=torch.uint8, device=dev))
            off = (-self.nc_raw.data_ptr()) % 256
            self.gacc = buf("gacc", lambda: torch.zeros(int(lib.pcr_ndp_chamfer_gacc_words(K)), dtype=torch.int64,
                                                        device=dev))
            c = _ChamferC()
            c.xs, c.tgt, c.K, c.M, c.trunc = self.xs.data_ptr(), self.t3.data_ptr(), K, M, 1e9
            c.d1, c.d2, c.i1, c.i2 = (self.d1.data_ptr(), self.d2.data_ptr(), self.i1.data_ptr(),
                                      self.i2.data_ptr())
            c.gacc, c.scratch = self.gacc.data_ptr(), self.nc_raw.data_ptr() + off
            self.nc = c
            t.gacc, t.gacc_k = self.gacc.data_ptr(), K
            self.loss_scratch = buf("loss_scratch", lambda: torch.zeros(int(lib.pcr_ndp_loss_scratch_bytes()),
                                                                       dtype=torch.uint8, device=dev))
            self.xs0 = s_sample.index_select(0, inds).contiguous()
            _lib.call("pcr_ndp_chamfer_prepare", ctypes.byref(c), _lib.ptr(self.xs0),
                      _lib.stream_handle(dev))
        self.desc = t

    def needs_warmup(self):
        # libpcr kernels only (no allocation inside a step): one warm-up per
        # pyramid loads the code objects before the first capture
        if self.shared.get("warm"):
            return False
        self.shared["warm"] = True
        return True

    def _rebuild_table(self):
        tab = (_AdamTensor * len(self.params))()
        for k, (p, g, m, v) in enumerate(zip(self.params, self.grads, self.m, self.v)):
            tab[k] = _AdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), 0)
        raw = np.frombuffer(bytes(tab), dtype=np.uint8).copy()
        self.table = torch.from_numpy(raw).to(self.s.device)

    def step(self):
        # every libpcr kernel of the iteration is gated on state[0]: after the
        # early-stop rule fired, the remaining replays of the level graph return
        # at once (registration.py:250-256 breaks out of the level)
        _lib.call("pcr_set_gate", _lib.ptr(self.state))
        try:
            self._step()
        finally:
            _lib.call("pcr_set_gate", None)

    def _step(self):
        cfg = self.cfg
        st = _lib.stream_handle(self.s.device)
        desc = ctypes.byref(self.desc)
        _lib.call("pcr_ndp_train_forward", desc, st)
        if self.use_nc:
            # the Chamfer with its gradient, then the loss and the early-stop rule in one launch
            _lib.call("pcr_ndp_chamfer_step", ctypes.byref(self.nc), st)
            _lib.call("pcr_ndp_chamfer_loss", _lib.ptr(self.d1), self.K, _lib.ptr(self.d2), self.M,
                      _lib.ptr(self.aux[6] if self.bce_on else None), self.N, float(cfg.w_reg), 1e9,
                      _lib.ptr(self.loss), _lib.ptr(self.log), _lib.ptr(self.ctr), int(cfg.iters),
                      _lib.ptr(self.state), float(cfg.break_threshold_ratio), int(cfg.max_break_count), 1e-4,
                      _lib.ptr(self.loss_scratch), st)
            _lib.call("pcr_ndp_train_backward", desc, _lib.ptr(self.part), self.CHUNK,
                      ctypes.cast(self.grad_ptrs, ctypes.c_void_p), st)
        else:
            self._chamfer_nnd(st)
            _lib.call("pcr_ndp_train_backward", desc, _lib.ptr(self.part), self.CHUNK,
                      ctypes.cast(self.grad_ptrs, ctypes.c_void_p), st)
            _lib.call("pcr_ndp_control", _lib.ptr(self.loss), _lib.ptr(self.state),
                      float(cfg.break_threshold_ratio), int(cfg.max_break_count), 1e-4, st)
        _lib.call("pcr_adam_masked", _lib.ptr(self.table), len(self.params), self.max_numel,
                  _lib.ptr(self.state), float(cfg.lr), 0.9, 0.999, 1e-8, st)

    def _chamfer_nnd(self, st):
        """The Chamfer pass on the nnd drop-in kernels (a1 forward, the glue, a2
        backward): subsets with repeated indices (no inverse map)."""
        from .nndistance import nnd_backward_cuda, nnd_forward_cuda
        cfg = self.cfg
        xs = self.xs if self.use_inv else self.xo.index_select(0, self.inds)[None].contiguous()
        nnd_forward_cuda(xs, self.t3, self.d1, self.d2, self.i1, self.i2)
        # loss (truncated Chamfer means + BCE), dL/dd1, dL/dd2, the log entry, the counter
        _lib.call("pcr_ndp_chamfer_glue", _lib.ptr(self.d1), self.K, _lib.ptr(self.d2), self.M,
                  _lib.ptr(self.aux[6] if self.bce_on else None), self.N, float(cfg.w_reg), 1e9,
                  _lib.ptr(self.gd1), _lib.ptr(self.gd2), _lib.ptr(self.loss), _lib.ptr(self.log),
                  _lib.ptr(self.ctr), int(cfg.iters), st)
        nnd_backward_cuda(xs, self.t3, self.gsub, self.gt, self.gd1, self.gd2, self.i1, self.i2)
        if not self.use_inv:
            self.gx.zero_()
            self.gx.index_add_(0, self.inds, self.gsub[0])


def optimize_deformation_pyramid(src_pcd, tgt_pcd, inds, config=None, NDP=None, use_graph=True,
                                 fused=True):
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
    shared = {}  # per-pyramid buffers of the levels (_Level)
    for level in range(NDP.n_hierarchy):
        NDP.gradient_setup(optimized_level=level)
        layer = NDP.pyramid[level]
        use_fused = fused and layer.input[0].weight.shape[0] == 128
        t0 = time.perf_counter()
        lv = (_LevelFused if use_fused else _Level)(layer, s_sample, t_sample, ind, level, cfg, shared)
        t1 = time.perf_counter()
        lv.run(use_graph)
        st = lv.state.cpu().numpy()
        t2 = time.perf_counter()
        info.append({"steps": int(st[3]), "evaluated": int(st[6]), "last_loss": float(st[4]),
                     "losses": lv.log[:int(st[6])].cpu().numpy(),
                     # which path ran: the fused HIP MLP kernels (width 128) or torch
                     # autograd, and the fused level Chamfer or the nnd drop-in kernels
                     "mlp": "fused" if use_fused else "torch",
                     "chamfer": "fused" if getattr(lv, "use_nc", False) else "nnd"})
        ev = getattr(lv, "replay_events", None)
        if ev is not None:
            info[-1]["replay_ms"] = ev[0].elapsed_time(ev[1])
            info[-1]["capture_ms"] = (lv.capture_done - t1) * 1e3
        if getattr(lv, "use_nc", False):
            # listed (uncertified) queries per direction of the last evaluated iteration
            hdr = lv.nc_raw[(lv.nc.scratch - lv.nc_raw.data_ptr()):][:88].cpu().numpy()
            h32 = hdr[:28].view(np.int32)
            info[-1]["fb_cnt"] = (int(h32[5]), int(h32[6]))
            if os.environ.get("PCR_NC_STATS", "0") != "0":
                # box path: queries, groups and leaves scanned over the level
                info[-1]["nc_stats"] = [int(v) for v in hdr[64:88].view(np.uint64)]
        info[-1]["setup_ms"] = (t1 - t0) * 1e3
        info[-1]["level_ms"] = (t2 - t0) * 1e3
        hist.append((lv.warped + tgt_mean).cpu().numpy())
        s_sample = lv.warped.clone()
    NDP.gradient_setup(optimized_level=-1)
    warped, _ = warp_pyramid(NDP, src_c)
    warped = warped + tgt_mean
    hist.append(warped.cpu().numpy())
    return warped, np.array(hist), {}, info


__all__ = ["NDPConfig", "NDPLayer", "DeformationPyramid", "optimize_deformation_pyramid"]
