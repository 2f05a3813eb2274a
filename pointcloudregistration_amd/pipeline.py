"""Batched pair pipeline (BASELINE configs[3]): for P resident
cloud pairs run, all on libpcr kernels,

  1. feature_match      exact mutual 1-NN in descriptor space      (a5)
  2. correspondences    mutual filter + compaction                  (a5)
  3. ransac_batch       hypothesize/verify, Philox stream           (a6/a7)
  4. icp_batch          point-to-point refinement                   (a8)
  5. nnd Chamfer        1-NN both ways between the aligned source and the
                        target (registration quality)              (a1/a3)

This is DataPreparation/RANSAC.py's per-pair loop (RANSAC.py:109-122:
execute_global_registration -> refine_registration -> keep the result) run for
P pairs per launch instead of one pair per Python iteration, with the
Chamfer/quality check of DataPreparation/QualityCheck.py:25-31 (squared form of
torch_nndistance).  One record per pair: T_ransac, T_icp, fitness/rmse of both,
chamfer, stats.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib, nndistance, registration as reg

RECORD_WIDTH = 40  # f64 per pair, see PairPipeline.records()


class _PipelineIO(ctypes.Structure):
    """pcr_pipeline_io (include/pcr_api.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("src_xyz", "tgt_xyz", "src_feat", "tgt_feat")] + \
        [(n, ctypes.c_int32) for n in ("P", "N", "M", "D")] + \
        [(n, ctypes.c_void_p) for n in ("pair_ids", "nn12", "corres", "n_corres", "T_ransac", "fit_ransac",
                                        "stats_ransac", "inlier_mask", "T_icp", "fit_icp", "stats_icp",
                                        "aligned", "d1", "d2", "i1", "i2", "records")]


@dataclass
class PipelineParams:
    ransac: reg.RansacParams
    icp: reg.IcpParams


def default_params(seed=0):
    """RANSAC.py's parameters: voxel 0.01 -> RANSAC d = 4*voxel = 0.04 (:37),
    ICP d = 0.02 (:95-98), mutual filter, n=3, EdgeLength(0.9), Distance(d),
    RANSACConvergenceCriteria(100000, 0.999), ICP criteria defaults."""
    return PipelineParams(reg.RansacParams(max_correspondence_distance=0.04, seed=seed),
                          reg.IcpParams(max_correspondence_distance=0.02))


class PairPipeline:
    """Holds device-resident inputs and per-stage outputs for P pairs.

    Buffer lifetime: the results of ``run()`` (the BatchResults' tensors, the
    Chamfer column) and ``records()`` are VIEWS of buffers preallocated once
    and rewritten by the next ``run()`` -- so a step allocates nothing and the
    whole step is one C-ABI call.  A caller that keeps results across steps
    takes ``records(copy=True)`` (or ``.clone()``s what it keeps)."""

    def __init__(self, src, tgt, src_feat, tgt_feat, params: PipelineParams, pair_ids=None,
                 device=None, context=0, graph=False):
        dev = device or torch.device("cuda", torch.cuda.current_device())
        # graph=True: the step is captured once into a HIP graph (after one eager
        # step) and replayed, the same records bit for bit; a step that cannot be
        # captured stays eager.  Measured (bench.py --graph): 9.72 vs 9.70 ms at
        # 256 pairs, and 2.74 vs 1.87 ms at 32 pairs, where the recorded
        # cooperative launches run slower -- off by default
        self.use_graph = bool(graph)
        self._graph = None
        self._graph_gen = -1
        self._graph_failed = False
        # libpcr workspace context (pcr_set_workspace_context): pipelines whose
        # steps run concurrently on different streams need different ones
        self.context = int(context)

        def d(x, dt):
            return torch.as_tensor(x).to(dev, dt).contiguous()

        self.src, self.tgt = d(src, torch.float32), d(tgt, torch.float32)
        self.src_feat, self.tgt_feat = d(src_feat, torch.float32), d(tgt_feat, torch.float32)
        self.P, self.N, self.M = self.src.shape[0], self.src.shape[1], self.tgt.shape[1]
        self.params = params
        self.pair_ids = None if pair_ids is None else d(pair_ids, torch.int32)
        self.device = dev
        self.stage_events = None
        # preallocated stage outputs: the one-call step (pcr_pipeline_step) writes
        # them all; the staged path (time_stages) fills the same records
        P, N, M = self.P, self.N, self.M
        i32, f64 = dict(dtype=torch.int32, device=dev), dict(dtype=torch.float64, device=dev)
        self.d1 = torch.empty(P, N, device=dev)
        self.d2 = torch.empty(P, M, device=dev)
        self.i1 = torch.empty(P, N, **i32)
        self.i2 = torch.empty(P, M, **i32)
        self.aligned = torch.empty_like(self.src)
        self.b_nn12 = torch.empty(P, N, **i32)
        self.b_corres = torch.empty(P, N, 2, **i32)
        self.b_ncor = torch.empty(P, **i32)
        self.T_r, self.fr_r, self.st_r = (torch.empty(P, 4, 4, **f64), torch.empty(P, 2, **f64),
                                          torch.empty(P, 5, **i32))
        self.mask = torch.empty(P, (N + 31) // 32, **i32)
        self.T_i, self.fr_i, self.st_i = (torch.empty(P, 4, 4, **f64), torch.empty(P, 2, **f64),
                                          torch.empty(P, 2, **i32))
        self.rec = torch.zeros(P, RECORD_WIDTH, **f64)
        io = _PipelineIO()
        io.src_xyz, io.tgt_xyz = self.src.data_ptr(), self.tgt.data_ptr()
        io.src_feat, io.tgt_feat = self.src_feat.data_ptr(), self.tgt_feat.data_ptr()
        io.P, io.N, io.M, io.D = P, N, M, self.src_feat.shape[2]
        io.pair_ids = None if self.pair_ids is None else self.pair_ids.data_ptr()
        for name, t in (("nn12", self.b_nn12), ("corres", self.b_corres), ("n_corres", self.b_ncor),
                        ("T_ransac", self.T_r), ("fit_ransac", self.fr_r), ("stats_ransac", self.st_r),
                        ("inlier_mask", self.mask), ("T_icp", self.T_i), ("fit_icp", self.fr_i),
                        ("stats_icp", self.st_i), ("aligned", self.aligned), ("d1", self.d1),
                        ("d2", self.d2), ("i1", self.i1), ("i2", self.i2), ("records", self.rec)):
            setattr(io, name, t.data_ptr())
        self.io = io
        self.c_ransac, self.c_icp = params.ransac.to_c(), params.icp.to_c()

    def _step_call(self):
        _lib.call("pcr_set_workspace_context", self.context)
        try:
            _lib.call("pcr_pipeline_step", ctypes.byref(self.io), ctypes.byref(self.c_ransac),
                      ctypes.byref(self.c_icp), _lib.stream_handle(self.device))
        finally:
            _lib.call("pcr_set_workspace_context", 0)

    def _capture(self):
        """One eager step (workspaces sized, code objects loaded), then the step
        recorded on a side stream into a HIP graph; on any capture error the
        pipeline stays eager."""
        self._step_call()
        cur = torch.cuda.current_stream(self.device)
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(cur)
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.stream(side):
                g.capture_begin()
                try:
                    self._step_call()
                finally:
                    g.capture_end()
        except Exception:  # noqa: BLE001 -- any refusal: eager from here on
            self._graph_failed = True
            torch.cuda.synchronize(self.device)
            return
        cur.wait_stream(side)
        self._graph = g
        self._graph_gen = _lib.generation()

    def _publish(self, rr, ir, ncor, corres, nn12):
        chamfer = self.rec[:, 36]
        self.last = (rr, ir, chamfer, ncor)
        self.corres = corres
        self.nn12 = nn12
        return rr, ir, chamfer

    def run(self, time_stages=False):
        if self.context and time_stages:
            raise ValueError("time_stages runs the stage calls in workspace context 0")
        if not time_stages:
            # the whole step in one host call, no round trip (csrc/pipeline.cpp)
            with torch.cuda.device(self.device):
                if self._graph is not None and self._graph_gen != _lib.generation():
                    self._graph = None  # pcr_shutdown freed the buffers it recorded
                if self.use_graph and self._graph is None and not self._graph_failed:
                    self._capture()
                if self.use_graph and self._graph is not None:
                    self._graph.replay()
                else:
                    self._step_call()
            rr = reg.BatchResult(self.T_r, self.fr_r[:, 0], self.fr_r[:, 1], self.st_r, None, self.mask)
            ir = reg.BatchResult(self.T_i, self.fr_i[:, 0], self.fr_i[:, 1], self.st_i, None)
            return self._publish(rr, ir, self.b_ncor, self.b_corres, self.b_nn12)
        # the same stages called one by one with events between them
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        ev[0].record()
        # feature NN + mutual filter (nn21 only where the filter reads it)
        corres, ncor, nn12 = reg.feature_correspondences(
            self.src_feat, self.tgt_feat, mutual_filter=self.params.ransac.mutual_filter,
            ransac_n=self.params.ransac.ransac_n)
        ev[1].record()
        rr = reg.ransac_batch(self.src, self.tgt, corres, ncor, self.params.ransac,
                              pair_ids=self.pair_ids, want_corr=False, want_mask=True)
        ev[2].record()
        ir = reg.icp_batch(self.src, self.tgt, rr.transformation, self.params.icp, want_corr=False)
        ev[3].record()
        T = ir.transformation
        aligned = reg.transform_batch(self.src, T, out=self.aligned)
        ev[4].record()
        nndistance.nnd_forward_cuda(aligned, self.tgt, self.d1, self.d2, self.i1, self.i2)
        io = _PipelineIO.from_buffer_copy(self.io)
        for name, t in (("nn12", nn12), ("corres", corres), ("n_corres", ncor),
                        ("T_ransac", rr.transformation), ("fit_ransac", None), ("stats_ransac", rr.stats),
                        ("T_icp", ir.transformation), ("fit_icp", None), ("stats_icp", ir.stats)):
            if t is not None:
                setattr(io, name, t.data_ptr())
        # fitness / rmse come as column views of (P, 2) buffers: pass the buffers
        io.fit_ransac = rr.fitness.data_ptr()
        io.fit_icp = ir.fitness.data_ptr()
        _lib.call("pcr_pipeline_records", ctypes.byref(io), _lib.stream_handle(self.device))
        ev[5].record()
        self.stage_events = ev
        return self._publish(rr, ir, ncor, corres, nn12)

    def stage_ms(self):
        """(feature_match, corres+ransac, icp, transform, chamfer) in ms of the last run."""
        ev = self.stage_events
        return [ev[k].elapsed_time(ev[k + 1]) for k in range(5)]

    def records(self, copy=False):
        """(P, RECORD_WIDTH) f64 per-pair result records (device), written by the
        step (pcr_pipeline_records): T_ransac (16), T_icp (16), RANSAC fitness /
        rmse, ICP fitness / rmse, Chamfer, RANSAC iterations, RANSAC status,
        correspondences after the mutual filter.  The buffer itself (valid until
        the next run()) unless copy=True."""
        return self.rec.clone() if copy else self.rec
