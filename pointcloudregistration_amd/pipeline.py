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

from dataclasses import dataclass

import torch

from . import nndistance, registration as reg

RECORD_WIDTH = 40  # f64 per pair, see PairPipeline.records()


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
    """Holds device-resident inputs and per-stage outputs for P pairs."""

    def __init__(self, src, tgt, src_feat, tgt_feat, params: PipelineParams, pair_ids=None,
                 device=None):
        dev = device or torch.device("cuda", torch.cuda.current_device())

        def d(x, dt):
            return torch.as_tensor(x).to(dev, dt).contiguous()

        self.src, self.tgt = d(src, torch.float32), d(tgt, torch.float32)
        self.src_feat, self.tgt_feat = d(src_feat, torch.float32), d(tgt_feat, torch.float32)
        self.P, self.N, self.M = self.src.shape[0], self.src.shape[1], self.tgt.shape[1]
        self.params = params
        self.pair_ids = None if pair_ids is None else d(pair_ids, torch.int32)
        self.device = dev
        self.stage_events = None
        # preallocated Chamfer buffers
        self.d1 = torch.empty(self.P, self.N, device=dev)
        self.d2 = torch.empty(self.P, self.M, device=dev)
        self.i1 = torch.empty(self.P, self.N, dtype=torch.int32, device=dev)
        self.i2 = torch.empty(self.P, self.M, dtype=torch.int32, device=dev)
        self.aligned = torch.empty_like(self.src)

    def run(self, time_stages=False):
        ev = None
        if time_stages:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
            ev[0].record()
        # feature NN + mutual filter (nn21 only where the filter reads it)
        corres, ncor, nn12 = reg.feature_correspondences(
            self.src_feat, self.tgt_feat, mutual_filter=self.params.ransac.mutual_filter,
            ransac_n=self.params.ransac.ransac_n)
        if ev:
            ev[1].record()
        rr = reg.ransac_batch(self.src, self.tgt, corres, ncor, self.params.ransac,
                              pair_ids=self.pair_ids, want_corr=False, want_mask=True)
        if ev:
            ev[2].record()
        ir = reg.icp_batch(self.src, self.tgt, rr.transformation, self.params.icp, want_corr=False)
        if ev:
            ev[3].record()
        T = ir.transformation
        aligned = reg.transform_batch(self.src, T, out=self.aligned)
        if ev:
            ev[4].record()
        nndistance.nnd_forward_cuda(aligned, self.tgt, self.d1, self.d2, self.i1, self.i2)
        chamfer = self.d1.mean(1, dtype=torch.float64) + self.d2.mean(1, dtype=torch.float64)
        if ev:
            ev[5].record()
            self.stage_events = ev
        self.last = (rr, ir, chamfer, ncor)
        self.corres = corres
        self.nn12 = nn12
        return rr, ir, chamfer

    def stage_ms(self):
        """(feature_match, corres+ransac, icp, transform, chamfer) in ms of the last run."""
        ev = self.stage_events
        return [ev[k].elapsed_time(ev[k + 1]) for k in range(5)]

    def records(self):
        """(P, RECORD_WIDTH) f64 per-pair result records (device)."""
        rr, ir, chamfer, ncor = self.last
        rec = torch.zeros(self.P, RECORD_WIDTH, dtype=torch.float64, device=self.device)
        rec[:, 0:16] = rr.transformation.reshape(self.P, 16)
        rec[:, 16:32] = ir.transformation.reshape(self.P, 16)
        rec[:, 32] = rr.fitness
        rec[:, 33] = rr.inlier_rmse
        rec[:, 34] = ir.fitness
        rec[:, 35] = ir.inlier_rmse
        rec[:, 36] = chamfer
        rec[:, 37] = rr.stats[:, 0].double()     # RANSAC iterations
        rec[:, 38] = rr.stats[:, 3].double()     # RANSAC status
        rec[:, 39] = ncor.double()               # correspondences after mutual filter
        return rec
