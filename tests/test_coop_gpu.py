"""Scheduling must not change any bit.

RANSAC: the verification sweeps of all pairs run speculatively on persistent
workgroups (ransac.hip); the sequential rule is replayed afterwards.  Whatever the
number of workgroups (PCR_RANSAC_WGS: 1 = every task in order on one workgroup,
where the skip/cut shortcuts see every earlier result), of target slots
(PCR_RANSAC_SLOTS: 0 = the best hypothesis' targets always come from one more
sweep) and of workgroups per task (PCR_RANSAC_SPLIT: 2 = each sweep in two
halves combined by the second to finish), the results equal the oracle's
sequential loop bit for bit.

ICP: iterations split over G = 1, 2, 4, 8 workgroups of a cooperative launch
(coop.h) must give the oracle's results bit for bit -- the split only changes who
adds which integer partial.  PCR_COOP_G forces the split (the library picks G from
the batch size: G > 1 only when the pairs alone cannot fill the CUs, e.g. 32 pairs
per GPU at 8 GPUs).  Also: ICP past its position checkpoint (> 8 iterations) and
clouds with more points than a split's threads."""
import os

import numpy as np
import pytest

from pointcloudregistration_amd import registration as reg
from pointcloudregistration_amd import synth

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy()


def _bits(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


@pytest.fixture()
def coop_g():
    old = os.environ.get("PCR_COOP_G")

    def set_g(g):
        os.environ["PCR_COOP_G"] = str(g)
    yield set_g
    if old is None:
        os.environ.pop("PCR_COOP_G", None)
    else:
        os.environ["PCR_COOP_G"] = old


@pytest.fixture()
def ransac_sched():
    keys = ("PCR_RANSAC_WGS", "PCR_RANSAC_SLOTS", "PCR_RANSAC_SPLIT", "PCR_RANSAC_SYNC")
    old = {k: os.environ.get(k) for k in keys}

    def set_sched(wgs, slots, split=None, sync=None):
        for k, v in zip(keys, (wgs, slots, split, sync)):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)
    yield set_sched
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("wgs,slots,split", [(None, None, None), (None, None, 1), (1, None, 2), (None, None, 8), (2, 0, 4),
                                             (2, 1, 1), (None, 0, 2), (3, 2, 2), (5, 2, 1)])
def test_ransac_speculative_bitexact_vs_oracle(oracle, ransac_sched, wgs, slots, split):
    P, n = 3, 4096
    B = synth.make_batch(P, n=n, m=n, d=32, base_seed=2000, feat_noise=1.0)
    ransac_sched(wgs, slots, split)
    prm = reg.RansacParams(max_correspondence_distance=0.04, seed=7)
    res = reg.register_feature_ransac_batch(B.src, B.tgt, B.src_feat, B.tgt_feat, prm,
                                            pair_ids=np.arange(P, dtype=np.int32) + 9)
    T, st, ct, mk = _np(res.transformation), _np(res.stats), _np(res.corr_tgt), _np(res.inlier_mask)
    for p in range(P):
        co = oracle.corres(oracle.featnn(B.src_feat[p], B.tgt_feat[p]),
                           oracle.featnn(B.tgt_feat[p], B.src_feat[p]), True, 3)
        r = oracle.ransac(B.src[p], B.tgt[p], co, 0.04, seed=7, pair_id=9 + p)
        assert _bits(T[p], r["T"])
        assert _bits(_np(res.fitness)[p], r["fitness"]) and _bits(_np(res.inlier_rmse)[p], r["inlier_rmse"])
        assert (st[p, 0], st[p, 1], st[p, 2], st[p, 3]) == (r["iters"], r["validated"], r["best_itr"], 1)
        cs = r["correspondence_set"]
        got = np.nonzero(ct[p] >= 0)[0]
        assert np.array_equal(got, cs[:, 0]) and np.array_equal(ct[p, got], cs[:, 1])
        bits = np.unpackbits(mk[p].view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(np.nonzero(bits)[0], cs[:, 0]) and st[p, 4] == len(cs)


def test_ransac_multi_round_low_inlier_ratio(oracle, ransac_sched):
    """Noisy descriptors -> a low inlier ratio -> est_k beyond the first round of
    1024 hypotheses: the later rounds continue the same sequential loop -- the
    device-gated second round [1024, max_iteration) and the host loop of
    4096-hypothesis rounds (PCR_RANSAC_SYNC=1) alike."""
    P, n = 2, 2048
    B = synth.make_batch(P, n=n, m=n, d=32, base_seed=3100, feat_noise=2.2)
    for wgs, slots, split, sync in ((None, None, None, None), (1, 0, 2, None), (5, 3, 1, None),
                                    (3, 1, 2, None), (None, None, None, 1), (3, 1, 2, 1)):
        ransac_sched(wgs, slots, split, sync)
        prm = reg.RansacParams(max_correspondence_distance=0.04, seed=3, max_iteration=6000)
        res = reg.register_feature_ransac_batch(B.src, B.tgt, B.src_feat, B.tgt_feat, prm)
        st = _np(res.stats)
        for p in range(P):
            co = oracle.corres(oracle.featnn(B.src_feat[p], B.tgt_feat[p]),
                               oracle.featnn(B.tgt_feat[p], B.src_feat[p]), True, 3)
            r = oracle.ransac(B.src[p], B.tgt[p], co, 0.04, seed=3, pair_id=p, max_iteration=6000)
            assert _bits(_np(res.transformation)[p], r["T"])
            assert (st[p, 0], st[p, 1], st[p, 2]) == (r["iters"], r["validated"], r["best_itr"])
            cs, ct = r["correspondence_set"], _np(res.corr_tgt)
            got = np.nonzero(ct[p] >= 0)[0]
            assert np.array_equal(got, cs[:, 0]) and np.array_equal(ct[p, got], cs[:, 1])
        assert st[:, 0].max() > 1024, st[:, 0]


@pytest.mark.parametrize("G", [1, 2, 3, 8])
@pytest.mark.parametrize("n,noise_init,r,relf", [(3000, 0.01, 0.02, 1e-6), (4096, 0.08, 0.1, 0.0),
                                                 (20000, 0.03, 0.05, 1e-6)])
def test_icp_split_bitexact_vs_oracle(oracle, coop_g, G, n, noise_init, r, relf):
    """relative_fitness = 0 runs all 30 iterations (past the position checkpoints
    at 8, 16 and 24 updates); 20000 points exceed a 512-thread split's threads."""
    P = 3
    B = synth.make_batch(P, n=n, m=n, d=8, base_seed=600 + n, feat_noise=1.0)
    rng = np.random.default_rng(n)
    init = np.zeros((P, 4, 4))
    for p in range(P):
        init[p, :3, :3] = synth.rotation_xyz(*rng.normal(0, noise_init, 3)) @ B.R[p]
        init[p, :3, 3] = B.t[p] + rng.normal(0, noise_init, 3)
        init[p, 3, 3] = 1
    coop_g(G)
    prm = reg.IcpParams(r, relative_fitness=relf, relative_rmse=relf)
    res = reg.icp_batch(B.src, B.tgt, init, prm)
    for p in range(P):
        o = oracle.icp(B.src[p], B.tgt[p], r, init=init[p], relative_fitness=relf, relative_rmse=relf)
        assert _bits(_np(res.transformation)[p], o["T"]), p
        assert _bits(_np(res.fitness)[p], o["fitness"]) and _bits(_np(res.inlier_rmse)[p], o["inlier_rmse"])
        assert tuple(_np(res.stats)[p]) == (o["iters"], o["n_corr"])
        assert int((_np(res.corr_tgt)[p] >= 0).sum()) == o["n_corr"]
    if relf == 0.0:
        assert _np(res.stats)[:, 0].max() == 30


def test_icp_library_chosen_uneven_split(oracle):
    """85 pairs (a 256-pair job's shard on 3 GPUs): the library picks G itself
    (3 on a 256-CU part), which does not divide the 1024 sum lanes -- every
    lane must still have an owner (a lane without one dropped its points from
    the means while they stayed in the count)."""
    os.environ.pop("PCR_COOP_G", None)
    P, n = 85, 2500
    B = synth.make_batch(P, n=n, m=n, d=8, base_seed=850, feat_noise=1.0)
    rng = np.random.default_rng(85)
    init = np.zeros((P, 4, 4))
    for p in range(P):
        init[p, :3, :3] = synth.rotation_xyz(*rng.normal(0, 0.02, 3)) @ B.R[p]
        init[p, :3, 3] = B.t[p] + rng.normal(0, 0.02, 3)
        init[p, 3, 3] = 1
    prm = reg.IcpParams(0.05)
    res = reg.icp_batch(B.src, B.tgt, init, prm)
    for p in range(P):
        o = oracle.icp(B.src[p], B.tgt[p], 0.05, init=init[p])
        assert _bits(_np(res.transformation)[p], o["T"]), p
        assert tuple(_np(res.stats)[p]) == (o["iters"], o["n_corr"])


@pytest.mark.parametrize("wgs,slots,split", [(None, None, None), (1, 0, 2), (4, 1, 1), (6, 1, 2)])
def test_ransac_speculative_mixed_batch(oracle, ransac_sched, wgs, slots, split):
    """One launch holding an invalid pair (K < ransac_n), ragged clouds and
    correspondence counts, and an iteration cap that is not a multiple of 64:
    the task list, the skip/cut shortcuts and the replay must still give every
    pair the oracle's sequential result (invalid pair: identity, status -1)."""
    P, n = 4, 2048
    B = synth.make_batch(P, n=n, m=n, d=32, base_seed=4400, feat_noise=1.0)
    cos, ns, ms = [], [1800, 2048, 2048, 1500], [2048, 1700, 2048, 2048]
    for p in range(P):
        nn12 = oracle.featnn(B.src_feat[p, :ns[p]], B.tgt_feat[p, :ms[p]])
        nn21 = oracle.featnn(B.tgt_feat[p, :ms[p]], B.src_feat[p, :ns[p]])
        cos.append(oracle.corres(nn12, nn21, True, 3))
    cos[2] = cos[2][:2]  # K = 2 < ransac_n: invalid
    K = max(len(c) for c in cos)
    C = np.zeros((P, K, 2), np.int32)
    for p, c in enumerate(cos):
        C[p, :len(c)] = c
    nc = np.array([len(c) for c in cos], np.int32)
    ransac_sched(wgs, slots, split)
    prm = reg.RansacParams(max_correspondence_distance=0.04, seed=5, max_iteration=333)
    res = reg.ransac_batch(B.src, B.tgt, C, nc, prm, n_src=np.array(ns, np.int32),
                           n_tgt=np.array(ms, np.int32), pair_ids=np.arange(P, dtype=np.int32))
    T, st, ct = _np(res.transformation), _np(res.stats), _np(res.corr_tgt)
    for p in range(P):
        if p == 2:
            assert np.array_equal(T[p], np.eye(4)) and st[p, 3] == -1
            continue
        r = oracle.ransac(B.src[p, :ns[p]], B.tgt[p, :ms[p]], cos[p], 0.04, seed=5, pair_id=p,
                          max_iteration=333)
        assert _bits(T[p], r["T"])
        assert (st[p, 0], st[p, 1], st[p, 2]) == (r["iters"], r["validated"], r["best_itr"])
        cs = r["correspondence_set"]
        got = np.nonzero(ct[p] >= 0)[0]
        assert np.array_equal(got, cs[:, 0]) and np.array_equal(ct[p, got], cs[:, 1])


@pytest.mark.parametrize("relf", [1e-6, 0.0])
def test_icp_tail_rebalance_bitexact(oracle, coop_g, relf):
    """A batch that fills the chip (G = 1) hands its last iterating pairs to a
    second, cooperative launch with several workgroups per pair (icp.hip's tail
    rebalancing): the same bits as one launch (PCR_ICP_TAIL=0) and as the
    oracle, with uneven iteration counts (per-pair init noise; relf = 0: all 30
    iterations, every pair listed)."""
    os.environ.pop("PCR_COOP_G", None)
    P, n = 200, 2000
    B = synth.make_batch(P, n=n, m=n, d=8, base_seed=4200, feat_noise=1.0)
    rng = np.random.default_rng(42)
    init = np.zeros((P, 4, 4))
    for p in range(P):
        s = 0.002 + 0.05 * rng.random()
        init[p, :3, :3] = synth.rotation_xyz(*rng.normal(0, s, 3)) @ B.R[p]
        init[p, :3, 3] = B.t[p] + rng.normal(0, s, 3)
        init[p, 3, 3] = 1
    prm = reg.IcpParams(0.05, relative_fitness=relf, relative_rmse=relf)
    old = os.environ.get("PCR_ICP_TAIL")
    try:
        os.environ["PCR_ICP_TAIL"] = "0"
        one = reg.icp_batch(B.src, B.tgt, init, prm)
        one = [_np(t).copy() for t in (one.transformation, one.fitness, one.inlier_rmse, one.stats, one.corr_tgt)]
        os.environ.pop("PCR_ICP_TAIL")
        two = reg.icp_batch(B.src, B.tgt, init, prm)
        two = [_np(t) for t in (two.transformation, two.fitness, two.inlier_rmse, two.stats, two.corr_tgt)]
    finally:
        if old is not None:
            os.environ["PCR_ICP_TAIL"] = old
    for a, b in zip(one, two):
        assert _bits(a, b)
    its = two[3][:, 0]
    assert its.max() > its.min()  or relf == 0.0
    for p in (0, int(np.argmax(its)), P - 1):
        o = oracle.icp(B.src[p], B.tgt[p], 0.05, init=init[p], relative_fitness=relf, relative_rmse=relf)
        assert _bits(two[0][p], o["T"]), p
        assert tuple(two[3][p]) == (o["iters"], o["n_corr"])


def test_icp_tail_concurrent_contexts_bitexact():
    """two ICP batches at once on two streams and two workspace
    contexts under pcr_set_concurrency(2), each large enough for the tail
    hand-off (P >= phase-2 grid / 2 with the grid sized to half the chip): the
    same bits as one launch per batch (PCR_ICP_TAIL=0), run one after the other."""
    import torch
    from pointcloudregistration_amd import _lib
    os.environ.pop("PCR_COOP_G", None)
    P, n = 160, 1500
    Bs = [synth.make_batch(P, n=n, m=n, d=8, base_seed=5100 + 1000 * k, feat_noise=1.0) for k in range(2)]
    inits = []
    rng = np.random.default_rng(7)
    for B in Bs:
        init = np.zeros((P, 4, 4))
        for p in range(P):
            s = 0.002 + 0.05 * rng.random()
            init[p, :3, :3] = synth.rotation_xyz(*rng.normal(0, s, 3)) @ B.R[p]
            init[p, :3, 3] = B.t[p] + rng.normal(0, s, 3)
            init[p, 3, 3] = 1
        inits.append(init)
    prm = reg.IcpParams(0.05)
    old = os.environ.get("PCR_ICP_TAIL")
    try:
        os.environ["PCR_ICP_TAIL"] = "0"
        want = []
        for B, init in zip(Bs, inits):
            r = reg.icp_batch(B.src, B.tgt, init, prm)
            want.append([_np(t).copy() for t in (r.transformation, r.fitness, r.inlier_rmse, r.stats)])
        os.environ.pop("PCR_ICP_TAIL")
        _lib.call("pcr_set_concurrency", 2)
        streams = [torch.cuda.Stream() for _ in range(2)]
        got = [None, None]
        for k in range(2):
            _lib.call("pcr_set_workspace_context", k)
            with torch.cuda.stream(streams[k]):
                got[k] = reg.icp_batch(Bs[k].src, Bs[k].tgt, inits[k], prm)
        _lib.call("pcr_set_workspace_context", 0)
        torch.cuda.synchronize()
    finally:
        _lib.call("pcr_set_concurrency", 1)
        _lib.call("pcr_set_workspace_context", 0)
        if old is not None:
            os.environ["PCR_ICP_TAIL"] = old
    for k in range(2):
        g = [_np(t) for t in (got[k].transformation, got[k].fitness, got[k].inlier_rmse, got[k].stats)]
        for a, b in zip(want[k], g):
            assert _bits(a, b), k
