"""C4 at its full size (BASELINE configs[3]): 256 pairs x 8192 points
x D=32 through the batched pipeline (pipeline.PairPipeline: feature NN both ways
-> mutual filter -> RANSAC -> ICP -> nnd Chamfer), exactly as bench.py runs it.

* 4 sampled pairs (first, last and two in between) are checked BIT FOR BIT
  against the oracle chain: nn12/nn21, the mutual correspondence set, RANSAC T /
  fitness / rmse / iterations / validations / best iteration, the inlier mask,
  ICP T / fitness / rmse / iterations / correspondence count, Chamfer.
* all 256 pairs are checked through properties: ground-truth RRE/RTE (ROPNet's
  metric, a12), the mutual-set invariants (every kept (i, j) has nn12[i] = j and
  nn21[j] = i; the count equals the number of mutual rows), records == stages.
"""
import numpy as np
import pytest
import torch

from pointcloudregistration_amd import nndistance
from pointcloudregistration_amd import registration as reg
from pointcloudregistration_amd import synth
from pointcloudregistration_amd.pipeline import PairPipeline, default_params

pytestmark = pytest.mark.gpu

P, N, D = 256, 8192, 32
SAMPLE = (0, 77, 190, 255)


@pytest.fixture(scope="module")
def c4():
    batch = synth.make_batch(P, n=N, m=N, d=D, base_seed=1000, feat_noise=1.0)
    params = default_params(seed=0)
    pipe = PairPipeline(batch.src, batch.tgt, batch.src_feat, batch.tgt_feat, params,
                        pair_ids=np.arange(P, dtype=np.int32))
    pipe.run()
    rec = pipe.records().cpu().numpy()
    pipe_corres, pipe_ncor = pipe.corres.cpu().numpy(), pipe.last[3].cpu().numpy()
    pipe_cham = [t.cpu().numpy() for t in (pipe.aligned, pipe.d1, pipe.d2, pipe.i1, pipe.i2)]
    # the same stages called one by one, keeping every intermediate
    nn12, nn21 = reg.feature_match(pipe.src_feat, pipe.tgt_feat)
    corres, ncor = reg.correspondences(nn12, nn21)
    rr = reg.ransac_batch(pipe.src, pipe.tgt, corres, ncor, params.ransac,
                          pair_ids=pipe.pair_ids, want_corr=True, want_mask=True)
    ir = reg.icp_batch(pipe.src, pipe.tgt, rr.transformation, params.icp, want_corr=True)
    aligned = reg.transform_batch(pipe.src, ir.transformation)
    cham = [torch.empty_like(pipe.d1), torch.empty_like(pipe.d2), torch.empty_like(pipe.i1),
            torch.empty_like(pipe.i2)]
    nndistance.nnd_forward_cuda(aligned, pipe.tgt, *cham)
    torch.cuda.synchronize()
    out = dict(batch=batch, params=params, rec=rec, pipe_corres=pipe_corres, pipe_ncor=pipe_ncor,
               nn12=nn12.cpu().numpy(),
               nn21=nn21.cpu().numpy(), corres=corres.cpu().numpy(), ncor=ncor.cpu().numpy(),
               T_r=rr.transformation.cpu().numpy(), fit_r=rr.fitness.cpu().numpy(),
               rmse_r=rr.inlier_rmse.cpu().numpy(), st_r=rr.stats.cpu().numpy(),
               mask=rr.inlier_mask.cpu().numpy(), ct_r=rr.corr_tgt.cpu().numpy(),
               T_i=ir.transformation.cpu().numpy(), fit_i=ir.fitness.cpu().numpy(),
               rmse_i=ir.inlier_rmse.cpu().numpy(), st_i=ir.stats.cpu().numpy(),
               pipe_cham=pipe_cham, cham=[t.cpu().numpy() for t in [aligned] + cham])
    return out


def _bits(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


def test_mutual_path_equals_both_directions(c4):
    """The pipeline's one-call mutual path (pcr_feature_correspondences: nn21
    only where the filter reads it, decided from certified screen values) gives
    every pair the correspondence set of the full nn12 / nn21 + filter."""
    assert np.array_equal(c4["pipe_ncor"], c4["ncor"])
    for p in range(P):
        k = int(c4["ncor"][p])
        assert np.array_equal(c4["pipe_corres"][p, :k], c4["corres"][p, :k]), p


def test_records_equal_stage_outputs(c4):
    rec = c4["rec"]
    assert _bits(rec[:, 0:16], c4["T_r"].reshape(P, 16))
    assert _bits(rec[:, 16:32], c4["T_i"].reshape(P, 16))
    assert _bits(rec[:, 32], c4["fit_r"]) and _bits(rec[:, 33], c4["rmse_r"])
    assert _bits(rec[:, 34], c4["fit_i"]) and _bits(rec[:, 35], c4["rmse_i"])
    assert np.array_equal(rec[:, 37], c4["st_r"][:, 0].astype(np.float64))
    assert np.array_equal(rec[:, 39], c4["ncor"].astype(np.float64))


def test_step_chamfer_equals_stage_chamfer(c4):
    """The one-call step forms the aligned sources inside the Chamfer's grid
    pass (pipeline.cpp, nnd_forward_grid_xf): the same aligned clouds, distances
    and indices as transform_batch + nnd_forward, bit for bit."""
    for got, want in zip(c4["pipe_cham"], c4["cham"]):
        assert _bits(got, want)
    # the record's Chamfer (written by the query kernel's last block per pair):
    # pipeline_records_kernel's order -- 256 lanes summing i = t, t + 256, ...
    # in f64, then a halving tree -- restated on the stage distances, bit for bit
    def lane_tree(d):
        acc = np.zeros((d.shape[0], 256))
        pad = np.zeros((d.shape[0], -d.shape[1] % 256), np.float32)
        rows = np.concatenate([d, pad], axis=1).astype(np.float64).reshape(d.shape[0], -1, 256)
        for k in range(rows.shape[1]):
            acc = acc + rows[:, k]
        h = 128
        while h:
            acc[:, :h] = acc[:, :h] + acc[:, h:2 * h]
            h //= 2
        return acc[:, 0]
    d1, d2 = c4["cham"][1], c4["cham"][2]
    want = lane_tree(d1) / d1.shape[1] + lane_tree(d2) / d2.shape[1]
    assert _bits(c4["rec"][:, 36], want)


def test_all_pairs_ground_truth_and_mutual_invariants(c4):
    b = c4["batch"]
    T = c4["T_i"]
    rre, rte = synth.rre_rte(T[:, :3, :3], T[:, :3, 3], b.R, b.t)
    assert np.all(c4["st_r"][:, 3] == 1), "every pair must find a hypothesis"
    assert np.median(rre) < 0.05 and rre.max() < 0.5, (np.median(rre), rre.max())
    assert np.median(rte) < 1e-3 and rte.max() < 5e-3, (np.median(rte), rte.max())
    nn12, nn21 = c4["nn12"], c4["nn21"]
    for p in range(P):
        k = int(c4["ncor"][p])
        co = c4["corres"][p, :k]
        assert np.all(nn12[p, co[:, 0]] == co[:, 1]) and np.all(nn21[p, co[:, 1]] == co[:, 0])
        mutual = nn21[p, nn12[p]] == np.arange(N)
        assert k == int(mutual.sum()) and np.array_equal(co[:, 0], np.nonzero(mutual)[0])
        # inlier mask == correspondence set of the best hypothesis
        bits = np.unpackbits(c4["mask"][p].view(np.uint8), bitorder="little")[:N].astype(bool)
        assert np.array_equal(bits, c4["ct_r"][p] >= 0)
        assert c4["st_r"][p, 4] == int(bits.sum())


@pytest.mark.parametrize("p", SAMPLE)
def test_sampled_pairs_bitexact_vs_oracle(c4, oracle, p):
    b, prm = c4["batch"], c4["params"]
    nn12 = oracle.featnn(b.src_feat[p], b.tgt_feat[p])
    nn21 = oracle.featnn(b.tgt_feat[p], b.src_feat[p])
    assert np.array_equal(c4["nn12"][p], nn12) and np.array_equal(c4["nn21"][p], nn21)
    co = oracle.corres(nn12, nn21, True, 3)
    assert c4["ncor"][p] == len(co) and np.array_equal(c4["corres"][p, :len(co)], co)
    r = oracle.ransac(b.src[p], b.tgt[p], co, prm.ransac.max_correspondence_distance,
                      seed=prm.ransac.seed, pair_id=p)
    assert _bits(c4["T_r"][p], r["T"])
    assert _bits(c4["fit_r"][p], r["fitness"]) and _bits(c4["rmse_r"][p], r["inlier_rmse"])
    assert tuple(c4["st_r"][p, :3]) == (r["iters"], r["validated"], r["best_itr"])
    cs = r["correspondence_set"]
    got = np.nonzero(c4["ct_r"][p] >= 0)[0]
    assert np.array_equal(got, cs[:, 0]) and np.array_equal(c4["ct_r"][p, got], cs[:, 1])
    o = oracle.icp(b.src[p], b.tgt[p], prm.icp.max_correspondence_distance, init=r["T"])
    assert _bits(c4["T_i"][p], o["T"])
    assert _bits(c4["fit_i"][p], o["fitness"]) and _bits(c4["rmse_i"][p], o["inlier_rmse"])
    assert tuple(c4["st_i"][p]) == (o["iters"], o["n_corr"])
    # Chamfer of the aligned pair: the record's f64 mean of the bit-exact distances
    T = o["T"]
    aligned = (b.src[p].astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)
    d1, d2, _, _ = oracle.nnd_forward(aligned[None], b.tgt[p][None])
    ch = d1.astype(np.float64).mean() + d2.astype(np.float64).mean()
    assert np.isclose(c4["rec"][p, 36], ch, rtol=1e-6)


@pytest.mark.parametrize("tail", ["1", "0"])
def test_graph_replay_equals_eager(c4, tail, monkeypatch):
    """`bench.py --graph` replays the step as one captured HIP graph: the same
    records bit for bit as the eager step, replay after replay.  At 256 pairs
    the step's ICP is one workgroup per pair plus, by default, the tail
    hand-off's second launch -- a cooperative one (its pair barriers need its
    workgroups co-resident), which the graph records as a node; the replays
    are checked with the hand-off (PCR_ICP_TAIL=1) and without it (0: one
    plain launch).  The eager records are the same either way (G is
    bit-neutral)."""
    monkeypatch.setenv("PCR_ICP_TAIL", tail)
    b = c4["batch"]
    pipe = PairPipeline(b.src, b.tgt, b.src_feat, b.tgt_feat, c4["params"],
                        pair_ids=np.arange(P, dtype=np.int32), graph=True)
    for _ in range(3):
        pipe.run()
        torch.cuda.synchronize()
        assert _bits(pipe.records().cpu().numpy(), c4["rec"])
    assert pipe._graph is not None  # captured (the runtime recorded every launch)


def test_graph_small_shard_equals_eager():
    """The 32-pair shard (cooperative ICP launch): captured or, if the runtime
    refuses to record it, eager -- the same records either way."""
    Ps = 32
    b = synth.make_batch(Ps, n=4096, m=4096, d=D, base_seed=1000, feat_noise=1.0)
    prm = default_params(seed=0)
    ids = np.arange(Ps, dtype=np.int32)
    eager = PairPipeline(b.src, b.tgt, b.src_feat, b.tgt_feat, prm, pair_ids=ids)
    eager.run()
    want = eager.records(copy=True).cpu().numpy()
    pipe = PairPipeline(b.src, b.tgt, b.src_feat, b.tgt_feat, prm, pair_ids=ids, graph=True)
    for _ in range(2):
        pipe.run()
        torch.cuda.synchronize()
        assert _bits(pipe.records().cpu().numpy(), want)
