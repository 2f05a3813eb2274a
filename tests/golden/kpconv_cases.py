"""Seeded inputs for the f2 KPConv helper cases (grid subsampling, radius
neighbours).  Shared by make_golden_kpconv.py and the tests."""
import numpy as np


def _cloud(rng, n, scale=1.0, offset=(0.0, 0.0, 0.0)):
    # a bumpy surface patch plus noise: many voxels hold several points
    u = rng.uniform(-1, 1, (n, 2))
    z = 0.3 * np.sin(3 * u[:, 0]) * np.cos(2 * u[:, 1])
    p = np.column_stack([u, z]) + 0.01 * rng.standard_normal((n, 3))
    return (p * scale + np.asarray(offset)).astype(np.float32)


def sub_case(name):
    rng = np.random.default_rng(sum(map(ord, name)))
    if name == "sub_two_clouds":
        p = np.concatenate([_cloud(rng, 3000), _cloud(rng, 2000, 1.3, (0.2, -0.1, 0.05))])
        f = rng.standard_normal((5000, 3)).astype(np.float32)
        return dict(points=p, batches=[3000, 2000], features=f, dl=0.1, max_p=0)
    if name == "sub_grid_aligned":
        k = rng.integers(-40, 40, (4000, 3))
        p = (k.astype(np.float32) * np.float32(0.05)).astype(np.float32)
        return dict(points=p, batches=[2500, 1500], features=None, dl=0.05, max_p=0)
    if name == "sub_max_p":
        p = np.concatenate([_cloud(rng, 1500), _cloud(rng, 900), _cloud(rng, 1200, 0.5)])
        f = rng.standard_normal((3600, 5)).astype(np.float32)
        return dict(points=p, batches=[1500, 900, 1200], features=f, dl=0.08, max_p=40)
    if name == "sub_single_voxel":
        p = np.concatenate([rng.uniform(0.31, 0.39, (700, 3)), rng.uniform(-5, 5, (1, 3))]).astype(np.float32)
        f = rng.standard_normal((701, 2)).astype(np.float32)
        return dict(points=p, batches=[700, 1], features=f, dl=0.1, max_p=0)
    if name == "sub_far":
        p = _cloud(rng, 3000, 20.0, (1.0e4, -3.0e3, 250.0))
        return dict(points=p, batches=[3000], features=None, dl=0.013, max_p=0)
    if name == "sub_many_small":
        sizes = rng.integers(1, 300, 24)
        p = np.concatenate([_cloud(rng, int(s), rng.uniform(0.2, 3)) for s in sizes])
        f = rng.standard_normal((p.shape[0], 1)).astype(np.float32)
        return dict(points=p, batches=sizes.tolist(), features=f, dl=0.05, max_p=0)
    raise KeyError(name)


SUB_CASES = ["sub_two_clouds", "sub_grid_aligned", "sub_max_p", "sub_single_voxel", "sub_far",
             "sub_many_small"]


def nb_case(name):
    rng = np.random.default_rng(sum(map(ord, name)))
    if name == "nb_self":
        s = np.concatenate([_cloud(rng, 2500), _cloud(rng, 1800, 1.2)])
        return dict(queries=s, supports=s, q_batches=[2500, 1800], s_batches=[2500, 1800], radius=0.09)
    if name == "nb_pool":
        s = np.concatenate([_cloud(rng, 3000), _cloud(rng, 2000)])
        q = np.concatenate([_cloud(rng, 700), _cloud(rng, 400)])
        return dict(queries=q, supports=s, q_batches=[700, 400], s_batches=[3000, 2000], radius=0.12)
    if name == "nb_upsample":
        s = np.concatenate([_cloud(rng, 600), _cloud(rng, 500)])
        q = np.concatenate([_cloud(rng, 2000), _cloud(rng, 1500)])
        return dict(queries=q, supports=s, q_batches=[2000, 1500], s_batches=[600, 500], radius=0.2)
    if name == "nb_sparse":
        s = _cloud(rng, 2000, 3.0)
        q = _cloud(rng, 800, 3.0)
        return dict(queries=q, supports=s, q_batches=[800], s_batches=[2000], radius=0.02)
    if name == "nb_empty_first":
        s = np.concatenate([_cloud(rng, 300), _cloud(rng, 1000)])
        q = _cloud(rng, 500)
        return dict(queries=q, supports=s, q_batches=[0, 500], s_batches=[300, 1000], radius=0.15)
    if name == "nb_dups":
        base = _cloud(rng, 400)
        s = np.concatenate([base, base[:150], base[:50]])
        return dict(queries=base, supports=s, q_batches=[400], s_batches=[600], radius=0.2)
    raise KeyError(name)


NB_CASES = ["nb_self", "nb_pool", "nb_upsample", "nb_sparse", "nb_empty_first", "nb_dups"]
