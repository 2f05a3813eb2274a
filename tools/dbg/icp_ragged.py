import sys, numpy as np
sys.path[:0] = ['.', 'oracle']
import oracle
from pointcloudregistration_amd import registration as reg, synth, formats
rng = np.random.default_rng(4)
S, G, T = [], [], []
for p, (n, m) in enumerate([(1200, 1100), (900, 1300), (1500, 1500)]):
    b = synth.make_pair(50 + p, n, m, 4)
    Tm = np.eye(4); Tm[:3, :3], Tm[:3, 3] = b[4], b[5]; Tm[:3, 3] += rng.normal(0, 0.01, 3)
    S.append(b[0]); G.append(b[1]); T.append(Tm)
prm = reg.IcpParams(0.03, 1e-6, 1e-6, 30)
for p in range(3):
    o = oracle.icp(S[p], G[p], 0.03, T[p])
    single = reg.icp_batch(S[p][None], G[p][None], T[p][None], prm)
    # same pair padded to 1500 with counts
    Sp = np.zeros((1, 1500, 3), np.float32); Sp[0, :len(S[p])] = S[p]
    Gp = np.zeros((1, 1500, 3), np.float32); Gp[0, :len(G[p])] = G[p]
    pad = reg.icp_batch(Sp, Gp, T[p][None], prm, n_src=np.array([len(S[p])], np.int32), n_tgt=np.array([len(G[p])], np.int32))
    print(p, 'oracle', o['n_corr'], o['fitness'], 'single', int(single.stats[0, 1]), float(single.fitness[0]),
          'padded', int(pad.stats[0, 1]), float(pad.fitness[0]), 'T eq', np.array_equal(o['T'], single.transformation[0].cpu().numpy()),
          np.array_equal(o['T'], pad.transformation[0].cpu().numpy()))
