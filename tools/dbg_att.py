import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import oracle_py as O
from yalm_amd import runtime as R
R.check(R.lib.yalm_set_device(0))
for (D, nh, nkv) in [(64, 8, 2), (32, 8, 8), (128, 32, 8), (64, 4, 4)]:
    for kv_len in [1, 5, 65, 300]:
        T = 4096
        rng = np.random.default_rng(kv_len * 7 + D)
        kb = rng.standard_normal(T * nkv * D).astype(np.float16)
        vb = rng.standard_normal(T * nkv * D).astype(np.float16)
        q = (rng.standard_normal(nh * D) * 2).astype(np.float32)
        xg, ag = R.mha(kb, vb, q, D, kv_len, T, nh, nkv)
        xo, ao = O.mha(kb, vb, q, D, kv_len, T, nh, nkv)
        ag = ag.reshape(nh, T)[:, :kv_len]; ao = ao.reshape(nh, T)[:, :kv_len]
        bad = np.abs(ag - ao) > 1e-4
        print(D, nh, nkv, kv_len, "xerr", float(np.max(np.abs(xg - xo))), "att bad", int(bad.sum()), "heads", sorted(set(np.nonzero(bad)[0].tolist())), ag[bad][:4], ao[bad][:4])
