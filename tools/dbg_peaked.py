"""Debug: the peaked Llama-3B-dims model's sampled text, GPU decode vs oracle per position."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py as O  # noqa: E402
from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime as R  # noqa: E402

cfg = M.LLAMA_32_3B.with_(max_seq_len=256)
n = 256
dm = R.DeviceModel.synthetic(cfg, seed=6, peak=M.PEAKED)
a, b = R.Decoder(dm), R.Decoder(dm)
rng = np.random.default_rng(77)
toks, lga = [1], []
for pos in range(n - 1):
    lg = a.forward(toks[-1], pos).astype(np.float64)
    lga.append(lg)
    pr = np.exp(lg - lg.max())
    toks.append(int(rng.choice(cfg.vocab_size, p=pr / pr.sum())))
worst_det = 0.0
for pos in range(n - 1):
    lg = b.forward(toks[pos], pos).astype(np.float64)
    worst_det = max(worst_det, float(np.max(np.abs(lg - lga[pos]))))
print("determinism: max |logits A - logits B| =", worst_det, flush=True)
om = O.OracleModel(cfg, O.synth_host_tensors_fast(cfg, seed=6, peak=M.PEAKED))
for pos in range(n - 1):
    lo = om.forward(toks[pos], pos).astype(np.float64)
    lg = lga[pos]
    e = np.max(np.abs(lg - lo)) / np.max(np.abs(lo))
    t = toks[pos + 1]
    lpo = lo[t] - lo.max() - np.log(np.exp(lo - lo.max()).sum())
    lpg = lg[t] - lg.max() - np.log(np.exp(lg - lg.max()).sum())
    if e > 1e-3 or not np.isfinite(lpo) or pos % 32 == 0 or lpo < -30:
        print(f"pos {pos}: tok {toks[pos]} -> {t}: logits rel {e:.2e}, log p oracle {lpo:.3f} gpu {lpg:.3f}, "
              f"max|lo| {np.max(np.abs(lo)):.1f}, argmax {int(np.argmax(lo))} / {int(np.argmax(lg))}", flush=True)
