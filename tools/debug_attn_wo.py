"""Debug aid (GPU): fused attention + Wo (attn_wo.h) vs the two separate
launches on the same weights, one forward at a few positions with the FFN
ablated (YALM_ABLATE=24: x = embedding + sum over layers of Wo . attention).
Prints the first differing rows of x and their ratio to the reference."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["YALM_ABLATE"] = os.environ.get("YALM_ABLATE", "24")

from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402


def main():
    runtime.check(runtime.lib.yalm_set_device(0))
    cfg = M.ModelConfig(dim=1024, hidden_dim=2048, head_dim=128, n_layers=int(os.environ.get("NL", "1")),
                        n_heads=16, n_kv_heads=4, vocab_size=1536, max_seq_len=72, rope_theta=10000.0,
                        act=M.SILU, weight_dtype=M.F16)
    t = M.synth_host_tensors(cfg, seed=5)
    decs = []
    for fused in (1, 0):
        os.environ["YALM_ATTN_WO"] = str(fused)
        dm = runtime.DeviceModel.from_arrays(cfg, t)
        dec = runtime.Decoder(dm)
        print("fused" if fused else "separate", "attn_wo =", dec.attn_wo, flush=True)
        decs.append((dm, dec))
    for pos, tok in enumerate([1, 17, 45]):
        xs = []
        for _, dec in decs:
            dec.forward(tok, pos)
            xs.append(dec.get_x().copy())
        a, b = xs
        d = np.abs(a - b)
        bad = np.nonzero(d > 1e-3 * (np.abs(b).max() + 1e-30))[0]
        print(f"pos {pos}: max|x| {np.abs(b).max():.4g} max diff {d.max():.4g} bad rows {len(bad)} first {bad[:24]}")
        if len(bad):
            r = bad[:8]
            print("   fused   ", a[r])
            print("   separate", b[r])
    for dm, dec in decs:
        dec.close()
        dm.close()


if __name__ == "__main__":
    main()
