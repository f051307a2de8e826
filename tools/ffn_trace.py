"""Timeline of the fused feed-forward launch (ffn.h) on a Mistral-7B-shaped
synthetic model: the last layer's launch of the last token, from the
per-workgroup s_memrealtime stamps (100 MHz) of yalm_ffn_trace; then the
launch's average time against the separate GLU + W2 launches.

usage: python tools/ffn_trace.py [--model mistral-7b] [--dtype fp16|fp8] [--ctx 32]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["YALM_FFN_TRACE"] = "1"

from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402


def q(v):
    return f"min {v.min():7.2f} med {np.median(v):7.2f} max {v.max():7.2f}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "fp8"])
    ap.add_argument("--ctx", type=int, default=32)
    ap.add_argument("--iters", type=int, default=64)
    args = ap.parse_args()
    runtime.check(runtime.lib.yalm_set_device(0))
    cfg = M.PRESETS[args.model].with_(weight_dtype=M.F16 if args.dtype == "fp16" else M.F8E5M2)
    dm = runtime.DeviceModel.synthetic(cfg, seed=1)
    dec = runtime.Decoder(dm)
    assert dec.ffn, "decoder does not run the fused feed-forward launch"
    for pos in range(args.ctx):
        dec.forward((7 * pos + 1) % cfg.vocab_size, pos, runtime.HYDRATE_KV_CACHE)
    dec.forward(5, args.ctx)
    tr = dec.ffn_trace().astype(np.int64)
    t0 = tr[:, 0].min()
    us = (tr[:, :6] - t0) / 100.0
    print(f"[{args.model} {args.dtype}] grid {len(tr)} workgroups; launch span {us[:, 5].max():.2f} us; "
          f"wave-0 items GLU {int(tr[0, 6] & 0xffffffff)} W2 {int(tr[0, 6] >> 32)}")
    names = ["start", "GLU partials done", "hb published", "all flags seen", "hb in LDS", "end"]
    for k, n in enumerate(names):
        print(f"{n:18s} {q(us[:, k])}")
    d = np.diff(us, axis=1)
    for k, n in enumerate(["GLU phase", "publish", "poll", "gather+barrier", "W2 phase"]):
        print(f"  dt {n:15s} {q(d[:, k])}")
    t_ffn = dec.time_kernel(7, args.iters) * 1e3
    t_glu = dec.time_kernel(3, args.iters) * 1e3
    t_w2 = dec.time_kernel(4, args.iters) * 1e3
    wb = M.DTYPE_BYTES[cfg.weight_dtype]
    b = 3 * cfg.hidden_dim * cfg.dim * wb
    print(f"fused launch {t_ffn:.2f} us ({b / t_ffn / 1e3:.0f} GB/s of weights)  vs  GLU {t_glu:.2f} + W2 {t_w2:.2f} "
          f"= {t_glu + t_w2:.2f} us (eager, layers rotated)")
    dec.close()
    dm.close()


if __name__ == "__main__":
    main()
