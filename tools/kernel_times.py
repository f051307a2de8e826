"""Per-kernel average device time (yalm_time_kernel: eager launches between HIP
events, layers rotated so weights come from HBM) for the decoder's kernels on a
synthetic model, with the kernel names. Compare variants via environment knobs.

usage: python tools/kernel_times.py [--model mistral-7b] [--dtype fp16|fp8] [--iters 64]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402

KINDS = {0: "QKV", 1: "attention", 2: "Wo", 3: "W1|W3+GLU", 4: "W2", 5: "logits", 8: "attn+Wo gran"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "fp8"])
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=16, help="positions hydrated first (attention kv_len = ctx + 1)")
    ap.add_argument("--ctxs", default="", help="comma-separated contexts, hydrated progressively (overrides --ctx)")
    ap.add_argument("--kernels", default="", help="comma-separated kernel ids (default: all)")
    args = ap.parse_args()
    runtime.check(runtime.lib.yalm_set_device(0))
    cfg = M.PRESETS[args.model].with_(weight_dtype=M.F16 if args.dtype == "fp16" else M.F8E5M2)
    dm = runtime.DeviceModel.synthetic(cfg, seed=1)
    dec = runtime.Decoder(dm)
    ctxs = [int(c) for c in args.ctxs.split(",")] if args.ctxs else [args.ctx]
    kids = [int(k) for k in args.kernels.split(",")] if args.kernels else list(KINDS)
    wb = M.DTYPE_BYTES[cfg.weight_dtype]
    nbytes = {0: (cfg.q_dim + 2 * cfg.kv_dim) * cfg.dim * wb, 2: cfg.dim * cfg.q_dim * wb,
              3: 2 * cfg.hidden_dim * cfg.dim * wb, 4: cfg.dim * cfg.hidden_dim * wb,
              5: cfg.vocab_size * cfg.dim * wb, 8: cfg.dim * cfg.q_dim * wb}
    env = {k: v for k, v in os.environ.items() if k.startswith("YALM_")}
    done = 0
    for ctx in ctxs:
        for pos in range(done, ctx):
            dec.forward((7 * pos + 1) % cfg.vocab_size, pos, runtime.HYDRATE_KV_CACHE)
        done = ctx
        dec.forward((7 * ctx + 1) % cfg.vocab_size, ctx)  # the step state at kv_len ctx + 1
        print(f"[{args.model} {args.dtype} kv_len {ctx + 1}] {env}")
        for kid in kids:
            if kid == 8 and not dec.attn_wo:
                continue
            us = dec.time_kernel(kid, args.iters) * 1e3
            gbs = nbytes.get(kid, 0) / (us * 1e-6) / 1e9 if kid in nbytes else 0
            print(f"  {kid} {KINDS[kid]:10s} {us:8.2f} us  {gbs:7.0f} GB/s  {dec.kernel_name(kid)}", flush=True)
    dec.close()
    dm.close()


if __name__ == "__main__":
    main()
