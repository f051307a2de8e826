"""Interleaved A/B of prefill settings in ONE process (cdna_hip_programming.md §5.4
rule 24): the forms are fixed when a decoder is created, so each variant gets its own
decoder (created under its environment) and each round runs every variant back to
back on the same weights and device.

usage: python tools/ab_prefill.py [--model llama-3.2-3b] [--n 4096] [--rounds 5]
                                  name=ENV=VAL[;ENV=VAL...] ...
       e.g.  2ph=YALM_PF_8P=0  8ph=YALM_PF_8P=1"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama-3.2-3b")
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=2)
ap.add_argument("variants", nargs="+")
args = ap.parse_args()

variants = []
for v in args.variants:
    name, _, rest = v.partition("=")
    env = dict(kv.split("=", 1) for kv in rest.split(";") if kv)
    variants.append((name, env))

cfg = M.PRESETS[args.model].with_(weight_dtype=M.F16, max_seq_len=max(args.n, 64))
n = args.n
q_dim, kv_dim = cfg.n_heads * cfg.head_dim, cfg.n_kv_heads * cfg.head_dim
gemm = 2 * n * (cfg.dim * (q_dim + 2 * kv_dim) + q_dim * cfg.dim + 3 * cfg.dim * cfg.hidden_dim)
attn = 4 * cfg.head_dim * cfg.n_heads * n * (n + 1) // 2
flops = cfg.n_layers * (gemm + attn) + 2 * n * cfg.dim * cfg.vocab_size

dm = runtime.DeviceModel.synthetic(cfg, seed=5)
decs = {}
for name, env in variants:
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    decs[name] = runtime.Decoder(dm)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
res = {name: [] for name, _ in variants}
for r in range(args.rounds):
    for name, _ in variants:
        res[name].append(decs[name].prefill_time(n, args.iters))
    print(json.dumps({"round": r, **{k: round(v[-1], 3) for k, v in res.items()}}), flush=True)
for name, ms in res.items():
    s = sorted(ms)
    print(json.dumps({"variant": name, "model": args.model, "n": n, "median_ms": round(s[len(s) // 2], 3),
                      "min_ms": round(s[0], 3), "tflops_at_median": round(flops / (s[len(s) // 2] * 1e-3) / 1e12, 1)}))
for d in decs.values():
    d.close()
dm.close()
