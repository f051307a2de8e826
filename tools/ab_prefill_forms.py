"""Interleaved A/B of prefill forms in ONE process through yalm_set_prefill_forms (the
production library: no A/B build needed): one decoder per variant on the same weights,
each round times every variant back to back (yalm_prefill_time).

usage: python tools/ab_prefill_forms.py [--model llama-3.2-3b] [--n 4096] [--rounds 5] name=SPEC ...
       e.g.  plain=ksplit:0  ksplit=   (an empty spec: the defaults)"""
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
ap.add_argument("--split", action="store_true", help="the split-operand precision form")
ap.add_argument("variants", nargs="+")
args = ap.parse_args()

cfg = M.PRESETS[args.model].with_(weight_dtype=M.F16, max_seq_len=max(args.n, 64))
dm = runtime.DeviceModel.synthetic(cfg, seed=5)
decs = {}
for v in args.variants:
    name, _, spec = v.partition("=")
    d = runtime.Decoder(dm)
    d.set_prefill_forms(spec)
    if args.split:
        d.set_prefill_precision(runtime.PREFILL_SPLIT)
    decs[name] = d
res = {k: [] for k in decs}
for r in range(args.rounds):
    for name, d in decs.items():
        res[name].append(d.prefill_time(args.n, args.iters))
    print(json.dumps({"round": r, **{k: round(v[-1], 3) for k, v in res.items()}}), flush=True)
for name, ms in res.items():
    s = sorted(ms)
    print(json.dumps({"variant": name, "model": args.model, "n": args.n, "split_form": args.split,
                      "median_ms": round(s[len(s) // 2], 3), "min_ms": round(s[0], 3)}))
for d in decs.values():
    d.close()
dm.close()
