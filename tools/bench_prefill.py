"""Config 4 of BASELINE.json on its own: Llama-3.2-3B fp16, 4k context, `-m perplexity`
as ONE batched MFMA prefill (yalm_prefill). Same measurement as the `prefill` object of
bench.py's default line (bench.prefill_leg), for other models / lengths.

usage: python tools/bench_prefill.py [--model llama-3.2-3b] [--n 4096] [--iters 3]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import prefill_leg  # noqa: E402
from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama-3.2-3b")
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--check", type=int, default=48, help="positions compared against the decode engine")
args = ap.parse_args()
print(json.dumps(prefill_leg(runtime, M, args.model, args.n, args.iters, args.check)), flush=True)
