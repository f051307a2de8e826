"""Config 4 of BASELINE.json: Llama-3.2-3B fp16, 4k context, `-m perplexity`
as ONE batched MFMA prefill (yalm_prefill) instead of the reference's 4095
sequential forwards (main.cpp:128-200). Synthetic weights of the real shape,
synthetic token ids. Prints one JSON line: ms per 4096-position pass (with
per-position log-probs), the MFMA utilisation against the dense f16 peak, the
same positions through the decode engine for scale, and a parity spot check
(first positions, prefill vs decode log p).

usage: python tools/bench_prefill.py [--model llama-3.2-3b] [--n 4096] [--iters 3]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402

MFMA_F16_PEAK_TFLOPS = 2500.0  # MI355X dense f16/bf16 (MI355X_MICROARCH.md; no sparsity)

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama-3.2-3b")
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--check", type=int, default=48, help="positions compared against the decode engine")
args = ap.parse_args()

cfg = M.PRESETS[args.model].with_(weight_dtype=M.F16, max_seq_len=max(args.n, 64))
n = args.n
q_dim, kv_dim = cfg.n_heads * cfg.head_dim, cfg.n_kv_heads * cfg.head_dim
gemm = 2 * n * (cfg.dim * (q_dim + 2 * kv_dim) + q_dim * cfg.dim + 3 * cfg.dim * cfg.hidden_dim)
attn = 4 * cfg.head_dim * cfg.n_heads * n * (n + 1) // 2
flops = cfg.n_layers * (gemm + attn) + 2 * n * cfg.dim * cfg.vocab_size

dm = runtime.DeviceModel.synthetic(cfg, seed=5)
dec = runtime.Decoder(dm)
ms = dec.prefill_time(n, args.iters)
tflops = flops / (ms * 1e-3) / 1e12

# parity spot check + sequential-decode rate on the same model
rng = np.random.default_rng(0)
tokens = rng.integers(0, cfg.vocab_size, size=args.check + 1).astype(np.int32)
lp_p = dec.prefill(tokens)
dec2 = runtime.Decoder(dm)
lp_d = []
t0 = time.perf_counter()
for pos in range(args.check):
    lg = dec2.forward(int(tokens[pos]), pos).astype(np.float64)
    m = lg.max()
    lp_d.append(lg[tokens[pos + 1]] - m - np.log(np.exp(lg - m).sum()))
seq_s = (time.perf_counter() - t0) / args.check
err = float(np.max(np.abs(lp_p[: args.check] - np.array(lp_d))))

print(json.dumps({
    "metric": f"prefill ms {args.model} fp16 {n}-position perplexity pass",
    "value": round(ms, 3),
    "unit": "ms",
    "higher_is_better": False,
    "tok_per_s": round(n / (ms * 1e-3), 1),
    "flops": flops,
    "mfma": {"achieved": round(tflops, 1), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
             "frac": round(tflops / MFMA_F16_PEAK_TFLOPS, 4)},
    "sequential_decode_ms_per_position": round(seq_s * 1e3, 3),
    "speedup_vs_sequential": round(seq_s * n / (ms * 1e-3), 1),
    "parity": {"positions": args.check, "max_abs_dlogp_vs_decode": err},
    "data": "synthetic weights of the real shape, synthetic token ids",
}), flush=True)
dec2.close()
dec.close()
dm.close()
