"""Per-phase timeline of the persistent decode engine (engine.h) on a
Mistral-7B-shaped synthetic model: the last launch's s_memrealtime stamps
(100 MHz) per CU and phase (yalm_engine_trace), summarised per phase kind over
layers 1..L-1 (medians over CUs, then over layers).

usage: python tools/engine_trace.py [--model mistral-7b] [--dtype fp16|fp8] [--tokens 8]
columns (us): seam = wait for the previous phase on every CU; in = input
gather (+ rmsnorm); rows = streaming the ring; epi = epilogue + publish;
crit = critical-path length of the phase (last publisher to last publisher);
stall = loader ring-full time inside the phase; ahead = ring slots landed
beyond the consumer position at phase start.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["YALM_ENGINE_TRACE"] = "1"
os.environ.setdefault("YALM_ENGINE", "1")

from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402

KINDS = ["qkv", "attn", "wo", "glu", "w2"]


def summarise(tr, L, label=""):
    tr = tr.astype(np.int64)
    E = 5 * L + 2
    start = tr[:, E - 1, 0]
    t0 = start.min()
    end = tr[:, E - 1, 3]
    print(f"{label}kernel span {(end.max() - t0) / 100:.1f} us; CU start spread {(start.max() - t0) / 100:.2f} us; "
          f"loader stall total median {np.median(tr[:, E - 1, 1]) / 100:.1f} us, loader finish "
          f"{(np.median(tr[:, E - 1, 2]) - t0) / 100:.1f} us; loader0 vmcnt-wait median "
          f"{np.median(tr[:, E - 1, 4]) / 100:.1f} us of lifetime {np.median(tr[:, E - 1, 5]) / 100:.1f} us")
    print(f"{'phase':8s} {'seam':>7s} {'in':>7s} {'rows':>7s} {'epi':>7s} {'crit':>7s} {'stall':>7s} {'ahead':>6s}")
    tot = 0.0
    for k, name in enumerate(KINDS + ["logits"]):
        phs = [l * 5 + k for l in range(1, L)] if name != "logits" else [5 * L]
        if name == "logits" and not tr[:, 5 * L, 3].any():
            continue
        cols = {c: [] for c in ("seam", "in", "rows", "epi", "crit", "stall", "ahead")}
        for ph in phs:
            prev = tr[:, ph - 1]
            cur = tr[:, ph]
            cols["seam"].append(np.median(cur[:, 0] - prev[:, 3]))
            cols["in"].append(np.median(cur[:, 1] - cur[:, 0]))
            cols["rows"].append(np.median(cur[:, 2] - cur[:, 1]))
            cols["epi"].append(np.median(cur[:, 3] - cur[:, 2]))
            cols["crit"].append(cur[:, 3].max() - prev[:, 3].max())
            cols["stall"].append(np.median(cur[:, 4] - prev[:, 4]))
            cols["ahead"].append(np.median(cur[:, 5] - cur[:, 6] / 8.0))
        v = {c: float(np.median(x)) for c, x in cols.items()}
        tot += v["crit"] * (L if name != "logits" else 1)
        print(f"{name:8s} {v['seam'] / 100:7.2f} {v['in'] / 100:7.2f} {v['rows'] / 100:7.2f} {v['epi'] / 100:7.2f} "
              f"{v['crit'] / 100:7.2f} {v['stall'] / 100:7.2f} {v['ahead']:6.1f}")
    print(f"sum of critical paths ~ {tot / 100:.1f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "fp8"])
    ap.add_argument("--tokens", type=int, default=8)
    ap.add_argument("--save", default="", help="write the raw (workgroups, phases, 8) trace as .npy")
    args = ap.parse_args()
    runtime.check(runtime.lib.yalm_set_device(0))
    cfg = M.PRESETS[args.model].with_(weight_dtype=M.F16 if args.dtype == "fp16" else M.F8E5M2)
    dm = runtime.DeviceModel.synthetic(cfg, seed=1)
    dec = runtime.Decoder(dm)
    assert dec.engine, "decoder is not running the persistent engine"
    for pos in range(12):
        dec.forward((7 * pos + 1) % cfg.vocab_size, pos, runtime.HYDRATE_KV_CACHE)
    dec.generate_greedy(5, 12, args.tokens)
    tr = dec.engine_trace()
    summarise(tr, cfg.n_layers, f"[{args.model} {args.dtype} greedy, kv {12 + args.tokens}] ")
    if args.save:
        np.save(args.save, tr)
    dec.close()
    dm.close()


if __name__ == "__main__":
    main()
