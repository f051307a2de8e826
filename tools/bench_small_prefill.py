"""Prompt hydration (the CLI's path, main.cpp:91-97 in the reference: one forward per
prompt token) at small T: yalm_prefill of T positions (KV cache only, no logits)
against T sequential HYDRATE forwards (graph replays) on the same model.

usage: python tools/bench_small_prefill.py [--model mistral-7b] [--ts 1,5,13,32,64,128,256]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--ts", default="1,5,13,32,64,128,256")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    runtime.check(runtime.lib.yalm_set_device(0))
    cfg = M.PRESETS[args.model].with_(weight_dtype=M.F16)
    dm = runtime.DeviceModel.synthetic(cfg, seed=1)
    dec = runtime.Decoder(dm)
    rng = np.random.default_rng(0)
    for T in [int(t) for t in args.ts.split(",")]:
        toks = rng.integers(3, cfg.vocab_size, size=T).astype(np.int32)
        dec.prefill(toks, 0, logprobs=False)  # warm-up (buffers, kernels)
        best_p = 1e9
        for _ in range(args.reps):
            t0 = time.perf_counter()
            dec.prefill(toks, 0, logprobs=False)
            best_p = min(best_p, time.perf_counter() - t0)
        for pos, t in enumerate(toks):  # warm-up (graph)
            dec.forward(int(t), pos, runtime.HYDRATE_KV_CACHE)
        runtime.check(runtime.lib.yalm_stream_sync(None))
        dec.device_step()
        best_s = 1e9
        for _ in range(args.reps):
            t0 = time.perf_counter()
            for pos, t in enumerate(toks):
                dec.forward(int(t), pos, runtime.HYDRATE_KV_CACHE)
            dec.device_step()  # syncs the decoder stream
            best_s = min(best_s, time.perf_counter() - t0)
        print(f"{args.model} T {T:4d}: prefill {best_p * 1e3:8.3f} ms   sequential {best_s * 1e3:8.3f} ms   "
              f"ratio {best_s / best_p:6.2f}", flush=True)
    dec.close()
    dm.close()


if __name__ == "__main__":
    main()
