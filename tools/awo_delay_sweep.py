"""Fused attention + Wo launch time (yalm_time_kernel 8) against one A/B knob at several
context lengths: by default the Wo workgroups' start delay (YALM_ATTN_WO_DELAY,
s_memrealtime ticks of 10 ns); --knob YALM_AWO_SPLITS sweeps the key splits per kv head.
Needs the A/B build (tools/build_ab_lib.sh wt ab; YALM_LIB=<that .so>): the product reads
no environment knobs.

usage: python tools/awo_delay_sweep.py [--dtype fp16|fp8] [--ctx 150,1023,4095] [--knob NAME] [--delays 0,20,100,200,300]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "fp8"])
    ap.add_argument("--ctx", default="150,1023,4095")
    ap.add_argument("--delays", default="0,20,100,200,300")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--knob", default="YALM_ATTN_WO_DELAY")
    args = ap.parse_args()
    runtime.check(runtime.lib.yalm_set_device(0))
    cfg = M.MISTRAL_7B.with_(weight_dtype=M.F16 if args.dtype == "fp16" else M.F8E5M2)
    dm = runtime.DeviceModel.synthetic(cfg, seed=1)
    ctxs = [int(c) for c in args.ctx.split(",")]
    delays = [int(d) for d in args.delays.split(",")]
    res = {}
    for d in delays:
        os.environ[args.knob] = str(d)
        dec = runtime.Decoder(dm)
        pos = 0
        for ctx in sorted(ctxs):
            toks = [(7 * p + 1) % cfg.vocab_size for p in range(pos, ctx)]
            if args.dtype == "fp16" and len(toks) > 64:
                dec.prefill(toks, pos, logprobs=False)
            else:
                for i, t in enumerate(toks):
                    dec.forward(t, pos + i, runtime.HYDRATE_KV_CACHE)
            pos = ctx
            dec.forward(5, ctx)
            pos = ctx + 1
            res[(d, ctx)] = dec.time_kernel(8, args.iters) * 1e3
            print(f"{args.knob} {d:4d}  kv_len {ctx + 1:5d}: {res[(d, ctx)]:7.2f} us", flush=True)
        dec.close()
    print(f"{args.dtype}: fused attention + Wo, us per launch (rows: {args.knob})")
    print("value  " + "".join(f"{'kv ' + str(c + 1):>10s}" for c in sorted(ctxs)))
    for d in delays:
        print(f"{d:5d}  " + "".join(f"{res[(d, c)]:10.2f}" for c in sorted(ctxs)))
    dm.close()


if __name__ == "__main__":
    main()
