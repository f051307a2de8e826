"""GEMV launch-geometry sweep (default: the row-block kernel, gpw = workgroups per CU) on the Mistral-7B-shaped synthetic model.
Times each weight-streaming kernel (HIP events, layers rotated so weights come
from HBM) for every (threads, unroll, gpw) candidate; prints GB/s.
usage: python tools/sweep_gemv.py [--dtype fp16|fp8] [--iters 64]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="fp16")
ap.add_argument("--iters", type=int, default=64)
ap.add_argument("--kinds", default="0,1,2,3,4")
ap.add_argument("--top", type=int, default=6)
args = ap.parse_args()

cfg = M.MISTRAL_7B.with_(weight_dtype=M.F16 if args.dtype == "fp16" else M.F8E5M2)
wb = M.DTYPE_BYTES[cfg.weight_dtype]
dm = runtime.DeviceModel.synthetic(cfg)
dec = runtime.Decoder(dm)
dec.forward(1, 0)
# kind -> (time_kernel id, bytes per launch, n_groups)
KINDS = {
    0: ("qkv", 0, (cfg.q_dim + 2 * cfg.kv_dim) * cfg.dim * wb, (cfg.q_dim + 2 * cfg.kv_dim) // 2),
    1: ("wo", 2, cfg.dim * cfg.q_dim * wb, cfg.dim),
    2: ("glu", 3, 2 * cfg.hidden_dim * cfg.dim * wb, cfg.hidden_dim),
    3: ("w2", 4, cfg.dim * cfg.hidden_dim * wb, cfg.dim),
    4: ("cls", 5, cfg.vocab_size * cfg.dim * wb, cfg.vocab_size // 2),
}
for kind in [int(k) for k in args.kinds.split(",")]:
    name, kid, nbytes, groups = KINDS[kind]
    dec.set_gemv_config(kind)
    auto = dec.time_kernel(kid, args.iters)
    print(f"{name}: auto {auto * 1e3:8.2f} us  {nbytes / auto / 1e6:7.0f} GB/s", flush=True)
    results = []
    for threads in (256, 512, 1024):
        for unroll in (2, 4, 8):
            for gpw in (1, 2, 3, 4):
                try:
                    dec.set_gemv_config(kind, threads, unroll, gpw)
                    t = dec.time_kernel(kid, args.iters)
                except runtime.YalmError as e:
                    print("  skip", threads, unroll, gpw, e)
                    continue
                results.append((t, threads, unroll, gpw))
    results.sort()
    for t, threads, unroll, gpw in results[:args.top]:
        print(f"   threads={threads} U={unroll} wg/cu={gpw:3d}: {t * 1e3:8.2f} us {nbytes / t / 1e6:7.0f} GB/s")
    dec.set_gemv_config(kind)
dec.close()
dm.close()
