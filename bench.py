"""Decode benchmark — BASELINE.json metric "decode tok/s Mistral-7B fp16 @1 GPU;
% of HBM bytes/token roofline" on config 2 (Mistral-7B fp16, 1x MI355X,
greedy -t 0, 256 tokens).

A step = one decode token: the whole per-token forward (embedding, 32
blocks, final norm, logits GEMV, device argmax feeding the next token) as one
hipGraph replay. Weights are random (no checkpoints offline) but of the real
architecture and size, generated in HBM before timing. The prompt is 13
synthetic token ids (the README prompt's length) hydrated first.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype fp16|fp8]
For N>1 launch under torch.distributed.run: each rank decodes its own
sequence on its GPU (replicas; no collective on the data path) and rank 0
reports total tokens / max-over-ranks time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PROMPT_LEN = 13


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "fp8"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample budget")
    ap.add_argument("--kernel-iters", type=int, default=64)
    ap.add_argument("--tp", action="store_true",
                    help="tensor parallel over the launched ranks (one sequence) instead of replicas")
    ap.add_argument("--tp-transport", default="rccl", choices=["rccl", "ipc"],
                    help="all-reduce transport for --tp: RCCL (one rank per GPU) or the IPC one-shot exchange")
    return ap.parse_args()


def pmc_traffic(kernel_match, dtype):
    """HBM bytes per launch of the dominant kernel from the newest committed
    rocprofv3 --pmc FETCH_SIZE pass that profiled it (profiles/*_pmc_fetch_size*.csv):
    median FETCH_SIZE (KB) x 1024 x 2 -- gfx950 counts half the bytes of 16 B/lane
    streaming reads (MI355X_MICROARCH.md §HBM). `kernel_match`: substrings that
    must all appear in the kernel name. None if no matching profile."""
    import csv
    import glob
    import statistics

    if dtype != "fp16":
        return None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_fetch_size*.csv")), reverse=True):
        rows = list(csv.DictReader(open(f)))
        vals = [float(r["Counter_Value"]) for r in rows
                if r["Counter_Name"] == "FETCH_SIZE" and all(k in r["Kernel_Name"] for k in kernel_match)]
        if vals:
            return int(statistics.median(vals) * 1024 * 2), os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(cfg, budget_s):
    """The CPU oracle (oracle/, restatement of the reference -d cpu path with
    its AVX2/F16C GEMV and OpenMP) on the same synthetic weights, timed on
    this host. Bounded sample: hydrate the prompt, then decode until the
    budget is spent (at least 2 tokens)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np

    import oracle_py as O

    threads = int(os.environ.get("YALM_CPU_THREADS", min(16, os.cpu_count() or 1)))
    O.set_threads(threads)
    host = O.synth_host_tensors_fast(cfg, seed=1)
    om = O.OracleModel(cfg, host)
    prompt = [(7 * i + 1) % cfg.vocab_size for i in range(PROMPT_LEN)]
    for pos, t in enumerate(prompt):
        om.forward(t, pos, 1 if pos == len(prompt) - 1 else 0)
    tok = int(np.argmax(om.buf["logits"]))
    n = 0
    t0 = time.perf_counter()
    while True:
        lg = om.forward(tok, PROMPT_LEN + n, 1)
        tok = int(np.argmax(lg))
        n += 1
        el = time.perf_counter() - t0
        if (el >= budget_s and n >= 2) or n >= 256:
            break
    del om, host
    return {
        "value": round(n / el, 4),
        "unit": "tok/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle -d cpu restatement, {n} greedy decode tokens after a {PROMPT_LEN}-token prompt, "
                  f"same synthetic Mistral-7B {'fp16' if cfg.weight_dtype == 1 else 'fp8'} weights, "
                  f"{threads} OpenMP threads, {el:.1f} s",
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    dev = local_rank
    if world > 1:
        import torch
        import torch.distributed as dist_mod

        # one rank per GPU; more ranks than GPUs (a 1-GPU rehearsal of the N > 1
        # path) share devices round-robin
        dev = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if torch.cuda.device_count() >= world:
            dist_mod.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist_mod.init_process_group("gloo")
        dist = dist_mod

    from yalm_amd import models as M
    from yalm_amd import runtime

    runtime.check(runtime.lib.yalm_set_device(dev))
    base = M.PRESETS[args.model]
    cfg = base.with_(weight_dtype=M.F16 if args.dtype == "fp16" else M.F8E5M2)

    if args.tp:
        # one sequence sharded over all ranks (Megatron split, RCCL all-reduce in the graph)
        dm = runtime.DeviceModel.synthetic(cfg, seed=1, tp=(rank, world))
        if args.tp_transport == "ipc":
            def gather(h):
                if dist is None:
                    return [h]
                out = [None] * world
                dist.all_gather_object(out, h)
                return out

            dec = runtime.Decoder(dm, tp_gather=gather)
        else:
            uid = [runtime.tp_unique_id() if rank == 0 else None]
            if dist is not None:
                dist.broadcast_object_list(uid, src=0)
            dec = runtime.Decoder(dm, tp_id=uid[0])
    else:
        dm = runtime.DeviceModel.synthetic(cfg, seed=1)
        dec = runtime.Decoder(dm)
    prompt = [(7 * i + 1) % cfg.vocab_size for i in range(PROMPT_LEN)]
    for pos, t in enumerate(prompt[:-1]):
        dec.forward(t, pos, runtime.HYDRATE_KV_CACHE)
    # first generated token; the device loop continues from there
    first = dec.generate_greedy(prompt[-1], PROMPT_LEN - 1, 1)[0]
    del first
    if args.warmup:
        dec.enqueue_greedy(args.warmup)
    runtime.check(runtime.lib.yalm_stream_sync(None))
    _, pos0 = dec.device_step()

    def barrier_sync():
        runtime.check(runtime.lib.yalm_stream_sync(None))
        dec.device_step()  # syncs the decoder stream
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    barrier_sync()
    t0 = time.perf_counter()
    dec.enqueue_greedy(args.steps)
    dec.device_step()
    t1 = time.perf_counter()
    barrier_sync()
    elapsed = t1 - t0
    if dist is not None:
        import torch

        tt = torch.tensor([elapsed], dtype=torch.float64,
                          device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    _, pos1 = dec.device_step()
    assert pos1 - pos0 == args.steps, (pos0, pos1)

    # ---- roofline of the dominant kernel: the fused feed-forward launch (rmsnorm +
    # W1/W3 + GLU + W2 + residual, 79.3% of the bytes) when the decoder runs it, else
    # the W1/W3 GEMV + SiLU-GLU (52.9% of the bytes)
    wb = M.DTYPE_BYTES[cfg.weight_dtype]
    hid_local = cfg.hidden_dim // (world if args.tp else 1)
    if dec.ffn:
        KID = 7
        # W1, W3, W2 + rms_ffn + x read + x rows written + hb written once
        kern_bytes = 3 * hid_local * cfg.dim * wb + 3 * cfg.dim * 4 + hid_local * 4
        match = ("ffn_kernel<WF16",)
    else:
        KID = 3
        kern_bytes = 2 * hid_local * cfg.dim * wb + 2 * cfg.dim * 4 + hid_local * 4
        match = ("gemv_rb_kernel<WF16", "PGlu")
    avg_ms = dec.time_kernel(KID, args.kernel_iters)
    achieved = kern_bytes / (avg_ms * 1e-3) / 1e9
    kname = dec.kernel_name(KID)
    traffic, traffic_src = pmc_traffic(match, args.dtype)

    toks = args.steps * (1 if args.tp else world)
    value = toks / elapsed
    kv_avg = (pos0 + pos1) / 2 + 1
    bytes_per_tok = cfg.weight_bytes_per_token() + cfg.kv_bytes_per_token(int(kv_avg))
    step_gbs = bytes_per_tok * (args.steps / elapsed) / 1e9  # per sequence
    n_seq = 1 if args.tp else world
    agg_gbs = step_gbs * n_seq  # all GPUs
    peak_all = HBM_PEAK_GBS * world

    out = {
        "metric": "decode tok/s Mistral-7B fp16 @1 GPU; % of HBM bytes/token roofline"
        if args.dtype == "fp16" else "decode tok/s Mistral-7B fp8 @1 GPU; % of HBM bytes/token roofline",
        "value": round(value, 3),
        "unit": "tok/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.tp else "weak",
        "vs_baseline": None,
        "dtype": "f16" if args.dtype == "fp16" else "f8e5m2",
        "data": "synthetic (random weights of the real Mistral-7B-v0.2 shape generated in HBM; "
                f"{PROMPT_LEN}-token synthetic prompt; greedy argmax on device)",
        "config": {
            "workload": f"{args.model} {args.dtype} batch-1 greedy decode, {args.steps} tokens"
                        f"{' (one sequence, tensor parallel)' if args.tp else '/GPU'}, "
                        f"kv_len {pos0 + 1}..{pos1}",
            "model": args.model,
            "global_batch": world,
            "seq_len": int(pos1),
            "parallelism": (f"tp{world}-{args.tp_transport}" if args.tp else
                            (f"replicas{world}" if world > 1 else "single")),
        },
        "step_roofline": {
            "bytes_per_token": int(bytes_per_tok),
            "achieved": round(agg_gbs, 1),
            "peak": peak_all,
            "unit": "GB/s",
            "frac": round(agg_gbs / peak_all, 4),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kname,
            "avg_launch_us": round(avg_ms * 1e3, 3),
            "algorithmic_bytes_per_launch": int(kern_bytes),
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
        },
        "cpu_baseline": None,
    }
    dec.close()
    dm.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
