"""Decode benchmark — BASELINE.json metric "decode tok/s Mistral-7B fp16 @1 GPU;
% of HBM bytes/token roofline".

N = 1: config 2 (Mistral-7B fp16, 1x MI355X, greedy -t 0); `--dtype fp8` is
config 3 (E5M2 weights). N > 1: config 5, one sequence tensor-parallel over N
GPUs (Megatron split, RCCL all-reduce captured in the per-token graph);
`--replicas` runs N independent decoders instead, `--tp-transport ipc` the IPC
one-shot exchange.

A step = one decode token: the whole per-token forward (embedding, 32 blocks,
final norm, logits GEMV, device argmax feeding the next token) as one hipGraph
replay. Weights are random (no checkpoints offline) but of the real
architecture and size, generated in HBM before timing. The prompt is 13
synthetic token ids (the README prompt's length) hydrated first.

At N = 1 fp16 the line also carries `fp8`: config 3, the same decode with E5M2
weights (a child run of this script; `--no-fp8` skips it), and `prefill`:
config 4 (Llama-3.2-3B, one 4096-position `-m perplexity` pass as a batched
MFMA prefill) with its own MFMA roofline (`--no-prefill` skips it).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype fp16|fp8]
With --gpus N > 1 and no WORLD_SIZE in the environment, the script starts N
rank processes itself (before any GPU call); under torch.distributed.run each
rank reads RANK / LOCAL_RANK / WORLD_SIZE. Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import socket
import subprocess
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
    ap.add_argument("--replicas", action="store_true",
                    help="N > 1: N independent decoders (one sequence per GPU) instead of tensor parallelism")
    ap.add_argument("--tp", action="store_true", help="tensor parallel even at N = 1 (TP1 through the transport)")
    ap.add_argument("--tp-transport", default="rccl", choices=["rccl", "ipc"],
                    help="all-reduce transport for tensor parallelism: RCCL (one rank per GPU) or the IPC one-shot exchange")
    ap.add_argument("--no-envelope", action="store_true")
    ap.add_argument("--no-prefill", action="store_true",
                    help="skip the config-4 leg (Llama-3.2-3B 4096-position batched prefill, N = 1 fp16 only)")
    ap.add_argument("--prefill-iters", type=int, default=3)
    ap.add_argument("--no-fp8", action="store_true",
                    help="skip the config-3 leg (the same decode with E5M2 weights, N = 1 fp16 runs only)")
    ap.add_argument("--no-long", action="store_true",
                    help="skip the long-context leg (decode at the full 4096-slot window into the sink regime)")
    ap.add_argument("--long-only", action="store_true",
                    help="run only the long-context leg (N = 1 fp16; for profiling) and print its JSON")
    ap.add_argument("--long-steps", type=int, default=64)
    ap.add_argument("--no-alt", action="store_true",
                    help="N > 1 over RCCL: skip the second measurement through the IPC exchange")
    ap.add_argument("--no-gpu-state", action="store_true",
                    help="skip the rocm-smi query (under a profiler: its preload would run inside rocm-smi too)")
    ap.add_argument("--eager", action="store_true",
                    help="single forwards launch their kernels directly instead of replaying graphs (profilers)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N > 1 on ONE GPU: every rank on device 0, its decoder stream on a disjoint block of "
                         "256/N CUs (yalm_stream_create_cu_part), IPC transport -- config 5's production launch "
                         "sequence rehearsed, not a scaling measurement")
    return ap.parse_args()


def spawn_ranks(n):
    """--gpus N without a launcher: start N copies of this script as ranks 0..N-1
    (each picks GPU LOCAL_RANK) and return the worst exit code. Nothing here has
    touched the GPU."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def gpu_state():
    """Partition modes and the top DPM level of each clock as rocm-smi reports
    them (a separate process). The current clock read at idle says nothing about
    the run, so the envelope measured in-process is the box calibration; this
    only shows whether a box is partitioned or clock-capped."""
    import re

    out = {}
    try:
        r = subprocess.run(["rocm-smi", "--showcomputepartition", "--showmemorypartition", "--json"],
                           capture_output=True, text=True, timeout=30)
        d = json.loads(r.stdout)
        card = d[sorted(d)[0]] if d else {}
        out.update({k: v for k, v in card.items() if "partition" in k.lower()})
        r = subprocess.run(["rocm-smi", "--showclkfrq"], capture_output=True, text=True, timeout=30)
        kind = None
        for line in r.stdout.splitlines():
            m = re.search(r"Supported (\w+) frequencies", line)
            if m:
                kind = m.group(1)
                continue
            f = re.search(r"(\d+)\s*Mhz", line, re.I)
            if kind and f:
                out[f"{kind}_max_mhz"] = max(out.get(f"{kind}_max_mhz", 0), int(f.group(1)))
    except Exception as e:  # report, never fail the bench on it
        out["error"] = repr(e)[:200]
    return out


def cgroup_cpus():
    """CPUs this process may use by its cgroup CPU quota (v2 cpu.max, v1
    cfs_quota/period), or None when unlimited / unreadable."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, q // p)
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(kernel_match):
    """HBM bytes per launch of the dominant kernel from the newest committed
    rocprofv3 --pmc FETCH_SIZE pass that profiled it (profiles/*_pmc_fetch_size*.csv):
    median FETCH_SIZE (KB) x 1024 x 2 -- gfx950 counts half the bytes of 16 B/lane
    streaming reads (MI355X_MICROARCH.md §HBM). `kernel_match`: substrings that
    must all appear in the kernel name (the weight type is part of it, so fp16 and
    fp8 passes never mix). None if no matching profile."""
    import csv
    import glob
    import statistics

    import re

    def run_order(f):  # profile prefixes r<round><run letters>: r6w < r6ah (a < z < aa < ah, spreadsheet order)
        m = re.match(r"r(\d+)([a-z]+)_", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_fetch_size*.csv")), key=run_order, reverse=True):
        rows = list(csv.DictReader(open(f)))
        vals = [float(r["Counter_Value"]) for r in rows
                if r["Counter_Name"] == "FETCH_SIZE" and all(k in r["Kernel_Name"] for k in kernel_match)]
        if vals:
            return int(statistics.median(vals) * 1024 * 2), os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(cfg, budget_s):
    """The CPU oracle (oracle/, restatement of the reference -d cpu path with
    its AVX2/F16C GEMV and OpenMP) on the same synthetic weights, timed on
    this host. Threads: nproc (BASELINE.md CPU-baseline plan), capped by the
    job's cgroup CPU quota -- on the GPU box nproc shows the whole machine (256)
    while the job may use 16 CPUs, and 256 OpenMP threads there ran 0.03 tok/s
    (profiles/r3_cpu_threads.txt). Bounded sample: hydrate the prompt, then
    decode until the budget is spent (at least 2 tokens)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np

    import oracle_py as O

    threads, nproc, quota, share = cpu_threads()
    host = O.synth_host_tensors_fast(cfg, seed=1)
    om = O.OracleModel(cfg, host)
    prompt = [(7 * i + 1) % cfg.vocab_size for i in range(PROMPT_LEN)]
    O.set_threads(threads)
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
        "cpu_model": cpu_model(),
        "nproc": nproc,
        "cgroup_cpus": quota,
        "sample": f"oracle -d cpu restatement, {n} greedy decode tokens after a {PROMPT_LEN}-token prompt, "
                  f"same synthetic Mistral-7B {'fp16' if cfg.weight_dtype == 1 else 'fp8'} weights, "
                  f"{threads} OpenMP threads = the host CPUs this job may use (nproc {nproc}, "
                  f"cgroup quota {quota}, OMP_NUM_THREADS {share or 'unset'}), {el:.1f} s",
    }


def cpu_threads():
    """(threads, nproc, cgroup quota, OMP_NUM_THREADS share) for the CPU baselines."""
    nproc = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)  # the harness's CPU share when no quota is readable
    return min(nproc, quota or share or nproc), nproc, quota, share


def prefill_cpu_baseline(model="llama-3.2-3b", n=4096, budget_s=12.0):
    """Config 4's CPU baseline: the reference's `-m perplexity` loop (main.cpp:174-184:
    one OUTPUT_LOGITS forward per position, then log(sample_prob(next)), sampler.cpp:11-25)
    restated by the oracle (orc_forward + orc_sample_prob) on the same synthetic
    Llama-3.2-3B fp16 weights, on this host's CPUs. Bounded sample: positions 0.. at the
    start of the context, then the same number at the end (pos n - k .., over a cache
    filled with seeded fp16 K/V rows: attention reads rows, not how they were made), each
    half given half the budget; the n-position pass time is the trapezoid of the two
    per-position costs (the per-position cost is linear in kv_len)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np

    import oracle_py as O
    from yalm_amd import models as M

    threads, nproc, quota, share = cpu_threads()
    cfg = M.PRESETS[model].with_(weight_dtype=M.F16, max_seq_len=n)
    host = O.synth_host_tensors_fast(cfg, seed=5)
    om = O.OracleModel(cfg, host)
    O.set_threads(threads)
    rng = np.random.default_rng(0)
    toks = rng.integers(0, cfg.vocab_size, size=n + 1)

    def run(p0):
        done, lp, t0 = 0, 0.0, time.perf_counter()
        while True:
            lg = om.forward(int(toks[p0 + done]), p0 + done, 1)
            lp += float(np.log(O.olib.orc_sample_prob(O.P(lg), cfg.vocab_size, int(toks[p0 + done + 1]))))
            done += 1
            el = time.perf_counter() - t0
            if (el >= budget_s / 2 and done >= 2) or done >= 64:
                return done, el / done

    k_head, s_head = run(0)
    late = n - 64
    for l in range(cfg.n_layers):  # the cache rows an n-position pass would hold before position `late`
        om.kcache[l][:late] = (rng.standard_normal((late, cfg.kv_dim)) * 1.3).astype(np.float16)
        om.vcache[l][:late] = (rng.standard_normal((late, cfg.kv_dim)) * 1.3).astype(np.float16)
    k_tail, s_tail = run(late)
    del om, host
    total = (s_head + s_tail) / 2 * n
    return {
        "value": round(total * 1e3, 1),
        "unit": "ms",
        "cores": threads,
        "kind": "port",
        "ms_per_position": [round(s_head * 1e3, 2), round(s_tail * 1e3, 2)],
        "cpu_model": cpu_model(),
        "nproc": nproc,
        "cgroup_cpus": quota,
        "sample": f"oracle restatement of the reference -m perplexity loop (forward + sample_prob per position, "
                  f"main.cpp:174-184), {model} fp16 synthetic weights: {k_head} positions from pos 0 and {k_tail} "
                  f"from pos {late} ({threads} OpenMP threads); value = the {n}-position pass extrapolated "
                  f"linearly in kv_len from the two per-position costs",
    }


MFMA_F16_PEAK_TFLOPS = 2500.0  # MI355X dense f16 (MI355X_MICROARCH.md; no sparsity)


def prefill_leg(runtime, M, model="llama-3.2-3b", n=4096, iters=3, check=48):
    """Config 4 (BASELINE.json): `-m perplexity` over an n-position context as ONE
    batched MFMA prefill (yalm_prefill) instead of the reference's n - 1 sequential
    forwards (main.cpp:128-200). Synthetic weights of the real shape, synthetic ids.
    Time = HIP events around `iters` whole passes on the decoder stream (yalm_prefill_time),
    flops = the GEMMs + causal attention + logits; a spot check of the first `check`
    positions' log p against the decode engine (the oracle check at these dims is
    tests/test_gpu_prefill_llama.py)."""
    import numpy as np

    check = max(1, check)
    cfg = M.PRESETS[model].with_(weight_dtype=M.F16, max_seq_len=max(n, 64))
    q_dim, kv_dim = cfg.n_heads * cfg.head_dim, cfg.n_kv_heads * cfg.head_dim
    gemm = 2 * n * (cfg.dim * (q_dim + 2 * kv_dim) + q_dim * cfg.dim + 3 * cfg.dim * cfg.hidden_dim)
    attn = 4 * cfg.head_dim * cfg.n_heads * n * (n + 1) // 2
    flops = cfg.n_layers * (gemm + attn) + 2 * n * cfg.dim * cfg.vocab_size
    dm = runtime.DeviceModel.synthetic(cfg, seed=5)
    dec = runtime.Decoder(dm)
    dec2 = None
    try:
        ms = dec.prefill_time(n, iters)
        tflops = flops / (ms * 1e-3) / 1e12
        rng = np.random.default_rng(0)
        tokens = rng.integers(0, cfg.vocab_size, size=check + 1).astype(np.int32)
        lp_p = dec.prefill(tokens)
        dec2 = runtime.Decoder(dm)
        lp_d = []
        t0 = time.perf_counter()
        for pos in range(check):
            lg = dec2.forward(int(tokens[pos]), pos).astype(np.float64)
            m = lg.max()
            lp_d.append(lg[tokens[pos + 1]] - m - np.log(np.exp(lg - m).sum()))
        seq_s = (time.perf_counter() - t0) / check
        err = float(np.max(np.abs(lp_p[:check] - np.array(lp_d))))
        # the split-operand precision form (yalm_set_prefill_precision SPLIT: every activation
        # operand as [hi | lo], what the CLI's -m perplexity runs), timed the same way
        dec.set_prefill_precision(runtime.PREFILL_SPLIT)
        ms_split = dec.prefill_time(n, max(1, iters - 1))
        lp_s = dec.prefill(tokens)
        err_split = float(np.max(np.abs(lp_s[:check] - np.array(lp_d))))
    finally:
        if dec2 is not None:
            dec2.close()
        dec.close()
        dm.close()
    return {
        "metric": f"prefill ms {model} fp16 {n}-position perplexity pass",
        "value": round(ms, 3),
        "unit": "ms",
        "higher_is_better": False,
        "iters": iters,
        "tok_per_s": round(n / (ms * 1e-3), 1),
        "flops": flops,
        "roofline": {"bound": "mfma", "achieved": round(tflops, 1), "peak": MFMA_F16_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(tflops / MFMA_F16_PEAK_TFLOPS, 4)},
        "sequential_decode_ms_per_position": round(seq_s * 1e3, 3),
        "speedup_vs_sequential": round(seq_s * n / (ms * 1e-3), 1),
        "spot_check": {"positions": check, "max_abs_dlogp_vs_decode": err},
        "split_form": {"value": round(ms_split, 3), "unit": "ms",
                       "what": "yalm_set_prefill_precision SPLIT (every f16 activation operand as [hi | lo]; "
                               "-m perplexity's form), 2x the matrix work, same algorithmic flops counted",
                       "tflops_algorithmic": round(flops / (ms_split * 1e-3) / 1e12, 1),
                       "max_abs_dlogp_vs_decode": err_split},
        "data": "synthetic weights of the real Llama-3.2-3B shape, synthetic token ids",
    }


def long_context_leg(runtime, M, cfg, dm, steps=64, fill=4080, warmup=4, kernel_iters=64):
    """Decode at the full 4096-slot window and into the StreamingLLM regime
    (infer.cpp:483-485: kv_sink 2, ring slots, kv_len = max_seq_len; the README's
    ~4800-token row, README.md:9-14). The cache is hydrated by one batched prefill
    of `fill` synthetic positions (yalm_prefill, the CLI's prompt path), then
    `steps` greedy tokens are timed from pos fill + 1 + warmup across
    pos max_seq_len. Also times, at the final state (kv_len = max_seq_len), the
    fused attention + Wo launch, the standalone split-KV attention and the plain
    Wo GEMV (HIP events on the decoder stream, layers rotated)."""
    import numpy as np

    dec = runtime.Decoder(dm)
    try:
        rng = np.random.default_rng(1)
        toks = rng.integers(3, cfg.vocab_size, size=fill).astype(np.int32)
        dec.prefill(toks, 0, logprobs=False)
        dec.generate_greedy(int(toks[-1]) % cfg.vocab_size, fill, 1)
        if warmup:
            dec.enqueue_greedy(warmup)
        _, pos0 = dec.device_step()
        t0 = time.perf_counter()
        dec.enqueue_greedy(steps)
        _, pos1 = dec.device_step()
        el = time.perf_counter() - t0
        kv = [M.kv_indices(cfg.max_seq_len, p)[2] for p in range(pos0, pos1)]
        kv_avg = float(np.mean(kv))
        bpt = cfg.weight_bytes_per_token() + cfg.kv_bytes_per_token(int(round(kv_avg)))
        value = steps / el
        kern = {}
        for kid, key in ((8, "attn_wo_us"), (1, "attention_us"), (2, "wo_gemv_us")):
            if kid == 8 and not dec.attn_wo:
                continue
            kern[key] = round(dec.time_kernel(kid, kernel_iters) * 1e3, 3)
        kvb = cfg.kv_bytes_per_token(cfg.max_seq_len) // cfg.n_layers  # K + V bytes one layer's attention reads
        wob = cfg.dim * cfg.q_dim * M.DTYPE_BYTES[cfg.weight_dtype]
        if "attention_us" in kern:
            kern["attention_kv_bytes"] = kvb
            kern["attention_gbs"] = round(kvb / (kern["attention_us"] * 1e-6) / 1e9, 1)
        if "attn_wo_us" in kern:
            kern["attn_wo_bytes"] = kvb + wob
            kern["attn_wo_gbs"] = round((kvb + wob) / (kern["attn_wo_us"] * 1e-6) / 1e9, 1)
    finally:
        dec.close()
    return {
        "metric": "decode tok/s Mistral-7B fp16 @1 GPU at the full 4096-slot window (sink regime)",
        "value": round(value, 3),
        "unit": "tok/s",
        "steps": steps,
        "ms_per_step": round(el / steps * 1e3, 4),
        "pos": [int(pos0), int(pos1)],
        "kv_len": [int(min(kv)), int(max(kv))],
        "hydrate": f"batched prefill of {fill} synthetic positions, then {warmup + 1} greedy warm-up tokens",
        "step_roofline": {"bytes_per_token": int(bpt), "achieved": round(bpt * value / 1e9, 1),
                          "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(bpt * value / 1e9 / HBM_PEAK_GBS, 4)},
        "kernels_at_kv_max": kern,
    }


def tp_bytes_per_token(cfg, size):
    """Algorithmic HBM bytes ONE rank reads per token under the Megatron split
    (include/yalm_hip.h): 1/size of every sharded matrix and of the classifier,
    the replicated norms and embedding row."""
    from yalm_amd import models as M

    wb = M.DTYPE_BYTES[cfg.weight_dtype]
    per_layer = 2 * cfg.dim * 4
    per_layer += (cfg.q_dim + 2 * cfg.kv_dim) // size * cfg.dim * wb
    per_layer += cfg.dim * cfg.q_dim // size * wb
    per_layer += 3 * cfg.dim * cfg.hidden_dim // size * wb
    return cfg.n_layers * per_layer + cfg.dim * wb + cfg.dim * 4 + cfg.vocab_size // size * cfg.dim * wb


def graph_kernels(dec):
    """Kernel launches per greedy token (the captured graph's kernel nodes); None when the
    decoder launches eagerly (--eager under the profiler)."""
    try:
        return dec.graph_kernels(2)
    except Exception:
        return None


def tp_info(mode, exch_us, kernels, cfg, agree):
    """The line's `tp` object. RCCL: 2 all-reduces per layer + the argmax gather, each
    its own collective launch (exchange_us = one all-reduce of x). IPC (tp_exchange.h): no
    exchange launches -- each exchange is pushed by its producer (Wo / W2 / argmax) and
    summed inside its consumer's x staging (exchange_us = the consumer side alone, timed as
    a launch of its own: an upper bound of what the folded form adds)."""
    n_ex = 2 * cfg.n_layers + 1
    out = {"exchange_us": round(exch_us, 3), "exchanges_per_token": n_ex, "kernels_per_token": kernels,
           "ranks_agree": agree}
    if mode == "tp-ipc":
        out["exchange_form"] = "folded into the producer and consumer kernels (no exchange launches)"
    else:
        out["exchange_ms_per_token"] = round(exch_us * n_ex / 1e3, 4)
    return out


def transport_candidates(world, tp, transport, replicas):
    """Decoder modes bench.py tries in order: the requested one, then (N > 1) the other
    tensor-parallel transport after RCCL, then independent replicas (N = 1: one GPU).
    A mode that cannot come up, or whose timed decode raises, on any rank moves every
    rank to the next."""
    if world == 1:
        first = f"tp-{transport}" if tp else "single"
        return [first] + (["single"] if first != "single" else [])
    first = "replica" if replicas else f"tp-{transport}"
    return [first] + (["tp-ipc"] if first == "tp-rccl" else []) + (["replica"] if first != "replica" else [])


def make_decoder(runtime, M, cfg, rank, world, mode, dist, launch=0, cu_part=None):
    """(DeviceModel, Decoder) for mode "single" | "replica" | "tp-rccl" | "tp-ipc"; cu_part:
    the decoder stream's CU block (the one-GPU rehearsal)."""
    if mode in ("single", "replica"):
        dm = runtime.DeviceModel.synthetic(cfg, seed=1)
        return dm, runtime.Decoder(dm, launch=launch, cu_part=cu_part)
    dm = runtime.DeviceModel.synthetic(cfg, seed=1, tp=(rank, world))
    if mode == "tp-ipc":
        def gather(h):
            out = [None] * world
            dist.all_gather_object(out, h)
            return out

        return dm, runtime.Decoder(dm, tp_gather=gather if world > 1 else (lambda h: [h]), launch=launch,
                                   cu_part=cu_part)
    uid = [runtime.tp_unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0)
    return dm, runtime.Decoder(dm, tp_id=uid[0], launch=launch, cu_part=cu_part)


def fp8_leg(args):
    """Config 3 beside config 2: the same decode with fp8 (E5M2) weights, as a child run of
    this script whose JSON line is parsed. Started BEFORE this process makes any GPU call (a
    child of a process holding the GPU is not started here)."""
    try:
        cmd = [sys.executable, os.path.abspath(__file__), "--dtype", "fp8", "--steps", str(args.steps),
               "--warmup", str(args.warmup), "--no-cpu-baseline", "--no-prefill", "--no-gpu-state",
               "--kernel-iters", str(args.kernel_iters)] + (["--no-envelope"] if args.no_envelope else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            raise RuntimeError(f"rc {r.returncode}: {(r.stderr or r.stdout)[-300:]}")
        d8 = json.loads(lines[-1])
        return {k: d8[k] for k in ("metric", "value", "unit", "ms_per_step", "dtype", "config", "step_roofline",
                                   "roofline") if k in d8}
    except Exception as e:  # report, never hide
        return {"error": repr(e)[:300]}


def main():
    args = parse()
    if args.long_only:
        args.no_fp8 = args.no_gpu_state = True
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        if any(k.startswith("ROCPROF") for k in os.environ):
            # under rocprofv3 the profiler's preload has initialised the GPU in this process:
            # starting rank processes from here would fork+exec a GPU-initialised process
            sys.exit("bench.py --gpus N under a profiler: start the ranks with a launcher outside it "
                     "(python -m torch.distributed.run ... bench.py) and put rocprofv3 on each rank's program")
        sys.exit(spawn_ranks(args.gpus))
    # stdout carries exactly one JSON line: whatever the libraries print there (RCCL's version
    # banner at communicator creation, HIP runtime notes) goes to stderr instead
    sys.stdout.flush()
    real_stdout = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist_mod

        # host-side control only (unique id, barriers, max-over-ranks time): gloo;
        # the data path is the decoder's own RCCL communicator / IPC exchange. A 300-s
        # timeout (default 30 min): if a transport fails on some ranks only, the others'
        # barriers raise (caught like the failure itself) instead of stalling the run
        import datetime

        dist_mod.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
        dist = dist_mod

    profiled = any(k.startswith("ROCPROF") for k in os.environ)
    fp8_leg_out = None
    if world == 1 and args.dtype == "fp16" and not args.no_fp8 and not profiled:
        fp8_leg_out = fp8_leg(args)  # before any GPU call of this process
    state = gpu_state() if local_rank == 0 and not (args.no_gpu_state or profiled) else None
    from yalm_amd import models as M
    from yalm_amd import runtime

    ndev = 1 if args.rehearse else (int(os.environ.get("YALM_BENCH_NDEV", "0")) or None)
    dev = local_rank if ndev is None else local_rank % ndev
    cu_part = (local_rank, world) if args.rehearse and world > 1 else None
    launch = runtime.LAUNCH_EAGER if args.eager else 0
    runtime.check(runtime.lib.yalm_set_device(dev))
    base = M.PRESETS[args.model]
    cfg = base.with_(weight_dtype=M.F16 if args.dtype == "fp16" else M.F8E5M2)

    candidates = transport_candidates(world, args.tp, "ipc" if args.rehearse else args.tp_transport, args.replicas)

    def all_ok(ok):
        """Every rank's verdict; a failed agreement (a peer that died or timed out inside
        another collective: ADVICE r5) counts as not ok, so the fallback chain goes on."""
        if dist is None:
            return ok
        oks = [None] * world
        try:
            dist.all_gather_object(oks, ok)
        except Exception:
            return False
        return all(bool(o) for o in oks)

    def timed_decode(dec, tp):
        """Hydrate the prompt, warm up, then time exactly args.steps greedy tokens
        between barrier + sync points; (max-over-ranks seconds, pos0, pos1, ranks agree)."""
        prompt = [(7 * i + 1) % cfg.vocab_size for i in range(PROMPT_LEN)]
        for pos, t in enumerate(prompt[:-1]):
            dec.forward(t, pos, runtime.HYDRATE_KV_CACHE)
        # first generated token; the device loop continues from there
        dec.generate_greedy(prompt[-1], PROMPT_LEN - 1, 1)
        if args.warmup:
            dec.enqueue_greedy(args.warmup)
        runtime.check(runtime.lib.yalm_stream_sync(None))
        _, pos0 = dec.device_step()

        def barrier_sync():
            runtime.check(runtime.lib.yalm_stream_sync(None))
            dec.device_step()  # syncs the decoder stream
            if dist is not None:
                dist.barrier()

        barrier_sync()
        t0 = time.perf_counter()
        dec.enqueue_greedy(args.steps)
        dec.device_step()
        t1 = time.perf_counter()
        barrier_sync()
        elapsed = t1 - t0
        tok1, pos1 = dec.device_step()
        assert pos1 - pos0 == args.steps, (pos0, pos1)
        agree = None
        if dist is not None:
            # every rank's whole greedy sequence since generate_greedy (first token, warm-up,
            # timed steps), hashed: ranks that diverge and meet again still disagree
            import hashlib

            seq = dec.device_tokens()
            h = hashlib.sha256(str(seq).encode()).hexdigest()
            allv = [None] * world
            dist.all_gather_object(allv, (elapsed, h, len(seq)))
            elapsed = max(v[0] for v in allv)
            if tp:  # every rank must have produced the same token sequence
                agree = len({(v[1], v[2]) for v in allv}) == 1
        return elapsed, pos0, pos1, agree

    fallback = None
    result = None
    for mode in candidates:
        dm = dec = None
        err = None
        try:
            dm, dec = make_decoder(runtime, M, cfg, rank, world, mode, dist, launch, cu_part)
        except Exception as e:
            err = f"{mode} failed on rank {rank}: {str(e)[:200]}"
        ok = all_ok(err is None)
        if ok and not args.long_only:
            try:
                result = timed_decode(dec, mode.startswith("tp-"))
            except Exception as e:
                err = f"{mode} decode failed on rank {rank}: {str(e)[:200]}"
            ok = all_ok(err is None)
        if ok:
            break
        fallback = (fallback + "; " if fallback else "") + (err or f"{mode} failed on another rank")
        for h in (dec, dm):
            if h is not None:
                try:
                    h.close()
                except Exception:
                    pass
        if mode == candidates[-1]:
            raise RuntimeError(fallback)
    tp = mode.startswith("tp-")
    tp_size = world if tp else 1
    if args.long_only:
        print(json.dumps(long_context_leg(runtime, M, cfg, dm, steps=args.long_steps,
                                          kernel_iters=args.kernel_iters)), file=real_stdout, flush=True)
        dec.close()
        dm.close()
        return

    elapsed, pos0, pos1, agree = result

    # ---- roofline of the dominant kernel: the W1/W3 GEMV + SiLU-GLU (52.9% of the bytes)
    wb = M.DTYPE_BYTES[cfg.weight_dtype]
    hid_local = cfg.hidden_dim // tp_size
    KID = 3
    kern_bytes = 2 * hid_local * cfg.dim * wb + 2 * cfg.dim * 4 + hid_local * 4
    wt = "WF16" if args.dtype == "fp16" else "WF8"
    avg_ms = dec.time_kernel(KID, args.kernel_iters)
    achieved = kern_bytes / (avg_ms * 1e-3) / 1e9
    kname = dec.kernel_name(KID)
    traffic, traffic_src = pmc_traffic((f"gemv_rb_kernel<{wt}", "PGlu"))
    exch_us = None
    kernels_per_token = graph_kernels(dec)
    if tp and tp_size > 1:
        exch_us = dec.time_kernel(6, args.kernel_iters) * 1e3
    env_ms = None
    if not args.no_envelope:
        if dist is not None:
            dist.barrier()
        env_ms = runtime.stream_envelope(kern_bytes, 16)

    toks = args.steps * (1 if tp else world)
    value = toks / elapsed
    kv_avg = (pos0 + pos1) / 2 + 1
    n_seq = 1 if tp else world
    if tp:
        rank_bytes = tp_bytes_per_token(cfg, tp_size) + cfg.kv_bytes_per_token(int(kv_avg)) // tp_size
    else:
        rank_bytes = cfg.weight_bytes_per_token() + cfg.kv_bytes_per_token(int(kv_avg))
    per_gpu_gbs = rank_bytes * (args.steps / elapsed) / 1e9
    bytes_per_tok = cfg.weight_bytes_per_token() + cfg.kv_bytes_per_token(int(kv_avg))

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
        "scaling": "strong" if tp else "weak",
        "vs_baseline": None,
        "dtype": "f16" if args.dtype == "fp16" else "f8e5m2",
        "data": "synthetic (random weights of the real Mistral-7B-v0.2 shape generated in HBM; "
                f"{PROMPT_LEN}-token synthetic prompt; greedy argmax on device)",
        "config": {
            "workload": f"{args.model} {args.dtype} batch-1 greedy decode, {args.steps} tokens"
                        f"{f' (one sequence, tensor parallel over {world} GPUs)' if tp and world > 1 else ''}"
                        f"{'/GPU' if not tp and world > 1 else ''}, kv_len {pos0 + 1}..{pos1}",
            "model": args.model,
            "global_batch": n_seq,
            "seq_len": int(pos1),
            "parallelism": (f"tp{tp_size}-{mode[3:]}" if tp else (f"replicas{world}" if world > 1 else "single")),
        },
        "step_roofline": {
            "bytes_per_token": int(bytes_per_tok),
            "bytes_per_token_per_gpu": int(rank_bytes),
            "achieved_per_gpu": round(per_gpu_gbs, 1),
            "peak_per_gpu": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(per_gpu_gbs / HBM_PEAK_GBS, 4),
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
            "envelope_us": round(env_ms * 1e3, 3) if env_ms else None,
            "envelope_gbs": round(kern_bytes / (env_ms * 1e-3) / 1e9, 1) if env_ms else None,
            "frac_of_envelope": round(env_ms / avg_ms, 4) if env_ms else None,
        },
        "gpu_state": state,
        "cpu_baseline": None,
    }
    out["kernels_per_token"] = kernels_per_token
    if tp and tp_size > 1:
        out["tp"] = tp_info(mode, exch_us, kernels_per_token, cfg, agree)
    if cu_part is not None:
        out["n_gpus"] = 1
        out["config"]["parallelism"] += "-rehearsal"
        out["rehearsal"] = (f"{world} rank processes on ONE MI355X, each decoder stream on a disjoint block of "
                            f"{256 // world} CUs (yalm_stream_create_cu_part): config 5's production launch sequence "
                            "(no shared-GPU gates), NOT a scaling number -- the ranks share one GPU's HBM")
    if fallback:
        out["fallback"] = fallback
    dec.close()
    if mode == "single" and args.dtype == "fp16" and not args.no_long:
        try:  # decode at long context (kv_len 4096, sink regime) on the same weights
            out["long_context"] = long_context_leg(runtime, M, cfg, dm, steps=args.long_steps,
                                                   kernel_iters=args.kernel_iters)
        except Exception as e:  # report, never hide
            out["long_context"] = {"error": repr(e)[:300]}
    dm.close()
    if mode == "tp-rccl" and world > 1 and not args.no_alt:
        # the same workload through the IPC one-shot exchange (include/yalm_hip.h), for
        # the all-reduce cost of RCCL's collective vs direct peer-mapped stores
        try:
            # every rank learns whether the IPC decoder came up everywhere before any rank
            # enters the timed decode (a rank that failed alone would otherwise meet the
            # others' barriers out of step)
            ok2, err2 = 1, None
            try:
                dm, dec = make_decoder(runtime, M, cfg, rank, world, "tp-ipc", dist, launch, cu_part)
            except Exception as e:
                ok2, err2 = 0, e
            oks2 = [None] * world
            dist.all_gather_object(oks2, ok2)
            if not all(oks2):
                if ok2:
                    dec.close()
                    dm.close()
                raise err2 or RuntimeError("the IPC decoder failed on another rank")
            e2, _, _, agree2 = timed_decode(dec, True)
            k2 = graph_kernels(dec)
            ex2 = dec.time_kernel(6, args.kernel_iters) * 1e3
            out["tp_ipc"] = {"value": round(args.steps / e2, 3), "ms_per_step": round(e2 / args.steps * 1e3, 4),
                             "exchange_us": round(ex2, 3), "kernels_per_token": k2, "ranks_agree": agree2}
            dec.close()
            dm.close()
            if agree2 and e2 < elapsed:
                # the line's value is the faster measured transport (both measured in this run,
                # same workload, same barriers and max-over-ranks clock); the other stays beside it
                out["tp_rccl"] = {"value": out["value"], "ms_per_step": out["ms_per_step"],
                                  "exchange_us": out["tp"]["exchange_us"],
                                  "kernels_per_token": out["kernels_per_token"], "ranks_agree": out["tp"]["ranks_agree"]}
                del out["tp_ipc"]
                out["value"] = round(args.steps / e2, 3)
                out["ms_per_step"] = round(e2 / args.steps * 1e3, 4)
                gbs = rank_bytes * (args.steps / e2) / 1e9
                out["step_roofline"]["achieved_per_gpu"] = round(gbs, 1)
                out["step_roofline"]["frac"] = round(gbs / HBM_PEAK_GBS, 4)
                out["config"]["parallelism"] = f"tp{tp_size}-ipc"
                out["kernels_per_token"] = k2
                out["tp"] = tp_info("tp-ipc", ex2, k2, cfg, agree2)
                out["tp"]["transport"] = "ipc (faster of the two measured)"
        except Exception as e:  # report, never hide
            out["tp_ipc"] = {"error": str(e)[:200]}
    if fp8_leg_out is not None:
        out["fp8"] = fp8_leg_out
    if world == 1 and args.dtype == "fp16" and not args.no_prefill:
        try:  # config 4 beside config 2 (the decoder above is closed: its HBM is free again)
            out["prefill"] = prefill_leg(runtime, M, iters=args.prefill_iters)
        except Exception as e:  # report, never hide
            out["prefill"] = {"error": repr(e)[:300]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"error": repr(e)}
        if isinstance(out.get("prefill"), dict) and "error" not in out["prefill"]:
            try:  # config 4's CPU baseline: the reference's sequential perplexity loop
                pc = prefill_cpu_baseline(budget_s=args.cpu_seconds)
                pc["speedup_gpu_vs_cpu"] = round(pc["value"] / out["prefill"]["value"], 1)
                out["prefill"]["cpu_baseline"] = pc
            except Exception as e:  # report, never hide
                out["prefill"]["cpu_baseline"] = {"error": repr(e)[:300]}
    if rank == 0:
        print(json.dumps(out), file=real_stdout, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if agree is False:
        sys.exit(3)


if __name__ == "__main__":
    main()
