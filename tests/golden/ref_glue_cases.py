"""Seeded inputs of the per-block glue cases pinned on the REFERENCE's own static
functions (oracle/ref_glue_harness.cpp: rmsnorm infer.cpp:134-144, rope 200-213,
softmax 170-185, clip 195-197, float_to_half / half_to_float 11-16). Inputs are
regenerated from the seeds here; tests/golden/ref_glue.npz holds the reference's
outputs (make_ref_glue_golden.py).

Composite cases follow _block_cpu's statement order (infer.cpp:265-317):
  kvrow:   rmsnorm(x, w) -> clip(qkv_clip) -> rope(pos) -> float_to_half, the K cache
           row of a block whose Wk is the identity (the f16 identity GEMV is exact, so
           the reference's matmul is the identity on these values);
  sinkrot: half_to_float(row) -> rope(pos 1) -> float_to_half, the sink rotation.
"""
import os

import numpy as np

GOLDEN = os.path.dirname(os.path.abspath(__file__))
FLT_MAX = float(np.finfo(np.float32).max)

POS = [0, 1, 17, 4095, 4096, 32767]

# (name, d, head_dim, theta, rotary_dim)
ROPE_GEOM = [
    ("mistral_q", 4096, 128, 1e6, 128),
    ("mistral_k", 1024, 128, 1e6, 128),
    ("llama3b_q", 3072, 128, 5e5, 128),
    ("partial64", 1024, 128, 1e4, 64),
    ("hd64", 512, 64, 1e4, 64),
]

CASES = []
for name, size, eps, scale in [("mistral", 4096, 1e-5, 3.0), ("llama3b", 3072, 1e-5, 1.0), ("tiny", 16, 1e-6, 1.0),
                               ("large_x", 4096, 1e-5, 1e3), ("small_x", 4096, 1e-5, 1e-3)]:
    CASES.append(dict(name=f"rmsnorm_{name}", op="rmsnorm", size=size, eps=eps, scale=scale))
for gname, d, hd, theta, rd in ROPE_GEOM:
    for pos in POS:
        CASES.append(dict(name=f"rope_{gname}_p{pos}", op="rope", d=d, head_dim=hd, theta=theta, rotary_dim=rd,
                          pos=pos))
for size, scale in [(1, 1.0), (17, 4.0), (4096, 8.0), (4096, 60.0)]:
    CASES.append(dict(name=f"softmax_{size}_s{int(scale)}", op="softmax", size=size, scale=scale))
CASES.append(dict(name="clip_half", op="clip", n=256, v=0.5))
CASES.append(dict(name="clip_max", op="clip", n=256, v=FLT_MAX))
CASES.append(dict(name="f2h_special", op="f2h"))
CASES.append(dict(name="f2h_random", op="f2h_random", n=4096))
CASES.append(dict(name="h2f_all", op="h2f"))
# composites at the Mistral kv geometry (kv_dim 1024) and a partial rotary geometry
for gname, d, hd, theta, rd, clip in [("mistral_k", 1024, 128, 1e6, 128, FLT_MAX), ("clip_k", 1024, 128, 1e6, 128, 0.5),
                                      ("partial64", 1024, 128, 1e4, 64, FLT_MAX)]:
    for pos in POS:
        CASES.append(dict(name=f"kvrow_{gname}_p{pos}", op="kvrow", d=d, head_dim=hd, theta=theta, rotary_dim=rd,
                          pos=pos, clip=clip, eps=1e-5))
for gname, d, hd, theta, rd in [("mistral_k", 1024, 128, 1e6, 128), ("partial64", 1024, 128, 1e4, 64)]:
    CASES.append(dict(name=f"sinkrot_{gname}", op="sinkrot", d=d, head_dim=hd, theta=theta, rotary_dim=rd))
CASE = {c["name"]: c for c in CASES}


def _seed(name: str) -> int:
    """FNV-1a of the case name (stable across processes, unlike hash())."""
    h = 2166136261
    for ch in name.encode():
        h = ((h ^ ch) * 16777619) & 0xFFFFFFFF
    return h


def f2h_special() -> np.ndarray:
    """float_to_half edge inputs: signed zeros, the f16 subnormal range and its rounding
    boundaries, halfway cases (ties to even), the overflow threshold, infinities."""
    v = [0.0, -0.0, 1.0, -1.0, 2.0 ** -24, 2.0 ** -25, 1.5 * 2.0 ** -25, 2.0 ** -26, 3 * 2.0 ** -25, 2.0 ** -14,
         2.0 ** -14 - 2.0 ** -25, 1 + 2.0 ** -11, 1 + 3 * 2.0 ** -11, 1 + 2.0 ** -11 + 2.0 ** -20, 65504.0,
         65519.0, 65519.996, 65520.0, 70000.0, -65520.0, 1e-8, 3.14159265, -2.718281828, float("inf"),
         float("-inf"), 2049.0, 2051.0, 4097.0, 0.1, 0.2, 0.3, 1.0 / 3.0]
    return np.array(v, np.float32)


def inputs(case: dict) -> dict:
    rng = np.random.default_rng(_seed(case["name"]))
    op = case["op"]
    if op == "rmsnorm":
        n = case["size"]
        return {"x": (rng.standard_normal(n) * case["scale"]).astype(np.float32),
                "w": (1.0 + 0.1 * rng.standard_normal(n)).astype(np.float32)}
    if op == "rope":
        return {"vec": rng.standard_normal(case["d"]).astype(np.float32)}
    if op == "softmax":
        x = (rng.standard_normal(case["size"]) * case["scale"]).astype(np.float32)
        return {"x": x}
    if op == "clip":
        x = (rng.standard_normal(case["n"]) * 2.0).astype(np.float32)
        x[:4] = [np.inf, -np.inf, 0.5, -0.5]
        return {"x": x}
    if op == "f2h":
        return {"x": f2h_special()}
    if op == "f2h_random":
        e = rng.integers(-30, 17, case["n"]).astype(np.float32)
        return {"x": (rng.standard_normal(case["n"]).astype(np.float32) * np.exp2(e)).astype(np.float32)}
    if op == "h2f":
        return {"x": np.arange(65536, dtype=np.uint32).astype(np.uint16)}
    if op == "kvrow":
        d = case["d"]
        return {"x": (rng.standard_normal(d) * 2.0).astype(np.float32),
                "w": (1.0 + 0.1 * rng.standard_normal(d)).astype(np.float32)}
    if op == "sinkrot":
        return {"row": rng.standard_normal(case["d"]).astype(np.float16).view(np.uint16)}
    raise ValueError(op)


def load_golden():
    return np.load(os.path.join(GOLDEN, "ref_glue.npz"), allow_pickle=False)
