"""Cases pinned on the REFERENCE's own CPU kernels (oracle/_ref/ref_infer =
/root/reference/src/infer.cpp compiled unmodified, see oracle/Makefile
`ref-infer`). Shared by the generator (make_ref_infer_golden.py, run where
/root/reference exists) and the tests (tests/test_ref_infer.py on CPU,
tests/test_gpu_ref_infer.py on the GPU box): every input is regenerated here
from a seed with numpy PCG64, so only outputs are committed
(tests/golden/ref_infer.npz).

Reference entry points (model.h:353-385):
  matmul_cpu f32 (infer.cpp:405-407 -> 48-59), matmul_cpu f16 (408-410 -> 63-98),
  mha_cpu (387-403 -> attn 216-248), ffn_cpu f32 (412-438).
"""
from __future__ import annotations

import os

import numpy as np

GOLDEN = os.path.dirname(os.path.abspath(__file__))

# Mistral-7B GEMV shapes (SURVEY §8d kernel microbench: test.cpp:307-359 shapes)
MISTRAL_GEMV = [("qkv", 4096, 6144), ("wo", 4096, 4096), ("w1", 4096, 14336), ("w2", 14336, 4096),
                ("wcls", 4096, 32000)]


def _cases():
    c = []
    # the reference's own kernel-test inputs (test.cpp:148-206, libstdc++ seeds)
    c.append(dict(name="tcpp_matmul_f32", op="matmul_f32", n=256, d=16, src="tcpp"))
    c.append(dict(name="tcpp_mha", op="mha", head_dim=16, kv_len=4, max_seq_len=4, n_heads=16, n_kv_heads=8,
                  src="tcpp"))
    c.append(dict(name="tcpp_ffn_gelu", op="ffn", hidden=256, dim=256, act=0, src="tcpp"))
    c.append(dict(name="tcpp_ffn_silu", op="ffn", hidden=256, dim=256, act=1, src="tcpp"))
    # Mistral-7B shapes, seeded normal data (weights N(0,1)*0.02, x N(0,1))
    for i, (tag, n, d) in enumerate(MISTRAL_GEMV):
        c.append(dict(name=f"mistral_{tag}_f16", op="matmul_f16", n=n, d=d, seed=100 + i))
    for i, (tag, n, d) in enumerate([("wo", 4096, 4096), ("w2", 14336, 4096)]):
        c.append(dict(name=f"mistral_{tag}_f32", op="matmul_f32", n=n, d=d, seed=200 + i))
    for i, kv in enumerate([1, 17, 256, 4096]):
        c.append(dict(name=f"mistral_mha_kv{kv}", op="mha", head_dim=128, kv_len=kv, max_seq_len=4096, n_heads=32,
                      n_kv_heads=8, seed=300 + i))
    c.append(dict(name="ffn_gelu_1024", op="ffn", hidden=3584, dim=1024, act=0, seed=400))
    c.append(dict(name="ffn_silu_1024", op="ffn", hidden=3584, dim=1024, act=1, seed=401))
    c.append(dict(name="mistral_ffn_silu_f32", op="ffn", hidden=14336, dim=4096, act=1, seed=402))
    return c


CASES = _cases()
CASE = {c["name"]: c for c in CASES}


def _tcpp():
    return dict(np.load(os.path.join(GOLDEN, "test_cpp_inputs.npz")))


def _normal(rng, shape, scale=1.0):
    a = rng.standard_normal(shape, dtype=np.float32)
    if scale != 1.0:
        a *= np.float32(scale)
    return a


def inputs(case: dict) -> dict:
    """The case's inputs as numpy arrays (weights (d, n) row-major as the .yalm
    layout, K/V (max_seq_len, n_kv_heads*head_dim) f16)."""
    op = case["op"]
    if case.get("src") == "tcpp":
        t = _tcpp()
        if op == "matmul_f32":
            return dict(x=t["matmul_x"].astype(np.float32), w=t["matmul_w"].reshape(16, 256).astype(np.float32))
        if op == "mha":
            return dict(q=t["mha_q"].astype(np.float32), kb=t["mha_kb"].astype(np.float16),
                        vb=t["mha_vb"].astype(np.float16))
        return dict(x=t["ffn_x"].astype(np.float32),
                    **{k: t["ffn_" + k].reshape(256, 256).astype(np.float32) for k in ("w1", "w2", "w3")})
    rng = np.random.default_rng(case["seed"])
    if op in ("matmul_f32", "matmul_f16"):
        n, d = case["n"], case["d"]
        x = _normal(rng, n)
        w = _normal(rng, (d, n), 0.02)
        return dict(x=x, w=w.astype(np.float16) if op == "matmul_f16" else w)
    if op == "mha":
        hd, nh, nkv, T = case["head_dim"], case["n_heads"], case["n_kv_heads"], case["max_seq_len"]
        q = _normal(rng, nh * hd)
        kb = _normal(rng, (T, nkv * hd)).astype(np.float16)
        vb = _normal(rng, (T, nkv * hd)).astype(np.float16)
        return dict(q=q, kb=kb, vb=vb)
    hidden, dim = case["hidden"], case["dim"]
    x = _normal(rng, dim)
    w1 = _normal(rng, (hidden, dim), 1.0 / np.sqrt(dim))
    w3 = _normal(rng, (hidden, dim), 1.0 / np.sqrt(dim))
    w2 = _normal(rng, (dim, hidden), 1.0 / np.sqrt(hidden))
    return dict(x=x, w1=w1, w2=w2, w3=w3)


def load_golden() -> dict:
    return dict(np.load(os.path.join(GOLDEN, "ref_infer.npz")))
