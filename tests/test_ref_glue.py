"""CPU tests: the C oracle's per-block glue is BIT-EXACT against the reference's own
static functions (rmsnorm infer.cpp:134-144, rope 200-213, softmax 170-185, clip
195-197, float_to_half / half_to_float 11-16), reached by a harness TU that #includes
the unmodified /root/reference/src/infer.cpp (oracle/_ref/ref_glue), on the committed
outputs in tests/golden/ref_glue.npz (make_ref_glue_golden.py). Composites follow
_block_cpu's order: the K cache row (rmsnorm -> clip -> rope -> float_to_half) and the
sink rotation (half_to_float -> rope(pos 1) -> float_to_half). Both sides are compiled
by gcc with the reference's flags, so equal bytes are the bar.

float_to_half is _cvtss_sh(x, 0) (round to nearest even): numpy's float16 cast is the
same function, which the oracle's f16 helpers and tests/oracle_py.py rely on.

Where oracle/_ref/ref_glue exists (this container), the reference binary is re-run live
and must reproduce the committed file."""
import hashlib
import os
import sys

import numpy as np
import pytest

import oracle_py as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import ref_glue_cases as C  # noqa: E402

G = C.load_golden()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rmsnorm(x, w, eps):
    o = np.zeros_like(x)
    O.olib.orc_rmsnorm(O.P(o), O.P(x), O.P(w), x.size, eps)
    return o


def rope(v, head_dim, pos, theta, rotary_dim):
    v = np.array(v, np.float32)
    O.olib.orc_rope(O.P(v), v.size, head_dim, pos, theta, rotary_dim)
    return v


def clip(x, v):  # infer.cpp:195-197 (comparisons only: exact)
    return np.where(x < -v, np.float32(-v), np.where(x > v, np.float32(v), x)).astype(np.float32)


def f2h(x):
    return np.asarray(x, np.float32).astype(np.float16).view(np.uint16)


def oracle_outputs(case):
    inp = C.inputs(case)
    op = case["op"]
    if op == "rmsnorm":
        return {"out": rmsnorm(inp["x"], inp["w"], case["eps"])}
    if op == "rope":
        return {"out": rope(inp["vec"], case["head_dim"], case["pos"], case["theta"], case["rotary_dim"])}
    if op == "softmax":
        o = np.zeros_like(inp["x"])
        O.olib.orc_softmax(O.P(o), O.P(inp["x"]), inp["x"].size)
        return {"out": o}
    if op == "clip":
        return {"out": clip(inp["x"], case["v"])}
    if op in ("f2h", "f2h_random"):
        return {"out": f2h(inp["x"])}
    if op == "h2f":
        return {"out": inp["x"].view(np.float16).astype(np.float32)}
    if op == "kvrow":
        xn = rmsnorm(inp["x"], inp["w"], case["eps"])
        k = rope(clip(xn, case["clip"]), case["head_dim"], case["pos"], case["theta"], case["rotary_dim"])
        return {"xn": xn, "k": k, "row": f2h(k)}
    if op == "sinkrot":
        k = rope(inp["row"].view(np.float16).astype(np.float32), case["head_dim"], 1, case["theta"],
                 case["rotary_dim"])
        return {"row": f2h(k)}
    raise ValueError(op)


@pytest.mark.parametrize("name", [c["name"] for c in C.CASES])
def test_oracle_glue_bit_exact_vs_reference(name):
    for k, a in oracle_outputs(C.CASE[name]).items():
        key = f"{name}/{k}"
        ref = G[key]
        bits = (lambda v: v.view(np.uint16 if v.dtype.itemsize == 2 else np.uint32).ravel())
        same = bits(np.ascontiguousarray(a)) == bits(ref)
        if a.dtype == np.float32:  # NaN payloads (h2f of the 1022 f16 NaNs): F16C quiets, numpy keeps
            same |= np.isnan(a.ravel()) & np.isnan(ref.ravel())
        bad = np.flatnonzero(~same)
        assert bad.size == 0, f"{key}: {bad.size} values differ, first at {bad[0]}: {a.ravel()[bad[0]]!r} " \
                              f"vs reference {ref.ravel()[bad[0]]!r}"
        if not np.isnan(a).any():
            assert sha(a) == str(G[key + "#sha256"])


def test_golden_covers_the_glue():
    ops = {c["op"] for c in C.CASES}
    assert {"rmsnorm", "rope", "softmax", "clip", "f2h", "h2f", "kvrow", "sinkrot"} <= ops
    pos = {c["pos"] for c in C.CASES if c["op"] == "rope"}
    assert {0, 1, 4095, 4096, 32767} <= pos
    assert any(c["op"] == "rope" and c["rotary_dim"] < c["head_dim"] for c in C.CASES)


REF_BIN = os.path.join(C.GOLDEN, "..", "..", "oracle", "_ref", "ref_glue")


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref/ref_glue not built (needs /root/reference)")
@pytest.mark.parametrize("name", ["rmsnorm_mistral", "rope_mistral_q_p32767", "rope_partial64_p4096",
                                  "softmax_4096_s60", "f2h_special", "kvrow_clip_k_p4095", "sinkrot_partial64"])
def test_reference_binary_reproduces_golden(name):
    import make_ref_glue_golden as MK

    for k, a in MK.run_case(C.CASE[name], REF_BIN).items():
        assert sha(a) == str(G[f"{name}/{k}#sha256"])
