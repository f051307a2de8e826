"""CPU tests: the C oracle (oracle/yalm_oracle.c) is BIT-EXACT against the
reference's own CPU kernels — matmul_cpu f32/f16, mha_cpu and ffn_cpu from
/root/reference/src/infer.cpp compiled unmodified (oracle/_ref/ref_infer) —
on the committed outputs in tests/golden/ref_infer.npz
(tests/golden/make_ref_infer_golden.py). Both sides are compiled by gcc with
the reference's flags (Makefile:36-39), so equal bytes are the bar.

Where oracle/_ref/ref_infer exists (this container), the reference binary is
also re-run live and must reproduce the committed file."""
import hashlib
import os
import sys

import numpy as np
import pytest

import oracle_py as O
from yalm_amd import models as M

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import ref_infer_cases as C  # noqa: E402

G = C.load_golden()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def oracle_outputs(case):
    inp = C.inputs(case)
    op = case["op"]
    if op.startswith("matmul"):
        return {"out": O.matmul(inp["x"], inp["w"], M.F32 if op == "matmul_f32" else M.F16)}
    if op == "mha":
        xout, att = O.mha(inp["kb"], inp["vb"], inp["q"], case["head_dim"], case["kv_len"], case["max_seq_len"],
                          case["n_heads"], case["n_kv_heads"])
        return {"xout": xout, "att": att.reshape(case["n_heads"], case["max_seq_len"])}
    return {"out": O.ffn(inp["x"], inp["w1"], inp["w2"], inp["w3"], case["act"], M.F32)}


@pytest.mark.parametrize("name", [c["name"] for c in C.CASES])
def test_oracle_bit_exact_vs_reference_kernels(name):
    case = C.CASE[name]
    for k, a in oracle_outputs(case).items():
        key = f"{name}/{k}"
        if key in G:
            ref = G[key]
            mine = a[:, :ref.shape[1]] if k == "att" else a
            bad = np.flatnonzero(mine.view(np.uint32).ravel() != ref.view(np.uint32).ravel())
            assert bad.size == 0, f"{key}: {bad.size} values differ, first at {bad[0]}: {mine.ravel()[bad[0]]!r} " \
                                  f"vs reference {ref.ravel()[bad[0]]!r}"
        assert sha(a) == str(G[key + "#sha256"]), f"{key}: bytes differ from the reference kernel"


REF_BIN = os.path.join(C.GOLDEN, "..", "..", "oracle", "_ref", "ref_infer")


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref/ref_infer not built (needs /root/reference)")
@pytest.mark.parametrize("name", ["tcpp_matmul_f32", "tcpp_mha", "tcpp_ffn_silu", "mistral_wo_f16",
                                  "mistral_mha_kv256"])
def test_reference_binary_reproduces_golden(name):
    import make_ref_infer_golden as MK

    for k, a in MK.run_case(C.CASE[name], REF_BIN).items():
        assert sha(a) == str(G[f"{name}/{k}#sha256"])
