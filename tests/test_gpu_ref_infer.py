"""GPU parity against the REFERENCE's own CPU kernels: the HIP test API
(yalm_matmul / yalm_mha / yalm_ffn, include/yalm_hip.h) on the seeded inputs of
tests/golden/ref_infer_cases.py, compared with the outputs that
/root/reference/src/infer.cpp's matmul_cpu / mha_cpu / ffn_cpu produced on the
same inputs (tests/golden/ref_infer.npz, made by
tests/golden/make_ref_infer_golden.py). The bars are the ones the oracle tests
use (tests/test_gpu_kernels.py), written here:
  GEMV        max|gpu - ref| / max|ref| < 2e-5    (fp32 sums in another order)
  mha xout    |gpu - ref| <= 2e-5 + 1e-4 |ref|;   att 2e-6 + 1e-4 |ref|
  ffn         max|gpu - ref| / max|ref| < 1e-4  (test.cpp:191-205 case also 1e-4 abs)
"""
import os
import sys

import numpy as np
import pytest

from yalm_amd import models as M

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import ref_infer_cases as C  # noqa: E402

pytestmark = pytest.mark.gpu

G = C.load_golden()


def rt():
    from yalm_amd import runtime

    return runtime


def relerr(a, b):
    return float(np.max(np.abs(a - b)) / (np.max(np.abs(b)) + 1e-30))


@pytest.mark.parametrize("name", [c["name"] for c in C.CASES])
def test_hip_vs_reference_kernels(name):
    case = C.CASE[name]
    inp = C.inputs(case)
    op = case["op"]
    if op.startswith("matmul"):
        g = rt().matmul(inp["x"], inp["w"], M.F32 if op == "matmul_f32" else M.F16)
        ref = G[f"{name}/out"]
        if case.get("src") == "tcpp":
            np.testing.assert_allclose(g, ref, atol=1e-4)  # test.cpp:17
        assert relerr(g, ref) < 2e-5
    elif op == "mha":
        xg, ag = rt().mha(inp["kb"], inp["vb"], inp["q"], case["head_dim"], case["kv_len"], case["max_seq_len"],
                          case["n_heads"], case["n_kv_heads"])
        np.testing.assert_allclose(xg, G[f"{name}/xout"], atol=2e-5, rtol=1e-4)
        key = f"{name}/att"
        if key in G:
            ag = ag.reshape(case["n_heads"], case["max_seq_len"])[:, :case["kv_len"]]
            np.testing.assert_allclose(ag, G[key], atol=2e-6, rtol=1e-4)
    else:
        g = rt().ffn(inp["x"], inp["w1"], inp["w2"], inp["w3"], case["act"], M.F32)
        ref = G[f"{name}/out"]
        if case.get("src") == "tcpp":
            np.testing.assert_allclose(g, ref, atol=1e-4)  # test.cpp:205
        assert relerr(g, ref) < 1e-4
