"""CPU tests: pin the C oracle against the reference's own known-answer test
and seeded kernel-test inputs, and against an independent float64 forward.
These run without a GPU (pytest -m "not gpu")."""
import os

import numpy as np
import pytest

import oracle_py as O
import ref_numpy as R
from yalm_amd import models as M


def test_attn_known_answer():
    """/root/reference/src/test.cpp:68-126 — exact one-hot attention KAT
    (2 heads, 1 kv head, head_dim 3, 4 tokens; q = 1e4 * one-hot)."""
    q = np.array([0.0, 1e4, 0.0, 0.0, 0.0, 1e4], np.float32)
    kb = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, -1, 0, 0], np.float16)
    vb = kb.copy()
    xout, att = O.mha(kb, vb, q, head_dim=3, kv_len=4, max_seq_len=4, n_heads=2, n_kv_heads=1)
    np.testing.assert_allclose(att[:4], [0, 1, 0, 0], atol=1e-4)  # test.cpp:118
    np.testing.assert_allclose(att[4:], [0, 0, 1, 0], atol=1e-4)  # test.cpp:120
    np.testing.assert_allclose(xout, [0, 1, 0, 0, 0, 1], atol=1e-4)  # test.cpp:121-125


@pytest.fixture(scope="module")
def tcpp(golden_dir):
    return dict(np.load(os.path.join(golden_dir, "test_cpp_inputs.npz")))


def test_reference_kernel_inputs_matmul(tcpp):
    """test.cpp:158-168 inputs (libstdc++ seeds 0,1): oracle f32 matmul vs float64."""
    w = tcpp["matmul_w"].reshape(16, 256)
    x = tcpp["matmul_x"]
    out = O.matmul(x, w, M.F32)
    np.testing.assert_allclose(out, w.astype(np.float64) @ x, atol=1e-4)  # test.cpp:17 criterion


def test_reference_kernel_inputs_mha(tcpp):
    """test.cpp:171-188 inputs: oracle mha vs float64 on the fp16-rounded K/V."""
    hd, nh, nkv, T = 16, 16, 8, 4
    kb = tcpp["mha_kb"].astype(np.float16)
    vb = tcpp["mha_vb"].astype(np.float16)
    q = tcpp["mha_q"]
    xout, att = O.mha(kb, vb, q, hd, T, T, nh, nkv)
    K = kb.astype(np.float64).reshape(T, nkv, hd)
    V = vb.astype(np.float64).reshape(T, nkv, hd)
    for h in range(nh):
        g = h // (nh // nkv)
        s = K[:, g] @ q[h * hd:(h + 1) * hd] / np.sqrt(hd)
        p = np.exp(s - s.max())
        p /= p.sum()
        np.testing.assert_allclose(att[h * T:(h + 1) * T], p, atol=1e-5)
        np.testing.assert_allclose(xout[h * hd:(h + 1) * hd], p @ V[:, g], atol=1e-4)


def test_reference_kernel_inputs_ffn(tcpp):
    """test.cpp:191-205 inputs (GELU, weights scaled 1/sqrt(256))."""
    x = tcpp["ffn_x"]
    w1 = tcpp["ffn_w1"].reshape(256, 256)
    w2 = tcpp["ffn_w2"].reshape(256, 256)
    w3 = tcpp["ffn_w3"].reshape(256, 256)
    out = O.ffn(x, w1, w2, w3, M.GELU, M.F32)
    hb = R.gelu(w1.astype(np.float64) @ x) * (w3.astype(np.float64) @ x)
    np.testing.assert_allclose(out, w2.astype(np.float64) @ hb, atol=1e-4)


def test_f16_gemv_reference_order():
    """infer.cpp:63-98: two 8-wide accumulators over 16-element chunks. A
    scalar restatement of exactly that order must be bit-identical."""
    rng = np.random.default_rng(0)
    n, d = 64, 5
    w = (rng.standard_normal((d, n)) * 0.1).astype(np.float16)
    x = rng.standard_normal(n).astype(np.float32)
    out = O.matmul(x, w, M.F16)
    wf = w.astype(np.float32)
    for i in range(d):
        lo = np.zeros(8, np.float32)
        hi = np.zeros(8, np.float32)
        for j in range(0, n, 16):
            lo = (wf[i, j:j + 8].astype(np.float64) * x[j:j + 8] + lo).astype(np.float32)  # fma: exact product
            hi = (wf[i, j + 8:j + 16].astype(np.float64) * x[j + 8:j + 16] + hi).astype(np.float32)
        s8 = (lo + hi).astype(np.float32)
        s4 = (s8[:4] + s8[4:]).astype(np.float32)
        s = np.float32(np.float32(s4[0] + s4[1]) + np.float32(s4[2] + s4[3]))
        assert out[i] == s, (i, out[i], s)


def test_fp8_matmul_equals_f16_twin():
    """fp8 semantics (defined here, the reference's is broken — SURVEY §0.2):
    E5M2 byte b == f16 bits b<<8, then the f16 GEMV; must equal the f16 path on
    the upcast twin bit-for-bit."""
    rng = np.random.default_rng(1)
    wb = rng.integers(0, 256, size=(7, 128), dtype=np.uint8)
    wb[(wb & 0x7C) == 0x7C] = 0x3C  # no inf/nan
    x = rng.standard_normal(128).astype(np.float32)
    twin = (wb.astype(np.uint16) << 8).view(np.float16)
    np.testing.assert_array_equal(O.matmul(x, wb, M.F8E5M2), O.matmul(x, twin, M.F16))


@pytest.mark.parametrize("dtype", [M.F32, M.F16, M.F8E5M2])
def test_synth_numpy_twin_bitexact(dtype):
    """The deterministic synthetic initialiser: numpy twin == C oracle, bitwise
    (the device kernel uses the same integer hash; checked on the GPU)."""
    n = 10007
    seed = M.synth_seed(3, "x")
    ref = M.synth_array(n, dtype, seed, 0.035, 1.0 if dtype == M.F32 else 0.0)
    if dtype == M.F32:
        a = np.empty(n, np.float32)
        O.olib.orc_synth_f32(O.P(a), n, seed, 0.035, 1.0)
    elif dtype == M.F16:
        a = np.empty(n, np.float16)
        O.olib.orc_synth_f16(O.P(a), n, seed, 0.035)
    else:
        a = np.empty(n, np.uint8)
        O.olib.orc_synth_f8(O.P(a), n, seed, 0.035)
    np.testing.assert_array_equal(a.view(np.uint8), ref.view(np.uint8))


def test_kv_indices():
    """infer.cpp:483-485 sliding window with 2 sinks."""
    assert M.kv_indices(8, 0) == (0, 0, 1)
    assert M.kv_indices(8, 7) == (0, 7, 8)
    assert M.kv_indices(8, 8) == (2, 2, 8)
    assert M.kv_indices(8, 13) == (2, 7, 8)
    assert M.kv_indices(8, 14) == (2, 2, 8)
    for pos in range(40):
        s, p, n = M.kv_indices(8, pos)
        a, b, c = (O.ctypes.c_int() for _ in range(3))
        O.olib.orc_kv_indices(8, pos, O.ctypes.byref(a), O.ctypes.byref(b), O.ctypes.byref(c))
        assert (s, p, n) == (a.value, b.value, c.value)


@pytest.mark.parametrize("dtype", [M.F32, M.F16, M.F8E5M2])
def test_oracle_forward_vs_float64(dtype):
    """End-to-end oracle forward vs the independent float64 restatement,
    through the sliding-window/sink regime (pos past max_seq_len)."""
    cfg = M.TINY.with_(weight_dtype=dtype, max_seq_len=16)
    t = M.synth_host_tensors(cfg, seed=5)
    om = O.OracleModel(cfg, t)
    rm = R.RefModel(cfg, t)
    tok = 7
    for pos in range(24):
        lo = om.forward(tok, pos)
        lr = rm.forward(tok, pos)
        err = np.max(np.abs(lo - lr)) / (np.max(np.abs(lr)) + 1e-30)
        assert err < 2e-3, (pos, err)
        tok = int(np.argmax(lr))


def test_sample_prob_and_argmax():
    lg = np.array([1.0, 3.0, 3.0, -2.0], np.float32)
    assert O.olib.orc_sample_argmax(O.P(lg), 4) == 1  # first max wins (sampler.cpp:31)
    p = O.olib.orc_sample_prob(O.P(lg), 4, 2)
    e = np.exp(lg - 3.0)
    assert abs(p - e[2] / e.sum()) < 1e-6
