"""GPU parity of the kernel-level test API (include/yalm_hip.h test section)
against the CPU oracle, mirroring the reference's test.cpp:148-206 (same
seeded inputs, same 1e-4 abs criterion) plus Mistral-7B shapes
(test.cpp:307-359 kernel_bench shapes) with a stated relative tolerance."""
import os

import numpy as np
import pytest

import oracle_py as O
from yalm_amd import models as M

pytestmark = pytest.mark.gpu

REL_TOL = 2e-5  # max|gpu - oracle| / max|oracle| for fp32-accumulated GEMVs


def rt():
    from yalm_amd import runtime

    return runtime


@pytest.fixture(scope="module")
def tcpp(golden_dir):
    return dict(np.load(os.path.join(golden_dir, "test_cpp_inputs.npz")))


def relerr(a, b):
    return float(np.max(np.abs(a - b)) / (np.max(np.abs(b)) + 1e-30))


def test_reference_matmul_case(tcpp):
    """test.cpp:158-168: f32 matmul, dim 256 -> 16, abs 1e-4."""
    w = tcpp["matmul_w"].reshape(16, 256)
    x = tcpp["matmul_x"]
    np.testing.assert_allclose(rt().matmul(x, w, M.F32), O.matmul(x, w, M.F32), atol=1e-4)


def test_reference_mha_case(tcpp):
    """test.cpp:171-188: head_dim 16, 16 heads / 8 kv heads, kv_len 4; att and xout at 1e-4."""
    kb = tcpp["mha_kb"].astype(np.float16)
    vb = tcpp["mha_vb"].astype(np.float16)
    q = tcpp["mha_q"]
    xg, ag = rt().mha(kb, vb, q, 16, 4, 4, 16, 8)
    xo, ao = O.mha(kb, vb, q, 16, 4, 4, 16, 8)
    np.testing.assert_allclose(ag, ao, atol=1e-4)
    np.testing.assert_allclose(xg, xo, atol=1e-4)


def test_reference_ffn_case(tcpp):
    """test.cpp:191-205: f32 ffn with GELU, abs 1e-4."""
    x = tcpp["ffn_x"]
    w1, w2, w3 = (tcpp[k].reshape(256, 256) for k in ("ffn_w1", "ffn_w2", "ffn_w3"))
    np.testing.assert_allclose(rt().ffn(x, w1, w2, w3, M.GELU, M.F32), O.ffn(x, w1, w2, w3, M.GELU, M.F32),
                               atol=1e-4)


def _weights(rng, d, n, dtype, scale=1.0):
    w = (rng.standard_normal((d, n)) * scale).astype(np.float32)
    if dtype == M.F16:
        return w.astype(np.float16)
    if dtype == M.F8E5M2:
        from yalm_amd.convert import f32_to_e5m2

        return f32_to_e5m2(w)
    return w


@pytest.mark.parametrize("dtype", [M.F32, M.F16, M.F8E5M2])
@pytest.mark.parametrize("n,d", [(4096, 14336), (4096, 6144), (14336, 4096), (4096, 32000), (512, 48), (2064, 80)])
def test_matmul_shapes(dtype, n, d):
    """Mistral GEMV shapes (W1/W3, QKV, W2, Wcls) and ragged ones (tail chunks)."""
    if dtype == M.F32 and n * d > 30_000_000:
        pytest.skip("f32 big shapes covered by f16/fp8")
    rng = np.random.default_rng(n + d)
    w = _weights(rng, d, n, dtype, 0.02)
    x = rng.standard_normal(n).astype(np.float32)
    g = rt().matmul(x, w, dtype)
    o = O.matmul(x, w, dtype)
    assert relerr(g, o) < REL_TOL


@pytest.mark.parametrize("kv_len", [1, 5, 127, 128, 129, 300, 1024, 4096])
@pytest.mark.parametrize("head_dim,n_heads,n_kv", [(128, 32, 8), (64, 8, 2), (128, 24, 8), (32, 8, 8)])
def test_mha_shapes(kv_len, head_dim, n_heads, n_kv):
    """Split-KV attention at Mistral/Llama-3B head layouts, kv_len across
    chunk boundaries (1 split .. 32 splits)."""
    max_seq_len = 4096
    rng = np.random.default_rng(kv_len * 7 + head_dim)
    kb = rng.standard_normal(max_seq_len * n_kv * head_dim).astype(np.float16)
    vb = rng.standard_normal(max_seq_len * n_kv * head_dim).astype(np.float16)
    q = (rng.standard_normal(n_heads * head_dim) * 2).astype(np.float32)
    xg, ag = rt().mha(kb, vb, q, head_dim, kv_len, max_seq_len, n_heads, n_kv)
    xo, ao = O.mha(kb, vb, q, head_dim, kv_len, max_seq_len, n_heads, n_kv)
    np.testing.assert_allclose(xg, xo, atol=2e-5, rtol=1e-4)
    np.testing.assert_allclose(ag, ao, atol=2e-6, rtol=1e-4)


def test_mha_attn_known_answer_gpu():
    """test.cpp:68-126 KAT adapted to a GPU-supported head_dim (16): q = 1e4 *
    one-hot saturates softmax to an exact one-hot; outputs are V rows."""
    hd, T = 16, 4
    q = np.zeros(2 * hd, np.float32)
    q[1] = 1e4
    q[hd + 2] = 1e4
    k = np.zeros((T, hd), np.float16)
    k[0, 0] = 1
    k[1, 1] = 1
    k[2, 2] = 1
    k[3, 0] = -1
    xout, att = rt().mha(k.reshape(-1), k.reshape(-1), q, hd, T, T, 2, 1)
    np.testing.assert_allclose(att[:T], [0, 1, 0, 0], atol=1e-4)
    np.testing.assert_allclose(att[T:], [0, 0, 1, 0], atol=1e-4)
    np.testing.assert_allclose(xout[:hd], k[1].astype(np.float32), atol=1e-4)
    np.testing.assert_allclose(xout[hd:], k[2].astype(np.float32), atol=1e-4)


@pytest.mark.parametrize("dtype", [M.F16, M.F8E5M2])
@pytest.mark.parametrize("act", [M.SILU, M.GELU])
def test_ffn_mistral_shape(dtype, act):
    rng = np.random.default_rng(3)
    dim, hidden = 4096, 14336
    w1 = _weights(rng, hidden, dim, dtype, 1 / 64)
    w3 = _weights(rng, hidden, dim, dtype, 1 / 64)
    w2 = _weights(rng, dim, hidden, dtype, 1 / 120)
    x = rng.standard_normal(dim).astype(np.float32)
    assert relerr(rt().ffn(x, w1, w2, w3, act, dtype), O.ffn(x, w1, w2, w3, act, dtype)) < 1e-4


def test_synth_device_matches_host_bitwise():
    """yalm_synth on the device == numpy/oracle twin (the bench's random
    Mistral weights are reproducible bit-for-bit on the host)."""
    runtime = rt()
    for dt, scale, off in ((M.F32, 0.2, 1.0), (M.F16, 0.035, 0.0), (M.F8E5M2, 0.035, 0.0)):
        n = 100003
        nb = n * M.DTYPE_BYTES[dt]
        p = runtime.lib.yalm_alloc(nb)
        seed = M.synth_seed(9, f"t{dt}")
        runtime.check(runtime.lib.yalm_synth(p, n, dt, seed, scale, off, None))
        runtime.check(runtime.lib.yalm_stream_sync(None))
        host = np.empty(nb, np.uint8)
        runtime.check(runtime.lib.yalm_download(host.ctypes.data, p, nb))
        runtime.lib.yalm_free(p)
        ref = M.synth_array(n, dt, seed, scale, off).view(np.uint8)
        np.testing.assert_array_equal(host, ref)


@pytest.mark.parametrize("n", [1024, 2064])
def test_fp8_every_byte_exact(n):
    """Every E5M2 byte value through the GEMV's fp8 unpack (v_cvt_pk_f32_bf8 on
    the row-block path n % 1024 == 0, the ragged path otherwise): row r holds
    byte r everywhere, x is one-hot, so out[r] must equal e5m2(r) exactly
    (NaN bytes give NaN; inf * 0 gives NaN, as in the float64 twin)."""
    w = np.repeat(np.arange(256, dtype=np.uint8)[:, None], n, axis=1)
    x = np.zeros(n, np.float32)
    x[n // 3] = 1.0
    g = rt().matmul(x, w, M.F8E5M2)
    ref = (M.e5m2_to_f32(w).astype(np.float64) * x.astype(np.float64)).sum(axis=1)
    fin = np.isfinite(ref)
    assert fin.sum() == 256 - 8  # 2 infinities + 6 NaNs -> non-finite sums
    np.testing.assert_array_equal(g[fin], ref[fin].astype(np.float32))
    assert np.all(np.isnan(g[~fin]))
