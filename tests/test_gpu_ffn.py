"""GPU parity of the fused feed-forward launch (yalm_amd/csrc/ffn.h): rmsnorm,
W1/W3 + SiLU/GELU-GLU and W2 + residual (infer.cpp:339-384; infer.cu:598-620,
270-288) as ONE launch whose hb hand-off is an in-launch seam over every
workgroup, against the CPU oracle and against the separate GLU and W2 launches.

Bars (stated here): logits max|gpu - oracle| / max|oracle|
< 1e-3; greedy tokens identical (through the sliding-window / sink regime past
max_seq_len); fused vs separate launches x and logits within 1e-5 relative (the
fp32 dot products are summed over 8 waves here, over the separate kernels' own
wave counts there); every W2 prefetch depth bitwise equal to the default;
replays bitwise identical; per-block x within 1e-4 of the oracle for any order
of layer launches (epoch-tagged flags).
"""
import os

import numpy as np
import pytest

import oracle_py as O
from yalm_amd import models as M

pytestmark = pytest.mark.gpu

# fused-path contract: fp16 / fp8, dim and hidden multiples of 512 (fp16) / 1024 (fp8) elements
BASE = M.ModelConfig(dim=1024, hidden_dim=2048, head_dim=128, n_layers=3, n_heads=16, n_kv_heads=4,
                     vocab_size=1536, max_seq_len=72, rope_theta=10000.0, act=M.SILU, weight_dtype=M.F16)

CASES = [
    ("f16", BASE),
    ("f16-gelu-tied", BASE.with_(act=M.GELU, tied=True)),
    ("f16-hidden3584-dim512-hd64", BASE.with_(dim=512, hidden_dim=3584, head_dim=64, rotary_dim=64, n_heads=8,
                                               n_kv_heads=2)),
    ("fp8", BASE.with_(n_heads=32, n_kv_heads=8, weight_dtype=M.F8E5M2)),
    ("fp8-hidden3072-gelu", BASE.with_(hidden_dim=3072, act=M.GELU, weight_dtype=M.F8E5M2)),
]


def rt():
    from yalm_amd import runtime

    return runtime


def relerr(a, b):
    return float(np.max(np.abs(a - b)) / (np.max(np.abs(b)) + 1e-30))


def make(cfg, seed, fused=True, t=None, env=None):
    runtime = rt()
    if t is None:
        t = M.synth_host_tensors(cfg, seed=seed)
    dm = runtime.DeviceModel.from_arrays(cfg, t)
    env = dict(env or {})
    env["YALM_FFN"] = "1" if fused else "0"
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        dec = runtime.Decoder(dm)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    assert dec.ffn == fused
    return t, dm, dec


@pytest.mark.parametrize("name,cfg", CASES, ids=[c[0] for c in CASES])
def test_ffn_forward_and_greedy_vs_oracle(name, cfg):
    """OUTPUT-mode logits at every position (hydrated prompt first), through
    pos >= max_seq_len (ring + sink rotation); then the device greedy loop."""
    t, dm, dec = make(cfg, seed=5)
    om = O.OracleModel(cfg, t)
    try:
        prompt = [1, 17, 45, 99, 3]
        for pos, tok in enumerate(prompt[:-1]):
            dec.forward(tok, pos, rt().HYDRATE_KV_CACHE)
            om.forward(tok, pos, 0)
        tok, pos = prompt[-1], len(prompt) - 1
        for i in range(cfg.max_seq_len + 8 - len(prompt)):
            lg = dec.forward(tok, pos + i)
            lo = om.forward(tok, pos + i)
            e = relerr(lg, lo)
            assert e < 1e-3, (i, e)
            to = int(O.olib.orc_sample_argmax(O.P(lo), cfg.vocab_size))
            srt = np.sort(lo)
            if srt[-1] - srt[-2] > 1e-3 * np.max(np.abs(lo)):
                assert int(np.argmax(lg)) == to, (i, int(np.argmax(lg)), to)
            tok = to
        p = pos + cfg.max_seq_len + 8 - len(prompt)
        assert dec.generate_greedy(tok, p, 12) == om.greedy(tok, p, 12)
    finally:
        dec.close()
        dm.close()


@pytest.mark.parametrize("name,cfg", [CASES[0], CASES[3]], ids=[CASES[0][0], CASES[3][0]])
def test_ffn_matches_separate_launches(name, cfg):
    """Same weights, same tokens: the fused launch against the separate GLU and
    W2 row-block launches (x after the forward and logits), 24 positions."""
    t, dm, dec = make(cfg, seed=7, fused=True)
    _, dm2, dec2 = make(cfg, seed=7, fused=False, t=t)
    try:
        tok = 11
        for pos in range(24):
            a = dec.forward(tok, pos)
            b = dec2.forward(tok, pos)
            assert relerr(a, b) < 1e-5, (pos, relerr(a, b))
            assert relerr(dec.get_x(), dec2.get_x()) < 1e-5
            tok = int(np.argmax(b))
    finally:
        dec.close()
        dec2.close()
        dm.close()
        dm2.close()


@pytest.mark.parametrize("P", ["0", "4", "12"])
def test_ffn_prefetch_depths(P):
    """Every compiled W2 prefetch depth across the seam (YALM_FFN_P) gives the
    default depth's logits bit for bit."""
    cfg = BASE
    t, dm, dec = make(cfg, seed=3, env={"YALM_FFN_P": P})
    _, dm2, dec2 = make(cfg, seed=3, t=t)
    try:
        tok = 4
        for pos in range(6):
            a = dec.forward(tok, pos)
            b = dec2.forward(tok, pos)
            np.testing.assert_array_equal(a, b)
            tok = int(np.argmax(b))
    finally:
        dec.close()
        dec2.close()
        dm.close()
        dm2.close()


def test_ffn_replay_deterministic():
    """Bitwise-identical logits and greedy tokens for the same token sequence on
    two decoders."""
    cfg = BASE
    outs = []
    for _ in range(2):
        t, dm, dec = make(cfg, seed=4)
        try:
            tok, got = 2, []
            for pos in range(20):
                lg = dec.forward(tok, pos)
                got.append(lg)
                tok = int(np.argmax(lg))
            got.append(np.array(dec.generate_greedy(tok, 20, 30), np.float32))
            outs.append(np.concatenate([g.ravel() for g in got]))
        finally:
            dec.close()
            dm.close()
    np.testing.assert_array_equal(outs[0], outs[1])


def test_ffn_block_hook_any_layer_order():
    """Block::block hook on the fused path: one layer run several times in a
    row, a forward stopped part-way, then full forwards. The hb flags carry the
    launch epoch, so no order of layer launches lets a workgroup gather a stale
    hb; x and logits match the oracle."""
    cfg = BASE
    t, dm, dec = make(cfg, seed=12)
    om = O.OracleModel(cfg, t)
    try:
        tok = 5
        for pos in range(4):
            lg = dec.forward(tok, pos)
            lo = om.forward(tok, pos)
            assert relerr(lg, lo) < 1e-3
            tok = int(np.argmax(lo))
        pos = 4
        kv_sink, kv_pos, kv_len = M.kv_indices(cfg.max_seq_len, pos)
        x0 = om.embed(tok)
        dec.set_x(x0)
        om.x[:] = x0
        for rep in range(3):
            dec.block(2, pos, kv_sink, kv_pos, kv_len)
            om.block(2, pos, kv_sink, kv_pos, kv_len)
            e = relerr(dec.get_x(), om.x)
            assert e < 1e-4, (rep, e)
            dec.set_x(om.x)
        dec.block(0, pos, kv_sink, kv_pos, kv_len)
        om.block(0, pos, kv_sink, kv_pos, kv_len)
        assert relerr(dec.get_x(), om.x) < 1e-4
        for pos in range(4, 12):
            lg = dec.forward(tok, pos)
            lo = om.forward(tok, pos)
            assert relerr(lg, lo) < 1e-3, (pos, relerr(lg, lo))
            tok = int(np.argmax(lo))
    finally:
        dec.close()
        dm.close()


def test_ffn_trace_and_timing():
    """The trace hook returns ordered stamps for every workgroup, and the
    fused launch is timeable through yalm_time_kernel (kernel id 7)."""
    cfg = BASE
    t, dm, dec = make(cfg, seed=1, env={"YALM_FFN_TRACE": "1"})
    try:
        dec.forward(1, 0)
        tr = dec.ffn_trace().astype(np.int64)
        assert tr.shape[0] >= 1
        for k in range(5):
            assert np.all(tr[:, k + 1] >= tr[:, k]), k
        assert dec.time_kernel(7, 4) > 0
        assert dec.kernel_name(7).startswith("ffn_kernel<")
    finally:
        dec.close()
        dm.close()
