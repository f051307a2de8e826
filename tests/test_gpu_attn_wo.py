"""GPU parity of the fused attention + Wo launch (yalm_amd/csrc/attn_wo.h): the
launch path's attention and output projection (+ residual) as one kernel whose
Wo weight stream overlaps the split-KV attention, against the CPU oracle and
against the two separate launches on the same weights.

Bars (stated here): logits max|gpu - oracle| / max|oracle|
< 1e-3; greedy tokens identical (through the sliding-window / sink regime past
max_seq_len, and with attention split over many chunks and merged); fused vs
separate launches < 1e-4 relative (only the fp32 summation order of Wo differs);
replays bitwise identical.
"""
import os

import numpy as np
import pytest

import oracle_py as O
from yalm_amd import models as M

pytestmark = pytest.mark.gpu

# fused-path contract: head_dim 128, Wo rows of 4 KB (XS = 1) or 8 KB (XS = 2)
BASE = M.ModelConfig(dim=1024, hidden_dim=2048, head_dim=128, n_layers=3, n_heads=16, n_kv_heads=4,
                     vocab_size=1536, max_seq_len=72, rope_theta=10000.0, act=M.SILU, weight_dtype=M.F16)

CASES = [
    ("f16-xs1-g4", BASE),
    ("f16-xs2-g4", BASE.with_(n_heads=32, n_kv_heads=8)),
    ("f16-xs1-g8-gelu-tied", BASE.with_(n_kv_heads=2, act=M.GELU, tied=True)),
    ("f16-xs1-g1-clip-rot64", BASE.with_(n_kv_heads=16, qkv_clip=0.5, rotary_dim=64)),
    ("fp8-xs1-g4", BASE.with_(n_heads=32, n_kv_heads=8, weight_dtype=M.F8E5M2)),
    ("fp8-xs2-g2", BASE.with_(n_heads=64, n_kv_heads=32, weight_dtype=M.F8E5M2)),
    ("f16-q_dim=dim", BASE.with_(dim=2048)),
]


def rt():
    from yalm_amd import runtime

    return runtime


def relerr(a, b):
    return float(np.max(np.abs(a - b)) / (np.max(np.abs(b)) + 1e-30))


def make(cfg, seed, fused=True, t=None, extra=None):
    runtime = rt()
    if t is None:
        t = M.synth_host_tensors(cfg, seed=seed)
    dm = runtime.DeviceModel.from_arrays(cfg, t)
    env = dict(extra or {})
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    try:
        dec = runtime.Decoder(dm, launch=0 if fused else runtime.LAUNCH_SEPARATE_ATTN_WO)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert dec.attn_wo == fused
    return t, dm, dec


@pytest.mark.parametrize("name,cfg", CASES, ids=[c[0] for c in CASES])
def test_attn_wo_forward_and_greedy_vs_oracle(name, cfg):
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


@pytest.mark.parametrize("name,cfg", CASES[:2] + CASES[4:5], ids=[c[0] for c in CASES[:2] + CASES[4:5]])
def test_attn_wo_matches_separate_launches(name, cfg):
    """Same weights, same tokens: fused vs separate attention and Wo launches
    (the residual x after the whole forward and the logits), 40 positions."""
    t, dm, dec = make(cfg, seed=7, fused=True)
    _, dm2, dec2 = make(cfg, seed=7, fused=False, t=t)
    try:
        tok = 11
        for pos in range(40):
            a = dec.forward(tok, pos)
            b = dec2.forward(tok, pos)
            assert relerr(a, b) < 1e-4, (pos, relerr(a, b))
            assert relerr(dec.get_x(), dec2.get_x()) < 1e-4
            tok = int(np.argmax(b))
    finally:
        dec.close()
        dec2.close()
        dm.close()
        dm2.close()


def test_attn_wo_long_context_split_attention():
    """kv_len up to 1040 (17 key chunks per kv head: one chunk per key split, a
    partial per (head, split) folded by that query head's merger workgroup; the
    last chunk is partial, 1040 = 16 x 64 + 16, so its rows past max_seq_len read
    as zeros through the per-chunk descriptor): greedy tokens equal the oracle's
    the whole way, then past max_seq_len."""
    cfg = BASE.with_(n_layers=2, max_seq_len=1040)
    t, dm, dec = make(cfg, seed=9)
    om = O.OracleModel(cfg, t)
    try:
        n = 1100
        assert dec.generate_greedy(3, 0, n) == om.greedy(3, 0, n)
    finally:
        dec.close()
        dm.close()


def test_attn_wo_stress_vs_separate():
    """Granule single-copy atomicity (attn_wo.h awo_ld8_sc1) under load: 32
    splits per kv head at kv_len up to 2048 (one workgroup then runs 1-32 chunks
    with its K/V loads double-buffered and one partial per workgroup) and 660
    replayed greedy forwards
    per decoder; the fused launch must give the same greedy tokens as the
    separate launches and every logits row within 1e-4 of them."""
    cfg = BASE.with_(n_layers=2, max_seq_len=2048, n_heads=32, n_kv_heads=8)
    t, dm, dec = make(cfg, seed=21)
    _, dm2, dec2 = make(cfg, seed=21, fused=False, t=t)
    try:
        for pos, tok in enumerate(range(1, 1400)):  # hydrate to kv_len 1400
            dec.forward(tok % cfg.vocab_size, pos, rt().HYDRATE_KV_CACHE)
            dec2.forward(tok % cfg.vocab_size, pos, rt().HYDRATE_KV_CACHE)
        a = dec.generate_greedy(7, 1399, 660)  # to pos 2059: past max_seq_len (ring + sinks)
        b = dec2.generate_greedy(7, 1399, 660)
        assert a == b
        for pos in range(2059, 2069):
            la = dec.forward(a[pos % 660], pos)
            lb = dec2.forward(a[pos % 660], pos)
            assert relerr(la, lb) < 1e-4, (pos, relerr(la, lb))
    finally:
        dec.close()
        dec2.close()
        dm.close()
        dm2.close()


def test_attn_wo_multichunk_workgroups_vs_oracle():
    """max_seq_len 4160 = 65 key chunks over 32 splits per kv head: past kv_len 2048
    a workgroup runs 2, then (kv_len > 4096) 3 chunks with the next chunk's K/V
    loaded before the current one is computed, and publishes ONE partial that the
    merger folds in split order. Greedy tokens equal the oracle's through the full
    window and past it (ring + sinks); fused and separate launches agree."""
    cfg = BASE.with_(n_layers=2, max_seq_len=4160, n_heads=32, n_kv_heads=8)
    t, dm, dec = make(cfg, seed=23)
    _, dm2, dec2 = make(cfg, seed=23, fused=False, t=t)
    om = O.OracleModel(cfg, t)
    try:
        n = 4200
        ref = om.greedy(5, 0, n)
        assert dec.generate_greedy(5, 0, n) == ref
        assert dec2.generate_greedy(5, 0, n) == ref
        for pos in (4190, 4191):
            lo = om.forward(ref[pos - 1], pos)
            assert relerr(dec.forward(ref[pos - 1], pos), lo) < 1e-3
            assert relerr(dec2.forward(ref[pos - 1], pos), lo) < 1e-3
    finally:
        dec.close()
        dec2.close()
        dm.close()
        dm2.close()


def test_attn_wo_time_kernel():
    """yalm_time_kernel id 8 times the fused launch with a fresh epoch per launch."""
    t, dm, dec = make(BASE, seed=3)
    try:
        for pos in range(8):
            dec.forward(1 + pos, pos, rt().HYDRATE_KV_CACHE)
        assert dec.time_kernel(8, 4) > 0
        assert "attn_wo" in dec.kernel_name(8)
    finally:
        dec.close()
        dm.close()


def test_attn_wo_replay_deterministic():
    """Bitwise-identical logits for the same token sequence on two decoders
    (ordered merges and reductions; epoch-tagged hand-off flags)."""
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


def test_attn_wo_block_hook_any_layer_order():
    """Block::block hook on the fused path: one layer run several
    times in a row, a forward stopped part-way, then full forwards. The done
    flags carry the launch epoch, so no order of layer launches can let a Wo
    workgroup read a stale attention output; x and logits match the oracle."""
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
        for rep in range(3):  # the same layer three times in a row
            dec.block(1, pos, kv_sink, kv_pos, kv_len)
            om.block(1, pos, kv_sink, kv_pos, kv_len)
            e = relerr(dec.get_x(), om.x)
            assert e < 1e-4, (rep, e)
            dec.set_x(om.x)
        dec.block(0, pos, kv_sink, kv_pos, kv_len)  # a forward stopped after layer 0
        om.block(0, pos, kv_sink, kv_pos, kv_len)
        assert relerr(dec.get_x(), om.x) < 1e-4
        for pos in range(4, 12):  # full forwards after the out-of-order launches
            lg = dec.forward(tok, pos)
            lo = om.forward(tok, pos)
            assert relerr(lg, lo) < 1e-3, (pos, relerr(lg, lo))
            tok = int(np.argmax(lo))
    finally:
        dec.close()
        dm.close()
