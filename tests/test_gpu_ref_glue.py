"""GPU: the HIP decode path's per-block glue against the REFERENCE's own functions
(tests/golden/ref_glue.npz: rmsnorm infer.cpp:134-144, clip 195-197, rope 200-213 and
float_to_half 11-16 of the unmodified infer.cpp, oracle/_ref/ref_glue).

A one-layer decoder whose Wq and Wk are the f16 identity (kv_dim = dim = 1024, 8 kv
heads x 128, the Mistral kv geometry) runs Block::block (yalm_block) at a chosen pos on
x = the case's input and rms_att = its weight: the fused QKV launch then writes
f16(rope(clip(rmsnorm(x) * w))) into K cache row kv_pos -- the identity GEMV is exact,
so that row is the reference's `kvrow` chain (infer.cpp:268, 277-292, 299). With
kv_sink = 2 (pos past the window) the same launch rotates the two sink rows by one
position (infer.cpp:303-317): compared with the reference's `sinkrot` chain.

Bars (the two devices round differently by construction: the reference sums x^2 in 8
FMA lanes and takes 1/sqrt by vrsqrtss + one Newton step, multiplies (x * w) * scale,
and calls libm cosf / sinf; the GPU sums in a wave tree, divides, multiplies
(x * scale) * w and calls device cosf / sinf): every f16 element within ONE f16 ulp of
the reference's, and at least 99% bit-identical. Measured (round 5, gpurun_out/r5b,
profiles/r5_glue_gpu.txt): 20 of 22 rows bit-identical, the other two (pos 4095) 1023 of
1024 elements identical and one 1 f16 ulp apart. Before the host computed the RoPE
frequencies the way the reference's compiled rope does (powf(theta, -(j * (1 /
rotary_dim))), yalm_hip.hip create_decoder), the pos-4095 row was 60 f16 ulps off.
"""
import os
import sys

import numpy as np
import pytest

from yalm_amd import models as M

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import ref_glue_cases as C  # noqa: E402

G = C.load_golden()
MAX_SEQ = 64
KV_POS = 5
MIN_EXACT = 0.99


def rt():
    from yalm_amd import runtime

    return runtime


def cfg_for(case):
    return M.ModelConfig(dim=case["d"], hidden_dim=256, head_dim=case["head_dim"], n_layers=1,
                         n_heads=case["d"] // case["head_dim"], n_kv_heads=case["d"] // case["head_dim"],
                         vocab_size=256, max_seq_len=MAX_SEQ, rope_theta=case["theta"],
                         rotary_dim=case["rotary_dim"], norm_eps=case.get("eps", 1e-5),
                         qkv_clip=case.get("clip", M.FLT_MAX), act=M.SILU, weight_dtype=M.F16)


class IdentityBlock:
    """Decoder over one layer with Wq = Wk = I (f16) and caller-owned KV caches."""

    def __init__(self, case, rms_w=None, k_init=None):
        R = rt()
        cfg = cfg_for(case)
        t = M.synth_host_tensors(cfg, seed=3)
        n = M.layer_names(0)
        eye = np.eye(cfg.dim, dtype=np.float16)
        t[n["wq"]] = eye
        t[n["wk"]] = eye
        if rms_w is not None:
            t[n["rms_att"]] = rms_w.astype(np.float32)
        self.cfg, self.R = cfg, R
        self.dm = R.DeviceModel.from_arrays(cfg, t)
        k = np.zeros((MAX_SEQ, cfg.kv_dim), np.float16) if k_init is None else k_init
        v = np.zeros((MAX_SEQ, cfg.kv_dim), np.float16)
        self.kp = R.lib.yalm_upload(k.ctypes.data, k.nbytes)
        self.vp = R.lib.yalm_upload(v.ctypes.data, v.nbytes)
        assert self.kp and self.vp
        self.dec = R.Decoder(self.dm, kv_caches=[(self.kp, self.vp)])

    def k_rows(self):
        out = np.zeros((MAX_SEQ, self.cfg.kv_dim), np.uint16)
        self.R.check(self.R.lib.yalm_download(out.ctypes.data, self.kp, out.nbytes))
        return out

    def close(self):
        self.dec.close()
        self.dm.close()
        self.R.lib.yalm_free(self.kp)
        self.R.lib.yalm_free(self.vp)


def f16_ulp_diff(a, b):
    """|a - b| in f16 ulps for same-sign finite values (bit distance of the ordered encodings)."""
    def ordered(u):
        u = u.astype(np.int32)
        return np.where(u & 0x8000, -(u & 0x7FFF), u)
    return np.abs(ordered(a) - ordered(b))


def check_row(got, ref, what):
    ulps = f16_ulp_diff(got, ref)
    exact = float(np.mean(ulps == 0))
    print(f"{what}: max {int(ulps.max())} f16 ulp, {exact * 100:.2f}% bit-identical")
    assert ulps.max() <= 1, (what, int(ulps.max()), int(np.argmax(ulps)))
    assert exact >= MIN_EXACT, (what, exact)


KV_CASES = [c["name"] for c in C.CASES if c["op"] == "kvrow"]


@pytest.mark.parametrize("name", KV_CASES)
def test_gpu_kv_row_vs_reference_glue(name):
    """rmsnorm -> Wk (identity) -> clip -> rope(pos) -> f16 K cache row, pos in {0, 1, 17,
    4095, 4096, 32767}, full and partial (rotary_dim 64 < head_dim 128) rotation."""
    case = C.CASE[name]
    inp = C.inputs(case)
    blk = IdentityBlock(case, rms_w=inp["w"])
    try:
        blk.dec.set_x(inp["x"])
        blk.dec.block(0, case["pos"], 0, KV_POS, KV_POS + 1)
        check_row(blk.k_rows()[KV_POS], G[f"{name}/row"], name)
    finally:
        blk.close()


@pytest.mark.parametrize("name", [c["name"] for c in C.CASES if c["op"] == "sinkrot"])
def test_gpu_sink_rotation_vs_reference_glue(name):
    """kv_sink = 2 (pos past max_seq_len): the QKV launch rotates sink rows 0 and 1 by
    one position, as infer.cpp:307-317 does with the reference's rope and f16 casts."""
    case = C.CASE[name]
    row = C.inputs(case)["row"]
    k = np.zeros((MAX_SEQ, case["d"]), np.uint16)
    k[0] = row
    k[1] = row
    blk = IdentityBlock(case, k_init=k.view(np.float16))
    try:
        blk.dec.set_x(np.ones(case["d"], np.float32))
        pos = MAX_SEQ + 7
        kv_sink, kv_pos, kv_len = M.kv_indices(MAX_SEQ, pos)
        blk.dec.block(0, pos, kv_sink, kv_pos, kv_len)
        rows = blk.k_rows()
        for r in (0, 1):
            check_row(rows[r], G[f"{name}/row"], f"{name} sink {r}")
    finally:
        blk.close()
