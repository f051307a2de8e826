"""GPU parity of the W1|W3 GEMV variants: the W3 stream rotated (YALM_GLU_W3_ROT=1,
gemv.h rb_perm) and W1/W3 interleaved row by row in a decoder copy
(YALM_GLU_INTERLEAVE=1). For the rotation: the workgroup streams its W3 rows in a rotated order and
parks every partial at its true (group, row), so the GLU output, the logits
and the greedy tokens are those of the unrotated kernel / the CPU oracle.
Bars: logits rel 1e-3 vs the oracle, greedy tokens identical, rotated vs
unrotated logits rel 1e-5 (the per-row chunk-to-wave dealing may differ)."""
import numpy as np
import pytest

import oracle_py as O
from yalm_amd import models as M

pytestmark = pytest.mark.gpu

CASES = [M.SMALL, M.SMALL.with_(hidden_dim=M.SMALL.hidden_dim + 64), M.SMALL.with_(weight_dtype=M.F8E5M2)]


@pytest.mark.parametrize("knob", ["YALM_GLU_W3_ROT", "YALM_GLU_INTERLEAVE"])
@pytest.mark.parametrize("cfg", CASES, ids=["small", "odd-groups", "fp8"])
def test_glu_w3_rotation(cfg, knob, monkeypatch):
    from yalm_amd import runtime

    t = M.synth_host_tensors(cfg, seed=21)
    dm = runtime.DeviceModel.from_arrays(cfg, t)
    monkeypatch.setenv(knob, "1")
    dec = runtime.Decoder(dm)
    monkeypatch.setenv(knob, "0")
    ref = runtime.Decoder(dm)
    om = O.OracleModel(cfg, t)
    try:
        tok = 3
        for pos in range(10):
            lg, lr, lo = dec.forward(tok, pos), ref.forward(tok, pos), om.forward(tok, pos)
            assert np.max(np.abs(lg - lo)) / np.max(np.abs(lo)) < 1e-3
            assert np.max(np.abs(lg - lr)) / np.max(np.abs(lr)) < 1e-5
            tok = int(np.argmax(lo))
        assert dec.generate_greedy(tok, 10, 12) == om.greedy(tok, 10, 12)
    finally:
        dec.close()
        ref.close()
        dm.close()
