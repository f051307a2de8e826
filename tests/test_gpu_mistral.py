"""Full-size parity: a Mistral-7B-shaped random-weight model (the bench
workload, BASELINE.json config 2) built in HBM by yalm_synth and, bit-for-bit
identically, on the host by the oracle's initialiser. Greedy tokens and
logits must agree with the CPU oracle."""
import numpy as np
import pytest

import oracle_py as O
from yalm_amd import models as M

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def relerr(a, b):
    return float(np.max(np.abs(a - b)) / (np.max(np.abs(b)) + 1e-30))


@pytest.mark.parametrize("dtype", [M.F16, M.F8E5M2])
def test_mistral_shape_greedy_parity(dtype):
    from yalm_amd import runtime

    cfg = M.MISTRAL_7B.with_(weight_dtype=dtype)
    dm = runtime.DeviceModel.synthetic(cfg, seed=1)
    dec = runtime.Decoder(dm)
    try:
        host = O.synth_host_tensors_fast(cfg, seed=1)
        # spot-check the initialiser on real tensors: device bytes == host bytes
        for name in ("model.layers.31.mlp.w2.weight", "model.norm.weight"):
            a = host[name]
            buf = np.empty(a.nbytes, np.uint8)
            runtime.check(runtime.lib.yalm_download(buf.ctypes.data, dm.ptrs[name], a.nbytes))
            np.testing.assert_array_equal(buf, a.reshape(-1).view(np.uint8))
        om = O.OracleModel(cfg, host)
        tok = 1
        for pos in range(6):
            lg = dec.forward(tok, pos)
            lo = om.forward(tok, pos)
            assert relerr(lg, lo) < 1e-3, (pos, relerr(lg, lo))
            tg, to = int(np.argmax(lg)), int(np.argmax(lo))
            assert tg == to, (pos, tg, to)
            tok = to
        # device greedy loop continues identically
        dev = dec.generate_greedy(tok, 6, 4)
        ref = om.greedy(tok, 6, 4)
        assert dev == ref
    finally:
        dec.close()
        dm.close()
