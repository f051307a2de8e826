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


@pytest.mark.parametrize("real", [None, M.REALISTIC], ids=["uniform", "realistic"])
def test_mistral_config2_256_tokens_vs_oracle(real):
    """The config-2 workload as written (BASELINE.json: Mistral-7B fp16, all 32 layers,
    256 greedy tokens after the bench's 13-token prompt, kv_len up to 268) against the
    CPU oracle step by step: logits within 1e-3 rel at every step, the device's argmax
    equal to the oracle's wherever the oracle's top-2 margin exceeds 1e-3 of max|logit|
    (the sequence then continues with the device's token), and the device greedy loop
    (one graph replay per token, argmax on the device) reproduces the sequence.

    realistic (round 5's "peaked" model only scaled the final norm by 2^3,
    an exact logit scale that could not change a token): models.REALISTIC, hidden states with
    a trained checkpoint's regimes -- peaked attention softmax (Wq / Wk x 24), three residual
    outlier channels of 10^2..10^3 (embedding columns, W2 rows), a GLU product above 65504 at
    every position in layer 1, a final norm x 4.5, a residual stream that dominates its
    branches (not chaotic: models.Realistic); next-token distributions peaked (top-1
    probability >= 0.5 at most steps, log ppl of the greedy text << ln(vocab)). The default
    synthetic model's are near-uniform (logit std ~1.2)."""
    from yalm_amd import runtime

    cfg = M.MISTRAL_7B.with_(weight_dtype=M.F16)
    dm = runtime.DeviceModel.synthetic(cfg, seed=1, real=real)
    dec = runtime.Decoder(dm)
    dec2 = runtime.Decoder(dm)
    try:
        om = O.OracleModel(cfg, O.synth_host_tensors_fast(cfg, seed=1, real=real))
        prompt = [(7 * i + 1) % cfg.vocab_size for i in range(13)]  # bench.py's prompt
        for pos, t in enumerate(prompt[:-1]):
            dec.forward(t, pos, runtime.HYDRATE_KV_CACHE)
            dec2.forward(t, pos, runtime.HYDRATE_KV_CACHE)
            om.forward(t, pos)
        tok, pos, seq, near_ties, worst, p1, lp = prompt[-1], len(prompt) - 1, [], 0, 0.0, [], []
        for _ in range(256):
            lg = dec.forward(tok, pos).astype(np.float64)
            lo = om.forward(tok, pos).astype(np.float64)
            worst = max(worst, relerr(lg, lo))
            lse = lo.max() + np.log(np.exp(lo - lo.max()).sum())
            p1.append(float(np.exp(lo.max() - lse)))
            lp.append(float(lo[int(np.argmax(lg))] - lse))
            assert relerr(lg, lo) < 1e-3, (pos, relerr(lg, lo))
            tg, to = int(np.argmax(lg)), int(np.argmax(lo))
            if tg != to:
                top = np.sort(lo)[-2:]
                assert (top[1] - top[0]) / np.max(np.abs(lo)) < 1e-3, (pos, tg, to)
                near_ties += 1
            seq.append(tg)
            tok, pos = tg, pos + 1
        p1 = np.array(p1)
        print(f"{'realistic' if real else 'uniform'}: 256 tokens, kv_len {len(prompt)}..{pos}: worst logits rel {worst:.2e}, near-tie steps "
              f"{near_ties}; oracle top-1 probability median {np.median(p1):.3f}, >= 0.5 at {np.mean(p1 >= 0.5):.0%} "
              f"of steps; log ppl of the greedy text {-np.mean(lp):.3f} (ln vocab {np.log(cfg.vocab_size):.2f})")
        assert near_ties <= 4
        if real is not None:
            assert np.mean(p1 >= 0.5) >= 0.5 and -np.mean(lp) < 0.25 * np.log(cfg.vocab_size)
        dev = dec2.generate_greedy(prompt[-1], len(prompt) - 1, 256)
        assert list(dev) == seq
    finally:
        dec.close()
        dec2.close()
        dm.close()
