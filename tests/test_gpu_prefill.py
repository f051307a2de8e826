"""GPU parity of the batched MFMA prefill path (include/yalm_hip.h "batched
prefill"): the GEMM and the causal attention against float64 numpy, and the
whole prefill against the decode engine (itself pinned to the CPU oracle by
test_gpu_decode.py), position by position.

Tolerances: the prefill rounds activations to f16 for the MFMA inputs (A
operands: normalised x, attention output, GLU output; P in attention), where
the reference keeps them f32 (infer.cpp). The GEMM itself accumulates in f32,
so on f16-exact inputs it is exact (test_gemm_exact_integers).
  * log p(next token): |prefill - decode| <= LP_ATOL (nats)
  * attention output: |o - o64| <= 4e-3 * max|v| + f16 rounding of o
"""
import numpy as np
import pytest

from yalm_amd import models as M

pytestmark = pytest.mark.gpu

LP_ATOL = 0.02  # nats, per position


def rt():
    from yalm_amd import runtime

    return runtime


@pytest.mark.parametrize("M_,N,K", [(128, 128, 64), (200, 256, 192), (37, 384, 128), (1, 128, 64)])
def test_gemm_exact_integers(M_, N, K):
    """Small asymmetric integers: every product and partial sum is exact in f32,
    so the MFMA GEMM (fragment maps, LDS swizzle, M tail) must match exactly."""
    rng = np.random.default_rng(M_ * N + K)
    a = rng.integers(-4, 5, size=(M_, K)).astype(np.float16)
    w = rng.integers(-4, 5, size=(N, K)).astype(np.float16)
    w[:, 0] += np.arange(N, dtype=np.float16) % 7  # break row/column symmetry
    c = rt().gemm_f16(a, w)
    ref = a.astype(np.int64) @ w.astype(np.int64).T
    np.testing.assert_array_equal(c, ref.astype(np.float32))


# GEMM forms (yalm_amd/csrc/prefill_gemm.h), chosen explicitly through
# yalm_set_prefill_forms (a decoder's, or with no decoder the yalm_gemm_f16 test hook's):
# "g16-256" / "g16-192" / "g16-128" / "g16-320" force the 256-row tile's width on every
# GEMM it divides (256 / 192 / 128 run the 8-phase gemm8p_kernel, "-2ph" the 2-phase
# gemm16_kernel, 320 is always 2-phase); "nopersist": one workgroup per tile instead of
# the persistent tile loop. The round-2 128 x 128 kernel and its stage / wide forms were
# removed in round 4.
G16_ALL = "qkv:{0},wo:{0},glu:{0},w2:{0},cls:{0},test:{0}"
FORMS = {"auto": "", "auto-qkv2": "qkv1:0",
         "g16-256": G16_ALL.format(256),
         "g16-256-2ph": G16_ALL.format(256) + ",8p:0", "g16-128": G16_ALL.format(128),
         "g16-192": G16_ALL.format(192),
         "g16-192-2ph": G16_ALL.format(192) + ",8p:0",
         "g16-128-2ph": G16_ALL.format(128) + ",8p:0",
         "g16-256-nopersist": G16_ALL.format(256) + ",persist:0",
         "g16-320": G16_ALL.format(320),
         "wnorm0": "wnorm:0"}  # the workgroup-per-row norm kernel (round 6 default: one wave per row)


@pytest.mark.parametrize("form", list(FORMS))
@pytest.mark.parametrize("M_,N,K", [(200, 256, 192), (37, 768, 128), (1, 256, 64), (513, 5120, 640), (300, 384, 64),
                                    (513, 512, 320), (260, 768, 448), (256, 256, 576), (70, 512, 128),
                                    (1100, 16384, 192)])
def test_gemm_forms_exact(form, M_, N, K):
    """Every tile form is exact on f16-exact integer data (any
    staging race or fragment-map error shows as a wrong integer); K tiles 1..10
    (odd and even counts: the 8-phase kernel's iteration covers two K tiles);
    1100 x 16384: more 256 x 256 tiles (320) than CUs, so the persistent tile loop runs."""
    rng = np.random.default_rng(M_ + N + K)
    a = rng.integers(-4, 5, size=(M_, K)).astype(np.float16)
    w = rng.integers(-4, 5, size=(N, K)).astype(np.float16)
    w[:, 0] += np.arange(N, dtype=np.float16) % 7
    rt().set_gemm_forms(FORMS[form])
    try:
        c = rt().gemm_f16(a, w)
    finally:
        rt().set_gemm_forms("")
    ref = a.astype(np.float64) @ w.astype(np.float64).T  # exact: small integers
    np.testing.assert_array_equal(c, ref.astype(np.float32))


@pytest.mark.parametrize("M_,N,K", [(300, 384, 512), (4096, 128, 3072)])
def test_gemm_random(M_, N, K):
    rng = np.random.default_rng(7)
    a = rng.standard_normal((M_, K)).astype(np.float16)
    w = (rng.standard_normal((N, K)) * 0.02).astype(np.float16)
    c = rt().gemm_f16(a, w)
    ref = a.astype(np.float64) @ w.astype(np.float64).T
    err = np.max(np.abs(c - ref)) / np.max(np.abs(ref))
    assert err < 1e-5, err


def _attn_ref(q, kc, vc, T, pos0, nh, nkv, D):
    q = q.astype(np.float64).reshape(T, nh, D)
    k = kc.astype(np.float64).reshape(-1, nkv, D)
    v = vc.astype(np.float64).reshape(-1, nkv, D)
    out = np.zeros((T, nh, D))
    G = nh // nkv
    for t in range(T):
        n = pos0 + t + 1
        for h in range(nh):
            s = k[:n, h // G] @ q[t, h] / np.sqrt(D)
            p = np.exp(s - s.max())
            p /= p.sum()
            out[t, h] = p @ v[:n, h // G]
    return out.reshape(T, nh * D)


@pytest.mark.parametrize("T,pos0", [(1, 0), (37, 0), (128, 0), (200, 0), (70, 50)])
@pytest.mark.parametrize("nh,nkv,D", [(8, 2, 64), (4, 4, 128), (6, 2, 128)])
def test_attn_prefill(T, pos0, nh, nkv, D):
    rng = np.random.default_rng(T * 31 + pos0 + D)
    q = rng.standard_normal((T, nh * D)).astype(np.float16)
    kc = rng.standard_normal((pos0 + T, nkv * D)).astype(np.float16)
    vc = rng.standard_normal((pos0 + T, nkv * D)).astype(np.float16)
    o = rt().attn_prefill(q, kc, vc, T, pos0, nh, nkv, D).astype(np.float64)
    ref = _attn_ref(q, kc, vc, T, pos0, nh, nkv, D)
    np.testing.assert_allclose(o, ref, atol=4e-3 * np.abs(vc).max(), rtol=2e-3)


def _decode_logprobs(dec, tokens):
    lp = []
    for pos, t in enumerate(tokens[:-1]):
        logits = dec.forward(int(t), pos).astype(np.float64)
        m = logits.max()
        lp.append(logits[tokens[pos + 1]] - m - np.log(np.exp(logits - m).sum()))
    return np.array(lp)


CFGS = {
    "small-d64": M.SMALL,
    "gqa-d128": M.ModelConfig(dim=512, hidden_dim=1024, head_dim=128, n_layers=3, n_heads=4, n_kv_heads=2,
                              vocab_size=1024, max_seq_len=320, rope_theta=1e6, act=M.SILU, weight_dtype=M.F16),
    # GELU-tanh GLU (the prefill's fast exp2 / rcp form vs the decode's tanhf)
    "gelu-d128": M.ModelConfig(dim=512, hidden_dim=1024, head_dim=128, n_layers=2, n_heads=4, n_kv_heads=2,
                               vocab_size=1024, max_seq_len=320, rope_theta=1e6, act=M.GELU, weight_dtype=M.F16),
    # QKV N 1280 = 4 x 320, Wo / W2 N 768 = 4 x 192, vocab 1920 = 10 x 192: the 192 / 320 tile widths
    "d768": M.ModelConfig(dim=768, hidden_dim=1536, head_dim=128, n_layers=2, n_heads=6, n_kv_heads=2,
                          vocab_size=1920, max_seq_len=320, rope_theta=1e6, act=M.SILU, weight_dtype=M.F16),
}


@pytest.mark.parametrize("cfg_name", ["gqa-d128", "d768"])
@pytest.mark.parametrize("form", ["auto", "auto-qkv2", "g16-256", "g16-256-2ph", "g16-128", "g16-128-2ph", "g16-192",
                                  "g16-192-2ph", "g16-320", "g16-256-nopersist"])
def test_prefill_forms_match_decode(form, cfg_name):
    """The whole prefill in each GEMM form (incl. the vocab-tiled logits epilogue, the
    one-launch two-depth QKV GEMM ("auto") and the k | v launch at a column offset over
    the [hi | lo] operand ("auto-qkv2", forced widths))."""
    cfg = CFGS[cfg_name]
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=4)
    tokens = np.random.default_rng(5).integers(0, cfg.vocab_size, size=90).astype(np.int32)
    dec_p = R.Decoder(dm)
    dec_p.set_prefill_forms(FORMS[form])
    dec_d = R.Decoder(dm)
    try:
        err = np.max(np.abs(dec_p.prefill(tokens)[:89] - _decode_logprobs(dec_d, tokens)))
        assert err <= LP_ATOL, (form, err)
    finally:
        dec_p.close()
        dec_d.close()
        dm.close()


@pytest.mark.parametrize("name", list(CFGS))
@pytest.mark.parametrize("n", [1, 61, 200])
def test_prefill_matches_decode(name, n):
    """Per-position log p(next) of one prefill pass vs the decode engine run
    position by position (the reference's perplexity loop), same weights."""
    cfg = CFGS[name]
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=3)
    rng = np.random.default_rng(n)
    tokens = rng.integers(0, cfg.vocab_size, size=n).astype(np.int32)
    dec_p = R.Decoder(dm)
    lp_p = dec_p.prefill(tokens)
    dec_d = R.Decoder(dm)
    lp_d = _decode_logprobs(dec_d, tokens)
    err = np.max(np.abs(lp_p[: n - 1] - lp_d)) if n > 1 else 0.0
    assert lp_p[n - 1] == 0.0
    assert err <= LP_ATOL, (name, n, err)
    # the KV cache the prefill wrote drives the decoder: the next step's logits agree
    nxt = int(rng.integers(0, cfg.vocab_size))
    if n < cfg.max_seq_len:
        lg_p = dec_p.forward(nxt, n)
        lg_d = dec_d.forward(int(tokens[-1]), n - 1) if n > 0 else None
        lg_d = dec_d.forward(nxt, n)
        rel = np.max(np.abs(lg_p - lg_d)) / np.max(np.abs(lg_d))
        assert rel < 5e-3, rel
    dec_p.close()
    dec_d.close()
    dm.close()


@pytest.mark.parametrize("cfg_name", ["gqa-d128", "d768", "gelu-d128"])
@pytest.mark.parametrize("n", [1, 5, 16, 17, 33, 64])
def test_prefill_short_prompt_paths(cfg_name, n):
    """Short prompts (T <= 64) run the split-K skinny GEMMs (prefill_skinny.h): their
    log p and the KV cache they leave (next decode step's logits) against the decode
    engine and against the 256-row-tile path of the same prompt (form skinny:0);
    every M-tile count 1..4 and the row tails."""
    cfg = CFGS[cfg_name]
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=8)
    tokens = np.random.default_rng(100 + n).integers(0, cfg.vocab_size, size=n).astype(np.int32)
    dec_s = R.Decoder(dm)
    dec_l = R.Decoder(dm)
    dec_l.set_prefill_forms("skinny:0")
    dec_r = R.Decoder(dm)
    dec_r.set_prefill_forms("skl:0")  # the skinny GEMMs' weights as register loads
    dec_d = R.Decoder(dm)
    try:
        lp_s, lp_l, lp_r = dec_s.prefill(tokens), dec_l.prefill(tokens), dec_r.prefill(tokens)
        np.testing.assert_array_equal(lp_s, lp_r)  # LDS-DMA or register weights: the same MFMA sequence
        np.testing.assert_allclose(lp_s, lp_l, atol=2e-3)  # the same f16 operands, another f32 sum order
        if n > 1:
            assert np.max(np.abs(lp_s[: n - 1] - _decode_logprobs(dec_d, tokens))) <= LP_ATOL
        dec_d.forward(int(tokens[-1]), n - 1)
        nxt = 7
        lg_s, lg_d = dec_s.forward(nxt, n), dec_d.forward(nxt, n)
        assert np.max(np.abs(lg_s - lg_d)) / np.max(np.abs(lg_d)) < 5e-3
    finally:
        dec_s.close()
        dec_l.close()
        dec_r.close()
        dec_d.close()
        dm.close()


def test_bench_prefill_leg():
    """bench.py's config-4 leg (the `prefill` object of the default line) on a small
    model: the fields the driver reads, a finite MFMA rate, and its spot check of the
    prefill's log p against the decode engine within LP_ATOL."""
    import bench

    R = rt()
    out = bench.prefill_leg(R, M, model="small", n=200, iters=1, check=8)
    assert out["unit"] == "ms" and out["value"] > 0 and out["higher_is_better"] is False
    rl = out["roofline"]
    assert rl["bound"] == "mfma" and 0 < rl["achieved"] and 0 < rl["frac"] < 1
    assert out["flops"] > 0 and out["tok_per_s"] > 0
    assert out["spot_check"]["max_abs_dlogp_vs_decode"] <= LP_ATOL
    assert out["split_form"]["value"] > 0 and out["split_form"]["max_abs_dlogp_vs_decode"] <= LP_ATOL


def _f16_twin(cfg8, t8):
    """The f16 model whose weights are the E5M2 model's, upcast exactly (byte b -> f16 bits
    b << 8): what the fp8 prefill's dequantised copy must compute with."""
    t16 = {}
    for name, a in t8.items():
        t16[name] = a if a.dtype == np.float32 else (a.astype(np.uint16) << 8).view(np.float16)
    return cfg8.with_(weight_dtype=M.F16), t16


@pytest.mark.parametrize("cfg_name", ["gqa-d128", "d768"])
@pytest.mark.parametrize("n", [13, 200])
def test_fp8_prefill_equals_f16_twin(cfg_name, n):
    """an fp8 (E5M2) model through yalm_prefill (per-layer exact upcast of
    the weights to f16, then the f16 MFMA GEMMs; the short-prompt skinny path at 13) is BIT
    for bit the prefill of its f16 twin -- log p and the KV cache (the next decode step's
    logits) -- and matches the fp8 decode engine run position by position within LP_ATOL."""
    cfg8 = CFGS[cfg_name].with_(weight_dtype=M.F8E5M2)
    t8 = M.synth_host_tensors(cfg8, seed=11)
    cfg16, t16 = _f16_twin(cfg8, t8)
    R = rt()
    dm8, dm16 = R.DeviceModel.from_arrays(cfg8, t8), R.DeviceModel.from_arrays(cfg16, t16)
    kvb = cfg8.max_seq_len * cfg8.kv_dim * 2
    caches = [[R.lib.yalm_alloc(kvb) for _ in range(2 * cfg8.n_layers)] for _ in range(2)]  # caller-owned K / V
    d8 = R.Decoder(dm8, kv_caches=list(zip(caches[0][0::2], caches[0][1::2])))
    d16 = R.Decoder(dm16, kv_caches=list(zip(caches[1][0::2], caches[1][1::2])))
    dd = R.Decoder(dm8)
    try:
        tokens = np.random.default_rng(31 + n).integers(0, cfg8.vocab_size, size=n).astype(np.int32)
        lp8, lp16 = d8.prefill(tokens), d16.prefill(tokens)
        np.testing.assert_array_equal(lp8, lp16)
        for p8, p16 in zip(caches[0], caches[1]):  # every K / V cache row the prefill wrote, bit for bit
            a, b = np.empty(kvb, np.uint8), np.empty(kvb, np.uint8)
            R.check(R.lib.yalm_download(a.ctypes.data, p8, kvb))
            R.check(R.lib.yalm_download(b.ctypes.data, p16, kvb))
            np.testing.assert_array_equal(a, b)
        assert np.max(np.abs(lp8[: n - 1] - _decode_logprobs(dd, tokens))) <= LP_ATOL
    finally:
        for h in (d8, d16, dd, dm8, dm16):
            h.close()
        for p in caches[0] + caches[1]:
            R.lib.yalm_free(p)


def test_prefill_range_guard_scales_glu_output():
    """a GLU product above 65504 (the f16 range; the reference keeps it in
    f32, infer.cpp:360-375) must not become inf. models.REALISTIC's spike layer gives one at
    every position: the range guard re-runs the pass with that layer's GLU output scaled by an
    exact power of two (prefill.h range_note), so log p and the next decode step match the
    decode engine, which keeps the product in f32."""
    cfg = M.LLAMA_32_3B.with_(n_layers=2, max_seq_len=256)  # the spike needs the real dims' norms
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=4, real=M.REALISTIC)
    dec_p, dec_d = R.Decoder(dm), R.Decoder(dm)
    try:
        for n in (17, 150):  # the skinny and the large-tile GEMMs
            tokens = np.random.default_rng(n).integers(0, cfg.vocab_size, size=n).astype(np.int32)
            lp = dec_p.prefill(tokens)
            passes, scaled = dec_p.prefill_info()
            assert passes == 2 and scaled == 1, (passes, scaled)
            assert np.all(np.isfinite(lp))
            ld = _decode_logprobs(dec_d, tokens)
            assert np.max(np.abs(lp[: n - 1] - ld)) <= LP_ATOL
            dec_d.forward(int(tokens[-1]), n - 1)
            lg_p, lg_d = dec_p.forward(7, n), dec_d.forward(7, n)
            assert np.max(np.abs(lg_p - lg_d)) / np.max(np.abs(lg_d)) < 5e-3
        # a model that fits: one pass
        dmu = R.DeviceModel.synthetic(cfg, seed=4)
        du = R.Decoder(dmu)
        du.prefill(np.arange(40, dtype=np.int32))
        assert du.prefill_info() == (1, 0)
        du.close()
        dmu.close()
    finally:
        dec_p.close()
        dec_d.close()
        dm.close()


def test_prefill_range_guard_refuses_unscalable_operand():
    """An operand the guard does not rescale (here the normalised x: an rms_att weight of
    1e6 puts one column of it past 65504) is refused with YALM_ERR_UNSUPPORTED instead of
    returning inf / NaN log-probs."""
    cfg = CFGS["gqa-d128"]
    t = M.synth_host_tensors(cfg, seed=4)
    t["model.layers.1.attn.norm.weight"][5] = 1e6
    R = rt()
    dm = R.DeviceModel.from_arrays(cfg, t)
    dec = R.Decoder(dm)
    try:
        with pytest.raises(R.YalmError) as ei:
            dec.prefill(np.arange(30, dtype=np.int32))
        assert "yalm error 3" in str(ei.value) and "normalised x" in str(ei.value), str(ei.value)
    finally:
        dec.close()
        dm.close()


@pytest.mark.parametrize("cfg_name", ["gqa-d128", "d768", "small-d64"])
@pytest.mark.parametrize("n", [40, 200])
def test_prefill_split_precision_form(cfg_name, n):
    """the split-operand form (yalm_set_prefill_precision SPLIT: the
    normalised x, Q, P, O and H as f16 [hi | lo] pairs, ~22 bits) against the decode engine
    (f32 activations, pinned to the oracle): an order of magnitude inside the fast form's
    LP_ATOL, and closer than the fast form on the same prompt; the KV cache it leaves drives
    the decoder. (T = 40: the short-prompt path switches to the large tiles in this form.)"""
    cfg = CFGS[cfg_name]
    R = rt()
    dm = R.DeviceModel.synthetic(cfg, seed=12)
    tokens = np.random.default_rng(7 + n).integers(0, cfg.vocab_size, size=n).astype(np.int32)
    dec_s, dec_f, dec_d = R.Decoder(dm), R.Decoder(dm), R.Decoder(dm)
    dec_s.set_prefill_precision(R.PREFILL_SPLIT)
    try:
        lp_s, lp_f = dec_s.prefill(tokens)[: n - 1], dec_f.prefill(tokens)[: n - 1]
        ld = _decode_logprobs(dec_d, tokens)
        es, ef = np.max(np.abs(lp_s - ld)), np.max(np.abs(lp_f - ld))
        print(f"{cfg_name} T {n}: max |d log p| split {es:.2e}, fast {ef:.2e}")
        assert es <= LP_ATOL / 10, es
        assert es < ef, (es, ef)
        dec_d.forward(int(tokens[-1]), n - 1)
        lg_s, lg_d = dec_s.forward(5, n), dec_d.forward(5, n)
        assert np.max(np.abs(lg_s - lg_d)) / np.max(np.abs(lg_d)) < 1e-3
    finally:
        for h in (dec_s, dec_f, dec_d, dm):
            h.close()
