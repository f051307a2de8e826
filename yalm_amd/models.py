"""Model configuration (reference Config, model.h:41-68 / model.cpp:17-75),
.yalm tensor naming (model.cpp:347-378) and synthetic random-weight models
of real shapes (there is no network for checkpoints: see DESIGN.md).
"""

from __future__ import annotations

import dataclasses

import numpy as np

F32, F16, BF16, F8E5M2 = 0, 1, 2, 3
GELU, SILU = 0, 1
FLT_MAX = 3.4028234663852886e38
KV_SINKS = 2  # model.h:12

DTYPE_NAMES = {"fp32": F32, "fp16": F16, "fp8": F8E5M2}
DTYPE_STRINGS = {F32: "F32", F16: "F16", F8E5M2: "F8_E5M2"}
DTYPE_BYTES = {F32: 4, F16: 2, F8E5M2: 1}


@dataclasses.dataclass
class ModelConfig:
    dim: int
    hidden_dim: int
    head_dim: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    vocab_size: int
    max_seq_len: int
    rope_theta: float = 10000.0
    rotary_dim: int = 0
    norm_eps: float = 1e-5
    act: int = SILU
    qkv_clip: float = FLT_MAX
    weight_dtype: int = F16
    tied: bool = False
    bos_token_id: int = 1
    eos_token_id: int = 2

    def __post_init__(self):
        if not self.rotary_dim:
            self.rotary_dim = self.head_dim

    @property
    def q_dim(self):
        return self.n_heads * self.head_dim

    @property
    def kv_dim(self):
        return self.n_kv_heads * self.head_dim

    def with_(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)

    def weight_bytes_per_token(self) -> int:
        """Algorithmic HBM bytes read per decode token, excluding the KV cache
        (SURVEY.md §8d): every layer's weights + norms, one embedding row, the
        final norm and the classifier."""
        wb = DTYPE_BYTES[self.weight_dtype]
        per_layer = 2 * self.dim * 4
        per_layer += (self.q_dim + 2 * self.kv_dim) * self.dim * wb  # wq wk wv
        per_layer += self.dim * self.q_dim * wb  # wo
        per_layer += 3 * self.dim * self.hidden_dim * wb  # w1 w2 w3
        return self.n_layers * per_layer + self.dim * wb + self.dim * 4 + self.vocab_size * self.dim * wb

    def kv_bytes_per_token(self, kv_len: int) -> int:
        """fp16 K and V rows read by attention at kv_len (2 * 2 B * kv_dim per row, per layer)."""
        return self.n_layers * 2 * 2 * self.kv_dim * kv_len

    def metadata(self) -> dict:
        """__metadata__ strings as convert.py writes them (convert.py:59-81)."""
        inv = {v: k for k, v in DTYPE_NAMES.items()}
        md = {
            "arch": "MistralForCausalLM",
            "dtype": inv[self.weight_dtype],
            "dim": str(self.dim),
            "hidden_dim": str(self.hidden_dim),
            "head_dim": str(self.head_dim),
            "n_layers": str(self.n_layers),
            "n_heads": str(self.n_heads),
            "n_kv_heads": str(self.n_kv_heads),
            "vocab_size": str(self.vocab_size),
            "max_seq_len": str(self.max_seq_len),
            "bos_token_id": str(self.bos_token_id),
            "eos_token_id": str(self.eos_token_id),
            "rope_theta": str(self.rope_theta),
            "rotary_dim": str(self.rotary_dim),
            "norm_eps": str(self.norm_eps),
            "norm_type": "rmsnorm",
            "act_type": "silu" if self.act == SILU else "gelu",
        }
        if self.qkv_clip != FLT_MAX:
            md["qkv_clip"] = str(self.qkv_clip)
        return md


def config_from_metadata(md: dict, context: int = 0, tied: bool = False) -> ModelConfig:
    """Config::from_yalm (model.cpp:17-75)."""
    dtype = md["dtype"]
    if dtype not in DTYPE_NAMES:
        raise ValueError(f"FATAL: unsupported dtype: {dtype}")
    max_seq_len = min(int(md["max_seq_len"]), 4096)  # model.cpp:33
    if context:
        max_seq_len = context
    act_str = md.get("act_type", "gelu")
    act = SILU if act_str == "silu" else GELU
    return ModelConfig(
        dim=int(md["dim"]),
        hidden_dim=int(md["hidden_dim"]),
        head_dim=int(md["head_dim"]),
        n_layers=int(md["n_layers"]),
        n_heads=int(md["n_heads"]),
        n_kv_heads=int(md["n_kv_heads"]),
        vocab_size=int(md["vocab_size"]),
        max_seq_len=max_seq_len,
        rope_theta=float(np.float32(float(md["rope_theta"]))),
        rotary_dim=int(md["rotary_dim"]),
        norm_eps=float(np.float32(float(md.get("norm_eps", "1e-5")))),
        act=act,
        qkv_clip=float(np.float32(float(md["qkv_clip"]))) if "qkv_clip" in md else FLT_MAX,
        weight_dtype=DTYPE_NAMES[dtype],
        tied=tied,
        bos_token_id=int(md.get("bos_token_id", "1")),
        eos_token_id=int(md.get("eos_token_id", "2")),
    )


# Real shapes (HF config.json values). Weights are synthetic.
MISTRAL_7B = ModelConfig(
    dim=4096, hidden_dim=14336, head_dim=128, n_layers=32, n_heads=32, n_kv_heads=8, vocab_size=32000,
    max_seq_len=4096, rope_theta=1e6, norm_eps=1e-5, act=SILU, weight_dtype=F16, tied=False,
)
LLAMA_32_3B = ModelConfig(
    dim=3072, hidden_dim=8192, head_dim=128, n_layers=28, n_heads=24, n_kv_heads=8, vocab_size=128256,
    max_seq_len=4096, rope_theta=5e5, norm_eps=1e-5, act=SILU, weight_dtype=F16, tied=True,
)
TINY = ModelConfig(
    dim=64, hidden_dim=128, head_dim=16, n_layers=2, n_heads=4, n_kv_heads=2, vocab_size=384, max_seq_len=64,
    rope_theta=10000.0, act=SILU, weight_dtype=F16,
)
SMALL = ModelConfig(
    dim=512, hidden_dim=1536, head_dim=64, n_layers=4, n_heads=8, n_kv_heads=2, vocab_size=2048, max_seq_len=256,
    rope_theta=10000.0, act=SILU, weight_dtype=F16,
)
PRESETS = {"mistral-7b": MISTRAL_7B, "llama-3.2-3b": LLAMA_32_3B, "tiny": TINY, "small": SMALL}


def layer_names(l: int) -> dict:
    p = f"model.layers.{l}."
    return {
        "rms_att": p + "attn.norm.weight",
        "rms_ffn": p + "mlp.norm.weight",
        "wq": p + "attn.wq.weight",
        "wk": p + "attn.wk.weight",
        "wv": p + "attn.wv.weight",
        "wo": p + "attn.wo.weight",
        "w1": p + "mlp.w1.weight",
        "w2": p + "mlp.w2.weight",
        "w3": p + "mlp.w3.weight",
    }


def tensor_shapes(c: ModelConfig) -> dict:
    """name -> (shape, is_norm) in .yalm naming (model.cpp:351-377)."""
    out = {"model.embed.weight": ((c.vocab_size, c.dim), False), "model.norm.weight": ((c.dim,), True)}
    if not c.tied:
        out["model.output.weight"] = ((c.vocab_size, c.dim), False)
    for l in range(c.n_layers):
        n = layer_names(l)
        out[n["rms_att"]] = ((c.dim,), True)
        out[n["rms_ffn"]] = ((c.dim,), True)
        out[n["wq"]] = ((c.q_dim, c.dim), False)
        out[n["wk"]] = ((c.kv_dim, c.dim), False)
        out[n["wv"]] = ((c.kv_dim, c.dim), False)
        out[n["wo"]] = ((c.dim, c.q_dim), False)
        out[n["w1"]] = ((c.hidden_dim, c.dim), False)
        out[n["w2"]] = ((c.dim, c.hidden_dim), False)
        out[n["w3"]] = ((c.hidden_dim, c.dim), False)
    return out


# ---- tensor parallelism (include/yalm_hip.h "tensor parallelism") ----
def tp_shard(c: ModelConfig, name: str, rank: int, size: int):
    """Megatron split of one .yalm tensor for rank/size: ("rows"|"cols", start,
    count) of its [out][in] matrix, or None when replicated (norms, embedding).
    The classifier ("model.output.weight", or the tied embedding used as
    wcls) is split by vocabulary rows."""
    if size == 1:
        return None
    if name in ("model.output.weight", "tp.wcls"):
        n = c.vocab_size // size
        return ("rows", rank * n, n)
    kind = name.rsplit(".", 2)[-2] if name.startswith("model.layers.") else None
    if kind in ("wq",):
        n = c.q_dim // size
        return ("rows", rank * n, n)
    if kind in ("wk", "wv"):
        n = c.kv_dim // size
        return ("rows", rank * n, n)
    if kind == "wo":
        n = c.q_dim // size
        return ("cols", rank * n, n)
    if kind in ("w1", "w3"):
        n = c.hidden_dim // size
        return ("rows", rank * n, n)
    if kind == "w2":
        n = c.hidden_dim // size
        return ("cols", rank * n, n)
    return None


def tp_check(c: ModelConfig, size: int) -> None:
    if c.n_heads % size or c.n_kv_heads % size or c.hidden_dim % size or c.vocab_size % size:
        raise ValueError(f"tensor parallel size {size} must divide n_heads, n_kv_heads, hidden_dim and vocab_size")


def shard_array(c: ModelConfig, name: str, a, rank: int, size: int):
    """Host-side slice of a full tensor (numpy) for rank/size."""
    sh = tp_shard(c, name, rank, size)
    if sh is None:
        return a
    kind, start, n = sh
    return a[start:start + n] if kind == "rows" else a[:, start:start + n]


# ---- deterministic synthetic init (same hash on device and in the oracle) ----
WEIGHT_SCALE = 0.035  # uniform [-a, a): std 0.02, the usual init scale
NORM_SCALE, NORM_OFFSET = 0.2, 1.0


def synth_seed(base: int, name: str) -> int:
    """Stable 64-bit seed per tensor name."""
    h = 1469598103934665603
    for ch in f"{base}:{name}".encode():
        h = ((h ^ ch) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def synth_params(name: str, is_norm: bool, peak: float = 1.0, real: "Realistic" = None, tied: bool = False):
    """(scale, offset) of a synthetic tensor. peak > 1 scales the final norm weight, so the
    logits spread peak x wider: the default model's logits have a std of ~1.2 (near-uniform
    next-token distributions). real: the realistic model's Wq / Wk gain and final-norm scale
    (its other features are patches, realistic_patch)."""
    if real is not None:
        peak = peak * real.final_norm
    if is_norm:
        k = peak if name == "model.norm.weight" else 1.0
        return NORM_SCALE * k, NORM_OFFSET * k
    if real is not None and name.endswith((".attn.wq.weight", ".attn.wk.weight")):
        return WEIGHT_SCALE * (real.qk_gain_tied if tied else real.qk_gain), 0.0
    if real is not None and name in ("model.embed.weight", "model.output.weight"):
        return WEIGHT_SCALE * (real.emb_gain_tied if tied else real.emb_gain), 0.0
    if real is not None and name.endswith((".attn.wo.weight", ".mlp.w2.weight")):
        return WEIGHT_SCALE * real.branch_gain, 0.0
    return WEIGHT_SCALE, 0.0


PEAKED = 8.0  # synth_params(peak=PEAKED): the final norm x 8 (round 5; a pure logit scale)


# ---- the realistic synthetic model ----
# Uniform random weights give hidden states no trained checkpoint has: near-uniform attention,
# no outlier channels, GLU products of order 1. This model keeps the deterministic synthetic
# weights and adds the regimes real checkpoints have (each a stated, seed-independent patch,
# applied identically to the device model and the oracle's host tensors):
#   * peaked attention softmax: Wq and Wk x qk_gain (reference infer.cpp:216-248 softmax);
#   * "massive activation" residual channels: three embedding columns set to outlier values of
#     10^2..10^3 (E5M2-exact), the W2 rows of those channels x w2_outlier_gain in every layer
#     (they keep growing), and -- as trained checkpoints have -- small norm weights there;
#   * a GLU spike: in one layer, glu_rows W1 / W3 rows read the largest outlier channel with
#     weight glu_value, so act(W1 x) * (W3 x) exceeds 65504 (the f16 range) at every position
#     (reference infer.cpp:360-375 keeps it in f32); their W2 columns x w2_spike_cols;
#   * a final-norm scale that is not a power of two (logits not an exact multiple of the
#     uniform model's);
#   * a residual stream that dominates its branches, as in trained models: the embedding and
#     classifier x emb_gain, Wo and W2 x branch_gain. With full-size branches a random-weight
#     model is chaotic (measured on the oracle, Mistral dims: a one-ulp change of ONE embedding
#     element moves the logits by 1.6e-3 at 16 layers with the other features on, 2.9e-4 for
#     the uniform model), so no two correct fp32 summation orders would agree to 1e-3 at 32
#     layers; with these gains it moves them by 4.4e-5 at 32 layers.
# Measured on the oracle (Mistral dims, 32 layers; Llama-3.2-3B dims, 28, tied): attention
# top weight median 0.89 / 0.86 in the last layers, residual outliers ~100 / 64 / 258 against
# other channels of std ~0.4 / 0.14, the layer-1 GLU product 1.6e5 / 8.4e4 at every position,
# top-1 next-token probability median 0.54 (Mistral) / 0.997 (Llama: the tied classifier
# favours the input token; log p of a uniformly random next token ~ -18).
@dataclasses.dataclass(frozen=True)
class Realistic:
    qk_gain: float = 24.0
    emb_gain: float = 16.0
    # tied models (the classifier IS the embedding): a residual dominated by a x16 embedding
    # makes the input token win by ~250 logits (measured, Llama dims); x4 leaves the layers'
    # updates a share of it (top-1 gap ~15, an unlikely token's log p ~ -18, finite in the
    # reference's f32 sample_prob), with the Wq / Wk gain raised to keep attention peaked
    emb_gain_tied: float = 4.0
    qk_gain_tied: float = 96.0
    branch_gain: float = 0.125
    final_norm: float = 4.5
    outliers: tuple = (96.0, -64.0, 256.0)
    outlier_norm: float = 1.0 / 64.0
    w2_outlier_gain: float = 8.0
    glu_value: float = 448.0
    glu_rows: int = 4
    w2_spike_cols: float = 1.0 / 4096.0


REALISTIC = Realistic()


def realistic_channels(c: ModelConfig) -> list:
    return [(c.dim * k) // 7 + 5 for k in (1, 3, 5)]


def realistic_glu_rows(c: ModelConfig, real: Realistic = REALISTIC) -> list:
    return [(c.hidden_dim * (k + 1)) // (real.glu_rows + 1) + 3 for k in range(real.glu_rows)]


def realistic_spike_layer(c: ModelConfig) -> int:
    return 1 if c.n_layers > 1 else 0


def realistic_names(c: ModelConfig) -> list:
    """The tensors realistic_patch changes."""
    out = ["model.embed.weight", "model.norm.weight"]
    for l in range(c.n_layers):
        n = layer_names(l)
        out += [n["rms_att"], n["rms_ffn"], n["w2"]]
        if l == realistic_spike_layer(c):
            out += [n["w1"], n["w3"]]
    return out


def decode_weights(a: np.ndarray, dtype: int) -> np.ndarray:
    """Stored weights (f32 / f16 / E5M2 bytes) -> float32, exactly."""
    if dtype == F8E5M2:
        return e5m2_to_f32(a)
    return a.astype(np.float32)


def encode_weights(v: np.ndarray, dtype: int) -> np.ndarray:
    """float32 -> stored weights: f16 round to nearest even; E5M2 through f16, then round
    to nearest even on the byte (the initialiser's rule, synth_array)."""
    v = np.asarray(v, np.float32)
    if dtype == F32:
        return v
    h16 = v.astype(np.float16)
    if dtype == F16:
        return h16
    hb = h16.view(np.uint16).astype(np.uint32)
    return ((hb + 0x7F + ((hb >> 8) & 1)) >> 8).astype(np.uint8)


def realistic_patch(c: ModelConfig, name: str, a: np.ndarray, real: Realistic = REALISTIC) -> None:
    """Patch one synthetic tensor (numpy, storage dtype, in place) into the realistic model."""
    ch = realistic_channels(c)
    wt = c.weight_dtype
    if name == "model.embed.weight":
        for cc, v in zip(ch, real.outliers):
            a[:, cc] = encode_weights(np.full(a.shape[0], v, np.float32), wt)
        return
    if name == "model.norm.weight" or name.endswith((".attn.norm.weight", ".mlp.norm.weight")):
        a[ch] = (a[ch] * np.float32(real.outlier_norm)).astype(np.float32)
        return
    if not name.startswith("model.layers."):
        return
    l = int(name.split(".")[2])
    n = layer_names(l)
    spike = l == realistic_spike_layer(c)
    rows = realistic_glu_rows(c, real)
    if name == n["w2"]:
        a[ch, :] = encode_weights(decode_weights(a[ch, :], wt) * np.float32(real.w2_outlier_gain), wt)
        if spike:
            a[:, rows] = encode_weights(decode_weights(a[:, rows], wt) * np.float32(real.w2_spike_cols), wt)
    elif spike and name in (n["w1"], n["w3"]):
        for r in rows:
            a[r, ch[2]] = encode_weights(np.array([real.glu_value], np.float32), wt)[0]


def apply_realistic(c: ModelConfig, tensors: dict, real: Realistic = REALISTIC) -> dict:
    for name in realistic_names(c):
        realistic_patch(c, name, tensors[name], real)
    return tensors


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)).astype(np.uint64)
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)).astype(np.uint64)
    return x ^ (x >> np.uint64(31))


def synth_array(n: int, dtype: int, seed: int, scale: float, offset: float = 0.0) -> np.ndarray:
    """numpy twin of the device/oracle initialiser (small sizes only)."""
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64)
        h = _splitmix64(np.uint64(seed) ^ (i * np.uint64(0xD1B54A32D192ED03)))
    s = ((h >> np.uint64(40)).astype(np.int64) - 8388608).astype(np.float32)
    k = np.float32(scale) * np.float32(1.0 / 8388608.0)
    if dtype == F32:
        # fmaf(s, k, offset): exact product (24-bit x 24-bit fits in f64), one rounding
        return (s.astype(np.float64) * np.float64(k) + np.float64(np.float32(offset))).astype(np.float32)
    v = (s * k).astype(np.float32)
    h16 = v.astype(np.float16)
    if dtype == F16:
        return h16
    hb = h16.view(np.uint16).astype(np.uint32)
    return ((hb + 0x7F + ((hb >> 8) & 1)) >> 8).astype(np.uint8)


def synth_host_tensors(c: ModelConfig, seed: int = 1, peak: float = 1.0, real: Realistic = None) -> dict:
    """All tensors of a synthetic model as numpy arrays (norms f32, weights in
    c.weight_dtype storage: f32 / f16 / uint8 E5M2 bits); real: the realistic model."""
    out = {}
    for name, (shape, is_norm) in tensor_shapes(c).items():
        scale, offset = synth_params(name, is_norm, peak, real, c.tied)
        dt = F32 if is_norm else c.weight_dtype
        n = int(np.prod(shape))
        out[name] = synth_array(n, dt, synth_seed(seed, name), scale, offset).reshape(shape)
    return apply_realistic(c, out, real) if real is not None else out


def e5m2_to_f32(b: np.ndarray) -> np.ndarray:
    """Exact: the E5M2 byte b is the f16 with bits b << 8."""
    return (b.astype(np.uint16) << 8).view(np.float16).astype(np.float32)


def rope_inv_freq(c: ModelConfig) -> np.ndarray:
    """The reference's compiled RoPE frequencies (infer.cpp:203 under -ffast-math:
    powf(theta, -(j * (1 / rotary_dim))), the form the decoder uploads); numpy's float32
    power stands in for glibc powf (may differ by an ulp: analysis tools only)."""
    j = np.arange(0, c.head_dim, 2).astype(np.float32)
    rinv = np.float32(1.0) / np.float32(c.rotary_dim)
    f = np.power(np.float32(c.rope_theta), -(j * rinv).astype(np.float32)).astype(np.float32)
    f[j >= c.rotary_dim] = 0.0
    return f.astype(np.float32)


def kv_indices(max_seq_len: int, pos: int):
    """infer.cpp:483-485"""
    kv_sink = KV_SINKS if pos >= max_seq_len else 0
    kv_pos = kv_sink + (pos - kv_sink) % (max_seq_len - kv_sink)
    kv_len = max_seq_len if pos >= max_seq_len else pos + 1
    return kv_sink, kv_pos, kv_len


def nbytes_model(c: ModelConfig) -> int:
    wb = DTYPE_BYTES[c.weight_dtype]
    tot = 0
    for _, (shape, is_norm) in tensor_shapes(c).items():
        tot += int(np.prod(shape)) * (4 if is_norm else wb)
    return tot

