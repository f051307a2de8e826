"""Independent float64 numpy restatement of the reference forward
(/root/reference/src/infer.cpp:254-523) — used to cross-check the C oracle
(which reproduces the reference's fp32 arithmetic order) and as a second,
order-free opinion on the GPU path. TEST INFRASTRUCTURE ONLY.
"""
import numpy as np

from yalm_amd import models as M


def w64(a, dtype):
    if dtype == M.F8E5M2 and a.dtype == np.uint8:
        return M.e5m2_to_f32(a).astype(np.float64)
    return a.astype(np.float64)


def rmsnorm(x, w, eps):
    return x / np.sqrt(np.mean(x * x) + eps) * w


def rope(v, head_dim, pos, theta, rotary_dim):
    v = v.copy()
    i = np.arange(0, v.shape[0], 2)
    j = i % head_dim
    freq = np.where(j >= rotary_dim, 0.0, 1.0 / np.power(float(np.float32(theta)), j / rotary_dim))
    ang = pos * freq
    c, s = np.cos(ang), np.sin(ang)
    v0, v1 = v[i].copy(), v[i + 1].copy()
    v[i] = v0 * c - v1 * s
    v[i + 1] = v0 * s + v1 * c
    return v


def silu(x):
    return x / (1 + np.exp(-x))


def gelu(x):
    return 0.5 * x * (1 + np.tanh(0.797885 * (x + 0.044715 * x ** 3)))


class RefModel:
    """allreduce / allgather: tensor-parallel hooks (identity for one device):
    with cfg = one rank's local dims and tensors = its shards (models.shard_array),
    x += allreduce(Wo_r o_r) and logits = allgather(Wcls_r x) restate the
    Megatron split of include/yalm_hip.h's yalm_decoder_create_tp."""

    def __init__(self, cfg: M.ModelConfig, tensors: dict, allreduce=None, allgather=None):
        self.allreduce = allreduce or (lambda v: v)
        self.allgather = allgather or (lambda v: v)
        self.c = cfg
        self.t = {k: w64(v, cfg.weight_dtype) if v.ndim == 2 else v.astype(np.float64) for k, v in tensors.items()}
        # the KV cache is fp16 in the reference (model.h:299-300)
        self.k = [np.zeros((cfg.max_seq_len, cfg.kv_dim), np.float16) for _ in range(cfg.n_layers)]
        self.v = [np.zeros((cfg.max_seq_len, cfg.kv_dim), np.float16) for _ in range(cfg.n_layers)]

    def block(self, l, x, pos, kv_sink, kv_pos, kv_len):
        c, t = self.c, self.t
        n = M.layer_names(l)
        xb = rmsnorm(x, t[n["rms_att"]], c.norm_eps)
        clip = c.qkv_clip
        q = np.clip(t[n["wq"]] @ xb, -clip, clip)
        k = np.clip(t[n["wk"]] @ xb, -clip, clip)
        v = np.clip(t[n["wv"]] @ xb, -clip, clip)
        q = rope(q, c.head_dim, pos, c.rope_theta, c.rotary_dim)
        k = rope(k, c.head_dim, pos, c.rope_theta, c.rotary_dim)
        self.k[l][kv_pos] = k.astype(np.float16)
        self.v[l][kv_pos] = v.astype(np.float16)
        for r in range(kv_sink):
            kk = rope(self.k[l][r].astype(np.float64), c.head_dim, 1, c.rope_theta, c.rotary_dim)
            self.k[l][r] = kk.astype(np.float16)
        G = c.n_heads // c.n_kv_heads
        K = self.k[l][:kv_len].astype(np.float64).reshape(kv_len, c.n_kv_heads, c.head_dim)
        V = self.v[l][:kv_len].astype(np.float64).reshape(kv_len, c.n_kv_heads, c.head_dim)
        out = np.zeros(c.q_dim)
        for h in range(c.n_heads):
            g = h // G
            s = K[:, g, :] @ q[h * c.head_dim:(h + 1) * c.head_dim] / np.sqrt(c.head_dim)
            p = np.exp(s - s.max())
            p /= p.sum()
            out[h * c.head_dim:(h + 1) * c.head_dim] = p @ V[:, g, :]
        x = x + self.allreduce(t[n["wo"]] @ out)
        xb = rmsnorm(x, t[n["rms_ffn"]], c.norm_eps)
        a = t[n["w1"]] @ xb
        hb = (silu(a) if c.act == M.SILU else gelu(a)) * (t[n["w3"]] @ xb)
        return x + self.allreduce(t[n["w2"]] @ hb)

    def forward(self, token, pos):
        c = self.c
        x = self.t["model.embed.weight"][token].copy()
        kv_sink, kv_pos, kv_len = M.kv_indices(c.max_seq_len, pos)
        for l in range(c.n_layers):
            x = self.block(l, x, pos, kv_sink, kv_pos, kv_len)
        x = rmsnorm(x, self.t["model.norm.weight"], c.norm_eps)
        wcls = self.t.get("model.output.weight", self.t.get("tp.wcls", self.t["model.embed.weight"]))
        return self.allgather(wcls @ x)
