"""ctypes wrapper of the CPU ORACLE (oracle/liboracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module, as the checker. It restates /root/reference/src/infer.cpp (see
oracle/yalm_oracle.h for the pinning status).
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from yalm_amd import models as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")


def _load():
    if not os.path.exists(ORACLE_LIB):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    return ctypes.CDLL(ORACLE_LIB)


olib = _load()
vp, ci, cf, cz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t


class OConfig(ctypes.Structure):
    _fields_ = [
        ("dim", ci), ("hidden_dim", ci), ("head_dim", ci), ("n_layers", ci), ("n_heads", ci),
        ("n_kv_heads", ci), ("vocab_size", ci), ("max_seq_len", ci), ("rope_theta", cf), ("rotary_dim", ci),
        ("norm_eps", cf), ("act", ci), ("qkv_clip", cf), ("weight_dtype", ci),
    ]


class OBlock(ctypes.Structure):
    _fields_ = [(n, vp) for n in ("rms_att", "rms_ffn", "wq", "wk", "wv", "wo", "w1", "w2", "w3", "key_cache",
                                  "value_cache")]


class OModel(ctypes.Structure):
    _fields_ = [("c", OConfig), ("emb", vp), ("rms_final", vp), ("wcls", vp), ("blocks", ctypes.POINTER(OBlock))]


class OState(ctypes.Structure):
    _fields_ = [(n, vp) for n in ("x", "xb", "xb2", "hb", "hb2", "q", "k", "v", "att", "logits")]


def _s(name, res, args):
    f = getattr(olib, name)
    f.restype = res
    f.argtypes = args


_s("orc_matmul_f32", None, [vp, vp, vp, ci, ci])
_s("orc_matmul_f16", None, [vp, vp, vp, ci, ci])
_s("orc_matmul_f8", None, [vp, vp, vp, ci, ci])
_s("orc_rmsnorm", None, [vp, vp, vp, ci, cf])
_s("orc_rope", None, [vp, ci, ci, ci, cf, ci])
_s("orc_softmax", None, [vp, vp, ci])
_s("orc_attn", None, [vp, vp, vp, vp, vp, ci, ci, ci])
_s("orc_mha", None, [vp, vp, vp, vp, vp, ci, ci, ci, ci, ci])
_s("orc_ffn", None, [vp, vp, vp, vp, vp, ci, ci, ci, ci])
_s("orc_block_forward", None, [ctypes.POINTER(OConfig), ctypes.POINTER(OBlock), ctypes.POINTER(OState), ci, ci, ci,
                               ci])
_s("orc_forward", None, [ctypes.POINTER(OModel), ctypes.POINTER(OState), ci, ci, ci])
_s("orc_sample_argmax", ci, [vp, ci])
_s("orc_sample_prob", cf, [vp, ci, ci])
_s("orc_synth_f32", None, [vp, cz, ctypes.c_uint64, cf, cf])
_s("orc_synth_f16", None, [vp, cz, ctypes.c_uint64, cf])
_s("orc_synth_f8", None, [vp, cz, ctypes.c_uint64, cf])
_s("orc_set_threads", None, [ci])
_s("orc_get_threads", ci, [])


def P(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"], "oracle needs contiguous arrays"
    return a.ctypes.data


def matmul(x, w, dtype):
    d, n = w.shape
    x = np.ascontiguousarray(x, np.float32)
    w = np.ascontiguousarray(w)
    out = np.zeros(d, np.float32)
    fn = {M.F32: olib.orc_matmul_f32, M.F16: olib.orc_matmul_f16, M.F8E5M2: olib.orc_matmul_f8}[dtype]
    fn(P(out), P(x), P(w), n, d)
    return out


def mha(kb, vb, q, head_dim, kv_len, max_seq_len, n_heads, n_kv_heads):
    kb = np.ascontiguousarray(kb, np.float16)
    vb = np.ascontiguousarray(vb, np.float16)
    q = np.ascontiguousarray(q, np.float32)
    xout = np.zeros(n_heads * head_dim, np.float32)
    att = np.zeros(n_heads * max_seq_len, np.float32)
    olib.orc_mha(P(xout), P(att), P(kb), P(vb), P(q), head_dim, kv_len, max_seq_len, n_heads, n_kv_heads)
    return xout, att


def attn(qh, kh, vh, head_dim, n_kv_heads, kv_len):
    qh = np.ascontiguousarray(qh, np.float32)
    kh = np.ascontiguousarray(kh, np.float16)
    vh = np.ascontiguousarray(vh, np.float16)
    xout = np.zeros(head_dim, np.float32)
    att = np.zeros(kv_len, np.float32)
    olib.orc_attn(P(xout), P(att), P(qh), P(kh), P(vh), head_dim, n_kv_heads, kv_len)
    return xout, att


def ffn(x, w1, w2, w3, act, dtype):
    hidden_dim, dim = w1.shape
    x = np.ascontiguousarray(x, np.float32)
    w1, w2, w3 = (np.ascontiguousarray(a) for a in (w1, w2, w3))
    out = np.zeros(dim, np.float32)
    olib.orc_ffn(P(out), P(x), P(w1), P(w2), P(w3), hidden_dim, dim, act, dtype)
    return out


def synth_host_tensors_fast(cfg: M.ModelConfig, seed: int = 1, peak: float = 1.0, real: "M.Realistic" = None) -> dict:
    """Full-size twin of DeviceModel.synthetic() built by the oracle's C
    initialiser (OpenMP): same hash, same bits; real: the realistic model's patches
    (models.realistic_patch) applied the same way."""
    out = {}
    for name, (shape, is_norm) in M.tensor_shapes(cfg).items():
        n = int(np.prod(shape))
        scale, offset = M.synth_params(name, is_norm, peak, real, cfg.tied)
        s = M.synth_seed(seed, name)
        if is_norm:
            a = np.empty(n, np.float32)
            olib.orc_synth_f32(P(a), n, s, scale, offset)
        elif cfg.weight_dtype == M.F32:
            a = np.empty(n, np.float32)
            olib.orc_synth_f32(P(a), n, s, scale, 0.0)
        elif cfg.weight_dtype == M.F16:
            a = np.empty(n, np.float16)
            olib.orc_synth_f16(P(a), n, s, scale)
        else:
            a = np.empty(n, np.uint8)
            olib.orc_synth_f8(P(a), n, s, scale)
        out[name] = a.reshape(shape)
    return M.apply_realistic(cfg, out, real) if real is not None else out


class OracleModel:
    """Model + InferenceState on the CPU (reference infer.cpp semantics)."""

    def __init__(self, cfg: M.ModelConfig, tensors: dict):
        self.cfg = cfg
        c = cfg
        self.t = {k: np.ascontiguousarray(v) for k, v in tensors.items()}
        self.oc = OConfig(c.dim, c.hidden_dim, c.head_dim, c.n_layers, c.n_heads, c.n_kv_heads, c.vocab_size,
                          c.max_seq_len, c.rope_theta, c.rotary_dim, c.norm_eps, c.act, c.qkv_clip, c.weight_dtype)
        self.kcache = [np.zeros((c.max_seq_len, c.kv_dim), np.float16) for _ in range(c.n_layers)]
        self.vcache = [np.zeros((c.max_seq_len, c.kv_dim), np.float16) for _ in range(c.n_layers)]
        self.blocks = (OBlock * c.n_layers)()
        for l in range(c.n_layers):
            n = M.layer_names(l)
            b = self.blocks[l]
            for k, name in n.items():
                setattr(b, k, P(self.t[name]))
            b.key_cache = P(self.kcache[l])
            b.value_cache = P(self.vcache[l])
        emb = self.t["model.embed.weight"]
        wcls = self.t.get("model.output.weight", emb)
        self.om = OModel(self.oc, P(emb), P(self.t["model.norm.weight"]), P(wcls), self.blocks)
        # xb2 holds the attention output (q_dim floats) and later the W2 output
        # (dim): the reference sizes it dim (its models have q_dim == dim); hb holds
        # the Wo output (dim floats, infer.cpp:332) before the GLU (hidden_dim): the
        # reference sizes it hidden_dim (its models have hidden_dim > dim)
        self.buf = {
            "x": np.zeros(c.dim, np.float32), "xb": np.zeros(c.dim, np.float32),
            "xb2": np.zeros(max(c.dim, c.q_dim), np.float32),
            "hb": np.zeros(max(c.hidden_dim, c.dim), np.float32), "hb2": np.zeros(c.hidden_dim, np.float32),
            "q": np.zeros(c.q_dim, np.float32), "k": np.zeros(c.kv_dim, np.float32),
            "v": np.zeros(c.kv_dim, np.float32), "att": np.zeros(c.n_heads * c.max_seq_len, np.float32),
            "logits": np.zeros(c.vocab_size, np.float32),
        }
        self.st = OState(**{k: P(v) for k, v in self.buf.items()})

    def forward(self, token: int, pos: int, mode: int = 1):
        olib.orc_forward(ctypes.byref(self.om), ctypes.byref(self.st), token, pos, mode)
        return self.buf["logits"].copy() if mode == 1 else None

    def block(self, layer, pos, kv_sink, kv_pos, kv_len):
        olib.orc_block_forward(ctypes.byref(self.oc), ctypes.byref(self.blocks[layer]), ctypes.byref(self.st), pos,
                               kv_sink, kv_pos, kv_len)

    @property
    def x(self):
        return self.buf["x"]

    def embed(self, token):
        e = self.t["model.embed.weight"][token]
        if self.cfg.weight_dtype == M.F8E5M2:
            return M.e5m2_to_f32(e)
        return e.astype(np.float32)

    def greedy(self, token: int, pos: int, n: int):
        """n argmax tokens, feeding each back (sampler.cpp:27-38)."""
        out = []
        for i in range(n):
            logits = self.forward(token, pos + i, 1)
            token = int(olib.orc_sample_argmax(P(logits), self.cfg.vocab_size))
            out.append(token)
        return out


def set_threads(n: int):
    olib.orc_set_threads(n)


def get_threads() -> int:
    return olib.orc_get_threads()
