"""HF checkpoint dir (config.json, tokenizer.json, *.safetensors) -> .yalm.

Own converter with the semantics of the reference /root/reference/convert.py
(numpy, no torch): metadata normalisation (convert.py:22-81), tokenizer blob
with sentencepiece '▁' -> ' ' or GPT-2 byte decoding and NUL -> BEL
(convert.py:83-125), Q/K rotary permutation to interleaved pairs
(permute_reverse, convert.py:145-158), f32 norms, weights cast to fp32 /
fp16 (round-to-nearest-even) / fp8 E5M2 (torch's fp8e5m2_from_fp32_value:
RNE, >= 2^16 -> inf), tied classifier when ``tie_word_embeddings`` is not
False (convert.py:200). MoE (Mixtral) checkpoints are out of scope.

Usage: python -m yalm_amd.convert [--dtype fp16] out.yalm hf_dir/
"""

from __future__ import annotations

import argparse
import json
import os

import numpy as np

from .yalmfile import read_yalm, write_yalm

SUPPORTED_ARCHITECTURES = ["LlamaForCausalLM", "MistralForCausalLM"]
SUPPORTED_DTYPES = ["fp32", "fp16", "fp8"]


def metadata_from_config(config: dict, dtype: str) -> dict:
    arch = config["architectures"][0]
    if arch not in SUPPORTED_ARCHITECTURES:
        raise ValueError(f"Architecture {arch} is not supported, must be one of {SUPPORTED_ARCHITECTURES}")
    if dtype not in SUPPORTED_DTYPES:
        raise ValueError(f"Data type {dtype} is not supported, must be one of {SUPPORTED_DTYPES}")
    head_dim = config.get("head_dim", config["hidden_size"] // config["num_attention_heads"])
    if config.get("attention_bias", False) or config.get("mlp_bias", False):
        raise ValueError("attention/mlp bias is not supported")
    if config["hidden_act"] not in ("gelu", "silu"):
        raise ValueError(f"unsupported hidden_act {config['hidden_act']}")
    md = {
        "arch": arch,
        "dtype": dtype,
        "dim": config["hidden_size"],
        "hidden_dim": config["intermediate_size"],
        "head_dim": head_dim,
        "n_layers": config["num_hidden_layers"],
        "n_heads": config["num_attention_heads"],
        "n_kv_heads": config.get("num_key_value_heads", config["num_attention_heads"]),
        "vocab_size": config["vocab_size"],
        "max_seq_len": config["max_position_embeddings"],
        "bos_token_id": config["bos_token_id"],
        "eos_token_id": config["eos_token_id"],
        "rope_theta": config.get("rope_theta", 10000.0),
        "rotary_dim": int(head_dim * config.get("partial_rotary_factor", 1)),
        "norm_eps": config["rms_norm_eps"],
        "norm_type": "rmsnorm",
        "act_type": config["hidden_act"],
    }
    # str() of the python value, as convert.py:63-80 does (floats print as 10000.0, 1e-05)
    return {k: str(v) for k, v in md.items()}


def gpt2_bytes_to_unicode() -> dict:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(2**8):
        if b not in bs:
            bs.append(b)
            cs.append(2**8 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def load_tokens(tokenizer_path: str, vocab_size: int) -> list:
    tokens = [""] * vocab_size
    with open(tokenizer_path, "r") as f:
        tok = json.load(f)
    gpt2 = not tok["model"].get("byte_fallback", False)
    vocab = tok["model"]["vocab"]
    if len(vocab) > vocab_size:
        raise ValueError("tokenizer vocab larger than vocab_size")
    for t, i in vocab.items():
        tokens[i] = t
    for added in tok["added_tokens"]:
        tokens[added["id"]] = added["content"]
    dec = {v: k for k, v in gpt2_bytes_to_unicode().items()}
    out = []
    for t in tokens:
        if gpt2:
            b = bytes([dec.get(c, 0) for c in t])
        else:
            b = t.replace("▁", " ").encode("utf-8")
        b = b.replace(b"\0", b"\7")
        out.append(b)
    return out


def permute_reverse(w: np.ndarray, heads: int, rotary_dim: int) -> np.ndarray:
    """Undo HF's rotate-half Q/K row order into interleaved (even, odd) pairs."""
    head_dim = w.shape[0] // heads
    assert rotary_dim <= head_dim
    w = w.reshape(heads, head_dim, -1)
    wr = w[:, :rotary_dim]
    wk = w[:, rotary_dim:]
    wr = wr.reshape(heads, 2, rotary_dim // 2, -1).transpose(0, 2, 1, 3).reshape(heads, rotary_dim, -1)
    return np.concatenate([wr, wk], axis=1).reshape(heads * head_dim, -1)


def f32_to_e5m2(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even f32 -> OCP E5M2 bits (torch c10 fp8e5m2_from_fp32_value)."""
    f = np.ascontiguousarray(x, np.float32).view(np.uint32)
    sign = f & np.uint32(0x80000000)
    a = f ^ sign
    fp32_inf = np.uint32(255 << 23)
    fp8_max = np.uint32(143 << 23)
    denorm_mask = np.uint32(134 << 23)
    res = np.zeros(a.shape, np.uint32)
    big = a >= fp8_max
    res[big] = np.where(a[big] > fp32_inf, 0x7F, 0x7C)
    small = (~big) & (a < np.uint32(113 << 23))
    if small.any():
        s = (a[small].view(np.float32) + denorm_mask.view(np.float32)).astype(np.float32).view(np.uint32)
        res[small] = s - denorm_mask
    norm = (~big) & (~small)
    if norm.any():
        v = a[norm].astype(np.uint64)
        mant_odd = (v >> 21) & 1
        v = v + ((15 - 127) << 23 & 0xFFFFFFFF) + 0xFFFFF + mant_odd
        res[norm] = ((v & 0xFFFFFFFF) >> 21).astype(np.uint32)
    return ((res & 0xFF) | (sign >> 24)).astype(np.uint8)


def _to_f32(t) -> np.ndarray:
    if t.dtype == "BF16":
        return (t.data.astype(np.uint32) << 16).view(np.float32).reshape(t.shape)
    if t.dtype in ("F32", "F16"):
        return t.data.astype(np.float32).reshape(t.shape)
    raise ValueError(f"unsupported source dtype {t.dtype}")


def convert(hf_dir: str, out_path: str, dtype: str = "fp16") -> None:
    with open(os.path.join(hf_dir, "config.json")) as f:
        config = json.load(f)
    md = metadata_from_config(config, dtype)
    vocab_size = int(md["vocab_size"])
    tokens = load_tokens(os.path.join(hf_dir, "tokenizer.json"), vocab_size)
    files = sorted(os.path.join(hf_dir, f) for f in os.listdir(hf_dir) if f.endswith(".safetensors"))
    if not files:
        raise FileNotFoundError(f"no .safetensors files found in {hf_dir}")
    src = {}
    opened = []
    for p in files:
        yd = read_yalm(p)
        opened.append(yd)
        for k, t in yd.tensors.items():
            assert k not in src
            src[k] = t

    def conv(name):
        a = _to_f32(src[name])
        if dtype == "fp32":
            return a, "F32"
        if dtype == "fp16":
            return a.astype(np.float16), "F16"
        return f32_to_e5m2(a), "F8_E5M2"

    tensors, dtypes = {}, {}

    def put(key, arr_dt):
        tensors[key], dtypes[key] = arr_dt

    put("model.embed.weight", conv("model.embed_tokens.weight"))
    n_heads, n_kv, rot = int(md["n_heads"]), int(md["n_kv_heads"]), int(md["rotary_dim"])
    for l in range(int(md["n_layers"])):
        p, q = f"model.layers.{l}.", f"model.layers.{l}."
        put(q + "attn.norm.weight", (_to_f32(src[p + "input_layernorm.weight"]), "F32"))
        for key, hf, heads in (("wq", "q_proj", n_heads), ("wk", "k_proj", n_kv)):
            a = permute_reverse(_to_f32(src[p + f"self_attn.{hf}.weight"]), heads, rot)
            src_key = f"__perm_{key}"
            src[src_key] = _F32View(a)
            put(q + f"attn.{key}.weight", conv(src_key))
        put(q + "attn.wv.weight", conv(p + "self_attn.v_proj.weight"))
        put(q + "attn.wo.weight", conv(p + "self_attn.o_proj.weight"))
        put(q + "mlp.norm.weight", (_to_f32(src[p + "post_attention_layernorm.weight"]), "F32"))
        put(q + "mlp.w1.weight", conv(p + "mlp.gate_proj.weight"))
        put(q + "mlp.w2.weight", conv(p + "mlp.down_proj.weight"))
        put(q + "mlp.w3.weight", conv(p + "mlp.up_proj.weight"))
    put("model.norm.weight", (_to_f32(src["model.norm.weight"]), "F32"))
    if config.get("tie_word_embeddings", None) == False:  # noqa: E712 (convert.py:200 semantics: absent -> tied)
        put("model.output.weight", conv("lm_head.weight"))
    blob = b"".join(t + b"\0" for t in tokens)
    put("tokenizer.tokens", (np.frombuffer(blob, np.uint8).copy(), "U8"))
    write_yalm(out_path, tensors, md, dtypes)
    for yd in opened:
        yd.close()


class _F32View:
    """Adapter so permuted f32 arrays go through the same conv() path."""

    dtype = "F32"

    def __init__(self, a):
        self.shape = a.shape
        self.data = np.ascontiguousarray(a, np.float32).reshape(-1)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("output", type=str)
    ap.add_argument("input", type=str)
    ap.add_argument("--dtype", type=str, default="fp16", choices=SUPPORTED_DTYPES)
    args = ap.parse_args(argv)
    convert(args.input, args.output, args.dtype)


if __name__ == "__main__":
    main()
