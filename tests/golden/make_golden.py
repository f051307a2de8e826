"""Build the committed golden fixtures under tests/golden/.

1. test_cpp_inputs.npz — the reference kernel test's seeded inputs
   (test.cpp:128-206), regenerated with libstdc++ by gen_test_cpp_inputs.cpp.
Run from the repo root: python tests/golden/make_golden.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def test_cpp_inputs():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "gen")
        subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "gen_test_cpp_inputs.cpp"), "-o", exe],
                       check=True)
        out = os.path.join(td, "in.bin")
        subprocess.run([exe, out], check=True)
        data = open(out, "rb").read()
    arrays = {}
    i = 0
    while i < len(data):
        nl = data.index(b"\n", i)
        name, n = data[i:nl].decode().split()
        n = int(n)
        arrays[name] = np.frombuffer(data[nl + 1: nl + 1 + 4 * n], np.float32).copy()
        i = nl + 1 + 4 * n + 1
    np.savez(os.path.join(HERE, "test_cpp_inputs.npz"), **arrays)
    print("wrote test_cpp_inputs.npz:", {k: v.shape for k, v in arrays.items()})




# ---------------------------------------------------------------------------
# 2. Tiny HF-format model dirs -> .yalm via the REFERENCE converter
#    (/root/reference/convert.py, run here only; its outputs are committed as
#    data fixtures so the GPU box never needs the reference).
TINY_HF = dict(vocab_size=384, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
               num_key_value_heads=2, max_position_embeddings=64, rope_theta=10000.0, rms_norm_eps=1e-5,
               hidden_act="silu", bos_token_id=1, eos_token_id=2)


def tiny_vocab(vocab_size):
    """<unk>,<s>,</s>, 256 byte-fallback tokens, then sentencepiece-style pieces."""
    vocab = ["<unk>", "<s>", "</s>"] + [f"<0x{i:02X}>" for i in range(256)]
    words = ["the", "thin", "is", "a", "large", "language", "model", "what", "of", "in", "and", "to", "it", "on",
             "pass", "key", "grass", "green", "sky", "blue", "sun", "yellow", "here", "we", "go", "there", "back",
             "again", "remember", "important", "info", "hidden", "inside", "lot", "irrelevant", "text", "find",
             "memorize", "them", "will", "quiz", "you", "about", "information", "meaning", "life", "Q", "A"]
    pieces = []
    for w in words:
        pieces += ["▁" + w, w]
    pieces += ["th", "in", "er", "an", "on", "at", "en", "is", "▁t", "▁a", "▁i", "▁s", "▁w",
               "▁▁", "▁▁▁▁", ".", ",", "?", "!", ":", "▁"]
    pieces += [chr(c) for c in range(ord("a"), ord("z") + 1)] + [str(d) for d in range(10)]
    seen = set(vocab)
    for p in pieces:
        if p not in seen and len(vocab) < vocab_size:
            vocab.append(p)
            seen.add(p)
    i = 0
    while len(vocab) < vocab_size:
        vocab.append(f"<extra_{i}>")
        i += 1
    return vocab


def write_hf_dir(path, hf=TINY_HF, seed=0, tie=False):
    """Synthetic HF checkpoint dir (config.json, tokenizer.json, model.safetensors)."""
    import json

    import torch
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    cfg = dict(hf, architectures=["MistralForCausalLM"], tie_word_embeddings=tie)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(cfg, f, indent=1)
    vocab = tiny_vocab(hf["vocab_size"])
    tok = {"model": {"type": "BPE", "byte_fallback": True, "vocab": {t: i for i, t in enumerate(vocab)}},
           "added_tokens": []}
    with open(os.path.join(path, "tokenizer.json"), "w") as f:
        json.dump(tok, f, indent=1)
    rng = np.random.Generator(np.random.PCG64(seed))
    d, h, L = hf["hidden_size"], hf["intermediate_size"], hf["num_hidden_layers"]
    nh, nkv = hf["num_attention_heads"], hf["num_key_value_heads"]
    hd = d // nh

    def w(*shape, s=0.1):
        return torch.from_numpy((rng.standard_normal(shape) * s).astype(np.float32))

    t = {"model.embed_tokens.weight": w(hf["vocab_size"], d, s=0.5)}
    for l in range(L):
        p = f"model.layers.{l}."
        t[p + "input_layernorm.weight"] = torch.from_numpy((1 + 0.1 * rng.standard_normal(d)).astype(np.float32))
        t[p + "self_attn.q_proj.weight"] = w(nh * hd, d)
        t[p + "self_attn.k_proj.weight"] = w(nkv * hd, d)
        t[p + "self_attn.v_proj.weight"] = w(nkv * hd, d)
        t[p + "self_attn.o_proj.weight"] = w(d, nh * hd)
        t[p + "post_attention_layernorm.weight"] = torch.from_numpy(
            (1 + 0.1 * rng.standard_normal(d)).astype(np.float32))
        t[p + "mlp.gate_proj.weight"] = w(h, d)
        t[p + "mlp.up_proj.weight"] = w(h, d)
        t[p + "mlp.down_proj.weight"] = w(d, h)
    t["model.norm.weight"] = torch.from_numpy((1 + 0.1 * rng.standard_normal(d)).astype(np.float32))
    if not tie:
        t["lm_head.weight"] = w(hf["vocab_size"], d, s=0.5)
    save_file(t, os.path.join(path, "model.safetensors"))


def reference_yalm_fixtures():
    ref = "/root/reference/convert.py"
    if not os.path.exists(ref):
        print("reference not present; keeping committed .yalm fixtures")
        return
    with tempfile.TemporaryDirectory() as td:
        for tie in (False, True):
            hfdir = os.path.join(td, f"hf_tie{int(tie)}")
            write_hf_dir(hfdir, tie=tie)
            for dt in ("fp32", "fp16", "fp8"):
                if tie and dt != "fp16":
                    continue
                out = os.path.join(HERE, f"tiny_{dt}{'_tied' if tie else ''}.yalm")
                subprocess.run([sys.executable, ref, "--dtype", dt, out, hfdir], check=True,
                               stdout=subprocess.DEVNULL)
                print("wrote", os.path.basename(out), os.path.getsize(out))


if __name__ == "__main__":
    test_cpp_inputs()
    reference_yalm_fixtures()
