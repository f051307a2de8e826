"""Which f16 rounding of the batched prefill (yalm_amd/csrc/prefill.h) moves log p
most? A float64 numpy emulation of the prefill at Llama-3.2-3B dims (synthetic
weights, the bench's initialiser) with each activation rounding switched on alone,
against the all-f32 emulation (K / V rounded to f16 as the reference does,
infer.cpp:299): max |d log p| per rounding point.

Rounding points: R1 the QKV A operand (normalised x; R1q / R1kv: for the q or the
k | v columns only), R2 Q, R3 P in attention,
R4 the attention output O (Wo's A operand), R5 the GLU A operand, R6 the GLU
output H (W2's A operand), R7 the classifier's A operand.

usage: python tools/prefill_precision_emul.py [--layers 2] [--n 128] [--peak 8]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_py as O  # noqa: E402
from yalm_amd import models as M  # noqa: E402


def f16(a):
    return a.astype(np.float16).astype(np.float64)


def rmsnorm(x, w, eps):
    x32 = x.astype(np.float32)
    ss = (x32.astype(np.float64) ** 2).sum(axis=1, keepdims=True)
    return (x * (1.0 / np.sqrt(ss / x.shape[1] + eps)) * w).astype(np.float64)


def run(cfg, t, tokens, R):
    c = cfg
    T = len(tokens)
    D, G = c.head_dim, c.n_heads // c.n_kv_heads
    emb = t["model.embed.weight"].astype(np.float64)
    x = emb[tokens].copy()
    inv = M.rope_inv_freq(c).astype(np.float64)
    ang = np.arange(T)[:, None] * inv[None, :]
    cos, sin = np.cos(ang), np.sin(ang)

    def rope(a, nh):
        a = a.reshape(T, nh, D // 2, 2)
        e, o = a[..., 0].copy(), a[..., 1].copy()
        a[..., 0] = e * cos[:, None, :] - o * sin[:, None, :]
        a[..., 1] = e * sin[:, None, :] + o * cos[:, None, :]
        return a.reshape(T, nh * D)

    mask = np.triu(np.ones((T, T), bool), 1)
    for l in range(c.n_layers):
        n = M.layer_names(l)
        W = {k: t[v].astype(np.float64) for k, v in n.items() if not k.startswith("rms")}
        xn = rmsnorm(x, t[n["rms_att"]].astype(np.float64), c.norm_eps)
        aq = f16(xn) if "R1" in R or "R1q" in R else xn
        akv = f16(xn) if "R1" in R or "R1kv" in R else xn
        q = rope(aq @ W["wq"].T, c.n_heads)
        k = f16(rope(akv @ W["wk"].T, c.n_kv_heads))
        v = f16(akv @ W["wv"].T)
        if "R2" in R:
            q = f16(q)
        o = np.zeros((T, c.q_dim))
        for h in range(c.n_heads):
            g = h // G
            s = q[:, h * D:(h + 1) * D] @ k[:, g * D:(g + 1) * D].T / np.sqrt(D)
            s[mask] = -np.inf
            m = s.max(axis=1, keepdims=True)
            p = np.exp(s - m)
            lsum = p.sum(axis=1, keepdims=True)
            if "R3" in R:
                p = f16(p)
            o[:, h * D:(h + 1) * D] = (p @ v[:, g * D:(g + 1) * D]) / lsum
        if "R4" in R:
            o = f16(o)
        x = x + o @ W["wo"].T
        xn = rmsnorm(x, t[n["rms_ffn"]].astype(np.float64), c.norm_eps)
        a = f16(xn) if "R5" in R else xn
        h1, h3 = a @ W["w1"].T, a @ W["w3"].T
        hh = h1 / (1.0 + np.exp(-h1)) * h3
        if "R6" in R:
            hh = f16(hh)
        x = x + hh @ W["w2"].T
    xn = rmsnorm(x, t["model.norm.weight"].astype(np.float64), c.norm_eps)
    a = f16(xn) if "R7" in R else xn
    wcls = t.get("model.output.weight", t["model.embed.weight"])
    lp = np.zeros(T - 1)
    for i0 in range(0, T - 1, 64):
        lg = a[i0:min(i0 + 64, T - 1)] @ wcls.astype(np.float64).T
        mx = lg.max(axis=1, keepdims=True)
        lse = mx[:, 0] + np.log(np.exp(lg - mx).sum(axis=1))
        idx = np.arange(i0, min(i0 + 64, T - 1))
        lp[idx] = lg[np.arange(len(idx)), tokens[idx + 1]] - lse
    return lp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--seed", type=int, default=6, help="synthetic weight seed")
    ap.add_argument("--tokseed", type=int, default=-1, help="token rng seed (default 1000 + layers)")
    ap.add_argument("--peak", type=float, default=1.0, help="final-norm scale (models.PEAKED = 8: a trained checkpoint's logit spread)")
    ap.add_argument("--sets", default="", help="comma-separated rounding sets to run, e.g. 'R1+R2,all-R1' (default: each alone, then all)")
    args = ap.parse_args()
    cfg = M.LLAMA_32_3B.with_(n_layers=args.layers, max_seq_len=max(args.n, 64))
    t = O.synth_host_tensors_fast(cfg, seed=args.seed, peak=args.peak)
    tseed = args.tokseed if args.tokseed >= 0 else 1000 + args.layers
    tokens = np.random.default_rng(tseed).integers(0, cfg.vocab_size, size=args.n)
    base = run(cfg, t, tokens, set())
    print(f"llama-3b dims, {args.layers} layers, {args.n} positions, peak {args.peak}; log ppl {-base.mean():.4f}")
    allr = {"R1", "R2", "R3", "R4", "R5", "R6", "R7"}
    sets = [{"R1"}, {"R2"}, {"R3"}, {"R4"}, {"R5"}, {"R6"}, {"R7"}, allr]
    if args.sets:
        sets = []
        for spec in args.sets.split(","):
            if spec == "all":
                sets.append(set(allr))
            elif spec.startswith("all-"):
                sets.append(allr - set(spec[4:].split("+")))
            else:
                sets.append(set(spec.split("+")))
    for R in sets:
        lp = run(cfg, t, tokens, R)
        d = np.abs(lp - base)
        print(f"  {'+'.join(sorted(R)):24s} max |d log p| {d.max():.2e}  p99 {np.quantile(d, 0.99):.2e}  "
              f"median {np.median(d):.2e}  |d log ppl| {abs(lp.mean() - base.mean()):.2e}", flush=True)


if __name__ == "__main__":
    main()
