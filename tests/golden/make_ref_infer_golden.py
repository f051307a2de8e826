"""Generates tests/golden/ref_infer.npz: outputs of the REFERENCE's own CPU
kernels (matmul_cpu f32/f16, mha_cpu, ffn_cpu from /root/reference/src/infer.cpp,
compiled unmodified by `make -C oracle ref-infer` into oracle/_ref/ref_infer)
on the seeded inputs of ref_infer_cases.py. Run here (the container that has
/root/reference); the npz is data only: per case the output vectors and the
sha256 of their exact bytes.

usage: python tests/golden/make_ref_infer_golden.py
"""
import hashlib
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import ref_infer_cases as C  # noqa: E402

REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_infer")
ATT_KEEP = 256  # attention rows are stored whole up to this kv_len, only hashed beyond


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run_case(case: dict, binary: str = REF_BIN) -> dict:
    """Runs the reference binary on one case; returns {output name: array}."""
    inp = C.inputs(case)
    with tempfile.TemporaryDirectory() as td:
        def f(name, a=None):
            p = os.path.join(td, name)
            if a is not None:
                np.ascontiguousarray(a).tofile(p)
            return p

        op = case["op"]
        if op.startswith("matmul"):
            args = [op, str(case["n"]), str(case["d"]), f("x", inp["x"]), f("w", inp["w"]), f("out")]
            subprocess.run([binary] + args, check=True)
            return {"out": np.fromfile(f("out"), np.float32)}
        if op == "mha":
            args = ["mha"] + [str(case[k]) for k in ("head_dim", "kv_len", "max_seq_len", "n_heads", "n_kv_heads")]
            args += [f("q", inp["q"]), f("kb", inp["kb"].view(np.uint16)), f("vb", inp["vb"].view(np.uint16)),
                     f("xout"), f("att")]
            subprocess.run([binary] + args, check=True)
            return {"xout": np.fromfile(f("xout"), np.float32),
                    "att": np.fromfile(f("att"), np.float32).reshape(case["n_heads"], case["max_seq_len"])}
        args = ["ffn", str(case["hidden"]), str(case["dim"]), str(case["act"]), f("x", inp["x"]),
                f("w1", inp["w1"]), f("w2", inp["w2"]), f("w3", inp["w3"]), f("out")]
        subprocess.run([binary] + args, check=True)
        return {"out": np.fromfile(f("out"), np.float32)}


def main():
    if not os.path.exists(REF_BIN):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref-infer"], check=True)
    data = {}
    for case in C.CASES:
        outs = run_case(case)
        for k, a in outs.items():
            key = f"{case['name']}/{k}"
            data[key + "#sha256"] = np.array(sha(a))
            if k == "att":
                if case["kv_len"] <= ATT_KEEP:
                    data[key] = a[:, :case["kv_len"]].copy()
            else:
                data[key] = a
        print(case["name"], {k: a.shape for k, a in outs.items()}, flush=True)
    np.savez_compressed(os.path.join(HERE, "ref_infer.npz"), **data)


if __name__ == "__main__":
    main()
