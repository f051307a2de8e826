"""Generates tests/golden/ref_glue.npz: outputs of the REFERENCE's own per-block glue
functions (static / inline in /root/reference/src/infer.cpp: rmsnorm, rope, softmax,
clip, float_to_half, half_to_float), reached by oracle/_ref/ref_glue, a harness TU
that #includes the unmodified infer.cpp (`make -C oracle ref-glue`), on the seeded
inputs of ref_glue_cases.py. Composite cases (kvrow, sinkrot) chain those calls in
_block_cpu's statement order (infer.cpp:265-317). Run here (the container that has
/root/reference); the npz is data only: per case the outputs and their sha256.

usage: python tests/golden/make_ref_glue_golden.py
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
import ref_glue_cases as C  # noqa: E402

REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_glue")


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


class Ref:
    """One call of the reference binary per glue function, through raw files."""

    def __init__(self, binary: str, td: str):
        self.bin, self.td, self.k = binary, td, 0

    def _f(self, a=None):
        self.k += 1
        p = os.path.join(self.td, f"f{self.k}")
        if a is not None:
            np.ascontiguousarray(a).tofile(p)
        return p

    def _run(self, *args):
        subprocess.run([self.bin] + [str(a) for a in args], check=True)

    def rmsnorm(self, x, w, eps):
        o = self._f()
        self._run("rmsnorm", x.size, repr(float(eps)), self._f(x), self._f(w), o)
        return np.fromfile(o, np.float32)

    def rope(self, v, head_dim, pos, theta, rotary_dim):
        o = self._f()
        self._run("rope", v.size, head_dim, pos, repr(float(theta)), rotary_dim, self._f(v), o)
        return np.fromfile(o, np.float32)

    def softmax(self, x):
        o = self._f()
        self._run("softmax", x.size, self._f(x), o)
        return np.fromfile(o, np.float32)

    def clip(self, x, v):
        o = self._f()
        self._run("clip", x.size, repr(float(v)), self._f(x), o)
        return np.fromfile(o, np.float32)

    def f2h(self, x):
        o = self._f()
        self._run("f2h", x.size, self._f(x), o)
        return np.fromfile(o, np.uint16)

    def h2f(self, x):
        o = self._f()
        self._run("h2f", x.size, self._f(x), o)
        return np.fromfile(o, np.float32)


def run_case(case: dict, binary: str = REF_BIN) -> dict:
    inp = C.inputs(case)
    with tempfile.TemporaryDirectory() as td:
        r = Ref(binary, td)
        op = case["op"]
        if op == "rmsnorm":
            return {"out": r.rmsnorm(inp["x"], inp["w"], case["eps"])}
        if op == "rope":
            return {"out": r.rope(inp["vec"], case["head_dim"], case["pos"], case["theta"], case["rotary_dim"])}
        if op == "softmax":
            return {"out": r.softmax(inp["x"])}
        if op == "clip":
            return {"out": r.clip(inp["x"], case["v"])}
        if op in ("f2h", "f2h_random"):
            return {"out": r.f2h(inp["x"])}
        if op == "h2f":
            return {"out": r.h2f(inp["x"])}
        if op == "kvrow":  # infer.cpp:268, 277-292, 299 (Wk = identity)
            xn = r.rmsnorm(inp["x"], inp["w"], case["eps"])
            k = r.clip(xn, case["clip"])
            k = r.rope(k, case["head_dim"], case["pos"], case["theta"], case["rotary_dim"])
            return {"xn": xn, "k": k, "row": r.f2h(k)}
        if op == "sinkrot":  # infer.cpp:307-317
            k = r.h2f(inp["row"])
            k = r.rope(k, case["head_dim"], 1, case["theta"], case["rotary_dim"])
            return {"row": r.f2h(k)}
        raise ValueError(op)


def main():
    if not os.path.exists(REF_BIN):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref-glue"], check=True)
    data = {}
    for case in C.CASES:
        outs = run_case(case)
        for k, a in outs.items():
            key = f"{case['name']}/{k}"
            data[key] = a
            data[key + "#sha256"] = np.array(sha(a))
    np.savez_compressed(os.path.join(HERE, "ref_glue.npz"), **data)
    print(len(C.CASES), "cases")


if __name__ == "__main__":
    main()
