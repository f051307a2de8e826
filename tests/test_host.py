"""C++20 host layer (yalm_amd/host): tokenizer parity with the Python twin on
the reference-converted fixture (CPU), and the yalm CLI end to end on the
GPU against the oracle's greedy tokens (the `-d cpu ... -t 0` contract of
BASELINE config 1/2 on a tiny model)."""
import os
import subprocess

import numpy as np
import pytest

from yalm_amd.tokenizer import Tokenizer
from yalm_amd.yalmfile import read_yalm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "yalm_amd", "host")
PROMPTS = [
    "the thin is",
    "What is a large language model?",
    "Q: What is the meaning of life?",
    "  spaces\tand\nnewlines  ",
    "héllo wörld — ünïcode ✓",
    "",
]


@pytest.fixture(scope="module")
def host_built():
    subprocess.run(["make", "-C", HOST, "-j4"], check=True, capture_output=True)
    return HOST


@pytest.mark.parametrize("prompt", PROMPTS)
def test_tokenizer_cpp_matches_python(host_built, golden_dir, prompt):
    path = os.path.join(golden_dir, "tiny_fp16.yalm")
    out = subprocess.run([os.path.join(host_built, "tok_dump"), path, prompt], capture_output=True, check=True)
    lines = out.stdout.decode().split("\n")
    ids = [int(t) for t in lines[0].split()]
    yd = read_yalm(path)
    tok = Tokenizer.from_yalm(yd)
    assert ids == tok.encode(prompt)
    prev = tok.bos_id
    for i, t in enumerate(ids[1:]):
        assert bytes.fromhex(lines[1 + i]) == tok.decode_one(prev, t)
        prev = t
    # decoding round trip: byte fallback covers every byte
    assert b"".join(tok.decode_one(-1, t) for t in ids[1:]) == prompt.encode()
    yd.close()


def test_cli_rejects_cpu_device(host_built, golden_dir):
    r = subprocess.run([os.path.join(host_built, "yalm"), os.path.join(golden_dir, "tiny_fp16.yalm"), "-d", "cpu",
                        "-i", "x"], capture_output=True)
    assert r.returncode == 1 and b"-d cpu" in r.stderr


def test_cli_usage(host_built):
    r = subprocess.run([os.path.join(host_built, "yalm")], capture_output=True)
    assert r.returncode == 1 and b"Usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("fname", ["tiny_fp16.yalm", "tiny_fp8.yalm", "tiny_fp32.yalm", "tiny_fp16_tied.yalm"])
@pytest.mark.parametrize("context", [0, 16])
def test_cli_greedy_matches_oracle(host_built, golden_dir, fname, context):
    """yalm <file> -d hip -m c -t 0 -n 40 [-T 16]: generated ids == oracle
    greedy on the same prompt (with -T 16 the decode runs 3x past the window:
    ring buffer + attention sinks)."""
    import oracle_py as O
    from yalm_amd import models as M

    path = os.path.join(golden_dir, fname)
    n = 40
    cmd = [os.path.join(host_built, "yalm"), path, "-d", "hip", "-m", "c", "-t", "0", "-n", str(n), "-i",
           "the thin is"]
    if context:
        cmd += ["-T", str(context)]
    r = subprocess.run(cmd, capture_output=True, env=dict(os.environ, YALM_PRINT_TOKENS="1"), timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    line = [l for l in r.stderr.decode().split("\n") if l.startswith("TOKENS:")][0]
    got = [int(t) for t in line[len("TOKENS:"):].split()]

    yd = read_yalm(path)
    tok = Tokenizer.from_yalm(yd)
    cfg = M.config_from_metadata(yd.metadata, context=context, tied="model.output.weight" not in yd.tensors)
    t = {k: np.array(v.data).reshape(v.shape) for k, v in yd.tensors.items()}
    yd.close()
    om = O.OracleModel(cfg, t)
    enc = tok.encode("the thin is")
    for pos, tk in enumerate(enc[:-1]):
        om.forward(tk, pos, 0)
    ref = []
    lg = om.forward(enc[-1], len(enc) - 1, 1)
    pos = len(enc)
    for _ in range(n):
        nt = int(np.argmax(lg))
        ref.append(nt)
        if nt in (cfg.eos_token_id,):
            break
        lg = om.forward(nt, pos, 1)
        pos += 1
    assert got == ref
