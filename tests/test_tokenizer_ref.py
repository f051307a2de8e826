"""CPU: tokenizer parity pinned on the REFERENCE tokenizer itself.

tests/golden/tokenizer_ref.json holds the ids and decode_one pieces that
/root/reference/src/tokenizer.cpp (compiled from its own source by
`make -C oracle ref`, oracle/ref_tok_harness.cpp) produces on the committed
reference-converted fixtures (generator: tests/golden/make_tok_golden.py).
Both of this repo's tokenizers must match them bit-exactly: the C++20 host
(yalm_amd/host/tokenizer.cpp, used by the CLI) and the Python twin
(yalm_amd/tokenizer.py). Where the reference binary is built (this container),
it is re-run live against the golden file too."""
import json
import os
import subprocess

import pytest

from yalm_amd.tokenizer import Tokenizer
from yalm_amd.yalmfile import read_yalm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "yalm_amd", "host")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_tok_dump")
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "tokenizer_ref.json")))
CASES = [(fx, i) for fx, entries in GOLD.items() for i in range(len(entries))]


def run(binary, path, prompt: bytes):
    out = subprocess.run([binary, path, prompt], capture_output=True, check=True).stdout.decode()
    lines = out.split("\n")
    ids = [int(t) for t in lines[0].split()]
    return ids, lines[1:len(ids)]


@pytest.fixture(scope="module")
def host_tok():
    subprocess.run(["make", "-C", HOST, "-j4", "tok_dump"], check=True, capture_output=True)
    return os.path.join(HOST, "tok_dump")


@pytest.mark.parametrize("fx,i", CASES)
def test_cpp_host_tokenizer_matches_reference(host_tok, golden_dir, fx, i):
    e = GOLD[fx][i]
    ids, pieces = run(host_tok, os.path.join(golden_dir, fx), bytes.fromhex(e["prompt_hex"]))
    assert ids == e["ids"]
    assert pieces == e["pieces_hex"]


@pytest.mark.parametrize("fx", sorted(GOLD))
def test_python_tokenizer_matches_reference(golden_dir, fx):
    yd = read_yalm(os.path.join(golden_dir, fx))
    tok = Tokenizer.from_yalm(yd)
    for e in GOLD[fx]:
        prompt = bytes.fromhex(e["prompt_hex"])
        ids = tok.encode(prompt)  # raw bytes: every byte reaches the trie as itself
        assert ids == e["ids"], prompt
        prev = tok.bos_id
        for t, piece in zip(ids[1:], e["pieces_hex"]):
            assert tok.decode_one(prev, t).hex() == piece
            prev = t
    yd.close()


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("fx", sorted(GOLD))
def test_reference_binary_reproduces_golden(golden_dir, fx):
    for e in GOLD[fx]:
        ids, pieces = run(REF_BIN, os.path.join(golden_dir, fx), bytes.fromhex(e["prompt_hex"]))
        assert ids == e["ids"] and pieces == e["pieces_hex"]
