"""Generates tests/golden/tokenizer_ref.json: token ids and decode_one pieces
produced by the REFERENCE tokenizer (/root/reference/src/tokenizer.cpp compiled
by `make -C oracle ref` into oracle/_ref/ref_tok_dump) on the committed
reference-converted fixtures. Run here (the container that has /root/reference);
the JSON is data only: prompts (hex), ids, hex pieces.

usage: python tests/golden/make_tok_golden.py
"""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_tok_dump")
FIXTURES = ["tiny_fp16.yalm", "tiny_fp16_tied.yalm", "tiny_fp32.yalm", "tiny_fp8.yalm"]

PROMPTS = [
    "the thin is",
    "What is a large language model?",
    "Q: What is the meaning of life?",
    "  spaces\tand\nnewlines  ",
    "héllo wörld — ünïcode ✓",
    "",
    "a",
    "the the the the the the the the the the",
    "inininininin theeeeee thin thing think",
    "\x01\x02\x7f control bytes",
    "emoji 😀🚀 and CJK 漢字",
    "x" * 300,
]
# every byte value 1..255 once (argv cannot carry NUL), including invalid UTF-8
RAW = [bytes(range(1, 128)), bytes(range(128, 256)), b"\xff\xfe broken \xc3 utf8 \xe2\x82"]


def run(binary, path, prompt: bytes):
    out = subprocess.run([binary, path, prompt], capture_output=True, check=True).stdout.decode()
    lines = out.split("\n")
    ids = [int(t) for t in lines[0].split()]
    return ids, lines[1:len(ids)]


def generate(binary=REF_BIN):
    data = {}
    for fx in FIXTURES:
        path = os.path.join(GOLDEN, fx)
        entries = []
        for p in [s.encode() for s in PROMPTS] + RAW:
            ids, pieces = run(binary, path, p)
            entries.append({"prompt_hex": p.hex(), "ids": ids, "pieces_hex": pieces})
        data[fx] = entries
    return data


if __name__ == "__main__":
    if not os.path.exists(REF_BIN):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    with open(os.path.join(GOLDEN, "tokenizer_ref.json"), "w") as f:
        json.dump(generate(), f, indent=0)
        f.write("\n")
    print("wrote tests/golden/tokenizer_ref.json")
