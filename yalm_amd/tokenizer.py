"""Python twin of the host tokenizer (yalm_amd/host/tokenizer.cpp), with the
reference semantics (/root/reference/src/tokenizer.cpp:3-107): greedy
longest-match over the vocabulary bytes with byte fallback, BOS-space strip in
decode_one. Used by tests and tools to build prompts without the C++ host."""

from __future__ import annotations


class Tokenizer:
    def __init__(self, vocab: list, bos_id: int, eos_id: int):
        self.vocab = vocab  # list[bytes]
        self.bos_id, self.eos_id = bos_id, eos_id
        self.eot_id = -1
        self.byte_fallback_start = -1
        for i, v in enumerate(vocab):
            if v == b"<0x00>":
                self.byte_fallback_start = i
            elif v in (b"<|eot_id|>", b"<|end|>", b"<|im_end|>"):
                self.eot_id = i
        self.trie: dict = {}
        for i, v in enumerate(vocab):
            node = self.trie
            for c in v:
                node = node.setdefault(c, {})
            node[None] = i  # later duplicates win

    @classmethod
    def from_yalm(cls, yd) -> "Tokenizer":
        blob = yd.tensors["tokenizer.tokens"].data.tobytes()
        vocab = blob.split(b"\0")[:-1]
        return cls(vocab, int(yd.metadata["bos_token_id"]), int(yd.metadata["eos_token_id"]))

    def encode(self, text, bos: bool = True) -> list:
        data = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        out = [self.bos_id] if bos else []
        i = 0
        while i < len(data):
            node, best, best_len, l = self.trie, -1, 0, 0
            while i + l < len(data) and data[i + l] in node:
                node = node[data[i + l]]
                l += 1
                if None in node:
                    best, best_len = node[None], l
            if best < 0:
                if self.byte_fallback_start >= 0:
                    out.append(data[i] + self.byte_fallback_start)
                i += 1
            else:
                out.append(best)
                i += best_len
        return out

    def decode_one(self, prev: int, token: int) -> bytes:
        piece = self.vocab[token]
        if prev == self.bos_id and piece[:1] == b" ":
            return piece[1:]
        if self.byte_fallback_start >= 0 and 0 <= token - self.byte_fallback_start < 256:
            return bytes([token - self.byte_fallback_start])
        return piece
