// tokenizer.h — greedy longest-match vocabulary encoder with byte fallback,
// the semantics of the reference tokenizer (/root/reference/src/tokenizer.cpp:
// 3-107): vocab from the NUL-separated "tokenizer.tokens" tensor, bos/eos from
// metadata, eot = <|eot_id|> / <|end|> / <|im_end|>, byte pieces for
// <0x00>..<0xFF>, BOS-following leading-space strip in decode_one.
#pragma once

#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "codec.h"

namespace yalm {

struct TokenTrie {
	std::unordered_map<char, std::unique_ptr<TokenTrie>> children;
	int token_id = -1;
};

struct Tokenizer {
	std::vector<std::string> vocab;
	TokenTrie vocab_trie;
	int bos_id = -1;
	int eos_id = -1;
	int eot_id = -1;
	int byte_fallback_start = -1;

	explicit Tokenizer(const YALMData &data);
	std::vector<int> encode(const std::string &text, bool encode_bos) const;
	std::string decode_one(int prev_token, int token) const;
	std::string encoding_to_debug_string(const std::vector<int> &encoding) const;
};

} // namespace yalm
