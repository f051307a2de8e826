#include "tokenizer.h"

#include <stdexcept>

namespace yalm {

Tokenizer::Tokenizer(const YALMData &data) {
	bos_id = std::stoi(data.metadata.at("bos_token_id").as_string());
	eos_id = std::stoi(data.metadata.at("eos_token_id").as_string());
	auto it = data.tensors.find("tokenizer.tokens");
	if (it == data.tensors.end())
		throw std::runtime_error("FATAL: missing tensor: tokenizer.tokens");
	const char *p = (const char *)it->second.data;
	const char *end = p + it->second.size;
	while (p < end) {
		const char *s = p;
		while (p < end && *p != '\0')
			++p;
		vocab.emplace_back(s, p - s);
		++p; // skip the NUL terminator
	}
	for (size_t i = 0; i < vocab.size(); ++i) {
		if (vocab[i] == "<0x00>")
			byte_fallback_start = (int)i;
		else if (vocab[i] == "<|eot_id|>" || vocab[i] == "<|end|>" || vocab[i] == "<|im_end|>")
			eot_id = (int)i;
	}
	for (size_t i = 0; i < vocab.size(); ++i) {
		TokenTrie *node = &vocab_trie;
		for (char c : vocab[i]) {
			auto &child = node->children[c];
			if (!child)
				child = std::make_unique<TokenTrie>();
			node = child.get();
		}
		node->token_id = (int)i; // later duplicates win, as in the reference
	}
}

std::string Tokenizer::decode_one(int prev_token, int token) const {
	const std::string &piece = vocab.at(token);
	if (prev_token == bos_id && !piece.empty() && piece[0] == ' ')
		return piece.substr(1);
	if (byte_fallback_start >= 0 && token >= byte_fallback_start && token - byte_fallback_start < 256)
		return std::string(1, (char)(token - byte_fallback_start));
	return piece;
}

std::vector<int> Tokenizer::encode(const std::string &text, bool encode_bos) const {
	std::vector<int> out;
	if (encode_bos)
		out.push_back(bos_id);
	size_t i = 0;
	while (i < text.size()) {
		const TokenTrie *node = &vocab_trie;
		int best = -1;
		size_t best_len = 0;
		for (size_t l = 0; i + l < text.size(); ++l) {
			auto it = node->children.find(text[i + l]);
			if (it == node->children.end())
				break;
			node = it->second.get();
			if (node->token_id >= 0) {
				best = node->token_id;
				best_len = l + 1;
			}
		}
		if (best < 0) {
			if (byte_fallback_start >= 0)
				out.push_back((unsigned char)text[i] + byte_fallback_start);
			i += 1;
		} else {
			out.push_back(best);
			i += best_len;
		}
	}
	return out;
}

std::string Tokenizer::encoding_to_debug_string(const std::vector<int> &encoding) const {
	std::string s;
	for (int t : encoding) {
		if (t == bos_id)
			s += "[<s>:" + std::to_string(t) + "]";
		else if (t == eos_id)
			s += "[</s>:" + std::to_string(t) + "]";
		else
			s += "[" + vocab.at(t) + ":" + std::to_string(t) + "]";
	}
	return s;
}

} // namespace yalm
