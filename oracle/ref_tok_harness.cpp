// ref_tok_harness.cpp — TEST INFRASTRUCTURE (oracle/_ref recipe, never shipped).
//
// Drives the REFERENCE tokenizer, compiled from its own source where it lies
// (/root/reference/src/tokenizer.cpp, with -iquote /root/reference/src and the
// reference's vendored nlohmann json), on a .yalm file. The reference loader
// (codec.cpp) needs spdlog, which the image lacks, so this harness fills the
// YALMData the Tokenizer constructor reads (metadata + the "tokenizer.tokens"
// tensor, codec.h:29-51) itself by parsing the .yalm layout: u64 header length,
// JSON header (with "__metadata__"), then the tensor bytes (codec.cpp:116-175).
//
// usage: ref_tok_dump model.yalm prompt
// prints the ids of tokenizer.encode(prompt, true) (tokenizer.cpp:57-94), then
// decode_one(prev, id) of each id after BOS, hex-escaped, one per line
// (tokenizer.cpp:44-55) — the same format as yalm_amd/host/tok_dump.
#include <cstdio>
#include <cstdint>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "tokenizer.h"

int main(int argc, char **argv) {
	if (argc != 3) {
		fprintf(stderr, "usage: ref_tok_dump model.yalm prompt\n");
		return 1;
	}
	std::ifstream f(argv[1], std::ios::binary);
	std::vector<char> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
	if (bytes.size() < 8)
		return 1;
	uint64_t hlen = 0;
	for (int i = 0; i < 8; ++i)
		hlen |= (uint64_t)(unsigned char)bytes[i] << (8 * i);
	json header = json::parse(bytes.begin() + 8, bytes.begin() + 8 + hlen);
	char *data = bytes.data() + 8 + hlen;
	YALMData yd;
	yd.data = bytes.data();
	yd.size = bytes.size();
	yd.metadata = header.at("__metadata__");
	const json &tj = header.at("tokenizer.tokens");
	Tensor t;
	t.name = "tokenizer.tokens";
	t.dtype = DType::U8;
	size_t b = tj.at("data_offsets")[0].get<size_t>(), e = tj.at("data_offsets")[1].get<size_t>();
	t.data = data + b;
	t.size = e - b;
	yd.tensors["tokenizer.tokens"] = t;

	Tokenizer tok(yd);
	std::vector<int> enc = tok.encode(argv[2], true);
	for (int id : enc)
		printf("%d ", id);
	printf("\n");
	int prev = tok.bos_id;
	for (size_t i = 1; i < enc.size(); ++i) {
		for (unsigned char c : tok.decode_one(prev, enc[i]))
			printf("%02x", c);
		printf("\n");
		prev = enc[i];
	}
	return 0;
}
