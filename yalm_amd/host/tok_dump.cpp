// tok_dump — test hook: prints the token ids the C++ tokenizer produces for a
// prompt (with BOS), then decode_one() of each id, hex-escaped, one per line.
#include <cstdio>

#include "tokenizer.h"

int main(int argc, char **argv) {
	if (argc != 3) {
		fprintf(stderr, "usage: tok_dump model.yalm prompt\n");
		return 1;
	}
	yalm::YALMData data;
	if (data.from_file(argv[1]) != 0)
		return 1;
	yalm::Tokenizer tok(data);
	auto enc = tok.encode(argv[2], true);
	for (int t : enc)
		printf("%d ", t);
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
