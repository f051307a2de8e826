// sample_dump — test hook for the host samplers (sampler.cpp, reference
// sampler.cpp:6-65) on fixed logits: no model, no GPU.
// usage: sample_dump logits.f32 seed temperature count [prob_index ...]
// prints the argmax, then `count` draws of Sampler(seed).sample(temperature),
// then sample_prob of each prob_index as a hex float (%a), one per line.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <memory>
#include <vector>

#include "sampler.h"

int main(int argc, char **argv) {
	if (argc < 5) {
		fprintf(stderr, "usage: sample_dump logits.f32 seed temperature count [prob_index ...]\n");
		return 1;
	}
	std::ifstream f(argv[1], std::ios::binary);
	std::vector<char> raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
	auto cfg = std::make_shared<yalm::Config>();
	cfg->vocab_size = (int)(raw.size() / sizeof(float));
	yalm::InferenceState st(cfg);
	std::copy(raw.begin(), raw.end(), (char *)st.logits());
	yalm::Sampler s(cfg, strtoull(argv[2], nullptr, 10));
	const float t = strtof(argv[3], nullptr);
	printf("%d\n", s.sample_argmax(st));
	for (int i = 0, n = atoi(argv[4]); i < n; ++i)
		printf("%d ", s.sample(st, t));
	printf("\n");
	for (int i = 5; i < argc; ++i)
		printf("%a\n", s.sample_prob(atoi(argv[i]), st));
	return 0;
}
