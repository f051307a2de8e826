#include "sampler.h"

#include <cfloat>
#include <cmath>
#include <cstdlib>

namespace yalm {

Sampler::Sampler(const std::shared_ptr<Config> config, uint64_t seed) : vocab_size(config->vocab_size) {
	std::srand((unsigned)seed);
}

static float max_logit(const float *logits, int n) {
	float m = -FLT_MAX;
	for (int i = 0; i < n; ++i)
		if (logits[i] > m)
			m = logits[i];
	return m;
}

float Sampler::sample_prob(int index, const InferenceState &s) const {
	const float *logits = s.logits();
	const float m = max_logit(logits, vocab_size);
	float sum = 0;
	for (int i = 0; i < vocab_size; ++i)
		sum += expf(logits[i] - m);
	return expf(logits[index] - m) / sum;
}

int Sampler::sample_argmax(const InferenceState &s) const {
	const float *logits = s.logits();
	int best = 0;
	float m = -FLT_MAX;
	for (int i = 0; i < vocab_size; ++i) {
		if (logits[i] > m) { // strict: the first maximum wins
			m = logits[i];
			best = i;
		}
	}
	return best;
}

int Sampler::sample(const InferenceState &s, float temperature) const {
	if (temperature == 0.0f)
		return sample_argmax(s);
	const float *logits = s.logits();
	const float m = max_logit(logits, vocab_size);
	float sum = 0;
	for (int i = 0; i < vocab_size; ++i)
		sum += expf((logits[i] - m) / temperature);
	const float r = std::rand() / (float)RAND_MAX;
	float cum = 0;
	for (int i = 0; i < vocab_size; ++i) {
		cum += expf((logits[i] - m) / temperature) / sum;
		if (cum >= r)
			return i;
	}
	return vocab_size - 1;
}

} // namespace yalm
