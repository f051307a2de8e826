// sampler.h — host samplers over the logits (reference sampler.cpp:11-65):
// softmax probability of one index, first-max argmax, temperature sampling
// with std::rand seeded at construction.
#pragma once

#include <cstdint>
#include <memory>

#include "model.h"

namespace yalm {

struct Sampler {
	int vocab_size = 0;
	Sampler(const std::shared_ptr<Config> config, uint64_t seed);
	float sample_prob(int index, const InferenceState &s) const;
	int sample_argmax(const InferenceState &s) const;
	int sample(const InferenceState &s, float temperature) const;
};

} // namespace yalm
