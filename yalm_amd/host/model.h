// model.h — C++20 host API with the reference's shape (Config, InferenceState,
// Block, Model: /root/reference/src/model.h:41-327) over the MI355X engine's
// C ABI (include/yalm_hip.h). No HIP/CUDA types appear here: the reference
// leaked cudaStream_t / cudaGraph_t into this header (model.h:4, 39, 70-79);
// the device state lives behind the opaque yalm_decoder.
//
// Device::HIP replaces Device::CUDA. The CPU device is the reference's own
// infer.cpp path and is not part of this engine;
// forward() on a CPU-resident model raises.
#pragma once

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/yalm_hip.h"
#include "codec.h"

namespace yalm {

constexpr int KV_SINKS = 2; // model.h:12

enum class ActivationType { GELU, SILU };
enum class LayerNormType { RMSNorm };
enum class Device { CPU, HIP };
enum class InferenceMode { HYDRATE_KV_CACHE, OUTPUT_LOGITS };

struct YalmRuntimeError : std::runtime_error {
	using std::runtime_error::runtime_error;
};
// Throws with yalm_last_error() when a C-ABI call fails.
void check(int rc, const char *what);

struct Config {
	int dim = 0, hidden_dim = 0, head_dim = 0, n_layers = 0, n_heads = 0, n_kv_heads = 0, vocab_size = 0,
	    max_seq_len = 0;
	float rope_theta = 10000.f;
	int rotary_dim = 0;
	float norm_eps = 1e-5f;
	ActivationType act = ActivationType::GELU;
	LayerNormType norm_type = LayerNormType::RMSNorm;
	float qkv_clip = 3.40282347e38f;
	int n_experts = 0, n_experts_active = 0;
	DType weight_dtype = DType::F16;

	// model.cpp:17-75 (max_seq_len = min(meta, 4096) unless context != 0)
	void from_yalm(YALMData &yalm, int context = 0);
	// Algorithmic HBM bytes for one token at position pos (the
	// classifier counted at the weight dtype, unlike model.cpp:99's fp32).
	size_t active_bytes(size_t pos) const;
	yalm_config to_c() const;
};

struct InferenceState {
	explicit InferenceState(std::shared_ptr<Config> config);
	~InferenceState();
	InferenceState(const InferenceState &) = delete;
	InferenceState &operator=(const InferenceState &) = delete;

	float *logits() const {
		return _logits; // host memory, valid after an OUTPUT_LOGITS forward
	}
	void cuda(); // reference name (model.cpp:323); selects the HIP device
	void hip() {
		cuda();
	}
	Device device() const {
		return _device;
	}
	InferenceMode mode() const {
		return _mode;
	}
	void set_mode(InferenceMode m) {
		_mode = m;
	}
	yalm_decoder decoder() const {
		return _decoder;
	}

private:
	friend struct Model;
	std::shared_ptr<Config> _config;
	Device _device = Device::CPU;
	InferenceMode _mode = InferenceMode::OUTPUT_LOGITS;
	float *_logits = nullptr;
	yalm_decoder _decoder = nullptr;
};

struct Block {
	Block(int layer_i, std::shared_ptr<Config> config, const Tensor *rms_att_weight, const Tensor *rms_ffn_weight,
	      const Tensor *wq, const Tensor *wk, const Tensor *wv, const Tensor *wo, const Tensor *w1, const Tensor *w2,
	      const Tensor *w3);
	~Block();
	void cuda(); // device weight upload (model.cpp:185-211)
	yalm_block_weights device_weights() const;

private:
	int _layer_i = 0;
	std::shared_ptr<Config> _config;
	Device _device = Device::CPU;
	const void *_rms_att = nullptr, *_rms_ffn = nullptr;
	const void *_wq = nullptr, *_wk = nullptr, *_wv = nullptr, *_wo = nullptr, *_w1 = nullptr, *_w2 = nullptr,
	           *_w3 = nullptr;
	std::vector<void *> _owned;
};

struct Model {
	std::shared_ptr<Config> config;
	std::vector<std::shared_ptr<Block>> blocks;
	const void *token_embedding_table = nullptr;
	const void *rms_final_weight = nullptr;
	const void *wcls = nullptr;

	Model(YALMData &yalm, int context = 0);
	~Model();
	Model(const Model &) = delete;
	Model &operator=(const Model &) = delete;

	// Model::forward (model.cpp:396-407). OUTPUT_LOGITS leaves logits in s.logits().
	void forward(InferenceState &s, int token, int pos, InferenceMode mode = InferenceMode::OUTPUT_LOGITS);
	// Greedy (-t 0) step on the device: forward + first-max argmax without
	// copying logits to the host. Returns the next token.
	int forward_greedy(InferenceState &s, int token, int pos);
	// Batched MFMA prefill of tokens[0..n) at positions pos0.. (yalm_prefill):
	// fills the KV cache; logprobs (may be null) gets log p(tokens[i+1]) per
	// position; split: the split-operand precision form (yalm_set_prefill_precision).
	// Returns false when this model's shape/dtype has no prefill path (f16 / fp8
	// weights, dims multiple of 128, head_dim 64|128), its activations leave the
	// prefill's f16 operand range, or YALM_NO_PREFILL=1; the caller then runs the
	// per-position forward.
	bool prefill(InferenceState &s, const int *tokens, int n, int pos0, float *logprobs, bool split = false);
	void cuda(); // Model::cuda (model.cpp:380-394)
	void hip() {
		cuda();
	}
	Device device() const {
		return _device;
	}

private:
	void ensure_decoder(InferenceState &s);
	Device _device = Device::CPU;
	bool _tied = false;
	std::vector<void *> _owned;
};

} // namespace yalm
