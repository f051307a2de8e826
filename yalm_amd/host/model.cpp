#include "model.h"

#include <cstdlib>

#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <iostream>

namespace yalm {

void check(int rc, const char *what) {
	if (rc != YALM_OK)
		throw YalmRuntimeError(std::string(what) + ": " + yalm_last_error());
}

static int meta_int(const Json &md, const char *k) {
	return std::stoi(md.at(k).as_string());
}

void Config::from_yalm(YALMData &yalm, int context) {
	const Json &md = yalm.metadata;
	dim = meta_int(md, "dim");
	hidden_dim = meta_int(md, "hidden_dim");
	head_dim = meta_int(md, "head_dim");
	n_layers = meta_int(md, "n_layers");
	n_heads = meta_int(md, "n_heads");
	n_kv_heads = meta_int(md, "n_kv_heads");
	vocab_size = meta_int(md, "vocab_size");
	n_experts = md.contains("n_experts") ? meta_int(md, "n_experts") : 0;
	n_experts_active = md.contains("n_experts_active") ? meta_int(md, "n_experts_active") : 0;
	max_seq_len = std::min(meta_int(md, "max_seq_len"), 4096);
	if (context)
		max_seq_len = context;
	rope_theta = std::stof(md.at("rope_theta").as_string());
	rotary_dim = meta_int(md, "rotary_dim");
	norm_eps = std::stof(md.value("norm_eps", "1e-5"));
	const std::string act_str = md.value("act_type", "gelu");
	if (act_str == "gelu") {
		act = ActivationType::GELU;
	} else if (act_str == "silu") {
		act = ActivationType::SILU;
	} else {
		std::cerr << "unsupported act_type, defaulting to gelu" << std::endl;
		act = ActivationType::GELU;
	}
	if (md.value("norm_type", "rmsnorm") != "rmsnorm")
		std::cerr << "unsupported norm_type, defaulting to rmsnorm" << std::endl;
	norm_type = LayerNormType::RMSNorm;
	qkv_clip = md.contains("qkv_clip") ? std::stof(md.at("qkv_clip").as_string()) : FLT_MAX;
	const std::string dtype = md.at("dtype").as_string();
	if (dtype == "fp32")
		weight_dtype = DType::F32;
	else if (dtype == "fp16")
		weight_dtype = DType::F16;
	else if (dtype == "fp8")
		weight_dtype = DType::F8E5M2;
	else
		throw std::runtime_error("FATAL: unsupported dtype: " + dtype);
	if (n_experts > 0)
		throw std::runtime_error("FATAL: mixture-of-experts models are CPU-only in the reference (infer.cu:865-867) "
		                         "and out of scope for this engine");
}

size_t Config::active_bytes(size_t pos) const {
	const size_t wsz = dtype_size(weight_dtype);
	size_t per_block = 2 * dim * sizeof(float);
	per_block += (size_t)n_heads * head_dim * dim * wsz;
	per_block += 2 * (size_t)n_kv_heads * head_dim * dim * wsz;
	per_block += (size_t)n_heads * head_dim * dim * wsz;
	per_block += 3 * (size_t)dim * hidden_dim * wsz;
	const size_t kv_len = std::min((size_t)max_seq_len, pos + 1);
	per_block += 2 * kv_len * n_kv_heads * head_dim * sizeof(f16_t);
	return dim * wsz + n_layers * per_block + dim * sizeof(float) + (size_t)vocab_size * dim * wsz;
}

yalm_config Config::to_c() const {
	yalm_config c{};
	c.dim = dim;
	c.hidden_dim = hidden_dim;
	c.head_dim = head_dim;
	c.n_layers = n_layers;
	c.n_heads = n_heads;
	c.n_kv_heads = n_kv_heads;
	c.vocab_size = vocab_size;
	c.max_seq_len = max_seq_len;
	c.rope_theta = rope_theta;
	c.rotary_dim = rotary_dim;
	c.norm_eps = norm_eps;
	c.act = act == ActivationType::SILU ? YALM_SILU : YALM_GELU;
	c.qkv_clip = qkv_clip;
	c.weight_dtype = (int)weight_dtype;
	return c;
}

// model.cpp:104-132
static const void *check_tensor(const Tensor *t, DType dt, std::array<int, 4> shape) {
	if (!t)
		throw std::runtime_error("FATAL: missing tensor");
	if (t->dtype != dt || t->shape != shape)
		throw std::runtime_error("FATAL: tensor mismatch for " + t->name + " (got " + dtype_to_string(t->dtype) +
		                         ", expected " + dtype_to_string(dt) + ")");
	return t->data;
}

static const Tensor *get_tensor(const YALMData &y, const std::string &key) {
	auto it = y.tensors.find(key);
	if (it == y.tensors.end())
		throw std::runtime_error("FATAL: missing tensor: " + key);
	return &it->second;
}

InferenceState::InferenceState(std::shared_ptr<Config> config) : _config(std::move(config)) {
	_logits = new float[_config->vocab_size]();
}

InferenceState::~InferenceState() {
	if (_decoder)
		yalm_decoder_destroy(_decoder);
	if (_device == Device::HIP)
		yalm_unregister_host(_logits);
	delete[] _logits;
}

void InferenceState::cuda() {
	if (_device != Device::CPU)
		return;
	_device = Device::HIP;
	// pinned logits so the OUTPUT copy is a straight DMA (model.cpp:338)
	check(yalm_register_host(_logits, sizeof(float) * _config->vocab_size), "register logits");
}

Block::Block(int layer_i, std::shared_ptr<Config> config, const Tensor *rms_att_weight, const Tensor *rms_ffn_weight,
             const Tensor *wq, const Tensor *wk, const Tensor *wv, const Tensor *wo, const Tensor *w1, const Tensor *w2,
             const Tensor *w3)
    : _layer_i(layer_i), _config(std::move(config)) {
	const Config &c = *_config;
	const DType dt = c.weight_dtype;
	_rms_att = check_tensor(rms_att_weight, DType::F32, {c.dim, 0, 0, 0});
	_rms_ffn = check_tensor(rms_ffn_weight, DType::F32, {c.dim, 0, 0, 0});
	_wq = check_tensor(wq, dt, {c.n_heads * c.head_dim, c.dim, 0, 0});
	_wk = check_tensor(wk, dt, {c.n_kv_heads * c.head_dim, c.dim, 0, 0});
	_wv = check_tensor(wv, dt, {c.n_kv_heads * c.head_dim, c.dim, 0, 0});
	_wo = check_tensor(wo, dt, {c.dim, c.n_heads * c.head_dim, 0, 0});
	_w1 = check_tensor(w1, dt, {c.hidden_dim, c.dim, 0, 0});
	_w2 = check_tensor(w2, dt, {c.dim, c.hidden_dim, 0, 0});
	_w3 = check_tensor(w3, dt, {c.hidden_dim, c.dim, 0, 0});
}

Block::~Block() {
	for (void *p : _owned)
		yalm_free(p);
}

static const void *upload(std::vector<void *> &owned, const void *host, size_t bytes) {
	void *d = yalm_upload(host, bytes);
	if (!d)
		throw YalmRuntimeError(std::string("upload: ") + yalm_last_error());
	owned.push_back(d);
	return d;
}

void Block::cuda() {
	if (_device != Device::CPU)
		return;
	const Config &c = *_config;
	const size_t wsz = dtype_size(c.weight_dtype);
	const size_t q_dim = (size_t)c.n_heads * c.head_dim, kv_dim = (size_t)c.n_kv_heads * c.head_dim;
	_rms_att = upload(_owned, _rms_att, c.dim * sizeof(float));
	_rms_ffn = upload(_owned, _rms_ffn, c.dim * sizeof(float));
	_wq = upload(_owned, _wq, q_dim * c.dim * wsz);
	_wk = upload(_owned, _wk, kv_dim * c.dim * wsz);
	_wv = upload(_owned, _wv, kv_dim * c.dim * wsz);
	_wo = upload(_owned, _wo, c.dim * q_dim * wsz);
	_w1 = upload(_owned, _w1, (size_t)c.hidden_dim * c.dim * wsz);
	_w2 = upload(_owned, _w2, (size_t)c.dim * c.hidden_dim * wsz);
	_w3 = upload(_owned, _w3, (size_t)c.hidden_dim * c.dim * wsz);
	_device = Device::HIP;
	// The KV cache is allocated (zeroed) by the decoder in HBM: no host copy
	// to upload (model.cpp:208-210 uploads a zero host array).
}

yalm_block_weights Block::device_weights() const {
	yalm_block_weights w{};
	w.rms_att = (const float *)_rms_att;
	w.rms_ffn = (const float *)_rms_ffn;
	w.wq = _wq;
	w.wk = _wk;
	w.wv = _wv;
	w.wo = _wo;
	w.w1 = _w1;
	w.w2 = _w2;
	w.w3 = _w3;
	return w;
}

Model::Model(YALMData &yalm, int context) {
	config = std::make_shared<Config>();
	config->from_yalm(yalm, context);
	std::cout << "loading model with dtype: " << dtype_to_string(config->weight_dtype) << std::endl;
	const Config &c = *config;
	token_embedding_table = check_tensor(get_tensor(yalm, "model.embed.weight"), c.weight_dtype,
	                                     {c.vocab_size, c.dim, 0, 0});
	for (int i = 0; i < c.n_layers; ++i) {
		const std::string p = "model.layers." + std::to_string(i) + ".";
		blocks.emplace_back(std::make_shared<Block>(
		    i, config, get_tensor(yalm, p + "attn.norm.weight"), get_tensor(yalm, p + "mlp.norm.weight"),
		    get_tensor(yalm, p + "attn.wq.weight"), get_tensor(yalm, p + "attn.wk.weight"),
		    get_tensor(yalm, p + "attn.wv.weight"), get_tensor(yalm, p + "attn.wo.weight"),
		    get_tensor(yalm, p + "mlp.w1.weight"), get_tensor(yalm, p + "mlp.w2.weight"),
		    get_tensor(yalm, p + "mlp.w3.weight")));
	}
	rms_final_weight = check_tensor(get_tensor(yalm, "model.norm.weight"), DType::F32, {c.dim, 0, 0, 0});
	_tied = yalm.tensors.count("model.output.weight") == 0;
	wcls = _tied ? token_embedding_table
	             : check_tensor(get_tensor(yalm, "model.output.weight"), c.weight_dtype, {c.vocab_size, c.dim, 0, 0});
}

Model::~Model() {
	blocks.clear();
	for (void *p : _owned)
		yalm_free(p);
}

void Model::cuda() {
	if (_device != Device::CPU)
		return;
	check(yalm_set_device(0), "set device");
	const Config &c = *config;
	const size_t wsz = dtype_size(c.weight_dtype);
	token_embedding_table = upload(_owned, token_embedding_table, (size_t)c.vocab_size * c.dim * wsz);
	for (auto &b : blocks)
		b->cuda();
	rms_final_weight = upload(_owned, rms_final_weight, c.dim * sizeof(float));
	// tied classifier: alias the uploaded embedding (the reference uploads it twice, model.cpp:388/393)
	wcls = _tied ? token_embedding_table : upload(_owned, wcls, (size_t)c.vocab_size * c.dim * wsz);
	_device = Device::HIP;
}

void Model::ensure_decoder(InferenceState &s) {
	if (s.device() != _device)
		throw std::runtime_error("FATAL: inference state device mismatch");
	if (_device != Device::HIP)
		throw std::runtime_error("this engine runs on the HIP device only: call model.cuda(); state.cuda() "
		                         "(the CPU path is the reference's own -d cpu)");
	if (s._decoder)
		return;
	std::vector<yalm_block_weights> bw;
	for (auto &b : blocks)
		bw.push_back(b->device_weights());
	yalm_model_weights mw{token_embedding_table, (const float *)rms_final_weight, wcls, bw.data()};
	const yalm_config cc = config->to_c();
	check(yalm_decoder_create(&cc, &mw, nullptr, &s._decoder), "decoder create");
}

void Model::forward(InferenceState &s, int token, int pos, InferenceMode mode) {
	ensure_decoder(s);
	s.set_mode(mode);
	check(yalm_forward(s._decoder, token, pos,
	                   mode == InferenceMode::OUTPUT_LOGITS ? YALM_OUTPUT_LOGITS : YALM_HYDRATE_KV_CACHE,
	                   mode == InferenceMode::OUTPUT_LOGITS ? s._logits : nullptr),
	      "forward");
}

bool Model::prefill(InferenceState &s, const int *tokens, int n, int pos0, float *logprobs, bool split) {
	const char *off = getenv("YALM_NO_PREFILL");
	if ((off && atoi(off) != 0) || n <= 0)
		return false;
	ensure_decoder(s);
	check(yalm_set_prefill_precision(s._decoder, split ? YALM_PREFILL_SPLIT : YALM_PREFILL_FAST), "prefill precision");
	const int r = yalm_prefill(s._decoder, tokens, n, pos0, logprobs);
	if (r == YALM_ERR_UNSUPPORTED)
		return false;
	check(r, "prefill");
	return true;
}

int Model::forward_greedy(InferenceState &s, int token, int pos) {
	ensure_decoder(s);
	int next = 0;
	check(yalm_generate_greedy(s._decoder, token, pos, 1, &next), "greedy step");
	return next;
}

} // namespace yalm
