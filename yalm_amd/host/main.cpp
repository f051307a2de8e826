// main.cpp — yalm-compatible CLI over the MI355X engine (flags and modes of
// /root/reference/src/main.cpp:17-428): completion, perplexity and passkey,
// -d device switch (cpu | cuda | hip prefixes), -m -n -t -i -f -T -l.
// -t 0 runs the greedy loop with the argmax on the device.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>

#include "model.h"
#include "sampler.h"
#include "tokenizer.h"

using namespace yalm;

static uint64_t now_ms() {
	return (uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
	           std::chrono::system_clock::now().time_since_epoch())
	    .count();
}

[[noreturn]] static void error_usage() {
	fprintf(stderr, "Usage:   yalm <checkpoint> [options]\n");
	fprintf(stderr, "Example: yalm model.yalm -i \"Q: What is the meaning of life?\"\n");
	fprintf(stderr, "Options:\n");
	fprintf(stderr, "  -h Display this help message\n");
	fprintf(stderr, "  -d [cpu,cuda,hip] which device to use (default - hip; cuda is an alias)\n");
	fprintf(stderr, "  -m [completion,passkey,perplexity] which mode to run in (default - completion)\n");
	fprintf(stderr, "  -T <int> sliding window context length (0 - max)\n");
	fprintf(stderr, "\nPerplexity mode options:\n  Choose one:\n    -i <string> input prompt\n");
	fprintf(stderr, "    -f <filepath> input file with prompt\n");
	fprintf(stderr, "Completion mode options:\n");
	fprintf(stderr, "  -n <int>    number of steps to run for in completion mode, default 256. 0 = max_seq_len, "
	                "-1 = infinite\n");
	fprintf(stderr, "  -t <float> temperature (default - 1.0)\n");
	fprintf(stderr, "  Choose one:\n    -i <string> input prompt\n    -f <filepath> input file with prompt\n");
	fprintf(stderr, "Passkey mode options:\n  -n <int>    number of junk lines to insert (default - 250)\n");
	fprintf(stderr, "  -l <int>    passkey position (-1 - random)\n");
	exit(1);
}

static bool print_token_ids() {
	const char *e = getenv("YALM_PRINT_TOKENS");
	return e && atoi(e) != 0;
}

// The sampler's seed: the clock, as the reference (main.cpp constructs Sampler(config,
// get_timestamp_ms())); YALM_SEED fixes it for reproducible runs (tests: the passkey
// value and position come from std::rand after Sampler's srand).
static uint64_t sampler_seed() {
	const char *e = getenv("YALM_SEED");
	return e ? strtoull(e, nullptr, 10) : now_ms();
}

static void setup_device(const std::string &device, Model &model, InferenceState &state) {
	if (device == "cpu") {
		fprintf(stderr, "error: -d cpu is the reference's own CPU backend (src/infer.cpp); this engine implements "
		                "the MI355X device path only. Use -d hip (or cuda).\n");
		exit(1);
	}
	std::cout << "Using HIP (MI355X)" << std::endl;
	model.cuda();
	state.cuda();
}

static std::vector<int> encode_prompt(const Tokenizer &tok, const std::string &prompt, bool show) {
	const uint64_t t0 = now_ms();
	std::vector<int> enc = tok.encode(prompt, true);
	const double s = (now_ms() - t0) / 1000.0;
	if (show)
		std::cout << tok.encoding_to_debug_string(enc) << std::endl;
	printf("Encoding stats: (%zu tokens, throughput: %.5gtok/s, latency: %.5gs/tok, total: %.5gs)\n\n", enc.size(),
	       enc.size() / s, s / enc.size(), s);
	return enc;
}

static void run_completion(const std::string &path, const std::string &device, const std::string &prompt,
                           int context, int num_steps, float temperature) {
	YALMData data;
	if (data.from_file(path) != 0) {
		fprintf(stderr, "error: cannot load %s\n", path.c_str());
		exit(1);
	}
	Model model(data, context);
	InferenceState state(model.config);
	Sampler sampler(model.config, sampler_seed());
	Tokenizer tokenizer(data);
	std::cout << "Model active bytes with full context window: " << model.config->active_bytes(model.config->max_seq_len)
	          << std::endl;
	if (num_steps == 0)
		num_steps = model.config->max_seq_len;
	setup_device(device, model, state);
	model.forward(state, 0, 0); // warm-up: captures the graph, touches all weights

	std::vector<int> encoding = encode_prompt(tokenizer, prompt, true);
	const bool greedy = temperature == 0.0f;
	const uint64_t start = now_ms();
	size_t read_bytes = 0;
	int next = 0;
	// hydrate all but the last prompt token in one batched prefill when the
	// model has that path (yalm_prefill) and there are at least 3 of them (one or
	// two positions are as fast as per-token forwards: profiles/r4m_delay_prefill.txt); the
	// last token goes through the per-token forward, which produces its logits /
	// greedy argmax
	size_t first = 0;
	if (encoding.size() >= 4 && (int)encoding.size() - 1 <= model.config->max_seq_len &&
	    model.prefill(state, encoding.data(), (int)encoding.size() - 1, 0, nullptr)) {
		first = encoding.size() - 1;
		for (size_t pos = 0; pos < first; ++pos)
			read_bytes += model.config->active_bytes(pos);
	}
	for (size_t pos = first; pos < encoding.size(); ++pos) {
		const bool last = pos + 1 == encoding.size();
		if (last && greedy)
			next = model.forward_greedy(state, encoding[pos], (int)pos);
		else
			model.forward(state, encoding[pos], (int)pos,
			              last ? InferenceMode::OUTPUT_LOGITS : InferenceMode::HYDRATE_KV_CACHE);
		read_bytes += model.config->active_bytes(pos);
	}
	const uint64_t end_hydrate = now_ms();
	std::string ids;
	for (int i = 0; i < num_steps || num_steps == -1; ++i) {
		const int token = greedy ? next : sampler.sample(state, temperature);
		std::cout << tokenizer.decode_one(encoding.back(), token) << std::flush;
		ids += std::to_string(token) + " ";
		encoding.push_back(token);
		if (token == tokenizer.eos_id || token == tokenizer.eot_id)
			break;
		const int pos = (int)encoding.size() - 1;
		if (greedy)
			next = model.forward_greedy(state, token, pos);
		else
			model.forward(state, token, pos);
		read_bytes += model.config->active_bytes(pos);
	}
	std::cout << "\n" << std::endl;
	if (print_token_ids())
		fprintf(stderr, "TOKENS: %s\n", ids.c_str());
	const double el = (now_ms() - start) / 1000.0;
	printf("Generation stats:\n  %zu tokens\n  throughput: %.5gtok/s\n  latency: %.5gs/tok\n  hydrate: %.5gs\n"
	       "  bandwidth: %.5gGB/s\n  total: %.5gs\n\n",
	       encoding.size(), encoding.size() / el, el / encoding.size(), (end_hydrate - start) / 1000.0,
	       (double)read_bytes / 1e9 / el, el);
}

static void run_perplexity(const std::string &path, const std::string &device, const std::string &prompt,
                           int context) {
	YALMData data;
	if (data.from_file(path) != 0) {
		fprintf(stderr, "error: cannot load %s\n", path.c_str());
		exit(1);
	}
	Model model(data, context);
	InferenceState state(model.config);
	Sampler sampler(model.config, sampler_seed());
	Tokenizer tokenizer(data);
	std::cout << "Model active bytes with full context window: " << model.config->active_bytes(model.config->max_seq_len)
	          << std::endl;
	setup_device(device, model, state);
	model.forward(state, 0, 0);
	std::vector<int> encoding = encode_prompt(tokenizer, prompt, true);
	double sum_logprob = 0.0, ss_logprob = 0.0;
	const uint64_t start = now_ms();
	size_t read_bytes = 0;
	const size_t N = encoding.size() - 1;
	// positions inside the context window in one batched prefill (per-position
	// log p from a vocab-tiled log-softmax on the device); the rest, past
	// max_seq_len (sliding window), position by position as in the reference
	size_t pos = 0;
	const size_t B = std::min(encoding.size(), (size_t)model.config->max_seq_len);
	std::vector<float> lps(B);
	// the split-operand precision form: every activation operand carries the f32 the
	// reference keeps to ~2^-22, so the perplexity is the reference's; a
	// model whose activations do not fit the prefill's operands (YALM_ERR_UNSUPPORTED) runs
	// position by position below, as the reference does
	if (B >= 2 && model.prefill(state, encoding.data(), (int)B, 0, lps.data(), true)) {
		for (; pos + 1 < B; ++pos) {
			const double lp = lps[pos];
			sum_logprob += lp;
			ss_logprob += lp * lp;
			read_bytes += model.config->active_bytes(pos);
		}
		std::cout << "\r Computing perplexity..." << pos << "/" << N << " (batched prefill)" << std::flush;
	}
	for (; pos + 1 < encoding.size(); ++pos) {
		std::cout << "\r Computing perplexity..." << pos + 1 << "/" << N << std::flush;
		model.forward(state, encoding[pos], (int)pos);
		read_bytes += model.config->active_bytes(pos);
		const double lp = std::log(sampler.sample_prob(encoding[pos + 1], state));
		sum_logprob += lp;
		ss_logprob += lp * lp;
	}
	std::cout << std::endl;
	const double el = (now_ms() - start) / 1000.0;
	const double ppl = std::exp(-sum_logprob / N);
	const double err = ppl * std::sqrt((ss_logprob - sum_logprob * sum_logprob / N) / N / N);
	printf("Stats:\n  %zu tokens\n  perplexity: %.5g ± %.5g\n  throughput: %.5gtok/s\n  latency: %.5gs/tok\n"
	       "  bandwidth: %.5gGB/s\n  total: %.5gs\n\n",
	       N, ppl, err, N / el, el / N, (double)read_bytes / 1e9 / el, el);
}

static void run_passkey(const std::string &path, const std::string &device, int context, int n_junk,
                        int passkey_pos) {
	YALMData data;
	if (data.from_file(path) != 0) {
		fprintf(stderr, "error: cannot load %s\n", path.c_str());
		exit(1);
	}
	Model model(data, context);
	InferenceState state(model.config);
	Sampler sampler(model.config, sampler_seed());
	Tokenizer tokenizer(data);
	std::cout << "Model active bytes with full context window: " << model.config->active_bytes(model.config->max_seq_len)
	          << std::endl;
	setup_device(device, model, state);
	model.forward(state, 0, 0);
	const std::string PREFIX = "There is an important info hidden inside a lot of irrelevant text. "
	                           "Find it and memorize them. I will quiz you about the important information there.";
	const std::string SUFFIX = " What is the pass key? The pass key is";
	// YALM_SEED (tests): re-seeded here, because the HIP runtime's initialisation above draws
	// from std::rand too (two runs with the same seed otherwise got different passkeys)
	if (getenv("YALM_SEED"))
		std::srand((unsigned)sampler_seed());
	const int passkey = std::rand() % 50000 + 1;
	const int ppos = passkey_pos == -1 ? std::rand() % n_junk : passkey_pos;
	std::string prompt = PREFIX;
	for (int i = 0; i < n_junk; i++) {
		if (i % n_junk == ppos)
			prompt += " The pass key is " + std::to_string(passkey) + ". Remember it. " + std::to_string(passkey) +
			          " is the pass key.";
		prompt += " The grass is green. The sky is blue. The sun is yellow. Here we go. There and back again.";
	}
	prompt += SUFFIX;
	std::vector<int> encoding = encode_prompt(tokenizer, prompt, false);
	printf("Passkey test:\n  prompt: %zu tokens\n  passkey: %d\n  passkey token index: ~%d\n\n", encoding.size(),
	       passkey, (int)(((float)ppos) / n_junk * encoding.size()));
	const size_t N = encoding.size();
	if (print_token_ids()) {
		std::string pids;
		for (int t : encoding)
			pids += std::to_string(t) + " ";
		fprintf(stderr, "PROMPT: %s\n", pids.c_str());
	}
	// the positions inside the context window before the last one in one batched prefill
	// (yalm_prefill; the reference hydrates them one forward each, main.cpp:228-232); the
	// rest -- past max_seq_len (sliding window + sinks) and the last prompt token, whose
	// logits start the answer -- one forward each
	size_t first = 0;
	const size_t H = std::min(N - 1, (size_t)model.config->max_seq_len);
	if (H >= 3 && model.prefill(state, encoding.data(), (int)H, 0, nullptr))
		first = H;
	for (size_t pos = first; pos < N; ++pos) {
		std::cout << "\r Running passkey test..." << pos + 1 << "/" << N << std::flush;
		model.forward(state, encoding[pos], (int)pos,
		              pos + 1 == N ? InferenceMode::OUTPUT_LOGITS : InferenceMode::HYDRATE_KV_CACHE);
	}
	std::cout << std::endl << SUFFIX << std::flush;
	if (const char *dump = getenv("YALM_DUMP_LOGITS")) { // test hook: the logits the answer starts from
		FILE *f = fopen(dump, "wb");
		if (!f || fwrite(state.logits(), sizeof(float), model.config->vocab_size, f) != (size_t)model.config->vocab_size) {
			fprintf(stderr, "error: cannot write %s\n", dump);
			exit(1);
		}
		fclose(f);
	}
	std::string ids;
	for (size_t pos = N; pos < N + 16; ++pos) {
		const int token = sampler.sample_argmax(state);
		std::cout << tokenizer.decode_one(encoding.back(), token) << std::flush;
		ids += std::to_string(token) + " ";
		encoding.push_back(token);
		if (token == tokenizer.eos_id || token == tokenizer.eot_id)
			break;
		model.forward(state, token, (int)pos);
	}
	std::cout << std::endl;
	if (print_token_ids())
		fprintf(stderr, "TOKENS: %s\n", ids.c_str());
}

int main(int argc, char *argv[]) {
	std::string checkpoint, device = "hip", mode = "completion", prompt, prompt_path;
	int context = 0, num_steps = 256, n_junk = 250, passkey_pos = -1;
	float temperature = 1.0f;
	if (argc < 2)
		error_usage();
	checkpoint = argv[1];
	for (int i = 2; i < argc; i += 2) {
		if (i + 1 >= argc || argv[i][0] != '-' || strlen(argv[i]) != 2)
			error_usage();
		const std::string v = argv[i + 1];
		switch (argv[i][1]) {
		case 'h': error_usage();
		case 'm':
			if (std::string("completion").starts_with(v))
				mode = "completion";
			else if (std::string("passkey").starts_with(v))
				mode = "passkey";
			else if (std::string("perplexity").starts_with(v))
				mode = "perplexity";
			else
				error_usage();
			break;
		case 'd':
			if (std::string("cpu").starts_with(v))
				device = "cpu";
			else if (std::string("cuda").starts_with(v) || std::string("hip").starts_with(v))
				device = "hip";
			else
				error_usage();
			break;
		case 'i': prompt = v; break;
		case 't': temperature = std::stof(v); break;
		case 'f': prompt_path = v; break;
		case 'T': context = std::stoi(v); break;
		case 'l': passkey_pos = std::stoi(v); break;
		case 'n':
			num_steps = std::stoi(v);
			n_junk = num_steps;
			break;
		default: error_usage();
		}
	}
	const int has_prompt = prompt.size() > 0, has_path = prompt_path.size() > 0;
	if (mode == "completion" || mode == "perplexity") {
		if (has_prompt + has_path != 1)
			error_usage();
		if (has_path) {
			std::ifstream f(prompt_path);
			if (!f.is_open()) {
				std::cerr << "Error: could not open file " << prompt_path << std::endl;
				return 1;
			}
			std::stringstream buf;
			buf << f.rdbuf();
			prompt = buf.str();
		}
	} else if (passkey_pos != -1 && (passkey_pos >= n_junk || passkey_pos < 0)) {
		std::cerr << "Error: passkey position must be between 0 and " << n_junk - 1 << std::endl;
		return 1;
	}
	fprintf(stderr, "[yalm] Using checkpoint: %s\n", checkpoint.c_str());
	try {
		if (mode == "completion")
			run_completion(checkpoint, device, prompt, context, num_steps, temperature);
		else if (mode == "passkey")
			run_passkey(checkpoint, device, context, n_junk, passkey_pos);
		else
			run_perplexity(checkpoint, device, prompt, context);
	} catch (const std::exception &e) {
		fprintf(stderr, "error: %s\n", e.what());
		return 1;
	}
	return 0;
}
