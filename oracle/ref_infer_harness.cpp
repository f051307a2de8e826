// ref_infer_harness.cpp — TEST INFRASTRUCTURE (oracle/_ref recipe, never shipped).
//
// Drives the REFERENCE CPU kernels, compiled unmodified from
// /root/reference/src/infer.cpp where it lies (oracle/Makefile target
// `ref-infer`), through the test hooks the reference itself exposes
// (model.h:353-385):
//   matmul_cpu(float*, float*, float*, n, d)   infer.cpp:405-407 -> matmul f32 48-59
//   matmul_cpu(float*, float*, f16_t*, n, d)   infer.cpp:408-410 -> matmul f16 63-98
//   mha_cpu(...)                               infer.cpp:387-403 -> attn 216-248
//   ffn_cpu(..., ActivationType)               infer.cpp:412-438
// model.h includes cuda_runtime_api.h; the genuine NVIDIA header shipped in the
// image (triton/backends/nvidia/include) satisfies it. infer.o is linked with
// --gc-sections, so _forward_cpu (which needs Block::block from model.cpp and
// therefore spdlog, absent) is dropped; no Block / InferenceState is built.
//
// usage (all buffers raw little-endian files):
//   ref_infer matmul_f32 n d x.f32 w.f32 out.f32
//   ref_infer matmul_f16 n d x.f32 w.f16 out.f32
//   ref_infer mha head_dim kv_len max_seq_len n_heads n_kv_heads q.f32 kb.f16 vb.f16 xout.f32 att.f32
//   ref_infer ffn hidden_dim dim act(0=gelu,1=silu) x.f32 w1.f32 w2.f32 w3.f32 out.f32
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "model.h"

template <typename T> static std::vector<T> load(const char *path, size_t n) {
	std::vector<T> v(n);
	FILE *f = fopen(path, "rb");
	if (!f || fread(v.data(), sizeof(T), n, f) != n) {
		fprintf(stderr, "ref_infer: cannot read %zu x %zu bytes from %s\n", n, sizeof(T), path);
		exit(2);
	}
	fclose(f);
	return v;
}

template <typename T> static void save(const char *path, const std::vector<T> &v) {
	FILE *f = fopen(path, "wb");
	if (!f || fwrite(v.data(), sizeof(T), v.size(), f) != v.size()) {
		fprintf(stderr, "ref_infer: cannot write %s\n", path);
		exit(2);
	}
	fclose(f);
}

int main(int argc, char **argv) {
	if (argc < 2) {
		fprintf(stderr, "usage: see the header of ref_infer_harness.cpp\n");
		return 1;
	}
	std::string op = argv[1];
	if ((op == "matmul_f32" || op == "matmul_f16") && argc == 7) {
		int n = atoi(argv[2]), d = atoi(argv[3]);
		std::vector<float> x = load<float>(argv[4], n), out(d);
		if (op == "matmul_f32") {
			std::vector<float> w = load<float>(argv[5], (size_t)n * d);
			matmul_cpu(out.data(), x.data(), w.data(), n, d);
		} else {
			std::vector<f16_t> w = load<f16_t>(argv[5], (size_t)n * d);
			matmul_cpu(out.data(), x.data(), w.data(), n, d);
		}
		save(argv[6], out);
		return 0;
	}
	if (op == "mha" && argc == 12) {
		int head_dim = atoi(argv[2]), kv_len = atoi(argv[3]), max_seq_len = atoi(argv[4]);
		int n_heads = atoi(argv[5]), n_kv_heads = atoi(argv[6]);
		size_t kv = (size_t)max_seq_len * n_kv_heads * head_dim;
		std::vector<float> q = load<float>(argv[7], (size_t)n_heads * head_dim);
		std::vector<f16_t> kb = load<f16_t>(argv[8], kv), vb = load<f16_t>(argv[9], kv);
		std::vector<float> xout((size_t)n_heads * head_dim), att((size_t)n_heads * max_seq_len, 0.0f);
		mha_cpu(xout.data(), att.data(), kb.data(), vb.data(), q.data(), head_dim, kv_len, max_seq_len, n_heads,
		        n_kv_heads);
		save(argv[10], xout);
		save(argv[11], att);
		return 0;
	}
	if (op == "ffn" && argc == 10) {
		int hidden = atoi(argv[2]), dim = atoi(argv[3]), act = atoi(argv[4]);
		std::vector<float> x = load<float>(argv[5], dim);
		std::vector<float> w1 = load<float>(argv[6], (size_t)hidden * dim);
		std::vector<float> w2 = load<float>(argv[7], (size_t)dim * hidden);
		std::vector<float> w3 = load<float>(argv[8], (size_t)hidden * dim);
		std::vector<float> out(dim);
		ffn_cpu(out.data(), x.data(), w1.data(), w2.data(), w3.data(), hidden, dim,
		        act ? ActivationType::SILU : ActivationType::GELU);
		save(argv[9], out);
		return 0;
	}
	fprintf(stderr, "ref_infer: bad arguments for '%s'\n", op.c_str());
	return 1;
}
