// Regenerates the seeded inputs of the reference's CPU-vs-GPU kernel test
// (/root/reference/src/test.cpp:128-206) with the same libstdc++ engines:
// std::default_random_engine(seed) + std::normal_distribution<float>(0, 1),
// value = dist(gen) * scale_factor (test.cpp:128-146). Own code; the values
// are data (fixtures), written as raw little-endian float32 in a fixed order.
// Build+run: tests/golden/make_golden.py
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

static std::vector<float> fill(size_t n, unsigned long seed, float scale = 1.0f) {
	std::default_random_engine gen(seed);
	std::normal_distribution<float> dist(0.0, 1.0);
	std::vector<float> v(n);
	for (size_t i = 0; i < n; i++)
		v[i] = dist(gen) * scale;
	return v;
}

static void put(FILE *f, const char *name, const std::vector<float> &v) {
	unsigned long long n = v.size();
	fprintf(f, "%s %llu\n", name, n);
	fwrite(v.data(), sizeof(float), v.size(), f);
	fputc('\n', f);
}

int main(int argc, char **argv) {
	const int head_dim = 16, n_heads = 16, dim = head_dim * n_heads, hidden_dim = dim, n_kv_heads = 8,
	          max_seq_len = 4;
	FILE *f = fopen(argc > 1 ? argv[1] : "test_cpp_inputs.bin", "wb");
	// matmul (test.cpp:158-168)
	put(f, "matmul_w", fill(dim * head_dim, 0));
	put(f, "matmul_x", fill(dim, 1));
	// mha (test.cpp:171-188): values then rounded to f16 with _cvtss_sh(v, 0)
	put(f, "mha_kb", fill(max_seq_len * n_kv_heads * head_dim, 0));
	put(f, "mha_vb", fill(max_seq_len * n_kv_heads * head_dim, 1));
	put(f, "mha_q", fill(n_heads * head_dim, 2));
	// ffn (test.cpp:191-205)
	put(f, "ffn_x", fill(dim, 0));
	put(f, "ffn_w1", fill(dim * hidden_dim, 1, 1.0 / sqrtf(dim)));
	put(f, "ffn_w2", fill(hidden_dim * dim, 2, 1.0 / sqrtf(hidden_dim)));
	put(f, "ffn_w3", fill(dim * hidden_dim, 3, 1.0 / sqrtf(dim)));
	fclose(f);
	return 0;
}
