// ref_glue_harness.cpp — TEST INFRASTRUCTURE (oracle/_ref recipe, never shipped).
//
// Drives the REFERENCE's per-block glue functions, which are `static` / `inline`
// in /root/reference/src/infer.cpp and so not reachable from another translation
// unit: this harness textually #includes the UNMODIFIED infer.cpp (found through
// -iquote /root/reference/src, compiled with the reference's flags, Makefile:36-39)
// and calls, on raw little-endian files:
//   rmsnorm   infer.cpp:134-144   ref_glue rmsnorm size eps x.f32 w.f32 out.f32
//   rope      infer.cpp:200-213   ref_glue rope d head_dim pos theta rotary_dim vec.f32 out.f32
//   softmax   infer.cpp:170-185   ref_glue softmax size x.f32 out.f32
//   clip      infer.cpp:195-197   ref_glue clip n v x.f32 out.f32
//   f2h / h2f infer.cpp:11-16     ref_glue f2h n x.f32 out.f16 ; ref_glue h2f n x.f16 out.f32
// No Block, InferenceState or Model is constructed (those need model.cpp, which needs
// spdlog, absent); with -ffunction-sections + --gc-sections the block / forward code the
// included file also defines is dropped. The statement ORDER of _block_cpu
// (infer.cpp:265-317: rmsnorm -> matmul -> clip -> rope -> float_to_half, and the sink
// rotation half_to_float -> rope(pos 1) -> float_to_half) is composed by the golden
// generator (tests/golden/make_ref_glue_golden.py) from these calls.
#include "infer.cpp"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

template <typename T> static std::vector<T> load(const char *path, size_t n) {
	std::vector<T> v(n);
	FILE *f = fopen(path, "rb");
	if (!f || fread(v.data(), sizeof(T), n, f) != n) {
		fprintf(stderr, "ref_glue: cannot read %zu x %zu bytes from %s\n", n, sizeof(T), path);
		exit(2);
	}
	fclose(f);
	return v;
}

template <typename T> static void save(const char *path, const std::vector<T> &v) {
	FILE *f = fopen(path, "wb");
	if (!f || fwrite(v.data(), sizeof(T), v.size(), f) != v.size()) {
		fprintf(stderr, "ref_glue: cannot write %s\n", path);
		exit(2);
	}
	fclose(f);
}

// The static functions are called through volatile pointers, so gcc compiles each as an
// ordinary out-of-line function. Called directly they were inlined into code gcc treats
// as executed once (main and what only main calls): no vectorisation, exact sqrt +
// division instead of rsqrt + Newton -- NOT the code _block_cpu runs. Out of line they
// get the same arithmetic as their inlined copies in the reference's forward (rmsnorm:
// 8-wide FMA sum, the same horizontal reduction, vrsqrtss + one Newton step; compared
// instruction by instruction with _block_cpu's copy).
static void (*volatile ref_rmsnorm)(float *, float *, float *, int, float) = rmsnorm;
static void (*volatile ref_rope)(float *, int, int, int, float, int) = rope;
static void (*volatile ref_softmax)(float *, float *, int) = softmax;

static int run(int argc, char **argv) {
	const std::string op = argv[1];
	if (op == "rmsnorm" && argc == 7) {
		const int n = atoi(argv[2]);
		const float eps = strtof(argv[3], nullptr);
		std::vector<float> x = load<float>(argv[4], n), w = load<float>(argv[5], n), o(n);
		ref_rmsnorm(o.data(), x.data(), w.data(), n, eps);
		save(argv[6], o);
		return 0;
	}
	if (op == "rope" && argc == 9) {
		const int d = atoi(argv[2]), head_dim = atoi(argv[3]), pos = atoi(argv[4]);
		const float theta = strtof(argv[5], nullptr);
		const int rotary_dim = atoi(argv[6]);
		std::vector<float> v = load<float>(argv[7], d);
		ref_rope(v.data(), d, head_dim, pos, theta, rotary_dim);
		save(argv[8], v);
		return 0;
	}
	if (op == "softmax" && argc == 5) {
		const int n = atoi(argv[2]);
		std::vector<float> x = load<float>(argv[3], n), o(n);
		ref_softmax(o.data(), x.data(), n);
		save(argv[4], o);
		return 0;
	}
	if (op == "clip" && argc == 6) {
		const int n = atoi(argv[2]);
		const float v = strtof(argv[3], nullptr);
		std::vector<float> x = load<float>(argv[4], n);
		for (float &e : x)
			e = clip(e, v);
		save(argv[5], x);
		return 0;
	}
	if (op == "f2h" && argc == 5) {
		const int n = atoi(argv[2]);
		std::vector<float> x = load<float>(argv[3], n);
		std::vector<f16_t> o(n);
		for (int i = 0; i < n; ++i)
			o[i] = float_to_half(x[i]);
		save(argv[4], o);
		return 0;
	}
	if (op == "h2f" && argc == 5) {
		const int n = atoi(argv[2]);
		std::vector<f16_t> x = load<f16_t>(argv[3], n);
		std::vector<float> o(n);
		for (int i = 0; i < n; ++i)
			o[i] = half_to_float(x[i]);
		save(argv[4], o);
		return 0;
	}
	fprintf(stderr, "ref_glue: bad op / argument count\n");
	return 1;
}

int main(int argc, char **argv) {
	if (argc < 2) {
		fprintf(stderr, "usage: see the header of ref_glue_harness.cpp\n");
		return 1;
	}
	return run(argc, argv);
}
