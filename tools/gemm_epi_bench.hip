// gemm_epi_bench.hip — what the prefill GEMM epilogues cost: the 8-phase kernel
// (prefill_gemm.h gemm8p_kernel) at the Llama-3.2-3B T = 4096 shapes with its product
// epilogue vs a null epilogue that keeps the accumulators alive (stores only on an
// impossible value), random f16 operands, interleaved rounds in one process.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -I yalm_amd/csrc \
//          -o tools/gemm_epi_bench tools/gemm_epi_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "prefill_gemm.h"

// round-5 epilogues (before the range guard and split forms), the A/B baseline
namespace pf {
template <int ACT>
struct E16GluR5 {
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	uint16_t *h;
	int ldh, M;
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(f32x4_t (&acc)[FI][FJ], int m0, int n0, int lane, int, int) const {
#pragma unroll
		for (int i = 0; i < FI; ++i)
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const int m = m0 + 16 * i + crow16(r, lane);
				if (m >= M)
					continue;
#pragma unroll
				for (int j = 0; j < FJ / 2; ++j)
					h[(size_t)m * ldh + n0 + 16 * j + (lane & 15)] =
					    f2h_bits(act_fast<ACT>(acc[i][j][r]) * acc[i][j + FJ / 2][r]);
			}
	}
};

struct E16QKVR5 {
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	uint16_t *q;
	uint16_t *kc, *vc;
	const float *rope;
	int M, q_dim, kv_dim, head_dim, pos0;
	float clip;
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(f32x4_t (&acc)[FI][FJ], int m0, int n0, int lane, int, int) const {
		const bool odd = lane & 1;
#pragma unroll
		for (int j = 0; j < FJ; ++j) {
			const int nb = __builtin_amdgcn_readfirstlane(n0 + 16 * j); // block's first column
			const int region = nb < q_dim ? 0 : (nb < q_dim + kv_dim ? 1 : 2);
			const int base = region == 0 ? 0 : (region == 1 ? q_dim : q_dim + kv_dim);
			const int nn = nb - base + (lane & 15); // column inside q / k / v
			const int fj = (nn % head_dim) >> 1;
			const bool rot = region != 2;
			uint16_t *const dst = (region == 0 ? q : (region == 1 ? kc : vc)) + nn;
			const int ld = region == 0 ? q_dim : kv_dim, roff = region == 0 ? 0 : pos0;
			constexpr int IB = FI < 4 ? FI : 4; // row fragments per batch of table loads
#pragma unroll
			for (int i0 = 0; i0 < FI; i0 += IB) {
				float2_t cs[IB][4];
#pragma unroll
				for (int i = 0; i < IB; ++i)
#pragma unroll
					for (int r = 0; r < 4; ++r) {
						const int m = min(m0 + 16 * (i0 + i) + crow16(r, lane), M - 1);
						cs[i][r] = *(const float2_t *)(rope + ((size_t)m * (head_dim >> 1) + fj) * 2);
					}
#pragma unroll
				for (int i = 0; i < IB; ++i)
#pragma unroll
					for (int r = 0; r < 4; ++r) {
						float v = acc[i0 + i][j][r];
						v = v < -clip ? -clip : (v > clip ? clip : v);
						const float p = dpp<0xB1>(v); // partner column (n ^ 1)
						const float ro = odd ? p * cs[i][r][1] + v * cs[i][r][0] : v * cs[i][r][0] - p * cs[i][r][1];
						const int m = m0 + 16 * (i0 + i) + crow16(r, lane);
						if (m < M)
							dst[(size_t)(roff + m) * ld] = f2h(rot ? ro : v);
					}
			}
		}
	}
};

} // namespace pf

struct E16Null {
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	float *sink;
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(pf::f32x4_t (&acc)[FI][FJ], int, int, int lane, int, int) const {
		float s = 0.f;
#pragma unroll
		for (int i = 0; i < FI; ++i)
#pragma unroll
			for (int j = 0; j < FJ; ++j)
				s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
		if (s == 1234567.0f)
			sink[lane] = s;
	}
};

// the 2-phase 256 x 320 kernel (gemm16_kernel), the Llama-3B QKV form
template <class EPI>
static float run320(const uint16_t *A, int M, int K, pf::BRowsPlain bm, int N, EPI e, int iters) {
	auto kern = pf::gemm16_kernel<EPI, pf::BRowsPlain, 320, 2>;
	constexpr size_t lds = pf::gemm16_lds<320>();
	hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
	const int nwg = ((M + 255) / 256) * (N / 320);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	hipLaunchKernelGGL(kern, dim3(nwg), dim3(512), lds, 0, A, K, M, K, K, bm, N, e, 0);
	hipEventRecord(e0, 0);
	for (int i = 0; i < iters; ++i)
		hipLaunchKernelGGL(kern, dim3(nwg), dim3(512), lds, 0, A, K, M, K, K, bm, N, e, 0);
	hipEventRecord(e1, 0);
	hipEventSynchronize(e1);
	float ms;
	hipEventElapsedTime(&ms, e0, e1);
	return ms * 1e3f / iters;
}

template <class EPI, class BMAP, int FJ0, int FJ1>
static float run(const uint16_t *A, int M, int K, BMAP bm, int N, EPI e, int iters) {
	auto kern = pf::gemm8p_kernel<EPI, BMAP, FJ0, FJ1>;
	constexpr size_t lds = pf::gemm8p_lds<FJ0, FJ1>();
	hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
	const int nwg = ((M + 255) / 256) * (N / (64 * (FJ0 + FJ1)));
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	hipLaunchKernelGGL(kern, dim3(nwg), dim3(512), lds, 0, A, K, M, K, K, bm, N, e, 0, N, K);
	hipEventRecord(e0, 0);
	for (int i = 0; i < iters; ++i)
		hipLaunchKernelGGL(kern, dim3(nwg), dim3(512), lds, 0, A, K, M, K, K, bm, N, e, 0, N, K);
	hipEventRecord(e1, 0);
	hipEventSynchronize(e1);
	float ms;
	hipEventElapsedTime(&ms, e0, e1);
	return ms * 1e3f / iters;
}

int main() {
	const int M = 4096;
	const size_t maxel = (size_t)16384 * 8192;
	std::vector<uint16_t> h(maxel);
	srand(3);
	for (auto &v : h) {
		_Float16 f = (_Float16)(((float)rand() / RAND_MAX - 0.5f) * 0.1f);
		__builtin_memcpy(&v, &f, 2);
	}
	uint16_t *A, *W, *H;
	float *X, *sink;
	hipMalloc(&A, (size_t)M * 8192 * 2);
	hipMalloc(&W, maxel * 2);
	hipMalloc(&H, (size_t)M * 8192 * 2);
	hipMalloc(&X, (size_t)M * 3072 * 4);
	hipMalloc(&sink, 256);
	hipMemcpy(A, h.data(), (size_t)M * 8192 * 2, hipMemcpyHostToDevice);
	hipMemcpy(W, h.data(), maxel * 2, hipMemcpyHostToDevice);
	hipMemset(X, 0, (size_t)M * 3072 * 4);
	pf::BSrc b{};
	b.p[0] = b.p[1] = b.p[2] = W;
	E16Null en;
	en.sink = sink;
	pf::E16Residual er;
	er.x = X;
	er.ldx = 3072;
	er.M = M;
	pf::E16Glu<1> eg;
	eg.h = H;
	eg.ldh = 8192;
	eg.M = M;
	uint16_t *Q, *KC, *VC;
	float *rope;
	hipMalloc(&Q, (size_t)M * 3072 * 2);
	hipMalloc(&KC, (size_t)M * 1024 * 2);
	hipMalloc(&VC, (size_t)M * 1024 * 2);
	hipMalloc(&rope, (size_t)M * 64 * 2 * 4);
	hipMemset(rope, 0, (size_t)M * 64 * 2 * 4);
	pf::E16GluR5<1> eg5;
	eg5.h = H;
	eg5.ldh = 8192;
	eg5.M = M;
	unsigned *rng;
	hipMalloc(&rng, 64);
	hipMemset(rng, 0, 64);
	eg.range = rng;
	pf::E16QKV eq;
	eq.q = Q;
	eq.kc = KC;
	eq.vc = VC;
	eq.rope = rope;
	eq.M = M;
	eq.q_dim = 3072;
	eq.kv_dim = 1024;
	eq.head_dim = 128;
	eq.pos0 = 0;
	eq.clip = 3.4e38f;
	pf::E16QKVR5 eq5;
	eq5.q = Q, eq5.kc = KC, eq5.vc = VC, eq5.rope = rope, eq5.M = M, eq5.q_dim = 3072, eq5.kv_dim = 1024;
	eq5.head_dim = 128, eq5.pos0 = 0, eq5.clip = 3.4e38f;
	eq.range = rng + 4;
	std::vector<float> t[12];
	for (int r = 0; r < 7; ++r) {
		b.end[0] = b.end[1] = b.end[2] = 3072;
		pf::BRowsPlain bp{b};
		t[0].push_back(run<pf::E16Residual, pf::BRowsPlain, 2, 1>(A, M, 3072, bp, 3072, er, 10)); // Wo
		t[1].push_back(run<E16Null, pf::BRowsPlain, 2, 1>(A, M, 3072, bp, 3072, en, 10));
		t[2].push_back(run<pf::E16Residual, pf::BRowsPlain, 2, 1>(A, M, 8192, bp, 3072, er, 10)); // W2
		t[3].push_back(run<E16Null, pf::BRowsPlain, 2, 1>(A, M, 8192, bp, 3072, en, 10));
		pf::BRowsGlu<64> bg{W, W + (size_t)8192 * 3072};
		t[4].push_back(run<pf::E16Glu<1>, pf::BRowsGlu<64>, 2, 2>(A, M, 3072, bg, 16384, eg, 10)); // W1|W3
		t[5].push_back(run<E16Null, pf::BRowsGlu<64>, 2, 2>(A, M, 3072, bg, 16384, en, 10));
		pf::BSrc bq{};
		bq.p[0] = W;
		bq.p[1] = W + (size_t)3072 * 3072;
		bq.p[2] = W + (size_t)4096 * 3072;
		bq.end[0] = 3072;
		bq.end[1] = 4096;
		bq.end[2] = 5120;
		t[6].push_back(run320<pf::E16QKV>(A, M, 3072, pf::BRowsPlain{bq}, 5120, eq, 10)); // QKV
		t[7].push_back(run320<E16Null>(A, M, 3072, pf::BRowsPlain{bq}, 5120, en, 10));
		t[8].push_back(run<pf::E16GluR5<1>, pf::BRowsGlu<64>, 2, 2>(A, M, 3072, bg, 16384, eg5, 10));
		t[9].push_back(run<pf::E16QKVR5, pf::BRowsPlain, 2, 2>(A, M, 3072, pf::BRowsPlain{bq}, 5120, eq5, 10));
		t[10].push_back(run<pf::E16QKV, pf::BRowsPlain, 2, 2>(A, M, 3072, pf::BRowsPlain{bq}, 5120, eq, 10));
		t[11].push_back(run<E16Null, pf::BRowsPlain, 2, 2>(A, M, 3072, pf::BRowsPlain{bq}, 5120, en, 10));
	}
	const char *nm[12] = {"Wo  residual", "Wo  null", "W2  residual", "W2  null", "GLU glu", "GLU null",
	                      "QKV qkv (2ph 320)", "QKV null (2ph 320)", "GLU glu r5", "QKV qkv r5 (8p)", "QKV qkv (8p)",
	                      "QKV null (8p)"};
	const double fl[12] = {2.0 * M * 3072 * 3072, 2.0 * M * 3072 * 3072, 2.0 * M * 3072 * 8192,
	                       2.0 * M * 3072 * 8192, 2.0 * M * 16384 * 3072, 2.0 * M * 16384 * 3072,
	                       2.0 * M * 5120 * 3072, 2.0 * M * 5120 * 3072, 2.0 * M * 16384 * 3072,
	                       2.0 * M * 5120 * 3072, 2.0 * M * 5120 * 3072, 2.0 * M * 5120 * 3072};
	for (int i = 0; i < 12; ++i) {
		std::sort(t[i].begin(), t[i].end());
		const float med = t[i][t[i].size() / 2];
		printf("%-20s median %7.1f us  min %7.1f us  %6.0f TFLOP/s\n", nm[i], med, t[i][0], fl[i] / (med * 1e-6) / 1e12);
	}
	return 0;
}
