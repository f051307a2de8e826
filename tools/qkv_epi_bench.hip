// qkv_epi_bench.hip — where the prefill's QKV / GLU epilogue time goes (prefill_gemm.h E16QKV,
// E16Glu) at the Llama-3.2-3B T = 4096 shapes, and a candidate: a 4 x 4 lane-quad transpose of
// each 16 x 16 C fragment (DPP, two steps) so every lane stores 4 consecutive f16 (8 B)
// instead of one f16 per element: a quarter of the store instructions, whole 32-B row pieces.
// Variants: prod (the product epilogue), notab (no RoPE table loads: constant cos / sin from
// the arguments), nostore (everything computed, stored only on an impossible value), tr4 (the
// transposed 8-byte stores). Interleaved rounds, medians.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -I yalm_amd/csrc \
//          -o tools/qkv_epi_bench tools/qkv_epi_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "prefill_gemm.h"

namespace pf {

// v[r] = C[row 4 q + r][col c] (q = lane >> 4, c = lane & 15) -> v[k] = C[row 4 q + (c & 3)][col 4 (c >> 2) + k]
__device__ __forceinline__ void quad_transpose(float (&v)[4], int lane) {
	const bool b2 = lane & 2, b1 = lane & 1;
	{
		const float s0 = b2 ? v[0] : v[2], s1 = b2 ? v[1] : v[3];
		const float r0 = dpp<0x4E>(s0), r1 = dpp<0x4E>(s1);
		if (b2)
			v[0] = r0, v[1] = r1;
		else
			v[2] = r0, v[3] = r1;
	}
	{
		const float s0 = b1 ? v[0] : v[1], s1 = b1 ? v[2] : v[3];
		const float r0 = dpp<0xB1>(s0), r1 = dpp<0xB1>(s1);
		if (b1)
			v[0] = r0, v[2] = r1;
		else
			v[1] = r0, v[3] = r1;
	}
}

// MODE 0 prod, 1 notab, 2 nostore, 3 tr4, 4 the tile's RoPE rows staged in LDS (one
// contiguous 128-KB copy: rows m0t .. m0t + 255 x 64 (cos, sin)), 5 = 4 + tr4
template <int MODE>
struct E16QKVd {
	static constexpr bool NEEDS_LDS = MODE >= 4;
	float *red = nullptr;
	uint16_t *q;
	uint16_t *kc, *vc;
	const float *rope;
	int M, q_dim, kv_dim, head_dim, pos0;
	float clip, c0 = 1.0f, s0 = 0.0f;
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(f32x4_t (&acc)[FI][FJ], int m0, int n0, int lane, int, int) const {
		const bool odd = lane & 1;
		const int m0t = m0 - (m0 % G_BM); // the tile's first row
		if constexpr (MODE >= 4) { // rows m0t .. m0t + 255 of the table: 128 KB, contiguous
			const float4_t *src = (const float4_t *)(rope + (size_t)m0t * (head_dim >> 1) * 2);
			float4_t *dst = (float4_t *)red;
			const int nrow = min(G_BM, M - m0t);
			const int n16 = nrow * (head_dim >> 1) * 2 / 4;
			for (int i = threadIdx.x; i < n16; i += G_THREADS)
				dst[i] = src[i];
			__syncthreads();
		}
#pragma unroll
		for (int j = 0; j < FJ; ++j) {
			const int nb = __builtin_amdgcn_readfirstlane(n0 + 16 * j);
			const int region = nb < q_dim ? 0 : (nb < q_dim + kv_dim ? 1 : 2);
			const int base = region == 0 ? 0 : (region == 1 ? q_dim : q_dim + kv_dim);
			const int nn = nb - base + (lane & 15);
			const int fj = (nn % head_dim) >> 1;
			const bool rot = region != 2;
			uint16_t *const dst0 = region == 0 ? q : (region == 1 ? kc : vc);
			const int ld = region == 0 ? q_dim : kv_dim, roff = region == 0 ? 0 : pos0;
			constexpr int IB = FI < 4 ? FI : 4;
#pragma unroll
			for (int i0 = 0; i0 < FI; i0 += IB) {
				float2_t cs[IB][4];
#pragma unroll
				for (int i = 0; i < IB; ++i)
#pragma unroll
					for (int r = 0; r < 4; ++r) {
						if constexpr (MODE == 1) {
							cs[i][r] = float2_t{c0, s0};
						} else if constexpr (MODE >= 4) {
							const int ml = min(m0 + 16 * (i0 + i) + crow16(r, lane), M - 1) - m0t;
							cs[i][r] = *(const float2_t *)(red + ((size_t)ml * (head_dim >> 1) + fj) * 2);
						} else {
							const int m = min(m0 + 16 * (i0 + i) + crow16(r, lane), M - 1);
							cs[i][r] = *(const float2_t *)(rope + ((size_t)m * (head_dim >> 1) + fj) * 2);
						}
					}
#pragma unroll
				for (int i = 0; i < IB; ++i) {
					float ov[4];
#pragma unroll
					for (int r = 0; r < 4; ++r) {
						float v = acc[i0 + i][j][r];
						v = v < -clip ? -clip : (v > clip ? clip : v);
						const float p = dpp<0xB1>(v);
						const float ro = odd ? p * cs[i][r][1] + v * cs[i][r][0] : v * cs[i][r][0] - p * cs[i][r][1];
						ov[r] = rot ? ro : v;
					}
					const int mb = m0 + 16 * (i0 + i);
					if constexpr (MODE == 3 || MODE == 5) {
						float hv[4];
#pragma unroll
						for (int r = 0; r < 4; ++r)
							hv[r] = __uint_as_float(f2h(ov[r]));
						quad_transpose(hv, lane);
						const int m = mb + 4 * (lane >> 4) + (lane & 3);
						const int col = nb - base + 4 * ((lane & 15) >> 2);
						if (m < M) {
							const uint32_t w0 = __float_as_uint(hv[0]) | (__float_as_uint(hv[1]) << 16);
							const uint32_t w1 = __float_as_uint(hv[2]) | (__float_as_uint(hv[3]) << 16);
							*(uint2 *)(dst0 + (size_t)(roff + m) * ld + col) = make_uint2(w0, w1);
						}
					} else {
#pragma unroll
						for (int r = 0; r < 4; ++r) {
							const int m = mb + crow16(r, lane);
							const uint16_t ob = f2h(ov[r]);
							if (MODE == 2 ? ob == 0x7c01 : m < M)
								dst0[(size_t)(roff + m) * ld + nn] = ob;
						}
					}
				}
			}
		}
	}
};

// GLU: MODE 0 prod (E16Glu<1> without the range note), 2 nostore, 3 tr4
template <int MODE>
struct E16GluD {
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	uint16_t *h;
	int ldh, M;
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(f32x4_t (&acc)[FI][FJ], int m0, int n0, int lane, int, int) const {
#pragma unroll
		for (int i = 0; i < FI; ++i)
#pragma unroll
			for (int j = 0; j < FJ / 2; ++j) {
				float hv[4];
#pragma unroll
				for (int r = 0; r < 4; ++r)
					hv[r] = act_fast<1>(acc[i][j][r]) * acc[i][j + FJ / 2][r];
				const int mb = m0 + 16 * i;
				if constexpr (MODE == 3) {
#pragma unroll
					for (int r = 0; r < 4; ++r)
						hv[r] = __uint_as_float(f2h_bits(hv[r]));
					quad_transpose(hv, lane);
					const int m = mb + 4 * (lane >> 4) + (lane & 3);
					const int col = n0 + 16 * j + 4 * ((lane & 15) >> 2);
					if (m < M) {
						const uint32_t w0 = __float_as_uint(hv[0]) | (__float_as_uint(hv[1]) << 16);
						const uint32_t w1 = __float_as_uint(hv[2]) | (__float_as_uint(hv[3]) << 16);
						*(uint2 *)(h + (size_t)m * ldh + col) = make_uint2(w0, w1);
					}
				} else {
#pragma unroll
					for (int r = 0; r < 4; ++r) {
						const int m = mb + crow16(r, lane);
						const uint16_t hb = f2h_bits(hv[r]);
						if (MODE == 2 ? hb == 0x7c01 : m < M)
							h[(size_t)m * ldh + n0 + 16 * j + (lane & 15)] = hb;
					}
				}
			}
	}
};

} // namespace pf

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

int main() {
	const int M = 4096;
	const size_t maxel = (size_t)16384 * 8192;
	std::vector<uint16_t> h(maxel);
	srand(3);
	for (auto &v : h) {
		_Float16 f = (_Float16)(((float)rand() / RAND_MAX - 0.5f) * 0.1f);
		__builtin_memcpy(&v, &f, 2);
	}
	uint16_t *A, *W, *H, *H2, *Q, *KC, *VC, *Q2, *KC2, *VC2;
	float *rope;
	hipMalloc(&A, (size_t)M * 8192 * 2);
	hipMalloc(&W, maxel * 2);
	hipMalloc(&H, (size_t)M * 8192 * 2);
	hipMalloc(&H2, (size_t)M * 8192 * 2);
	hipMalloc(&Q, (size_t)M * 3072 * 2);
	hipMalloc(&KC, (size_t)M * 1024 * 2);
	hipMalloc(&VC, (size_t)M * 1024 * 2);
	hipMalloc(&Q2, (size_t)M * 3072 * 2);
	hipMalloc(&KC2, (size_t)M * 1024 * 2);
	hipMalloc(&VC2, (size_t)M * 1024 * 2);
	hipMalloc(&rope, (size_t)M * 64 * 2 * 4);
	hipMemcpy(A, h.data(), (size_t)M * 8192 * 2, hipMemcpyHostToDevice);
	hipMemcpy(W, h.data(), maxel * 2, hipMemcpyHostToDevice);
	{ // a real RoPE table (pos, theta 500000): the check below compares the two store forms
		std::vector<float> rt((size_t)M * 64 * 2);
		for (int m = 0; m < M; ++m)
			for (int f = 0; f < 64; ++f) {
				const double a = m * pow(500000.0, -f / 64.0);
				rt[((size_t)m * 64 + f) * 2] = (float)cos(a);
				rt[((size_t)m * 64 + f) * 2 + 1] = (float)sin(a);
			}
		hipMemcpy(rope, rt.data(), rt.size() * 4, hipMemcpyHostToDevice);
	}
	pf::BSrc bq{};
	bq.p[0] = W;
	bq.p[1] = W + (size_t)3072 * 3072;
	bq.p[2] = W + (size_t)4096 * 3072;
	bq.end[0] = 3072;
	bq.end[1] = 4096;
	bq.end[2] = 5120;
	const pf::BRowsPlain bp{bq};
	const pf::BRowsGlu<64> bg{W, W + (size_t)8192 * 3072};
	auto qkv = [&](auto e, uint16_t *q, uint16_t *k, uint16_t *v) {
		e.q = q, e.kc = k, e.vc = v, e.rope = rope, e.M = M, e.q_dim = 3072, e.kv_dim = 1024, e.head_dim = 128;
		e.pos0 = 0, e.clip = 3.4e38f;
		return e;
	};
	auto e0 = qkv(pf::E16QKVd<0>{}, Q, KC, VC);
	auto e1 = qkv(pf::E16QKVd<1>{}, Q, KC, VC);
	auto e2 = qkv(pf::E16QKVd<2>{}, Q, KC, VC);
	auto e3 = qkv(pf::E16QKVd<3>{}, Q2, KC2, VC2);
	auto e4 = qkv(pf::E16QKVd<4>{}, Q2, KC2, VC2);
	auto e5 = qkv(pf::E16QKVd<5>{}, Q2, KC2, VC2);
	pf::E16GluD<0> g0;
	g0.h = H, g0.ldh = 8192, g0.M = M;
	pf::E16GluD<2> g2;
	g2.h = H, g2.ldh = 8192, g2.M = M;
	pf::E16GluD<3> g3;
	g3.h = H2, g3.ldh = 8192, g3.M = M;
	const int NV = 14;
	std::vector<float> t[NV];
	for (int r = 0; r < 7; ++r) {
		t[0].push_back(run<decltype(e0), pf::BRowsPlain, 2, 2>(A, M, 3072, bp, 5120, e0, 10));
		t[1].push_back(run<decltype(e1), pf::BRowsPlain, 2, 2>(A, M, 3072, bp, 5120, e1, 10));
		t[2].push_back(run<decltype(e2), pf::BRowsPlain, 2, 2>(A, M, 3072, bp, 5120, e2, 10));
		t[3].push_back(run<decltype(e3), pf::BRowsPlain, 2, 2>(A, M, 3072, bp, 5120, e3, 10));
		t[4].push_back(run320<decltype(e0)>(A, M, 3072, bp, 5120, e0, 10));
		t[5].push_back(run320<decltype(e3)>(A, M, 3072, bp, 5120, e3, 10));
		t[6].push_back(run320<decltype(e2)>(A, M, 3072, bp, 5120, e2, 10));
		t[7].push_back(run<pf::E16GluD<0>, pf::BRowsGlu<64>, 2, 2>(A, M, 3072, bg, 16384, g0, 10));
		t[8].push_back(run<pf::E16GluD<2>, pf::BRowsGlu<64>, 2, 2>(A, M, 3072, bg, 16384, g2, 10));
		t[9].push_back(run<pf::E16GluD<3>, pf::BRowsGlu<64>, 2, 2>(A, M, 3072, bg, 16384, g3, 10));
		t[10].push_back(run<decltype(e4), pf::BRowsPlain, 2, 2>(A, M, 3072, bp, 5120, e4, 10));
		t[11].push_back(run<decltype(e5), pf::BRowsPlain, 2, 2>(A, M, 3072, bp, 5120, e5, 10));
		t[12].push_back(run320<decltype(e4)>(A, M, 3072, bp, 5120, e4, 10));
		t[13].push_back(run320<decltype(e5)>(A, M, 3072, bp, 5120, e5, 10));
	}
	const char *nm[NV] = {"QKV 8p prod", "QKV 8p notab", "QKV 8p nostore", "QKV 8p tr4", "QKV 320 prod",
	                      "QKV 320 tr4", "QKV 320 nostore", "GLU 8p prod", "GLU 8p nostore", "GLU 8p tr4",
	                      "QKV 8p ldstab", "QKV 8p ldstab+tr4", "QKV 320 ldstab", "QKV 320 ldstab+tr4"};
	for (int i = 0; i < NV; ++i) {
		std::sort(t[i].begin(), t[i].end());
		printf("%-18s median %7.1f us  min %7.1f us\n", nm[i], t[i][t[i].size() / 2], t[i][0]);
	}
	// the transposed stores must write exactly what the product form writes
	auto same = [](const uint16_t *a, const uint16_t *b, size_t n) {
		std::vector<uint16_t> x(n), y(n);
		hipMemcpy(x.data(), a, n * 2, hipMemcpyDeviceToHost);
		hipMemcpy(y.data(), b, n * 2, hipMemcpyDeviceToHost);
		size_t d = 0;
		for (size_t i = 0; i < n; ++i)
			d += x[i] != y[i];
		return d;
	};
	run<decltype(e0), pf::BRowsPlain, 2, 2>(A, M, 3072, bp, 5120, e0, 1);
	run<decltype(e3), pf::BRowsPlain, 2, 2>(A, M, 3072, bp, 5120, e3, 1);
	printf("tr4 vs prod mismatches (8p): Q %zu K %zu V %zu\n", same(Q, Q2, (size_t)M * 3072),
	       same(KC, KC2, (size_t)M * 1024), same(VC, VC2, (size_t)M * 1024));
	run<decltype(e5), pf::BRowsPlain, 2, 2>(A, M, 3072, bp, 5120, e5, 1);
	hipDeviceSynchronize();
	printf("ldstab+tr4 vs prod mismatches (8p): Q %zu K %zu V %zu\n", same(Q, Q2, (size_t)M * 3072),
	       same(KC, KC2, (size_t)M * 1024), same(VC, VC2, (size_t)M * 1024));
	run320<decltype(e0)>(A, M, 3072, bp, 5120, e0, 1);
	run320<decltype(e4)>(A, M, 3072, bp, 5120, e4, 1);
	hipDeviceSynchronize();
	printf("ldstab vs prod mismatches (320): Q %zu K %zu V %zu\n", same(Q, Q2, (size_t)M * 3072),
	       same(KC, KC2, (size_t)M * 1024), same(VC, VC2, (size_t)M * 1024));
	run<pf::E16GluD<0>, pf::BRowsGlu<64>, 2, 2>(A, M, 3072, bg, 16384, g0, 1);
	run<pf::E16GluD<3>, pf::BRowsGlu<64>, 2, 2>(A, M, 3072, bg, 16384, g3, 1);
	hipDeviceSynchronize();
	printf("tr4 vs prod mismatches: Q %zu K %zu V %zu H %zu\n", same(Q, Q2, (size_t)M * 3072),
	       same(KC, KC2, (size_t)M * 1024), same(VC, VC2, (size_t)M * 1024), same(H, H2, (size_t)M * 8192));
	return 0;
}
