// attn_pf_bench.hip — the prefill's causal attention kernel alone, on the Llama-3.2-3B
// attention shape (24 q / 8 kv heads x 128, T = 4096, pos0 = 0), random f16 data:
// per-launch time from HIP events over back-to-back launches, TFLOP/s (causal
// FLOPs 4 D heads T (T + 1) / 2), variants interleaved in one process, and every
// variant's output compared with variant 0's (max |diff|).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -I yalm_amd/csrc \
//          -o tools/attn_pf_bench tools/attn_pf_bench.hip   (the product flags of prefill.hip, Makefile)
// usage: tools/attn_pf_bench [T] [rounds] [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "prefill.h"

// round-3 kernel as committed before the softmax rework (baseline of the A/B)
namespace pf {
template <int D>
__global__ __launch_bounds__(THREADS) void attn_prefill_kernel_r3(const uint16_t *__restrict__ Q,
                                                               const uint16_t *__restrict__ kc,
                                                               const uint16_t *__restrict__ vc, int T, int pos0,
                                                               int n_heads, int n_kv, uint16_t *__restrict__ O) {
	static_assert(D == 64 || D == 128, "head_dim");
	constexpr int DCH = D / 8;
	extern __shared__ __attribute__((aligned(16))) uint16_t asmem[];
	uint16_t *const Kb = asmem;               // [2][AKT * D]
	uint16_t *const Vb = asmem + 2 * AKT * D; // [2][AKT * D]
	const int lane = threadIdx.x & 63, l32 = lane & 31, hh = lane >> 5;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int qb = gridDim.x - 1 - blockIdx.x; // heaviest (latest) query blocks first
	const int h = blockIdx.y, g = h / (n_heads / n_kv);
	const int q_dim = n_heads * D, kv_dim = n_kv * D;
	const int qw0 = qb * AQ + wave * 32; // this wave's first query row
	const int qrow = qw0 + l32;          // this lane's query
	const int qpos = pos0 + qrow;
	// scores in log2 units: exp2(s * log2(e) / sqrt(D) - m)
	const float sl2 = 1.4426950408889634f / sqrtf((float)D);
	const int kv_rows = pos0 + T; // valid cache rows (masked keys past a query are never used)

	half8_t qf[D / 16]; // B operand of S^T = K Q^T: Q[query = l32][d = 16 s + 8 h ..]
	{
		const uint16_t *qp = Q + (size_t)min(qrow, T - 1) * q_dim + h * D + 8 * hh;
#pragma unroll
		for (int s = 0; s < D / 16; ++s)
			qf[s] = *(const half8_t *)(qp + 16 * s);
	}
	f32x16_t o[D / 32]; // O^T tiles: rows = d (32 jd + crow), column = query
#pragma unroll
	for (int jd = 0; jd < D / 32; ++jd)
		o[jd] = f32x16_t{};
	float m = -FLT_MAX, l = 0.0f;
	const int qmax_blk = min(qb * AQ + AQ, T) - 1; // last query row of the block
	const int ntile = (pos0 + qmax_blk) / AKT + 1; // key tiles up to its position
	// transposed-read lane geometry (ds_read_b64_tr_b16: 16-lane groups, 4 rows x 16 columns)
	const int gi = lane & 15, gq = gi >> 2, gp = gi & 3;
	const int dgrp = 16 * ((lane >> 4) & 1);

	stage_kv<D, false>(Kb, kc, 0, kv_rows, kv_dim, g, wave, lane);
	stage_kv<D, true>(Vb, vc, 0, kv_rows, kv_dim, g, wave, lane);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	int cur = 0;
	for (int kt = 0; kt < ntile; ++kt) {
		const int key0 = kt * AKT;
		if (kt + 1 < ntile) { // next tile's LDS-DMA overlaps this tile's math
			stage_kv<D, false>(Kb + (cur ^ 1) * AKT * D, kc, key0 + AKT, kv_rows, kv_dim, g, wave, lane);
			stage_kv<D, true>(Vb + (cur ^ 1) * AKT * D, vc, key0 + AKT, kv_rows, kv_dim, g, wave, lane);
		}
		const uint16_t *Ks = Kb + cur * AKT * D;
		const uint16_t *Vs = Vb + cur * AKT * D;

		// ---- S^T = K Q^T: two 32-key blocks; register r of block j is key key0 + 32 j + crow(r, lane)
		f32x16_t st[2];
#pragma unroll
		for (int j = 0; j < 2; ++j) {
			st[j] = f32x16_t{};
			const int kr = 32 * j + l32;
#pragma unroll
			for (int s = 0; s < D / 16; ++s) {
				const int kcnk = 2 * s + hh;
				const half8_t ka = *(const half8_t *)(Ks + kr * D + 8 * (kcnk ^ (kr % DCH)));
				st[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ka, qf[s], st[j], 0, 0, 0);
			}
		}
		// ---- online softmax for this lane's query (causal mask on the diagonal tiles)
		const bool diag = key0 + AKT - 1 > pos0 + qw0;
		float mx = -FLT_MAX;
#pragma unroll
		for (int j = 0; j < 2; ++j)
#pragma unroll
			for (int r = 0; r < 16; ++r) {
				float v = st[j][r] * sl2;
				if (diag && key0 + 32 * j + crow(r, lane) > qpos)
					v = -FLT_MAX;
				st[j][r] = v;
				mx = fmaxf(mx, v);
			}
		mx = fmaxf(mx, xor32(mx)); // the other lane half holds the other 32 keys
		const float mn = fmaxf(m, mx);
		const float alpha = __builtin_amdgcn_exp2f(m - mn);
		m = mn;
		float ls = 0.0f;
		half8_t pb[2][2]; // P^T fragments: [block j][k-step s]
#pragma unroll
		for (int j = 0; j < 2; ++j)
#pragma unroll
			for (int r = 0; r < 16; ++r) {
				const float p = __builtin_amdgcn_exp2f(st[j][r] - mn);
				ls += p;
				pb[j][r >> 3][r & 7] = (_Float16)p;
			}
		ls += xor32(ls);
		l = l * alpha + ls;
#pragma unroll
		for (int jd = 0; jd < D / 32; ++jd)
			o[jd] *= alpha;
		// ---- O^T += V^T P^T
#pragma unroll
		for (int j = 0; j < 2; ++j)
#pragma unroll
			for (int s = 0; s < 2; ++s) {
				const int klo = 32 * j + 16 * s + 4 * hh + gq; // keys of elements 0..3 (row gq of the 4-row block)
#pragma unroll
				for (int jd = 0; jd < D / 32; ++jd) {
					const int d = 32 * jd + dgrp + 4 * gp;
					const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
					    (YALM_LDS short4_t *)(Vs + klo * D + 8 * ((d >> 3) ^ ((klo & 3) << 1)) + (d & 7)));
					const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YALM_LDS short4_t *)(
					    Vs + (klo + 8) * D + 8 * ((d >> 3) ^ (((klo + 8) & 3) << 1)) + (d & 7)));
					half8_t va;
#pragma unroll
					for (int e = 0; e < 4; ++e) {
						va[e] = __builtin_bit_cast(_Float16, (short)lo[e]);
						va[4 + e] = __builtin_bit_cast(_Float16, (short)hi[e]);
					}
					o[jd] = __builtin_amdgcn_mfma_f32_32x32x16_f16(va, pb[j][s], o[jd], 0, 0, 0);
				}
			}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads(); // next tile landed; this tile's K / V reads are done
		cur ^= 1;
	}
	// ---- normalise and store O[query][h * D + d] (f16, the Wo GEMM's A operand); d = 32 jd + crow(r)
	if (qrow < T) {
		const float inv = 1.0f / l;
		uint16_t *op = O + (size_t)qrow * q_dim + h * D;
#pragma unroll
		for (int jd = 0; jd < D / 32; ++jd)
#pragma unroll
			for (int r4 = 0; r4 < 4; ++r4) { // registers 4 r4 .. 4 r4 + 3 are 4 consecutive d
				const int d = 32 * jd + 8 * r4 + 4 * hh;
				uint32_t w0 = (uint32_t)f2h_bits(o[jd][4 * r4 + 0] * inv) | ((uint32_t)f2h_bits(o[jd][4 * r4 + 1] * inv) << 16);
				uint32_t w1 = (uint32_t)f2h_bits(o[jd][4 * r4 + 2] * inv) | ((uint32_t)f2h_bits(o[jd][4 * r4 + 3] * inv) << 16);
				*(uint2 *)(op + d) = make_uint2(w0, w1);
			}
	}
}

} // namespace pf

#define CK(x)                                                                                                          \
	do {                                                                                                               \
		hipError_t e_ = (x);                                                                                           \
		if (e_ != hipSuccess) {                                                                                        \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                  \
			exit(1);                                                                                                   \
		}                                                                                                              \
	} while (0)

static __host__ uint16_t h16(float f) {
	_Float16 h = (_Float16)f;
	uint16_t u;
	memcpy(&u, &h, 2);
	return u;
}
static __host__ float f16(uint16_t u) {
	_Float16 h;
	memcpy(&h, &u, 2);
	return (float)h;
}

struct Variant {
	const char *name;
	void (*launch)(const uint16_t *, const uint16_t *, const uint16_t *, int, int, int, int, uint16_t *, hipStream_t);
};

static void launch_v0(const uint16_t *Q, const uint16_t *kc, const uint16_t *vc, int T, int pos0, int nh, int nkv,
                      uint16_t *O, hipStream_t st) {
	const dim3 grid((T + pf::AQ - 1) / pf::AQ, nh);
	pf::attn_prefill_kernel_r3<128><<<grid, pf::THREADS, pf::attn_prefill_lds<128>(), st>>>(Q, kc, vc, T, pos0, nh, nkv, O);
}
// the product kernel (prefill.h) with the product launch geometry (prefill.hip launch_attn_prefill)
static void launch_v1(const uint16_t *Q, const uint16_t *kc, const uint16_t *vc, int T, int pos0, int nh, int nkv,
                      uint16_t *O, hipStream_t st) {
	const dim3 grid(nh, (T + pf::AQ - 1) / pf::AQ);
	pf::attn_prefill_kernel<128><<<grid, pf::THREADS, pf::attn_prefill_lds<128>(), st>>>(Q, kc, vc, T, pos0, nh, nkv, O);
}

// 32-key tiles: half the LDS per workgroup (32 KB) and fewer registers, so 3 workgroups per CU
static void launch_v2(const uint16_t *Q, const uint16_t *kc, const uint16_t *vc, int T, int pos0, int nh, int nkv,
                      uint16_t *O, hipStream_t st) {
	const dim3 grid(nh, (T + pf::AQ - 1) / pf::AQ);
	pf::attn_prefill_kernel<128, 32><<<grid, pf::THREADS, pf::attn_prefill_lds<128, 32>(), st>>>(Q, kc, vc, T, pos0, nh,
	                                                                                          nkv, O);
}

// the split-operand precision form (Q and O [hi | lo]; here Q's lo half reads the next row's
// hi, O writes 2x wide: a timing of the doubled MFMA work, not a numerics check)
static uint16_t *g_q2 = nullptr, *g_o2 = nullptr;
static void launch_split(const uint16_t *Q, const uint16_t *kc, const uint16_t *vc, int T, int pos0, int nh, int nkv,
						 uint16_t *O, hipStream_t st) {
	const dim3 grid(nh, (T + pf::AQ - 1) / pf::AQ);
	pf::attn_prefill_kernel<128, 64, true><<<grid, pf::THREADS, pf::attn_prefill_lds<128>(), st>>>(g_q2, kc, vc, T, pos0,
	                                                                                              nh, nkv, g_o2);
	(void)Q;
	(void)O;
}

int main(int argc, char **argv) {
	const int T = argc > 1 ? atoi(argv[1]) : 4096;
	const int rounds = argc > 2 ? atoi(argv[2]) : 5;
	const int iters = argc > 3 ? atoi(argv[3]) : 10;
	const int nh = 24, nkv = 8, D = 128, pos0 = 0;
	const size_t qn = (size_t)T * nh * D, kn = (size_t)(pos0 + T) * nkv * D;
	std::vector<uint16_t> hq(qn), hk(kn), hv(kn);
	srand(1);
	auto rnd = [] { return (float)rand() / RAND_MAX * 2.0f - 1.0f; };
	for (auto &x : hq)
		x = h16(rnd() * 2.0f);
	for (auto &x : hk)
		x = h16(rnd() * 2.0f);
	for (auto &x : hv)
		x = h16(rnd());
	uint16_t *q, *k, *v;
	CK(hipMalloc(&q, qn * 2));
	CK(hipMalloc(&k, kn * 2));
	CK(hipMalloc(&v, kn * 2));
	CK(hipMemcpy(q, hq.data(), qn * 2, hipMemcpyHostToDevice));
	CK(hipMemcpy(k, hk.data(), kn * 2, hipMemcpyHostToDevice));
	CK(hipMemcpy(v, hv.data(), kn * 2, hipMemcpyHostToDevice));
	CK(hipFuncSetAttribute((const void *)pf::attn_prefill_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize,
	                       (int)pf::attn_prefill_lds<128>()));
	CK(hipFuncSetAttribute((const void *)pf::attn_prefill_kernel_r3<128>, hipFuncAttributeMaxDynamicSharedMemorySize,
	                       (int)pf::attn_prefill_lds<128>()));
	CK(hipFuncSetAttribute((const void *)pf::attn_prefill_kernel<128, 32>, hipFuncAttributeMaxDynamicSharedMemorySize,
	                       (int)pf::attn_prefill_lds<128, 32>()));
	CK(hipFuncSetAttribute((const void *)pf::attn_prefill_kernel<128, 64, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
	                       (int)pf::attn_prefill_lds<128>()));
	CK(hipMalloc(&g_q2, 2 * qn * 2));
	CK(hipMalloc(&g_o2, 2 * qn * 2));
	CK(hipMemset(g_q2, 0, 2 * qn * 2));
	std::vector<Variant> vs = {{"product", launch_v1}, {"r3", launch_v0}, {"split", launch_split}};
	const int nv = (int)vs.size();
	std::vector<uint16_t *> outs(nv);
	for (auto &o : outs)
		CK(hipMalloc(&o, qn * 2));
	hipStream_t st;
	CK(hipStreamCreate(&st));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	const double flops = 4.0 * D * nh * (double)T * (T + 1) / 2;
	std::vector<std::vector<float>> ms(nv);
	for (int r = 0; r < rounds; ++r) {
		for (int i = 0; i < nv; ++i) {
			vs[i].launch(q, k, v, T, pos0, nh, nkv, outs[i], st);
			CK(hipEventRecord(e0, st));
			for (int it = 0; it < iters; ++it)
				vs[i].launch(q, k, v, T, pos0, nh, nkv, outs[i], st);
			CK(hipEventRecord(e1, st));
			CK(hipEventSynchronize(e1));
			float t;
			CK(hipEventElapsedTime(&t, e0, e1));
			ms[i].push_back(t / iters);
		}
	}
	std::vector<uint16_t> ref(qn), got(qn);
	CK(hipMemcpy(ref.data(), outs[0], qn * 2, hipMemcpyDeviceToHost));
	for (int i = 0; i < nv; ++i) {
		CK(hipMemcpy(got.data(), outs[i], qn * 2, hipMemcpyDeviceToHost));
		double md = 0;
		for (size_t j = 0; j < qn; ++j)
			md = fmax(md, fabs((double)f16(got[j]) - f16(ref[j])));
		std::vector<float> s = ms[i];
		std::sort(s.begin(), s.end());
		printf("%-12s T=%d median %.1f us min %.1f us  %.0f TFLOP/s  max|diff vs %s| %.3g\n", vs[i].name, T,
		       s[s.size() / 2] * 1e3, s[0] * 1e3, flops / (s[s.size() / 2] * 1e-3) / 1e12, vs[0].name, md);
	}
	return 0;
}
