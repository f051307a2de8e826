// xk_prefetch_bench.hip — can a streaming kernel's tail warm the caches for the next kernel's
// first loads? Two back-to-back weight streams A (bytes_a) and B (bytes_b), 256 workgroups of
// 512 threads each, contiguous slice per workgroup, 16-byte nontemporal loads U = 4 deep (the
// GEMV kernels' access pattern). Variant "pre": when a workgroup of A issues its LAST round of
// loads it also loads the first `pre_kb` of the slice the same-index workgroup of B will read
// first (same blockIdx -> same XCD), with a chosen cache policy. Reports A+B time per pair,
// rotated through a 4-GB pool so every stream comes from HBM.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/xk_prefetch_bench tools/xk_prefetch_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../yalm_amd/csrc/device_common.h"

#define CK(x)                                                                                                          \
	do {                                                                                                               \
		hipError_t e_ = (x);                                                                                           \
		if (e_ != hipSuccess) {                                                                                        \
			printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                                           \
			return 1;                                                                                                  \
		}                                                                                                              \
	} while (0)

constexpr int THREADS = 512, U = 4, NWG = 256;
constexpr size_t ROUND = (size_t)THREADS * 16 * U; // bytes one workgroup has in flight

// POL: 0 = none, 1 = plain load, 2 = nontemporal load
template <int POL>
__global__ __launch_bounds__(THREADS) void stream_k(const char *w, size_t per_wg, const char *nxt, size_t nxt_per_wg,
                                                    int pre_rounds, float *sink) {
	const char *p = w + blockIdx.x * per_wg;
	float acc = 0.f;
	for (size_t o = 0; o < per_wg; o += ROUND) {
		u32x4_t v[U];
		for (int u = 0; u < U; ++u)
			v[u] = load_nt16(p + o + (size_t)(u * THREADS + threadIdx.x) * 16);
		if (POL && o + ROUND >= per_wg) { // last round: touch the head of the next kernel's slice
			const char *q = nxt + blockIdx.x * nxt_per_wg;
			for (int r = 0; r < pre_rounds; ++r)
				for (int u = 0; u < U; ++u) {
					const u32x4_t t = POL == 1 ? load16(q + r * ROUND + (size_t)(u * THREADS + threadIdx.x) * 16)
					                           : load_nt16(q + r * ROUND + (size_t)(u * THREADS + threadIdx.x) * 16);
					acc += __uint_as_float(t[1] & 0x3fffffffu);
				}
		}
		for (int u = 0; u < U; ++u)
			acc += __uint_as_float(v[u][0] & 0x3fffffffu);
	}
	if (acc == 12345.f)
		sink[blockIdx.x] = acc;
}

int main() {
	hipStream_t s;
	CK(hipStreamCreate(&s));
	const size_t pool = 4ull << 30;
	char *w;
	float *sink;
	CK(hipMalloc(&w, pool));
	CK(hipMemset(w, 0, pool));
	CK(hipMalloc(&sink, NWG * 4));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	struct Pair {
		const char *name;
		size_t a, b;
	} pairs[] = {{"fp8 GLU -> W2 (117.4 / 58.7 MB)", 117440512, 58720256},
	             {"fp16 GLU -> W2 (234.9 / 117.4 MB)", 234881024, 117440512},
	             {"fp8 W2 -> QKV (58.7 / 25.2 MB)", 58720256, 25165824}};
	for (const Pair &pr : pairs) {
		const size_t pa = pr.a / NWG / ROUND * ROUND, pb = pr.b / NWG / ROUND * ROUND;
		const size_t ta = pa * NWG, tb = pb * NWG;
		printf("--- %s\n", pr.name);
		for (int pol = 0; pol <= 2; ++pol)
			for (int rounds : {1, 2, 4}) {
				if (pol == 0 && rounds > 1)
					continue;
				size_t off = 0;
				auto run = [&](int reps) {
					for (int i = 0; i < reps; ++i) {
						if (off + ta + tb > pool)
							off = 0;
						const char *a = w + off, *b = w + off + ta;
						off += ta + tb;
						if (pol == 0)
							stream_k<0><<<NWG, THREADS, 0, s>>>(a, pa, b, pb, 0, sink);
						else if (pol == 1)
							stream_k<1><<<NWG, THREADS, 0, s>>>(a, pa, b, pb, rounds, sink);
						else
							stream_k<2><<<NWG, THREADS, 0, s>>>(a, pa, b, pb, rounds, sink);
						stream_k<0><<<NWG, THREADS, 0, s>>>(b, pb, nullptr, 0, 0, sink);
					}
				};
				run(10);
				CK(hipEventRecord(e0, s));
				const int reps = 200;
				run(reps);
				CK(hipEventRecord(e1, s));
				CK(hipEventSynchronize(e1));
				float ms;
				CK(hipEventElapsedTime(&ms, e0, e1));
				const float us = ms * 1e3f / reps;
				printf("  %-12s pre %d x %3zu KB per wg: A+B %7.2f us  (%.0f GB/s over A+B bytes)\n",
				       pol == 0 ? "no prefetch" : pol == 1 ? "plain load" : "nt load", pol ? rounds : 0,
				       pol ? ROUND >> 10 : 0, us, (ta + tb) / us / 1e3);
			}
	}
	return 0;
}
