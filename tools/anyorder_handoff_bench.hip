// anyorder_handoff_bench.hip — what a DEPENDENT kernel pair gains from hipExtAnyOrderLaunch
// (eager launches only: a hipGraph capture drops the flag, tools/anyorder_probe.hip).
// A = a GLU-like producer: 256 workgroups stream WA bytes, then each writes its block of the
// output h (n_h floats in 256 blocks). B = a W2-like consumer: 256 workgroups stream WB bytes
// and need ALL of h before they can use their weights.
//   barrier:    A <<<>>>, B <<<>>>: h written with plain stores, read plain after the boundary.
//   any-order:  B launched with the flag, so its workgroups land next to A's tail: A writes h as
//               {value, tag} granules (one agent-scope 64-bit store each, the last element of
//               each block doubling as the block's sentinel); B issues its first weight round,
//               polls the 256 sentinels (one 8-byte load per lane x 4) until every tag is this
//               pair's, then gathers h granules (every tag checked).
// Tags grow by one per pair, so the buffer is never reset. Reports time per pair.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/anyorder_handoff_bench tools/anyorder_handoff_bench.hip
#include <hip/hip_ext.h>
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

constexpr int THREADS = 512, U = 4, NWG = 256, NH = 14336, BLK = NH / NWG; // 56 h values per A workgroup
constexpr size_t ROUND = (size_t)THREADS * 16 * U;
constexpr unsigned long long SPIN = 200000000ull; // 2 s of s_memrealtime: a bounded wait

__device__ __forceinline__ float stream_rounds(const char *p, size_t bytes, float acc) {
	for (size_t o = 0; o < bytes; o += ROUND) {
		u32x4_t v[U];
		for (int u = 0; u < U; ++u)
			v[u] = load_nt16(p + o + (size_t)(u * THREADS + threadIdx.x) * 16);
		for (int u = 0; u < U; ++u)
			acc += __uint_as_float(v[u][0] & 0x3fffffffu);
	}
	return acc;
}

// producer: stream, then this block of h (plain floats, or granules tagged `tag`)
template <bool GRAN>
__global__ __launch_bounds__(THREADS) void prod_k(const char *w, size_t per_wg, float *h, unsigned long long *hg,
                                                  unsigned tag, float *sink) {
	const float acc = stream_rounds(w + blockIdx.x * per_wg, per_wg, 0.f);
	const float v = acc * 1e-30f + (float)(blockIdx.x * BLK + threadIdx.x);
	if (acc == 12345.f)
		sink[blockIdx.x] = acc;
	if (threadIdx.x < BLK) {
		const int i = blockIdx.x * BLK + threadIdx.x;
		if (GRAN)
			__hip_atomic_store(hg + i, (unsigned long long)__float_as_uint(v) | ((unsigned long long)tag << 32),
			                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		else
			h[i] = v;
	}
}

// consumer: first weight round in flight, then all of h (after the boundary, or through the
// sentinels + a tag-checked gather), staged in LDS, then the rest of the stream
template <bool GRAN>
__global__ __launch_bounds__(THREADS) void cons_k(const char *w, size_t per_wg, const float *h,
                                                  const unsigned long long *hg, unsigned tag, float *sink,
                                                  unsigned *err) {
	__shared__ float hs[NH];
	const char *p = w + blockIdx.x * per_wg;
	u32x4_t v0[U];
	for (int u = 0; u < U; ++u)
		v0[u] = load_nt16(p + (size_t)(u * THREADS + threadIdx.x) * 16);
	const unsigned long long dl = __builtin_amdgcn_s_memrealtime() + SPIN;
	if (GRAN) {
		// sentinels: lane j of every wave polls blocks j, j + 64, ... (4 per lane)
		const int lane = threadIdx.x & 63;
		for (;;) {
			bool ok = true;
			for (int k = 0; k < NWG / 64; ++k) {
				const unsigned long long g = __hip_atomic_load(hg + (size_t)(k * 64 + lane) * BLK + BLK - 1,
				                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				ok = ok && (unsigned)(g >> 32) == tag;
			}
			if (__all(ok))
				break;
			if (__builtin_amdgcn_s_memrealtime() > dl) {
				if (lane == 0)
					__hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				break;
			}
			__builtin_amdgcn_s_sleep(1);
		}
		// gather: all of this thread's granules issued at once, then every tag checked (the
		// whole batch re-read on a stale one)
		constexpr int PER = (NH + THREADS - 1) / THREADS; // 28 granules per thread
		for (;;) {
			unsigned long long g[PER];
#pragma unroll
			for (int k = 0; k < PER; ++k) {
				const int i = min(k * THREADS + (int)threadIdx.x, NH - 1);
				g[k] = __hip_atomic_load(hg + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
			bool ok = true;
#pragma unroll
			for (int k = 0; k < PER; ++k)
				ok = ok && (unsigned)(g[k] >> 32) == tag;
			if (ok || __builtin_amdgcn_s_memrealtime() > dl) {
#pragma unroll
				for (int k = 0; k < PER; ++k)
					if (k * THREADS + (int)threadIdx.x < NH)
						hs[k * THREADS + threadIdx.x] = __uint_as_float((unsigned)g[k]);
				break;
			}
		}
	} else {
		for (int i = threadIdx.x; i < NH / 4; i += THREADS)
			*(float4_t *)&hs[4 * i] = *(const float4_t *)(h + 4 * i);
	}
	__syncthreads();
	float acc = hs[(threadIdx.x * 7) % NH];
	for (int u = 0; u < U; ++u)
		acc += __uint_as_float(v0[u][0] & 0x3fffffffu);
	acc = stream_rounds(p + ROUND, per_wg - ROUND, acc);
	if (acc == 12345.f)
		sink[blockIdx.x] = acc;
}

int main() {
	hipStream_t s;
	CK(hipStreamCreate(&s));
	const size_t pool = 4ull << 30;
	char *w;
	float *sink, *h;
	unsigned long long *hg;
	unsigned *err;
	CK(hipMalloc(&w, pool));
	CK(hipMemset(w, 0, pool));
	CK(hipMalloc(&sink, NWG * 4));
	CK(hipMalloc(&h, NH * 4));
	CK(hipMalloc(&hg, NH * 8));
	CK(hipMemset(hg, 0, NH * 8));
	CK(hipMalloc(&err, 4));
	CK(hipMemset(err, 0, 4));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	struct Pair {
		const char *name;
		size_t a, b;
	} pairs[] = {{"fp8 GLU -> W2 (117.4 / 58.7 MB)", 117440512, 58720256},
	             {"fp16 GLU -> W2 (234.9 / 117.4 MB)", 234881024, 117440512}};
	unsigned tag = 0;
	for (const Pair &pr : pairs) {
		const size_t pa = pr.a / NWG / ROUND * ROUND, pb = pr.b / NWG / ROUND * ROUND;
		const size_t ta = pa * NWG, tb = pb * NWG;
		printf("--- %s\n", pr.name);
		for (int mode = 0; mode < 3; ++mode) {
			size_t off = 0;
			auto pair = [&]() -> hipError_t {
				if (off + ta + tb > pool)
					off = 0;
				const char *a = w + off, *b = w + off + ta;
				off += ta + tb;
				++tag;
				if (mode == 0) {
					prod_k<false><<<NWG, THREADS, 0, s>>>(a, pa, h, hg, tag, sink);
					cons_k<false><<<NWG, THREADS, 0, s>>>(b, pb, h, hg, tag, sink, err);
				} else if (mode == 1) { // granule hand-off, barrier launches (its cost alone)
					prod_k<true><<<NWG, THREADS, 0, s>>>(a, pa, h, hg, tag, sink);
					cons_k<true><<<NWG, THREADS, 0, s>>>(b, pb, h, hg, tag, sink, err);
				} else { // the consumer launched any-order, the producer after a barrier as usual
					prod_k<true><<<NWG, THREADS, 0, s>>>(a, pa, h, hg, tag, sink);
					hipExtLaunchKernelGGL(cons_k<true>, dim3(NWG), dim3(THREADS), 0, s, nullptr, nullptr, 1, b, pb,
					                      (const float *)h, (const unsigned long long *)hg, tag, sink, err);
				}
				return hipGetLastError();
			};
			for (int i = 0; i < 10; ++i)
				CK(pair());
			CK(hipEventRecord(e0, s));
			const int reps = 200;
			for (int i = 0; i < reps; ++i)
				CK(pair());
			CK(hipEventRecord(e1, s));
			CK(hipEventSynchronize(e1));
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			unsigned e = 0;
			CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
			printf("  %-44s A+B %7.2f us per pair%s\n",
			       mode == 0   ? "barrier, plain h"
			       : mode == 1 ? "barrier, granule h (hand-off cost alone)"
			                   : "consumer any-order, granule h",
			       ms * 1e3f / reps, e ? "  [WAIT GAVE UP]" : "");
		}
	}
	return 0;
}
