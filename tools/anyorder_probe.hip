// anyorder_probe.hip — does hipExtAnyOrderLaunch let a kernel start before its predecessor
// in the same stream has finished, on gfx950 / ROCm 7.2? (hip_ext.h says the flag is not
// supported on GFX9 boards.) Two independent weight-stream kernels A then B (the GEMV access
// pattern: 256 workgroups x 512 threads, 16-byte nontemporal loads), launched with <<<>>> or
// with hipExtLaunchKernelGGL(..., flags = hipExtAnyOrderLaunch); each workgroup stamps
// s_memrealtime at start and end. Reports the pair's time and B's first start against A's
// last end (negative = the kernels overlapped).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/anyorder_probe tools/anyorder_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

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
constexpr size_t ROUND = (size_t)THREADS * 16 * U;

__global__ __launch_bounds__(THREADS) void stream_k(const char *w, size_t per_wg, float *sink,
                                                    unsigned long long *stamps) {
	const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
	const char *p = w + blockIdx.x * per_wg;
	float acc = 0.f;
	for (size_t o = 0; o < per_wg; o += ROUND) {
		u32x4_t v[U];
		for (int u = 0; u < U; ++u)
			v[u] = load_nt16(p + o + (size_t)(u * THREADS + threadIdx.x) * 16);
		for (int u = 0; u < U; ++u)
			acc += __uint_as_float(v[u][0] & 0x3fffffffu);
	}
	if (acc == 12345.f)
		sink[blockIdx.x] = acc;
	__syncthreads();
	if (threadIdx.x == 0) {
		stamps[2 * blockIdx.x] = t0;
		stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
	}
}

int main() {
	hipStream_t s;
	CK(hipStreamCreate(&s));
	const size_t pool = 4ull << 30;
	char *w;
	float *sink;
	unsigned long long *st;
	CK(hipMalloc(&w, pool));
	CK(hipMemset(w, 0, pool));
	CK(hipMalloc(&sink, NWG * 4));
	CK(hipMalloc(&st, 2 * 2 * NWG * 8));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	const size_t pa = 117440512 / NWG / ROUND * ROUND, pb = 58720256 / NWG / ROUND * ROUND;
	const size_t ta = pa * NWG, tb = pb * NWG;
	for (int flags = 0; flags <= 1; ++flags) {
		size_t off = 0;
		auto pair = [&](unsigned long long *sa, unsigned long long *sb) -> hipError_t {
			if (off + ta + tb > pool)
				off = 0;
			const char *a = w + off, *b = w + off + ta;
			off += ta + tb;
			if (!flags) {
				stream_k<<<NWG, THREADS, 0, s>>>(a, pa, sink, sa);
				stream_k<<<NWG, THREADS, 0, s>>>(b, pb, sink, sb);
				return hipGetLastError();
			}
			hipExtLaunchKernelGGL(stream_k, dim3(NWG), dim3(THREADS), 0, s, nullptr, nullptr, 1, a, pa, sink, sa);
			hipExtLaunchKernelGGL(stream_k, dim3(NWG), dim3(THREADS), 0, s, nullptr, nullptr, 1, b, pb, sink, sb);
			return hipGetLastError();
		};
		for (int i = 0; i < 10; ++i)
			CK(pair(st, st + 2 * NWG));
		CK(hipEventRecord(e0, s));
		const int reps = 200;
		for (int i = 0; i < reps; ++i)
			CK(pair(st, st + 2 * NWG));
		CK(hipEventRecord(e1, s));
		CK(hipEventSynchronize(e1));
		float ms;
		CK(hipEventElapsedTime(&ms, e0, e1));
		std::vector<unsigned long long> h(4 * NWG);
		CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
		unsigned long long a_end = 0, b_start = ~0ull, a_start = ~0ull, b_end = 0;
		for (int i = 0; i < NWG; ++i) {
			a_start = std::min(a_start, h[2 * i]);
			a_end = std::max(a_end, h[2 * i + 1]);
			b_start = std::min(b_start, h[2 * NWG + 2 * i]);
			b_end = std::max(b_end, h[2 * NWG + 2 * i + 1]);
		}
		printf("%s: A+B %.2f us per pair (%.0f GB/s); last pair: A %.2f us, B starts %.2f us after A's last end, B %.2f us\n",
		       flags ? "hipExtAnyOrderLaunch" : "<<<>>>            ", ms * 1e3f / reps, (ta + tb) / (ms * 1e3f / reps) / 1e3,
		       (a_end - a_start) / 100.0, ((double)b_start - (double)a_end) / 100.0, (b_end - b_start) / 100.0);
	}
	// the same pairs captured into a hipGraph (20 pairs per graph): does the capture keep the flag?
	for (int flags = 0; flags <= 1; ++flags) {
		size_t off = 0;
		hipGraph_t g;
		hipGraphExec_t ge;
		CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
		for (int i = 0; i < 20; ++i) {
			if (off + ta + tb > pool)
				off = 0;
			const char *a = w + off, *b = w + off + ta;
			off += ta + tb;
			if (!flags) {
				stream_k<<<NWG, THREADS, 0, s>>>(a, pa, sink, st);
				stream_k<<<NWG, THREADS, 0, s>>>(b, pb, sink, st + 2 * NWG);
			} else {
				hipExtLaunchKernelGGL(stream_k, dim3(NWG), dim3(THREADS), 0, s, nullptr, nullptr, 1, a, pa, sink, st);
				hipExtLaunchKernelGGL(stream_k, dim3(NWG), dim3(THREADS), 0, s, nullptr, nullptr, 1, b, pb, sink,
				                      st + 2 * NWG);
			}
		}
		CK(hipStreamEndCapture(s, &g));
		CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
		for (int i = 0; i < 3; ++i)
			CK(hipGraphLaunch(ge, s));
		CK(hipEventRecord(e0, s));
		const int reps = 10;
		for (int i = 0; i < reps; ++i)
			CK(hipGraphLaunch(ge, s));
		CK(hipEventRecord(e1, s));
		CK(hipEventSynchronize(e1));
		float ms;
		CK(hipEventElapsedTime(&ms, e0, e1));
		printf("graph, %s: A+B %.2f us per pair\n", flags ? "hipExtAnyOrderLaunch" : "<<<>>>            ",
		       ms * 1e3f / (reps * 20));
		CK(hipGraphExecDestroy(ge));
		CK(hipGraphDestroy(g));
	}
	return 0;
}
