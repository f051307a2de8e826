// mall_prefetch_bench.hip — does warming the first megabytes of a weight stream in the
// Infinity Cache (MALL) / L2 shorten the next stream kernel's ramp?
// A decode GEMV streams its rows as one contiguous window moving through the matrix
// (row group g -> workgroup g % NB), so its first loads are the matrix's first few MB.
// Sequences, back to back on one stream, the timed kernel bracketed by events:
//   cold : S(X, 235 MB) -> [S(Y, 117 MB)]
//   warm : P(Y, first W MB) -> S(X) -> [S(Y)]      (does the warm survive X's nt stream?)
//   hot  : S(X) -> P(Y, first W MB) -> [S(Y)]      (prefetch right before)
// S = 256 workgroups x 512 threads, wave w reads 1-KB chunks w, w + 2048, ... (U = 4 in
// flight, 16-B nontemporal loads); P = plain 16-B loads of the first W MB.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mall_prefetch_bench tools/mall_prefetch_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void stream_k(const u32x4 *__restrict__ p, size_t nchunks, unsigned *out) {
	const size_t W = (size_t)gridDim.x * 8;
	const size_t w = blockIdx.x * 8 + (threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	unsigned acc = 0;
	for (size_t c = w; c < nchunks; c += 4 * W) {
		u32x4 v[4];
#pragma unroll
		for (int u = 0; u < 4; ++u) {
			const size_t cc = c + u * W;
			v[u] = cc < nchunks ? __builtin_nontemporal_load(p + cc * 64 + lane) : u32x4{0, 0, 0, 0};
		}
#pragma unroll
		for (int u = 0; u < 4; ++u)
			acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

__global__ __launch_bounds__(256) void prefetch_k(const u32x4 *__restrict__ p, size_t n16, unsigned *out) {
	unsigned acc = 0;
	for (size_t i = blockIdx.x * 256ul + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
		acc ^= p[i][0];
	if (acc == 0x12345678u)
		out[1] = acc;
}

int main() {
	const size_t XB = 235ull << 20, YB = 117ull << 20;
	u32x4 *x, *y, *z;
	unsigned *out;
	hipMalloc(&x, XB);
	hipMalloc(&y, YB);
	hipMalloc(&z, 512ull << 20);
	hipMalloc(&out, 64);
	hipMemset(x, 1, XB);
	hipMemset(y, 2, YB);
	hipMemset(z, 3, 512ull << 20);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	auto S = [&](const u32x4 *p, size_t bytes) { stream_k<<<256, 512>>>(p, bytes / 1024, out); };
	auto P = [&](const u32x4 *p, size_t bytes) { prefetch_k<<<256, 256>>>(p, bytes / 16, out); };
	auto flush = [&]() { S(z, 512ull << 20); };
	const size_t Ws[] = {0, 2ull << 20, 8ull << 20, 32ull << 20};
	const char *names[] = {"cold", "warm", "hot"};
	for (size_t W : Ws) {
		for (int mode = 0; mode < 3; ++mode) {
			if (W == 0 && mode)
				continue;
			std::vector<float> t;
			for (int it = 0; it < 15; ++it) {
				flush();
				if (mode == 1)
					P(y, W);
				S(x, XB);
				if (mode == 2)
					P(y, W);
				hipEventRecord(e0, 0);
				S(y, YB);
				hipEventRecord(e1, 0);
				hipEventSynchronize(e1);
				float ms;
				hipEventElapsedTime(&ms, e0, e1);
				if (it >= 3)
					t.push_back(ms * 1e3f);
			}
			std::sort(t.begin(), t.end());
			printf("%-5s prefetch %3zu MB: S(Y 117 MB) median %.2f us min %.2f us\n", names[mode], W >> 20,
			       t[t.size() / 2], t[0]);
		}
	}
	return 0;
}
