// stream_bench.hip — calibration microbenchmark: time of a pure read-only
// HBM stream (sum-reduce of N bytes, 16 B/lane nt loads) as a function of N,
// to separate the per-launch fixed cost T0 from the steady-state bandwidth B
// (T(N) = T0 + N/B) that bounds the decode GEMVs.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_bench tools/stream_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(512) void stream_read(const u32x4 *__restrict__ p, size_t n16, size_t per_wave,
                                                   unsigned *out) {
	const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
	const int lane = threadIdx.x & 63;
	size_t base = wave * per_wave;
	size_t end = base + per_wave < n16 ? base + per_wave : n16;
	unsigned acc = 0;
	for (size_t i = base + lane; i < end; i += 64 * U) {
		u32x4 v[U];
#pragma unroll
		for (int u = 0; u < U; ++u) {
			size_t j = i + (size_t)u * 64;
			v[u] = j < end ? __builtin_nontemporal_load(p + j) : u32x4{0, 0, 0, 0};
		}
#pragma unroll
		for (int u = 0; u < U; ++u)
			acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

template <int U>
static float run(const u32x4 *buf, size_t maxb, size_t bytes, size_t per_wave_bytes, int threads, unsigned *out) {
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	const size_t n16 = bytes / 16;
	const size_t per_wave = per_wave_bytes / 16;
	const size_t waves = (n16 + per_wave - 1) / per_wave;
	const int wpb = threads / 64;
	const int blocks = (int)((waves + wpb - 1) / wpb);
	float tot = 0;
	const int iters = 20;
	for (int it = 0; it < iters; ++it) {
		const u32x4 *p = buf + (it & 1) * (maxb / 16);
		hipEventRecord(e0, 0);
		stream_read<U><<<blocks, threads>>>(p, n16, per_wave, out);
		hipEventRecord(e1, 0);
		hipEventSynchronize(e1);
		float ms;
		hipEventElapsedTime(&ms, e0, e1);
		if (it >= 2)
			tot += ms;
	}
	return tot / (iters - 2) * 1e3f;
}

int main() {
	const size_t maxb = 1ull << 30;
	u32x4 *buf;
	unsigned *out;
	hipMalloc(&buf, maxb * 2);
	hipMalloc(&out, 64);
	hipMemset(buf, 1, maxb * 2);
	const size_t sizes_mb[] = {16, 33, 50, 117, 235, 470};
	for (size_t mb : sizes_mb) {
		const size_t bytes = mb << 20;
		float best = 1e9;
		char desc[128] = "";
		for (size_t pw : {4096ul, 8192ul, 16384ul, 32768ul, 65536ul, 131072ul})
			for (int thr : {256, 512})
				for (int u : {2, 4, 8}) {
					float t = u == 2 ? run<2>(buf, maxb, bytes, pw, thr, out)
					          : u == 4 ? run<4>(buf, maxb, bytes, pw, thr, out)
					                   : run<8>(buf, maxb, bytes, pw, thr, out);
					if (getenv("SB_ALL"))
						printf("  size=%zu per_wave=%zuKB thr=%d U=%d: %.2f us\n", mb, pw / 1024, thr, u, t);
					if (t < best) {
						best = t;
						snprintf(desc, sizeof desc, "per_wave=%zuKB threads=%d U=%d", pw / 1024, thr, u);
					}
				}
		printf("size=%4zu MB best %8.2f us -> %6.0f GB/s  (%s)\n", mb, best, bytes / (best * 1e-6) / 1e9, desc);
	}
	return 0;
}
