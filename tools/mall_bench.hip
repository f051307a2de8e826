// mall_bench.hip — does a prefetch pass leave weights in the Infinity Cache
// (MALL, 256 MiB) so that the next kernel's streaming read of them is faster?
// Measures the read time of a W-byte buffer (Wo-sized: 32 MiB) by the decode
// GEMV access pattern (16 B/lane nt loads, one workgroup per CU, rows dealt
// round-robin) after (a) a cache flush (cold), (b) a flush + a prefetch
// kernel that touches every line with plain / nt loads, timed separately.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mall_bench tools/mall_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                                                                         \
	do {                                                                                                               \
		hipError_t e_ = (x);                                                                                           \
		if (e_ != hipSuccess) {                                                                                        \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                  \
			exit(1);                                                                                                   \
		}                                                                                                              \
	} while (0)

// consumer: 8 KB blocks dealt round-robin over 256 workgroups of 512 threads, U = 4
template <bool NT>
__global__ __launch_bounds__(512) void consume(const char *p, size_t bytes, unsigned *out) {
	const int w = blockIdx.x, v = threadIdx.x >> 6, lane = threadIdx.x & 63;
	const size_t nblk = bytes / 8192;
	unsigned acc = 0;
	for (size_t j = w; j < nblk; j += gridDim.x) {
		const char *q = p + j * 8192 + v * 1024 + lane * 16;
		u32x4 x = NT ? __builtin_nontemporal_load((const u32x4 *)q) : *(const u32x4 *)q;
		acc ^= x[0] ^ x[1] ^ x[2] ^ x[3];
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

// prefetcher: every lane touches one dword per 64-byte segment... here 16 B per lane, whole lines
template <int MODE> // 0 plain, 1 nt, 2 one dword per 128-B line (plain)
__global__ __launch_bounds__(256) void prefetch(const char *p, size_t bytes, unsigned *out) {
	unsigned acc = 0;
	const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
	if (MODE == 2) {
		for (size_t i = tid; i < bytes / 128; i += nth)
			acc ^= *(const unsigned *)(p + i * 128);
	} else {
		for (size_t i = tid; i < bytes / 16; i += nth) {
			u32x4 x = MODE == 1 ? __builtin_nontemporal_load((const u32x4 *)p + i) : ((const u32x4 *)p)[i];
			acc ^= x[0] ^ x[1] ^ x[2] ^ x[3];
		}
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

int main() {
	setvbuf(stdout, NULL, _IONBF, 0);
	const size_t W = 32ull << 20, FL = 1ull << 30;
	char *w, *fl;
	unsigned *out;
	CHK(hipMalloc(&w, W));
	CHK(hipMalloc(&fl, FL));
	CHK(hipMalloc(&out, 64));
	CHK(hipMemset(w, 1, W));
	CHK(hipMemset(fl, 2, FL));
	hipEvent_t e0, e1, e2;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	CHK(hipEventCreate(&e2));
	auto flush = [&] { prefetch<1><<<4096, 256>>>(fl, FL, out); };
	auto run = [&](const char *name, int pmode, bool nt_consumer) {
		float tp = 0, tc = 0;
		const int it = 10;
		for (int i = 0; i < it; ++i) {
			flush();
			CHK(hipEventRecord(e0, 0));
			if (pmode == 0)
				prefetch<0><<<2048, 256>>>(w, W, out);
			else if (pmode == 1)
				prefetch<1><<<2048, 256>>>(w, W, out);
			else if (pmode == 2)
				prefetch<2><<<2048, 256>>>(w, W, out);
			CHK(hipEventRecord(e1, 0));
			if (nt_consumer)
				consume<true><<<256, 512>>>(w, W, out);
			else
				consume<false><<<256, 512>>>(w, W, out);
			CHK(hipEventRecord(e2, 0));
			CHK(hipEventSynchronize(e2));
			float a, b;
			CHK(hipEventElapsedTime(&a, e0, e1));
			CHK(hipEventElapsedTime(&b, e1, e2));
			if (i) {
				tp += a;
				tc += b;
			}
		}
		tp = tp / (it - 1) * 1e3f, tc = tc / (it - 1) * 1e3f;
		printf("%-40s prefetch %7.2f us   consume %7.2f us (%5.2f TB/s)\n", name, tp, tc, W / (tc * 1e-6) / 1e12);
	};
	run("cold, nt consumer", -1, true);
	run("cold, plain consumer", -1, false);
	run("plain prefetch, nt consumer", 0, true);
	run("plain prefetch, plain consumer", 0, false);
	run("nt prefetch, nt consumer", 1, true);
	run("line-touch prefetch, nt consumer", 2, true);
	run("line-touch prefetch, plain consumer", 2, false);
	return 0;
}
