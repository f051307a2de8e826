// concurrency_check.hip — do kernels on two HIP streams run concurrently on this
// box? Two single-workgroup kernels that each spin 200 us, on one stream vs on
// two streams; also 256-workgroup variants (one per CU) to check co-residency.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/concurrency_check tools/concurrency_check.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                                                         \
	do {                                                                                                               \
		hipError_t e_ = (x);                                                                                           \
		if (e_ != hipSuccess) {                                                                                        \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                  \
			exit(1);                                                                                                   \
		}                                                                                                              \
	} while (0)

__global__ __launch_bounds__(512) void spin(unsigned long long ticks, unsigned long long *stamp) {
	__shared__ float pad[12000];
	const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
	pad[threadIdx.x] = 0;
	while (__builtin_amdgcn_s_memrealtime() - t0 < ticks)
		__builtin_amdgcn_s_sleep(10);
	if (threadIdx.x == 0 && blockIdx.x == 0) {
		stamp[0] = t0;
		stamp[1] = __builtin_amdgcn_s_memrealtime() + (unsigned long long)pad[5];
	}
}

int main() {
	hipStream_t s[2];
	CHK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
	CHK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
	unsigned long long *st;
	CHK(hipMalloc(&st, 64));
	hipEvent_t e0, e1, ej;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	CHK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
	const unsigned long long ticks = 20000; // 200 us at 100 MHz
	for (int blocks : {1, 256}) {
		for (int ns = 1; ns <= 2; ++ns) {
			float best = 1e9f;
			for (int it = 0; it < 5; ++it) {
				CHK(hipEventRecord(e0, 0));
				CHK(hipStreamWaitEvent(s[0], e0, 0));
				CHK(hipStreamWaitEvent(s[1], e0, 0));
				spin<<<blocks, 512, 0, s[0]>>>(ticks, st);
				spin<<<blocks, 512, 0, s[ns - 1]>>>(ticks, st + 2);
				CHK(hipEventRecord(ej, s[0]));
				CHK(hipStreamWaitEvent(0, ej, 0));
				CHK(hipEventRecord(ej, s[1]));
				CHK(hipStreamWaitEvent(0, ej, 0));
				CHK(hipEventRecord(e1, 0));
				CHK(hipEventSynchronize(e1));
				float ms;
				CHK(hipEventElapsedTime(&ms, e0, e1));
				if (ms < best)
					best = ms;
			}
			unsigned long long h[4];
			CHK(hipMemcpy(h, st, 32, hipMemcpyDeviceToHost));
			printf("blocks=%3d streams=%d: %7.1f us (2 x 200 us kernels); second kernel started %+.1f us after the first\n",
			       blocks, ns, best * 1e3, ((long long)h[2] - (long long)h[0]) * 0.01);
		}
	}
	return 0;
}
