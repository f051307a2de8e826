// Where does the dispatcher put the workgroups of a 2-per-CU grid? Each of 512
// workgroups (256 threads, 70 KB LDS: at most 2 per CU, like the fused attention + Wo
// launch) records its XCC / SE / CU and waits (bounded) until every workgroup has
// arrived, so the placement is the co-resident one. Prints, per workgroup b < 256,
// whether b + 256 landed on the same CU.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/placement_bench tools/placement_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                                     \
	do {                                                                                           \
		hipError_t e = (x);                                                                        \
		if (e != hipSuccess) {                                                                     \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                                 \
			exit(1);                                                                               \
		}                                                                                          \
	} while (0)

__global__ __launch_bounds__(256) void place(unsigned *ids, unsigned *arrived, int n) {
	extern __shared__ unsigned lds[];
	if (threadIdx.x == 0) {
		const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
		const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20); // XCC_ID
		lds[0] = hw;
		ids[2 * blockIdx.x] = hw;
		ids[2 * blockIdx.x + 1] = xcc;
		__hip_atomic_fetch_add(arrived, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
		while (__hip_atomic_load(arrived, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)n &&
		       __builtin_amdgcn_s_memrealtime() - t0 < 20000000ull) // 0.2 s
			__builtin_amdgcn_s_sleep(8);
	}
	__syncthreads();
}

int main() {
	const int n = 512;
	unsigned *ids, *arr;
	CHK(hipMalloc(&ids, 2 * n * 4));
	CHK(hipMalloc(&arr, 4));
	CHK(hipMemset(arr, 0, 4));
	CHK(hipFuncSetAttribute((const void *)place, hipFuncAttributeMaxDynamicSharedMemorySize, 70 * 1024));
	hipLaunchKernelGGL(place, dim3(n), dim3(256), 70 * 1024, 0, ids, arr, n);
	CHK(hipDeviceSynchronize());
	unsigned h[2 * n], a = 0;
	CHK(hipMemcpy(h, ids, sizeof(h), hipMemcpyDeviceToHost));
	CHK(hipMemcpy(&a, arr, 4, hipMemcpyDeviceToHost));
	printf("arrived %u of %d\n", a, n);
	auto cu = [&](int b) {
		const unsigned hw = h[2 * b], x = h[2 * b + 1] & 15;
		return (x << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
	};
	int same = 0;
	for (int b = 0; b < n / 2; ++b)
		same += cu(b) == cu(b + n / 2);
	printf("b and b+256 on the same CU: %d of %d\n", same, n / 2);
	// distinct CUs among the first 256
	int distinct = 0;
	for (int b = 0; b < n / 2; ++b) {
		bool dup = false;
		for (int c = 0; c < b; ++c)
			dup = dup || cu(c) == cu(b);
		distinct += !dup;
	}
	printf("distinct CUs among b < 256: %d\n", distinct);
	for (int b = 0; b < 48; ++b) {
		int partner = -1;
		for (int c = 0; c < n; ++c)
			if (c != b && cu(c) == cu(b))
				partner = c;
		printf("b %3d: xcc %u se %u sh %u cu %2u  co-resident with b %d\n", b, h[2 * b + 1] & 15, (h[2 * b] >> 13) & 7,
		       (h[2 * b] >> 12) & 1, (h[2 * b] >> 8) & 15, partner);
	}
	return 0;
}
