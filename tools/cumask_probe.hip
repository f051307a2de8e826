// Which CUs does a CU-masked stream (hipExtStreamCreateWithCUMask) run on? For
// N = 2 / 4 / 8 "ranks" and two mask layouts (contiguous 256/N-bit blocks; bit i to
// rank i mod N), every rank's stream runs a 1024-workgroup grid whose workgroups
// record XCC / SE / SH / CU (HW_ID, XCC_ID) and linger ~20 us so the grid spreads.
// Prints, per layout and N: CUs each rank used, XCCs touched, and whether any two
// ranks shared a CU. Then two ranks' kernels handshake through a flag (bounded
// spin): with disjoint masks rank 0's grid filling its CUs cannot starve rank 1's.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/cumask_probe tools/cumask_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <set>
#include <vector>

#define CHK(x)                                                                                                         \
	do {                                                                                                               \
		hipError_t e = (x);                                                                                            \
		if (e != hipSuccess) {                                                                                         \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                                                     \
			exit(1);                                                                                                   \
		}                                                                                                              \
	} while (0)

__global__ __launch_bounds__(256) void place(unsigned *ids) {
	if (threadIdx.x == 0) {
		const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
		const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20); // XCC_ID
		ids[2 * blockIdx.x] = hw;
		ids[2 * blockIdx.x + 1] = xcc;
		const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
		while (__builtin_amdgcn_s_memrealtime() - t0 < 2000ull) // ~20 us at 100 MHz
			__builtin_amdgcn_s_sleep(4);
	}
	__syncthreads();
}

// rank 0: every workgroup spins until rank 1's kernel has set *flag (bounded 50 ms);
// rank 1: one workgroup sets it. Records whether each rank-0 workgroup saw the flag.
__global__ __launch_bounds__(256) void handshake(unsigned *flag, unsigned *seen, int setter) {
	if (threadIdx.x == 0) {
		if (setter) {
			__hip_atomic_store(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
		} else {
			const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
			unsigned v = 0;
			while (!(v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) &&
			       __builtin_amdgcn_s_memrealtime() - t0 < 5000000ull) // 50 ms
				__builtin_amdgcn_s_sleep(8);
			seen[blockIdx.x] = v;
		}
	}
	__syncthreads();
}

static unsigned cu_key(unsigned hw, unsigned xcc) {
	return ((xcc & 15) << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
}

static std::vector<uint32_t> make_mask(int ncu, int layout, int r, int N) {
	std::vector<uint32_t> m((ncu + 31) / 32, 0u);
	for (int i = 0; i < ncu; ++i) {
		const bool on = layout == 0 ? (i / (ncu / N)) == r : (i % N) == r;
		if (on)
			m[i / 32] |= 1u << (i % 32);
	}
	return m;
}

int main() {
	int ncu = 0;
	CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	printf("CUs: %d\n", ncu);
	const int nb = 1024;
	unsigned *ids;
	CHK(hipMalloc(&ids, 2 * nb * 4));
	std::vector<unsigned> h(2 * nb);
	for (int layout = 0; layout < 2; ++layout) {
		for (int N : {2, 4, 8}) {
			std::vector<std::set<unsigned>> used(N);
			for (int r = 0; r < N; ++r) {
				auto m = make_mask(ncu, layout, r, N);
				hipStream_t s;
				CHK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
				std::vector<uint32_t> back(m.size(), 0);
				CHK(hipExtStreamGetCUMask(s, (uint32_t)back.size(), back.data()));
				int pop = 0;
				for (uint32_t w : back)
					pop += __builtin_popcount(w);
				CHK(hipMemsetAsync(ids, 0xff, 2 * nb * 4, s));
				hipLaunchKernelGGL(place, dim3(nb), dim3(256), 0, s, ids);
				CHK(hipStreamSynchronize(s));
				CHK(hipMemcpy(h.data(), ids, 2 * nb * 4, hipMemcpyDeviceToHost));
				std::set<unsigned> xccs;
				for (int b = 0; b < nb; ++b) {
					used[r].insert(cu_key(h[2 * b], h[2 * b + 1]));
					xccs.insert(h[2 * b + 1] & 15);
				}
				printf("layout %s N %d rank %d: mask popcount %d (get-back), CUs used %zu, XCCs touched %zu {",
				       layout ? "interleaved" : "contiguous", N, r, pop, used[r].size(), xccs.size());
				for (unsigned x : xccs)
					printf(" %u", x);
				printf(" }\n");
				CHK(hipStreamDestroy(s));
			}
			int shared = 0;
			for (int a = 0; a < N; ++a)
				for (int b = a + 1; b < N; ++b)
					for (unsigned k : used[a])
						shared += used[b].count(k);
			printf("layout %s N %d: CUs shared between ranks: %d\n", layout ? "interleaved" : "contiguous", N, shared);
		}
	}
	// handshake: rank 0 fills its half of the chip with spinning workgroups, rank 1's kernel
	// (launched after) must still get a CU
	for (int layout = 0; layout < 2; ++layout) {
		unsigned *flag, *seen;
		CHK(hipMalloc(&flag, 4));
		CHK(hipMalloc(&seen, 4 * 2048));
		CHK(hipMemset(flag, 0, 4));
		CHK(hipMemset(seen, 0, 4 * 2048));
		hipStream_t s0, s1;
		auto m0 = make_mask(ncu, layout, 0, 2), m1 = make_mask(ncu, layout, 1, 2);
		CHK(hipExtStreamCreateWithCUMask(&s0, (uint32_t)m0.size(), m0.data()));
		CHK(hipExtStreamCreateWithCUMask(&s1, (uint32_t)m1.size(), m1.data()));
		const int n0 = 2048; // 8 per CU of rank 0's 128: more than fit
		hipLaunchKernelGGL(handshake, dim3(n0), dim3(256), 0, s0, flag, seen, 0);
		hipLaunchKernelGGL(handshake, dim3(1), dim3(256), 0, s1, flag, seen, 1);
		CHK(hipStreamSynchronize(s0));
		CHK(hipStreamSynchronize(s1));
		std::vector<unsigned> sv(n0);
		CHK(hipMemcpy(sv.data(), seen, 4 * n0, hipMemcpyDeviceToHost));
		int ok = 0;
		for (unsigned v : sv)
			ok += v == 1;
		printf("handshake layout %s: rank-0 workgroups that saw rank 1's flag: %d of %d\n",
		       layout ? "interleaved" : "contiguous", ok, n0);
		CHK(hipStreamDestroy(s0));
		CHK(hipStreamDestroy(s1));
		CHK(hipFree(flag));
		CHK(hipFree(seen));
	}
	return 0;
}
