// persist_bench.hip — go/no-go microbenchmark for a persistent decode-layer
// engine: the byte stream of one Mistral-7B fp16 decode layer
// (QKV 48 MiB, Wo 32 MiB, W1|W3 224 MiB, W2 112 MiB) with the five
// all-to-all seams of the real layer (QKV -> attention -> Wo -> GLU -> W2 ->
// next layer), timed three ways:
//   launches : one streaming kernel per GEMV + a small "attention" kernel per
//              layer (today's engine, kernel boundaries as seams)
//   persist  : one 256-workgroup launch (1 per CU) per layer, in-launch seams
//              (sharded arrival counters, sc1 hand-off vector) — optionally
//              with the next phase's first U weight items issued BEFORE the
//              seam wait (prefetch across the dependency)
//   persist-all : the same, 32 layers in one launch
// Weights are only XOR-reduced (no math); the hand-off vector gather is real.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/persist_bench tools/persist_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                                                                         \
	do {                                                                                                               \
		hipError_t e_ = (x);                                                                                           \
		if (e_ != hipSuccess) {                                                                                        \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                  \
			exit(1);                                                                                                   \
		}                                                                                                              \
	} while (0)

constexpr int NWG = 256, THR = 512, NWAVE = THR / 64, ITEM = 1024;
constexpr int NPH = 4;
constexpr int ATT_WGS = 24, ATT_BYTES = 32768;

struct Args {
	const char *base;
	size_t layer_bytes;
	size_t off[NPH];
	unsigned per_wg[NPH]; // bytes per workgroup per phase
	int gather[NPH];      // floats gathered before the phase
	int l0, nl;
	unsigned *counters; // 8 shards, 32 words apart
	unsigned *endc, *epoch, *err;
	float *vec;
	const char *kv;
	unsigned *out;
};

__device__ __forceinline__ u32x4 ldnt(const char *p) { return __builtin_nontemporal_load((const u32x4 *)p); }

__device__ __forceinline__ unsigned ld_sc1u(const unsigned *p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1f(const float *p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte sc1 (L1-bypassing) load through a raw buffer resource (aux bit 4 = sc1 on gfx950)
__device__ __forceinline__ f32x4 ld_sc1x4(const float *base, unsigned byte_off) {
	__amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 0x7fffffff, 0x00020000);
	return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16));
}
__device__ __forceinline__ void st_sc1f(float *p, float v) {
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 lanes 0..7 poll the 8 shards until their sum reaches target
__device__ __forceinline__ void seam_wait(const Args &a, unsigned target, int tid) {
	if (tid < 64) {
		const int lane = tid;
		long spins = 0;
		while (true) {
			unsigned c = ld_sc1u(a.counters + (lane & 7) * 32);
			// every aligned group of 8 lanes sums the 8 shards (all 64 lanes must exit together)
			for (int o = 1; o < 8; o <<= 1)
				c += __shfl_xor(c, o, 64);
			if ((int)(c - target) >= 0)
				break;
			if (++spins > (1l << 18) || ld_sc1u(a.err) != 0) {
				if (lane == 0)
					atomicCAS(a.err, 0u, 0x10000u + target);
				break;
			}
			__builtin_amdgcn_s_sleep(1);
		}
	}
	__syncthreads();
}

__device__ __forceinline__ void seam_arrive(const Args &a, int tid) {
	__syncthreads(); // every wave done with the phase
	if (tid == 0)
		__hip_atomic_fetch_add(a.counters + (blockIdx.x & 7) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The wave's items of all phases form ONE stream t = 0..T-1; slot u is
// refilled with item t+U right after item t is consumed, unconditionally (the
// address clamps at T-1), so hipcc's vmcnt bookkeeping stays static (a
// conditional refill makes it wait vmcnt(0) before every load) and the
// refills issued in a phase's tail ARE the next phase's prefetch across the
// seam. PREFETCH=false drains before each seam instead (vmcnt(0)).
template <int U, bool PREFETCH, bool GATHER_ALL>
__global__ __launch_bounds__(THR, 1) void persist_kernel(Args a) {
	__shared__ __attribute__((aligned(16))) float vec[14336];
	__shared__ unsigned sh_epoch;
	const int w = blockIdx.x, tid = threadIdx.x, lane = tid & 63, v = tid >> 6;
	if (tid == 0)
		sh_epoch = ld_sc1u(a.epoch);
	__syncthreads();
	const unsigned E = sh_epoch;
	const unsigned seams_per_launch = 5 * a.nl - 1;
	unsigned seam = 0;
	unsigned acc = 0;
	int cstart[NPH + 1];
	cstart[0] = 0;
	for (int p = 0; p < NPH; ++p)
		cstart[p + 1] = cstart[p] + (int)(a.per_wg[p] / ITEM / NWAVE);
	const int per_layer = cstart[NPH];
	const int T = per_layer * a.nl; // multiple of U for this workload

	auto addr = [&](int t) {
		const int li = t / per_layer, r = t - li * per_layer;
		const int p = r < cstart[1] ? 0 : r < cstart[2] ? 1 : r < cstart[3] ? 2 : 3;
		const int j = r - cstart[p];
		return a.base + (size_t)(a.l0 + li) * a.layer_bytes + a.off[p] + ((size_t)(j * NWG + w) * NWAVE + v) * ITEM +
		       lane * 16;
	};
	auto gather = [&](int n) {
		if (GATHER_ALL || v == 0) {
			const int step = GATHER_ALL ? THR : 64;
			for (int i = (GATHER_ALL ? tid : lane) * 4; i < n; i += step * 4)
				*(f32x4 *)&vec[i] = ld_sc1x4(a.vec, i * 4);
		}
		__syncthreads();
	};
	auto next_target = [&]() { return 256u * (E * seams_per_launch + (++seam)); };

	u32x4 buf[U];
#pragma unroll
	for (int u = 0; u < U; ++u)
		buf[u] = ldnt(addr(u));
	gather(a.gather[0]);
	int r = 0, p = 0; // position within the layer, current phase
	for (int k = 0; k < T; k += U) {
#pragma unroll
		for (int u = 0; u < U; ++u) {
			const int t = k + u;
			if (r == per_layer)
				r = 0;
			const int np = r < cstart[1] ? 0 : r < cstart[2] ? 1 : r < cstart[3] ? 2 : 3;
			if (t > 0 && np != p) { // phase boundary: publish, seam, gather
				if (!PREFETCH)
					asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				acc += __float_as_uint(vec[(tid * 7) % a.gather[p]]);
				if (v == 0) {
					const int outs = (p == 2 ? 14336 : 4096) / NWG;
					if (lane < outs)
						st_sc1f(a.vec + w * outs + lane, (float)(acc & 0xff));
					asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				}
				seam_arrive(a, tid);
				seam_wait(a, next_target(), tid);
				if (np == 1) { // attention: 24 workgroups read KV, publish, seam
					if (w < ATT_WGS) {
						float s = 0.f;
						const float *kb = (const float *)(a.kv + (size_t)w * ATT_BYTES);
#pragma unroll
						for (int i = tid * 4; i < ATT_BYTES / 4; i += THR * 4) {
							f32x4 tt = ld_sc1x4(kb, i * 4);
							s += tt[0] + tt[1] + tt[2] + tt[3];
						}
						if (tid == 0)
							st_sc1f(a.vec + w, s);
						asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
					}
					seam_arrive(a, tid);
					seam_wait(a, next_target(), tid);
				}
				gather(a.gather[np]);
				p = np;
			}
			acc ^= buf[u][0] ^ buf[u][1] ^ buf[u][2] ^ buf[u][3];
			buf[u] = ldnt(addr(min(t + U, T - 1)));
			++r;
		}
	}
	acc += __float_as_uint(vec[(tid * 7) % a.gather[p]]);
	__syncthreads();
	if (tid == 0) {
		const unsigned t = __hip_atomic_fetch_add(a.endc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (t == 256u * (E + 1) - 1)
			__hip_atomic_fetch_add(a.epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	if (acc == 0x12345678u)
		a.out[0] = acc;
}

// Coordinator variant: wave 0 streams nothing — it publishes, arrives and
// polls with no weight loads queued ahead of its poll (in-order vmcnt: a poll
// behind U prefetch loads returns only after them). Waves 1..7 stream and keep
// their refills running across every seam (the prefetch).
template <int U>
__global__ __launch_bounds__(THR, 1) void persist_coord_kernel(Args a) {
	__shared__ __attribute__((aligned(16))) float vec[14336];
	__shared__ unsigned sh_epoch;
	constexpr int NS = NWAVE - 1;
	const int w = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
	const int v = __builtin_amdgcn_readfirstlane(tid >> 6);
	if (tid == 0)
		sh_epoch = ld_sc1u(a.epoch);
	__syncthreads();
	const unsigned E = sh_epoch;
	const unsigned seams_per_launch = 5 * a.nl - 1;
	unsigned seam = 0;
	unsigned acc = 0;
	auto next_target = [&]() { return 256u * (E * seams_per_launch + (++seam)); };
	auto gather = [&](int n) {
		for (int i = tid * 4; i < n; i += THR * 4)
			*(f32x4 *)&vec[i] = ld_sc1x4(a.vec, i * 4);
		__syncthreads();
	};
	// per-phase item counts of this wave (items s, s+NS, ... of the WG's phase slice)
	int NP[NPH], cum[NPH + 1];
	cum[0] = 0;
	for (int p = 0; p < NPH; ++p) {
		const int tot = (int)(a.per_wg[p] / ITEM);
		NP[p] = v == 0 ? 0 : (tot > v - 1 ? (tot - 1 - (v - 1)) / NS + 1 : 0);
		cum[p + 1] = cum[p] + NP[p];
	}
	const int per_layer = cum[NPH];
	const int T = per_layer * a.nl;
	auto addr = [&](int t) {
		const int li = t / per_layer, r = t - li * per_layer;
		const int p = r < cum[1] ? 0 : r < cum[2] ? 1 : r < cum[3] ? 2 : 3;
		const int it = (v - 1) + NS * (r - cum[p]); // item within the WG slice
		const int blk = it / NWAVE, sub = it - blk * NWAVE;
		return a.base + (size_t)(a.l0 + li) * a.layer_bytes + a.off[p] + ((size_t)(blk * NWG + w) * NWAVE + sub) * ITEM +
		       lane * 16;
	};
	const char *dummy = (const char *)a.vec + lane * 16;
	// seam sequence identical for all waves: after each phase except the last of the launch
	auto do_seam = [&](int p_done, int np) {
		// streamers: partials would go to LDS here
		__syncthreads();
		if (v == 0) {
			const int outs = (p_done == 2 ? 14336 : 4096) / NWG;
			if (lane < outs)
				st_sc1f(a.vec + w * outs + lane, (float)(acc & 0xff));
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			if (lane == 0)
				__hip_atomic_fetch_add(a.counters + (w & 7) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		seam_wait(a, next_target(), tid);
		if (np == 1) {
			if (w < ATT_WGS) {
				float s = 0.f;
				const float *kb = (const float *)(a.kv + (size_t)w * ATT_BYTES);
				for (int i = tid * 4; i < ATT_BYTES / 4; i += THR * 4) {
					f32x4 tt = ld_sc1x4(kb, i * 4);
					s += tt[0] + tt[1] + tt[2] + tt[3];
				}
				if (tid == 0)
					st_sc1f(a.vec + w, s);
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			}
			__syncthreads();
			if (tid == 0)
				__hip_atomic_fetch_add(a.counters + (w & 7) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			seam_wait(a, next_target(), tid);
		}
		gather(a.gather[np]);
	};

	gather(a.gather[0]);
	if (v == 0) {
		// coordinator: walk the same seam sequence
		for (int li = 0; li < a.nl; ++li)
			for (int p = 0; p < NPH; ++p)
				if (!(li == a.nl - 1 && p == NPH - 1))
					do_seam(p, (p + 1) % NPH);
	} else {
		u32x4 buf[U];
#pragma unroll
		for (int u = 0; u < U; ++u)
			buf[u] = ldnt(u < T ? addr(u) : dummy);
		int r = 0;
		for (int k = 0; k < T; k += U) {
#pragma unroll
			for (int u = 0; u < U; ++u) {
				const int t = k + u;
				if (t < T) {
					if (r == per_layer)
						r = 0;
					const int p = r < cum[1] ? 0 : r < cum[2] ? 1 : r < cum[3] ? 2 : 3; // (every phase non-empty here)
					acc ^= buf[u][0] ^ buf[u][1] ^ buf[u][2] ^ buf[u][3];
					++r;
					if (r == cum[p + 1] && t + 1 < T) // last item of this phase: seam after it
						do_seam(p, (p + 1) % NPH);
				}
				buf[u] = ldnt(t + U < T ? addr(t + U) : dummy);
			}
		}
	}
	acc += __float_as_uint(vec[(tid * 7) % 4096]);
	__syncthreads();
	if (tid == 0) {
		const unsigned t = __hip_atomic_fetch_add(a.endc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (t == 256u * (E + 1) - 1)
			__hip_atomic_fetch_add(a.epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	if (acc == 0x12345678u)
		a.out[0] = acc;
}

// pure streaming in the persistent geometry: the same item stream, no seams
template <int U>
__global__ __launch_bounds__(THR, 1) void persist_noseam_kernel(Args a) {
	const int w = blockIdx.x, tid = threadIdx.x, lane = tid & 63, v = tid >> 6;
	int cstart[NPH + 1];
	cstart[0] = 0;
	for (int p = 0; p < NPH; ++p)
		cstart[p + 1] = cstart[p] + (int)(a.per_wg[p] / ITEM / NWAVE);
	const int per_layer = cstart[NPH];
	const int T = per_layer * a.nl;
	auto addr = [&](int t) {
		const int li = t / per_layer, r = t - li * per_layer;
		const int p = r < cstart[1] ? 0 : r < cstart[2] ? 1 : r < cstart[3] ? 2 : 3;
		const int j = r - cstart[p];
		return a.base + (size_t)(a.l0 + li) * a.layer_bytes + a.off[p] + ((size_t)(j * NWG + w) * NWAVE + v) * ITEM +
		       lane * 16;
	};
	unsigned acc = 0;
	u32x4 buf[U];
#pragma unroll
	for (int u = 0; u < U; ++u)
		buf[u] = ldnt(addr(u));
	for (int k = 0; k < T; k += U) {
#pragma unroll
		for (int u = 0; u < U; ++u) {
			acc ^= buf[u][0] ^ buf[u][1] ^ buf[u][2] ^ buf[u][3];
			buf[u] = ldnt(addr(min(k + u + U, T - 1)));
		}
	}
	if (acc == 0x12345678u)
		a.out[0] = acc + tid;
}

// ---- launches baseline: today's geometry (many small workgroups, 16 KB per wave, U=4)
__global__ __launch_bounds__(512) void stream_kernel(const char *p, size_t bytes, const float *vec, int gather,
                                                     unsigned *out) {
	__shared__ float xs[4096];
	const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
	const int lane = threadIdx.x & 63;
	const size_t per_wave = 16384;
	const char *b = p + wave * per_wave + lane * 16;
	u32x4 r[4];
#pragma unroll
	for (int u = 0; u < 4; ++u)
		r[u] = ldnt(b + u * 1024);
	for (int i = threadIdx.x; i < gather && i < 4096; i += blockDim.x)
		xs[i] = vec[i];
	__syncthreads();
	unsigned acc = 0;
#pragma unroll
	for (int k = 0; k < 16; k += 4)
#pragma unroll
		for (int u = 0; u < 4; ++u) {
			acc ^= r[u][0] ^ r[u][1] ^ r[u][2] ^ r[u][3];
			if (k + u + 4 < 16)
				r[u] = ldnt(b + (k + u + 4) * 1024);
		}
	acc += __float_as_uint(xs[threadIdx.x & 4095]);
	if (acc == 0x12345678u)
		out[0] = acc;
}
__global__ __launch_bounds__(256) void att_kernel(const char *kv, float *vec) {
	float s = 0.f;
	for (int i = threadIdx.x; i < ATT_BYTES / 4; i += 256)
		s += ((const float *)(kv + (size_t)blockIdx.x * ATT_BYTES))[i];
	if (threadIdx.x == 0)
		vec[blockIdx.x] = s;
}

// ---- overlapped launches: kernel k runs on stream k % 2, so it is dispatched
// while kernel k-1 still runs; it issues its first U weight loads, then waits
// for k-1's arrival counter (sc1 poll by one lane), gathers the hand-off
// vector with sc1 loads and streams the rest. Completion: sc1 stores,
// vmcnt(0), one agent-scope add per workgroup.
template <int U, int SLEEP>
__global__ __launch_bounds__(512) void chain_kernel(const char *p, size_t bytes, int k, unsigned *counters, int nb_prev,
                                                    float *vec, int gather, unsigned *err, unsigned *out) {
	__shared__ __attribute__((aligned(16))) float xs[14336];
	const int w = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
	const int v = __builtin_amdgcn_readfirstlane(tid >> 6);
	const int nb = gridDim.x;
	// items: 1 KB, block j*nb + w (8 KB) split over the 8 waves
	const int nblk = (int)(bytes / 8192);
	const int mine = (nblk - w + nb - 1) / nb; // blocks of this WG; 1 item per wave per block
	auto addr = [&](int j) { return p + ((size_t)(j * nb + w) * 8 + v) * 1024 + lane * 16; };
	const char *dummy = (const char *)vec + lane * 16;
	u32x4 buf[U];
	if (v != 0 || k == 0) {
#pragma unroll
		for (int u = 0; u < U; ++u)
			buf[u] = ldnt(u < mine ? addr(u) : dummy);
	}
	if (k > 0) {
		if (tid == 0) { // wave 0 has no loads queued ahead of its poll (in-order vmcnt)
			long spins = 0;
			// 8 replicas of each counter (128 B apart); poll this XCD's
			while ((int)(ld_sc1u(counters + ((k - 1) * 8 + (w & 7)) * 32) - nb_prev) < 0) {
				if (++spins > (1l << 22)) {
					atomicCAS(err, 0u, 0x10000u + k);
					break;
				}
				__builtin_amdgcn_s_sleep(SLEEP);
			}
		}
		__syncthreads();
		if (v == 0) {
#pragma unroll
			for (int u = 0; u < U; ++u)
				buf[u] = ldnt(u < mine ? addr(u) : dummy);
		}
	}
	for (int i = tid * 4; i < gather; i += 512 * 4)
		*(f32x4 *)&xs[i] = ld_sc1x4(vec, i * 4);
	__syncthreads();
	unsigned acc = 0;
	for (int kk = 0; kk < mine; kk += U) {
#pragma unroll
		for (int u = 0; u < U; ++u) {
			const int j = kk + u;
			if (j < mine)
				acc ^= buf[u][0] ^ buf[u][1] ^ buf[u][2] ^ buf[u][3];
			buf[u] = ldnt(j + U < mine ? addr(j + U) : dummy);
		}
	}
	acc += __float_as_uint(xs[(tid * 7) % gather]);
	if (tid < 16)
		st_sc1f(vec + w * 16 + tid, (float)(acc & 0xff));
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if (tid < 8) // one add per replica
		__hip_atomic_fetch_add(counters + (k * 8 + tid) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	if (acc == 0x12345678u)
		out[0] = acc;
}
template <int SLEEP>
__global__ __launch_bounds__(256) void chain_att_kernel(const char *kv, float *vec, int k, unsigned *counters,
                                                        int nb_prev, unsigned *err) {
	if (threadIdx.x == 0) {
		long spins = 0;
		while ((int)(ld_sc1u(counters + ((k - 1) * 8 + (blockIdx.x & 7)) * 32) - nb_prev) < 0) {
			if (++spins > (1l << 22)) {
				atomicCAS(err, 0u, 0x10000u + k);
				break;
			}
			__builtin_amdgcn_s_sleep(SLEEP);
		}
	}
	__syncthreads();
	float s = 0.f;
	const float *kb = (const float *)(kv + (size_t)blockIdx.x * ATT_BYTES);
	for (int i = threadIdx.x * 4; i < ATT_BYTES / 4; i += 256 * 4) {
		f32x4 t = ld_sc1x4(kb, i * 4);
		s += t[0] + t[1] + t[2] + t[3];
	}
	if (threadIdx.x == 0)
		st_sc1f(vec + blockIdx.x, s);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if (threadIdx.x < 8)
		__hip_atomic_fetch_add(counters + (k * 8 + threadIdx.x) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main(int argc, char **argv) {
	setvbuf(stdout, NULL, _IONBF, 0);
	const int L = 32;
	const size_t sz[NPH] = {48ull << 20, 32ull << 20, 224ull << 20, 112ull << 20};
	size_t layer = 0, off[NPH];
	for (int p = 0; p < NPH; ++p) {
		off[p] = layer;
		layer += sz[p];
	}
	int ncu = 0;
	CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	if (ncu < NWG) {
		printf("need %d CUs, have %d\n", NWG, ncu);
		return 1;
	}
	char *w;
	CHK(hipMalloc(&w, layer * L));
	CHK(hipMemset(w, 1, layer * L));
	char *kv;
	CHK(hipMalloc(&kv, ATT_WGS * ATT_BYTES));
	CHK(hipMemset(kv, 0, ATT_WGS * ATT_BYTES));
	float *vec;
	CHK(hipMalloc(&vec, 14336 * 4));
	CHK(hipMemset(vec, 0, 14336 * 4));
	unsigned *ctr;
	CHK(hipMalloc(&ctr, 4096));
	CHK(hipMemset(ctr, 0, 4096));
	unsigned *out;
	CHK(hipMalloc(&out, 64));
	hipEvent_t e0, e1;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	const double tot_bytes = (double)layer * L;
	auto report = [&](const char *name, float ms) {
		printf("%-34s %8.1f us/layer  %6.2f TB/s  (%.3f ms / %d layers)\n", name, ms * 1e3 / L,
		       tot_bytes / (ms * 1e-3) / 1e12, ms, L);
	};
	auto timeit = [&](auto fn) {
		float best = 1e30f;
		for (int it = 0; it < 6; ++it) {
			CHK(hipEventRecord(e0, 0));
			fn();
			CHK(hipEventRecord(e1, 0));
			CHK(hipEventSynchronize(e1));
			float ms;
			CHK(hipEventElapsedTime(&ms, e0, e1));
			if (it >= 1 && ms < best)
				best = ms;
		}
		return best;
	};

	// launches baseline
	{
		float ms = timeit([&] {
			for (int l = 0; l < L; ++l) {
				for (int p = 0; p < NPH; ++p) {
					const int blocks = (int)(sz[p] / 16384 / 8);
					stream_kernel<<<blocks, 512>>>(w + l * layer + off[p], sz[p], vec, 4096, out);
					if (p == 0)
						att_kernel<<<ATT_WGS, 256>>>(kv, vec);
				}
			}
		});
		report("launches (5 kernels/layer)", ms);
	}
	{
		// same kernels, one stream, flags unused (k = 0 path) except the gather: reference for the chain
		unsigned *cc, *cerr;
		CHK(hipMalloc(&cc, 4 * 32 * 8 * 200));
		CHK(hipMalloc(&cerr, 4));
		CHK(hipMemset(cerr, 0, 4));
		hipStream_t s2[2];
		CHK(hipStreamCreateWithFlags(&s2[0], hipStreamNonBlocking));
		CHK(hipStreamCreateWithFlags(&s2[1], hipStreamNonBlocking));
		hipEvent_t ej;
		CHK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
		auto chain = [&](int nstreams, int SL) {
			CHK(hipMemsetAsync(cc, 0, 4 * 32 * 8 * 200, 0));
			CHK(hipEventRecord(ej, 0));
			CHK(hipStreamWaitEvent(s2[0], ej, 0));
			CHK(hipStreamWaitEvent(s2[1], ej, 0));
			int k = 0, nb_prev = 0;
			for (int l = 0; l < L; ++l) {
				for (int p = 0; p < NPH; ++p) {
					hipStream_t st = s2[nstreams == 2 ? (k & 1) : 0];
					const int g = p == 3 ? 14336 : 4096;
					if (SL == 1)
						chain_kernel<4, 1><<<256, 512, 0, st>>>(w + l * layer + off[p], sz[p], k, cc, nb_prev, vec, g, cerr, out);
					else
						chain_kernel<4, 8><<<256, 512, 0, st>>>(w + l * layer + off[p], sz[p], k, cc, nb_prev, vec, g, cerr, out);
					nb_prev = 256;
					++k;
					if (p == 0) {
						st = s2[nstreams == 2 ? (k & 1) : 0];
						if (SL == 1)
							chain_att_kernel<1><<<ATT_WGS, 256, 0, st>>>(kv, vec, k, cc, nb_prev, cerr);
						else
							chain_att_kernel<8><<<ATT_WGS, 256, 0, st>>>(kv, vec, k, cc, nb_prev, cerr);
						nb_prev = ATT_WGS;
						++k;
					}
				}
			}
			CHK(hipEventRecord(ej, s2[0]));
			CHK(hipStreamWaitEvent(0, ej, 0));
			CHK(hipEventRecord(ej, s2[1]));
			CHK(hipStreamWaitEvent(0, ej, 0));
		};
		for (int ns = 1; ns <= 2; ++ns)
			for (int U : {1, 8}) {
				float ms = timeit([&] { chain(ns, U); });
				unsigned e;
				CHK(hipMemcpy(&e, cerr, 4, hipMemcpyDeviceToHost));
				char nm[96];
				snprintf(nm, sizeof nm, "chain %d stream(s) sleep=%d%s", ns, U, e ? " SEAM TIMEOUT" : "");
				report(nm, ms);
				if (e)
					exit(1);
			}
	}
	Args a{};
	a.base = w;
	a.layer_bytes = layer;
	for (int p = 0; p < NPH; ++p) {
		a.off[p] = off[p];
		a.per_wg[p] = (unsigned)(sz[p] / NWG);
	}
	a.gather[0] = 4096, a.gather[1] = 4096, a.gather[2] = 4096, a.gather[3] = 14336;
	a.counters = ctr;
	a.endc = ctr + 512;
	a.epoch = ctr + 544;
	a.err = ctr + 576;
	a.vec = vec;
	a.kv = kv;
	a.out = out;
	auto runp = [&](auto kern, int U, bool PF, bool GA, bool ALL) {
		CHK(hipMemset(ctr, 0, 4096));
		float ms = timeit([&] {
			if (ALL) {
				a.l0 = 0, a.nl = L;
				kern<<<NWG, THR>>>(a);
			} else {
				for (int l = 0; l < L; ++l) {
					a.l0 = l, a.nl = 1;
					kern<<<NWG, THR>>>(a);
				}
			}
		});
		unsigned err;
		CHK(hipMemcpy(&err, a.err, 4, hipMemcpyDeviceToHost));
		char nm[96];
		snprintf(nm, sizeof nm, "persist%s U=%d pf=%d gather=%s", ALL ? "-all" : "", U, PF, GA ? "all" : "w0");
		report(nm, ms);
		if (err) {
			unsigned c[1];
			CHK(hipMemcpy(c, a.counters, 4, hipMemcpyDeviceToHost));
			printf("  SEAM TIMEOUT err=%x shard0=%u\n", err, c[0]);
			exit(1);
		}
	};
#define RUNP(U, PF, GA, ALL) runp(persist_kernel<U, PF, GA>, U, PF, GA, ALL)
	for (int all = 0; all < 2; ++all) {
		auto noseam = [&](auto kern, int U) {
			float ms = timeit([&] {
				if (all) {
					a.l0 = 0, a.nl = L;
					kern<<<NWG, THR>>>(a);
				} else {
					for (int l = 0; l < L; ++l) {
						a.l0 = l, a.nl = 1;
						kern<<<NWG, THR>>>(a);
					}
				}
			});
			char nm[96];
			snprintf(nm, sizeof nm, "noseam%s U=%d", all ? "-all" : "", U);
			report(nm, ms);
		};
		noseam(persist_noseam_kernel<8>, 8);
		noseam(persist_noseam_kernel<16>, 16);
	}
	auto runc = [&](auto kern, int U, bool ALL) {
		CHK(hipMemset(ctr, 0, 4096));
		float ms = timeit([&] {
			if (ALL) {
				a.l0 = 0, a.nl = L;
				kern<<<NWG, THR>>>(a);
			} else {
				for (int l = 0; l < L; ++l) {
					a.l0 = l, a.nl = 1;
					kern<<<NWG, THR>>>(a);
				}
			}
		});
		unsigned err;
		CHK(hipMemcpy(&err, a.err, 4, hipMemcpyDeviceToHost));
		char nm[96];
		snprintf(nm, sizeof nm, "coord%s U=%d", ALL ? "-all" : "", U);
		report(nm, ms);
		if (err) {
			printf("  SEAM TIMEOUT err=%x\n", err);
			exit(1);
		}
	};
	runc(persist_coord_kernel<4>, 4, false);
	runc(persist_coord_kernel<8>, 8, false);
	runc(persist_coord_kernel<16>, 16, false);
	runc(persist_coord_kernel<4>, 4, true);
	runc(persist_coord_kernel<8>, 8, true);
	runc(persist_coord_kernel<16>, 16, true);
	runc(persist_coord_kernel<24>, 24, true);
	RUNP(8, false, true, false);
	RUNP(8, true, true, false);
	RUNP(16, true, true, false);
	RUNP(16, true, false, false);
	RUNP(8, true, true, true);
	RUNP(16, true, true, true);
	RUNP(16, true, false, true);
	RUNP(24, true, true, true);
	return 0;
}
