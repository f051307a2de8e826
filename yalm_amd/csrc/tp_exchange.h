// tp_exchange.h — the tensor-parallel all-reduce of x folded into the kernels on
// either side of it (IPC transport; BASELINE config 5).
//
// Megatron split (include/yalm_hip.h): after the Wo and the W2 GEMVs every rank holds
// a partial of x (rank 0's includes the residual), and every rank needs the sum. The
// round-2..4 form wrote the partial into the rank's own buffer, then ONE extra
// single-workgroup kernel per exchange signalled the peers, waited for them and pulled
// and summed every rank's partial: 2 exchanges x (launch + round trips) per layer, 7
// launches per layer against 4 on one GPU. Here there is no exchange kernel:
//   * PRODUCER (the Wo workgroups of the fused attention + Wo launch, the W2 GEMV, the
//     argmax): each workgroup PUSHES its rows to slot [parity][this rank] of EVERY
//     rank's buffer (system-scope stores: the bytes leave the writer at once), waits for
//     them (vmcnt(0)), and takes a ticket; the last workgroup of the launch bumps
//     xdone[this rank] in every rank's control words.
//   * CONSUMER (the next GEMV's x staging: GLU after Wo, next layer's QKV / the logits
//     after W2): waits until xdone[p] >= xdone[own] for every rank p (this rank's own
//     count is final: its producer finished before the consumer launched), then sums
//     the N slots in rank order -- bit-identical x on every rank -- while its weight
//     stream is already in flight, and writes x back for the next residual.
// Strict alternation of the two parities holds by construction: exchange k uses parity
// k & 1 where k = this rank's produced-exchange count, and a peer's producer k + 2 (same
// parity) can only start after its consumer k + 1, which needs this rank's producer k + 1,
// which runs after this rank's consumer k. Every rank runs the same exchange sequence
// (the API's lockstep rule), whatever the graph (HYDRATE / LOGITS / GREEDY, yalm_block):
// no sequence number is derived from the forward's structure.
//
// Buffer per rank (yalm_tp_ipc_alloc, hipDeviceMallocUncached: never cached in a
// reader's L2, so a pushed value cannot be shadowed by a stale line), mapped on every
// rank: [2 parities][n ranks][S floats] slots, then control words: xdone[64] (exchanges
// produced by each source rank, toward this rank), ticket, error.
#pragma once

#include "device_common.h"

#define TPX_TIMEOUT 200000000ull // 2 s of s_memrealtime (100 MHz)
#define TPX_CTRL_WORDS 128       // xdone[64], ticket, error, padding

struct TpX {
	float *const *bufs; // [n] this rank's buffer and the peers' (IPC-mapped), device array
	int rank, n, S;     // this rank, ranks, floats per (parity, source) slot
	float *xw;          // consumer: where the summed x is written back (the decoder's x)
	__device__ __forceinline__ unsigned *ctrl(int p) const {
		return (unsigned *)(bufs[p] + 2 * (size_t)n * S);
	}
	__device__ __forceinline__ float *slot(int p, unsigned par, int src) const {
		return bufs[p] + ((size_t)(par & 1u) * n + src) * S;
	}
};

__device__ __forceinline__ unsigned tpx_ld(const unsigned *p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void tpx_st(float *p, float v) {
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float tpx_ldf(const float *p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Exchanges this rank has produced so far; a producer pushes into parity tpx_seq & 1.
__device__ __forceinline__ unsigned tpx_seq(const TpX &t) {
	return tpx_ld(t.ctrl(t.rank) + t.rank);
}

// Producer: element i of this rank's slot, on every rank (own first).
__device__ __forceinline__ void tpx_put(const TpX &t, unsigned par, int i, float v) {
	for (int k = 0; k < t.n; ++k) {
		const int p = t.rank + k < t.n ? t.rank + k : t.rank + k - t.n;
		tpx_st(t.slot(p, par, t.rank) + i, v);
	}
}

// Producer tail, called by every thread of each of the launch's `nprod` producer
// workgroups after its pushes: the stores are drained (their writes acknowledged), the
// workgroup takes a ticket; the last one resets the ticket and bumps xdone[rank] on
// every rank.
__device__ __forceinline__ void tpx_arrive(const TpX &t, int nprod) {
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if (threadIdx.x == 0) {
		unsigned *tk = t.ctrl(t.rank) + 64;
		const unsigned v = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
		if (v == (unsigned)nprod - 1u) {
			__hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); // every workgroup's pushes before the counts
			for (int k = 0; k < t.n; ++k) {
				const int p = t.rank + k < t.n ? t.rank + k : t.rank + k - t.n;
				__hip_atomic_fetch_add(t.ctrl(p) + t.rank, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			}
		}
	}
}

// Consumer: every wave waits (lane p polls rank p's count) until each rank has produced
// as many exchanges as this rank; returns the parity to read. A wait past TPX_TIMEOUT
// gives up (results wrong) and sets the error word, reported by the next sync call.
__device__ __forceinline__ unsigned tpx_wait(const TpX &t) {
	const unsigned *c = t.ctrl(t.rank);
	const unsigned want = tpx_ld(c + t.rank);
	const int lane = threadIdx.x & 63;
	const unsigned *mine = c + (lane < t.n ? lane : t.rank);
	const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + TPX_TIMEOUT;
	for (;;) {
		if (__all((int)(tpx_ld(mine) - want) >= 0))
			break;
		__builtin_amdgcn_s_sleep(1);
		if (__builtin_amdgcn_s_memrealtime() > deadline) {
			if (lane == 0)
				__hip_atomic_store((unsigned *)c + 65, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			break;
		}
	}
	return (want - 1u) & 1u;
}

// Consumer: the summed x (rank order) of parity par into LDS xs[0, n), optionally
// rmsnorm'ed (infer.cpp:134-144, the statement order of stage_x), and workgroup 0 writes
// the raw sum back to t.xw. Four floats per thread per pass; every rank's loads issued
// before the adds.
template <bool NORM, int NMAX = 8>
__device__ __forceinline__ void tpx_stage_x(float *xs, const TpX &t, unsigned par, const float *__restrict__ normw,
                                            int n, float eps) {
	const int tid = threadIdx.x, nthreads = blockDim.x;
	// the own buffer through a buffer resource: 16-byte sc0 sc1 (system-scope) loads the
	// compiler tracks (cachepolicy 0x11), instead of four 4-byte atomic loads each
	const uint64_t ba = (uint64_t)t.bufs[t.rank];
	const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)ba), hi = __builtin_amdgcn_readfirstlane((uint32_t)(ba >> 32));
	const __amdgpu_buffer_rsrc_t own = __builtin_amdgcn_make_buffer_rsrc(
	    (void *)(((uint64_t)hi << 32) | lo), (short)0, (int)(2u * (uint32_t)t.n * (uint32_t)t.S * 4u), 0x00020000);
	const uint32_t base = ((par & 1u) * (uint32_t)t.n) * (uint32_t)t.S * 4u, rstride = (uint32_t)t.S * 4u;
	float ss = 0.0f;
	for (int i = tid * 4; i < n; i += nthreads * 4) {
		float4_t v[NMAX];
#pragma unroll
		for (int r = 0; r < NMAX; ++r)
			if (r < t.n)
				v[r] = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(
				                                        own, base + (uint32_t)r * rstride + (uint32_t)i * 4u, 0, 0x11));
		float4_t a = v[0];
#pragma unroll
		for (int r = 1; r < NMAX; ++r)
			if (r < t.n)
				a += v[r];
		*(float4_t *)(xs + i) = a;
		if (blockIdx.x == 0)
			*(float4_t *)(t.xw + i) = a;
		if constexpr (NORM)
			ss = sumsq4(ss, a);
	}
	if constexpr (NORM) {
		float *red = xs + ((n + 3) & ~3);
		ss = wave_sum(ss);
		if ((tid & 63) == 0)
			red[tid >> 6] = ss;
		__syncthreads();
		float tot = 0.0f;
		for (int w = 0; w < nthreads / YALM_WAVE; ++w)
			tot += red[w];
		const float scale = 1.0f / sqrtf(tot / n + eps);
		for (int i = tid * 4; i < n; i += nthreads * 4) {
			float4_t v = *(const float4_t *)(xs + i);
			const float4_t w = *(const float4_t *)(normw + i);
			v[0] = v[0] * scale * w[0];
			v[1] = v[1] * scale * w[1];
			v[2] = v[2] * scale * w[2];
			v[3] = v[3] * scale * w[3];
			*(float4_t *)(xs + i) = v;
		}
	}
	__syncthreads();
}
