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
//     argmax, the logits GEMV of an OUTPUT forward): each row value is PUSHED to slot
//     [parity][this rank] of EVERY rank's buffer as an 8-byte {value, tag} granule, ONE
//     system-scope store each: the data is its own ready flag (the granule hand-off of
//     attn_wo.h, across processes) -- no drain, no counter, no last-arriver.
//   * CONSUMER (the next GEMV's x staging: GLU after Wo, next layer's QKV / the logits
//     after W2): loads the N slots' granules of its x, re-reading until every tag is this
//     exchange's, sums them in rank order -- bit-identical x on every rank -- while its
//     weight stream is already in flight, and (workgroup 0) writes x back for the next
//     residual.
// The exchange index g = StepState.xbase + ex: step_begin_kernel (and yalm_block's
// set_step_full_kernel, the timing hooks' bump) reserves this forward's exchanges
// [xbase, xbase + n_ex) and every launch knows its own ex statically (Wo of layer l:
// 2 l, W2: 2 l + 1, the logits / argmax: 2 L). Exchange g uses parity g & 1 and tag g + 1
// (zeroed memory never matches). Consecutive exchanges alternate parity, and a peer's
// producer g + 2 (the same parity) runs only after its consumer g + 1, which needs this
// rank's producer g + 1, which runs after this rank's consumer g: a slot is never
// rewritten while it is read. Every rank runs the same exchange sequence (the API's
// lockstep rule).
//
// Round 5 first cut (measured, TP1 on one MI355X, rocprofv3): per-rank exchange counters
// bumped by the producer launch's last workgroup (drain, ticket, fence, remote atomics)
// and a counter poll before the consumer's loads cost +4.2 us per W2, +5.2 per attention
// + Wo, +1.8 / +2.2 per GLU / QKV launch over one GPU -- three serialised round trips at
// every producer's tail. Granules leave one.
//
// Buffer per rank (yalm_tp_ipc_alloc, hipDeviceMallocUncached: never cached in a
// reader's L2, so a pushed granule cannot be shadowed by a stale line), mapped on every
// rank: [2 parities][n ranks][S granules], then control words (error).
#pragma once

#include "device_common.h"

#define TPX_TIMEOUT 200000000ull // 2 s of s_memrealtime (100 MHz)
#define TPX_CTRL_WORDS 64        // error word + padding (in floats)

struct TpX {
	float *const *bufs;     // [n] this rank's buffer and the peers' (IPC-mapped), device array
	int rank, n, S;         // this rank, ranks, granules per (parity, source) slot
	float *xw;              // consumer: where the summed x is written back (the decoder's x)
	const StepState *step;  // xbase: this forward's first exchange index
	int ex;                 // this launch's exchange within the forward
	__device__ __forceinline__ unsigned long long *slot(int p, unsigned par, int src) const {
		return (unsigned long long *)bufs[p] + ((size_t)(par & 1u) * n + src) * S;
	}
	__device__ __forceinline__ unsigned *err() const {
		return (unsigned *)((unsigned long long *)bufs[rank] + 2 * (size_t)n * S);
	}
	// this launch's exchange index (one load of the step state, a kernel-start read)
	__device__ __forceinline__ unsigned g() const { return step->xbase + (unsigned)ex; }
};

// Producer: element i of this rank's slot of exchange g, on every rank (own first).
__device__ __forceinline__ void tpx_put(const TpX &t, unsigned g, int i, float v) {
	const unsigned long long gr = (unsigned long long)__float_as_uint(v) | ((unsigned long long)(g + 1u) << 32);
	for (int k = 0; k < t.n; ++k) {
		const int p = t.rank + k < t.n ? t.rank + k : t.rank + k - t.n;
		__hip_atomic_store(t.slot(p, g, t.rank) + i, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	}
}

// Consumer: one granule of source rank src (element i) of exchange g, waited for (bounded;
// a wait that gives up sets the error word, reported by the next sync call).
__device__ __forceinline__ float tpx_get1(const TpX &t, unsigned g, int src, int i, unsigned long long deadline) {
	const unsigned long long *s = t.slot(t.rank, g, src) + i;
	for (;;) {
		const unsigned long long v = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		if ((unsigned)(v >> 32) == g + 1u)
			return __uint_as_float((unsigned)v);
		if (__builtin_amdgcn_s_memrealtime() > deadline) {
			__hip_atomic_store(t.err(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			return __uint_as_float((unsigned)v);
		}
		__builtin_amdgcn_s_sleep(1);
	}
}

// Consumer: the summed x (rank order) of exchange g into LDS xs[0, n), optionally
// rmsnorm'ed (infer.cpp:134-144, the statement order of stage_x), and workgroup 0 writes
// the raw sum back to t.xw. Per pass a thread loads 4 elements of every rank (2 x 16-byte
// sc0 sc1 loads of 2 granules each, through a buffer resource so the compiler tracks
// them), all issued before any check; a pass re-reads until every tag in the wave is g + 1.
template <bool NORM, int NMAX = 8>
__device__ __forceinline__ void tpx_stage_x(float *xs, const TpX &t, unsigned g, const float *__restrict__ normw,
                                            int n, float eps) {
	const int tid = threadIdx.x, nthreads = blockDim.x;
	const uint64_t ba = (uint64_t)t.bufs[t.rank];
	const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)ba), hi = __builtin_amdgcn_readfirstlane((uint32_t)(ba >> 32));
	const __amdgpu_buffer_rsrc_t own = __builtin_amdgcn_make_buffer_rsrc(
	    (void *)(((uint64_t)hi << 32) | lo), (short)0, (int)(2u * (uint32_t)t.n * (uint32_t)t.S * 8u), 0x00020000);
	const uint32_t base = ((g & 1u) * (uint32_t)t.n) * (uint32_t)t.S * 8u, rstride = (uint32_t)t.S * 8u;
	const unsigned tag = g + 1u;
	const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + TPX_TIMEOUT;
	float ss = 0.0f;
	for (int i = tid * 4; i < n; i += nthreads * 4) {
		u32x4_t v[NMAX][2];
		for (;;) {
#pragma unroll
			for (int r = 0; r < NMAX; ++r)
				if (r < t.n) {
					const uint32_t o = base + (uint32_t)r * rstride + (uint32_t)i * 8u;
					v[r][0] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(own, o, 0, 0x11));
					v[r][1] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(own, o + 16u, 0, 0x11));
				}
			bool ok = true;
#pragma unroll
			for (int r = 0; r < NMAX; ++r)
				if (r < t.n)
					ok = ok && v[r][0][1] == tag && v[r][0][3] == tag && v[r][1][1] == tag && v[r][1][3] == tag;
			if (__all(ok))
				break;
			if (__builtin_amdgcn_s_memrealtime() > deadline) {
				if ((tid & 63) == 0)
					__hip_atomic_store(t.err(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
				break;
			}
			__builtin_amdgcn_s_sleep(1);
		}
		float4_t a;
		{
			const uint32_t e0 = v[0][0][0], e1 = v[0][0][2], e2 = v[0][1][0], e3 = v[0][1][2];
			a = float4_t{__uint_as_float(e0), __uint_as_float(e1), __uint_as_float(e2), __uint_as_float(e3)};
		}
#pragma unroll
		for (int r = 1; r < NMAX; ++r)
			if (r < t.n) {
				const uint32_t e0 = v[r][0][0], e1 = v[r][0][2], e2 = v[r][1][0], e3 = v[r][1][2];
				a += float4_t{__uint_as_float(e0), __uint_as_float(e1), __uint_as_float(e2), __uint_as_float(e3)};
			}
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
