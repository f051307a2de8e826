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
// Consumer staging reads N x 32 KB of granules per workgroup (x of 4096): past this many ranks
// a collect launch of TPX_COLLECT_WG workgroups sums x once instead (the collect form).
// tools/tpx_stage_bench.hip, MI355X, 256 x 512-thread workgroups + a 29 MB weight stream (a
// TP8 W1|W3): staging in the consumer 11.1 / 11.4 / 12.6 / 15.2 us at N = 1 / 2 / 4 / 8,
// collect (32 workgroups) + plain staging 11.6 / 11.9 / 12.3 / 13.2, one GPU's plain 9.5.
#define TPX_STAGE_MAX_RANKS 4
#define TPX_COLLECT_WG 32

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

// A consumer's wait gives up at its deadline (2 s: the error word is set and reported by the
// next sync call), or, after 10 us, as soon as an earlier wait of this rank has given up:
// the results are invalid and reported already, and a forward of 2 L + 1 exchanges must not
// spend 2 s on each of them (a failed transport on real xGMI then costs one timeout, not
// minutes, and bench.py's other transport is still measured).
__device__ __forceinline__ bool tpx_give_up(const TpX &t, unsigned long long deadline) {
	const unsigned long long now = __builtin_amdgcn_s_memrealtime();
	if (now > deadline) {
		__hip_atomic_store(t.err(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		return true;
	}
	return now + TPX_TIMEOUT > deadline + 1000ull &&
	       __hip_atomic_load(t.err(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}

// Consumer: one granule of source rank src (element i) of exchange g, waited for (bounded,
// tpx_give_up).
__device__ __forceinline__ float tpx_get1(const TpX &t, unsigned g, int src, int i, unsigned long long deadline) {
	const unsigned long long *s = t.slot(t.rank, g, src) + i;
	for (;;) {
		const unsigned long long v = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		if ((unsigned)(v >> 32) == g + 1u || tpx_give_up(t, deadline))
			return __uint_as_float((unsigned)v);
		__builtin_amdgcn_s_sleep(1);
	}
}

// Consumer view of exchange g in this rank's own buffer: a buffer resource over both
// parities (a granule past the end reads as 0: tag 0 never matches), the parity's base.
struct TpxView {
	__amdgpu_buffer_rsrc_t own;
	uint32_t base, rstride; // byte offset of slot [g & 1][0], bytes per source slot
	unsigned tag;           // g + 1
};

__device__ __forceinline__ TpxView tpx_view(const TpX &t, unsigned g) {
	TpxView w;
	const uint64_t ba = (uint64_t)t.bufs[t.rank];
	const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)ba), hi = __builtin_amdgcn_readfirstlane((uint32_t)(ba >> 32));
	w.own = __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0,
	                                          (int)(2u * (uint32_t)t.n * (uint32_t)t.S * 8u), 0x00020000);
	w.base = ((g & 1u) * (uint32_t)t.n) * (uint32_t)t.S * 8u;
	w.rstride = (uint32_t)t.S * 8u;
	w.tag = g + 1u;
	return w;
}

// Elements [i, i + 4) of every source rank < nr: 2 x 16-byte sc0 sc1 loads (2 granules each)
// per rank, all issued before any is used. Lanes with i >= n load nothing useful (an
// out-of-range offset reads zeros) and are ignored by the check.
template <int NMAX>
__device__ __forceinline__ void tpx_load_pass(u32x4_t (&v)[NMAX][2], const TpxView &w, int nr, int i, int n) {
#pragma unroll
	for (int r = 0; r < NMAX; ++r)
		if (r < nr) {
			const uint32_t o = i < n ? w.base + (uint32_t)r * w.rstride + (uint32_t)i * 8u : 0x80000000u;
			v[r][0] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(w.own, o, 0, 0x11));
			v[r][1] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(w.own, o + 16u, 0, 0x11));
		}
}

// Re-reads the pass until every tag in the wave is this exchange's (bounded: a give-up sets
// the error word), then sums the ranks in rank order.
template <int NMAX>
__device__ __forceinline__ float4_t tpx_sum_pass(u32x4_t (&v)[NMAX][2], const TpxView &w, const TpX &t, int i, int n,
                                                 unsigned long long deadline) {
	for (;;) {
		bool ok = true;
#pragma unroll
		for (int r = 0; r < NMAX; ++r)
			if (r < t.n)
				ok = ok && v[r][0][1] == w.tag && v[r][0][3] == w.tag && v[r][1][1] == w.tag && v[r][1][3] == w.tag;
		if (__all(ok || i >= n))
			break;
		if (__any(tpx_give_up(t, deadline))) // (wave-uniform exit)
			break;
		__builtin_amdgcn_s_sleep(1);
		tpx_load_pass<NMAX>(v, w, t.n, i, n);
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
	return a;
}

// The first PPRE passes of a consumer's x staging, loaded ahead of its weight stream (vmcnt
// completes in order: granule loads issued behind the weight loads wait for them, and a
// pass-by-pass loop serialised one uncached round trip per pass -- measured +1.8 / +2.0 us
// per GLU / QKV launch at TP1). 8 VGPRs per rank slot (TPX_NMAX) and pass, plus the norm weights' 4 per pass.
constexpr int TPX_NMAX = TPX_STAGE_MAX_RANKS;
template <int PPRE>
struct TpxPre {
	u32x4_t v[PPRE][TPX_NMAX][2];
	float4_t nw[PPRE];
};

template <bool NORM, int THREADS, int PPRE>
__device__ __forceinline__ void tpx_prefetch(TpxPre<PPRE> &pre, const TpxView &w, const TpX &t,
                                             const float *__restrict__ normw, int n) {
#pragma unroll
	for (int p = 0; p < PPRE; ++p)
		if (p * THREADS * 4 < n) {
			const int i = (p * THREADS + (int)threadIdx.x) * 4;
			tpx_load_pass<TPX_NMAX>(pre.v[p], w, t.n, i, n);
			if constexpr (NORM)
				pre.nw[p] = *(const float4_t *)(normw + (i < n ? i : n - 4));
		}
}

// Consumer: the summed x (rank order) of the exchange into LDS xs[0, n), optionally
// rmsnorm'ed (infer.cu:526 / infer.cpp:134-144, the statement order of stage_x), and
// workgroup 0 writes the raw sum back to t.xw. Passes past PPRE load here.
template <bool NORM, int THREADS, int PPRE>
__device__ __forceinline__ void tpx_stage_x(float *xs, const TpX &t, const TpxView &w, TpxPre<PPRE> &pre,
                                            const float *__restrict__ normw, int n, float eps) {
	const int tid = threadIdx.x;
	const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + TPX_TIMEOUT;
	float ss = 0.0f;
	auto put = [&](int i, const float4_t &a) {
		if (i < n) {
			*(float4_t *)(xs + i) = a;
			if (blockIdx.x == 0)
				*(float4_t *)(t.xw + i) = a;
			if constexpr (NORM)
				ss = sumsq4(ss, a);
		}
	};
#pragma unroll
	for (int p = 0; p < PPRE; ++p)
		if (p * THREADS * 4 < n) {
			const int i = (p * THREADS + tid) * 4;
			put(i, tpx_sum_pass<TPX_NMAX>(pre.v[p], w, t, i, n, deadline));
		}
	for (int i0 = PPRE * THREADS * 4; i0 < n; i0 += THREADS * 4) {
		const int i = i0 + tid * 4;
		u32x4_t v[TPX_NMAX][2];
		tpx_load_pass<TPX_NMAX>(v, w, t.n, i, n);
		put(i, tpx_sum_pass<TPX_NMAX>(v, w, t, i, n, deadline));
	}
	if constexpr (NORM) {
		float *red = xs + ((n + 3) & ~3);
		ss = wave_sum(ss);
		if ((tid & 63) == 0)
			red[tid >> 6] = ss;
		__syncthreads();
		float tot = 0.0f;
		for (int wv = 0; wv < THREADS / YALM_WAVE; ++wv)
			tot += red[wv];
		const float scale = 1.0f / sqrtf(tot / n + eps);
		auto norm = [&](int i, const float4_t &nw) {
			float4_t v = *(const float4_t *)(xs + i);
			v[0] = v[0] * scale * nw[0];
			v[1] = v[1] * scale * nw[1];
			v[2] = v[2] * scale * nw[2];
			v[3] = v[3] * scale * nw[3];
			*(float4_t *)(xs + i) = v;
		};
#pragma unroll
		for (int p = 0; p < PPRE; ++p) {
			const int i = (p * THREADS + tid) * 4;
			if (i < n)
				norm(i, pre.nw[p]);
		}
		for (int i = (PPRE * THREADS + tid) * 4; i < n; i += THREADS * 4)
			norm(i, *(const float4_t *)(normw + i));
	}
	__syncthreads();
}
