// gemv.h — weight-streaming GEMV for batch-1 decode on gfx950.
//
// Replaces the reference's warp-per-row GEMVs (infer.cu:216-336, 598-620):
//   * one wave64 owns a group of R weight rows and streams them with 16-byte
//     non-temporal loads (U chunks of 64 lanes x 16 B in flight per row),
//   * the activation vector is staged once per workgroup in LDS as fp32 —
//     optionally rmsnorm'ed on the way in (fusing infer.cu:526-539 into the
//     consumer, removing the 1-workgroup norm launch),
//   * wave64 xor-butterfly reduction, then a per-use epilogue policy:
//       PStore     out[row]  = acc                 (logits, test matmul, W2 in ffn test)
//       PResidual  out[row] += acc                 (Wo, W2: fused_matmul_add_residuals)
//       PQKV       clip + RoPE + fp16 KV-cache write, pairs of rows (fused_qkv_matmul_clip
//                  + fused_rope_and_cache_update + rotate_sink_tokens)
//       PGlu       act(W1 row) * (W3 row)          (fused_ffn_w1_w3_glu_act)
// Accumulation is fp32 (weights widened exactly: f16 -> f32, E5M2 -> f16 -> f32).
#pragma once

#include <type_traits>

#include "device_common.h"
#include "tp_exchange.h"

#define GEMV_THREADS 256

#ifdef YALM_WG_TRACE
__device__ unsigned long long *yalm_wg_trace;
#endif

template <class WT, int R_>
struct PStore {
	static constexpr int R = R_;
	const char *W;
	int n;
	float *out;
	int n_groups;
	__device__ __forceinline__ void prologue() const {}
	__device__ __forceinline__ const char *row(int g, int r) const {
		return W + (size_t)(g * R + r) * n * WT::BYTES;
	}
	__device__ __forceinline__ void finish(int g, const float *acc, int lane) const {
		if (lane < R)
			out[g * R + lane] = acc[lane];
	}
	__device__ __forceinline__ void finish_all(int g, const float *acc) const {
#pragma unroll
		for (int r = 0; r < R; ++r)
			out[g * R + r] = acc[r];
	}
};

template <class WT, int R_>
struct PResidual {
	static constexpr int R = R_;
	const char *W;
	int n;
	float *out;
	int n_groups;
	__device__ __forceinline__ void prologue() const {}
	__device__ __forceinline__ const char *row(int g, int r) const {
		return W + (size_t)(g * R + r) * n * WT::BYTES;
	}
	__device__ __forceinline__ void finish(int g, const float *acc, int lane) const {
		if (lane < R)
			out[g * R + lane] += acc[lane];
	}
	__device__ __forceinline__ void finish_all(int g, const float *acc) const {
#pragma unroll
		for (int r = 0; r < R; ++r)
			out[g * R + r] += acc[r];
	}
	// the residual rows, read before the weight stream (gemv_rb_kernel): the epilogue's
	// read-modify-write then costs no load round trip at the tail
	static constexpr bool PRE = true;
	__device__ __forceinline__ float pre(int g, int r) const { return out[g * R + r]; }
	__device__ __forceinline__ void finish_pre(int g, const float *acc, const float *xr) const {
#pragma unroll
		for (int r = 0; r < R; ++r)
			out[g * R + r] = xr[r] + acc[r];
	}
};

// policies with a pre(g, r) / finish_pre epilogue (PRE = true)
template <class P, class = void>
struct gemv_early : std::false_type {};
template <class P>
struct gemv_early<P, std::void_t<decltype(P::EARLY)>> : std::bool_constant<P::EARLY> {};

struct NoEarly {};
template <class P, bool = gemv_early<P>::value>
struct early_of {
	using type = NoEarly;
};
template <class P>
struct early_of<P, true> {
	using type = typename P::Early;
};

template <class P, class = void>
struct gemv_pre : std::false_type {};
template <class P>
struct gemv_pre<P, std::void_t<decltype(P::PRE)>> : std::bool_constant<P::PRE> {};

// out[row] = base[row] + acc: the tensor-parallel Wo / W2 partial of rank 0,
// which also carries the residual into the all-reduce (other ranks: PStore).
template <class WT, int R_>
struct PAddTo {
	static constexpr int R = R_;
	const char *W;
	int n;
	float *out;
	const float *base;
	int n_groups;
	__device__ __forceinline__ void prologue() const {}
	__device__ __forceinline__ const char *row(int g, int r) const {
		return W + (size_t)(g * R + r) * n * WT::BYTES;
	}
	__device__ __forceinline__ void finish(int g, const float *acc, int lane) const {
		if (lane < R)
			out[g * R + lane] = base[g * R + lane] + acc[lane];
	}
	__device__ __forceinline__ void finish_all(int g, const float *acc) const {
#pragma unroll
		for (int r = 0; r < R; ++r)
			out[g * R + r] = base[g * R + r] + acc[r];
	}
};

// IPC tensor-parallel producer (tp_exchange.h): row value (+ the residual base on rank 0)
// pushed into this rank's slot of every rank's exchange buffer, at element offset + row, as
// {value, tag} granules: no tail, no counter (the granule is its own ready flag).
template <class WT, int R_>
struct PPush {
	static constexpr int R = R_;
	const char *W;
	int n;
	const float *base; // residual (rank 0's x) or null
	TpX t;
	int offset;
	int n_groups;
	mutable unsigned xg = 0; // this launch's exchange index (read in prologue, ahead of the stream's end)
	__device__ __forceinline__ void prologue() const { xg = t.g(); }
	__device__ __forceinline__ const char *row(int g, int r) const {
		return W + (size_t)(g * R + r) * n * WT::BYTES;
	}
	static constexpr bool PRE = true;
	__device__ __forceinline__ float pre(int g, int r) const { return base ? base[g * R + r] : 0.0f; }
	__device__ __forceinline__ void finish_pre(int g, const float *acc, const float *xr) const {
#pragma unroll
		for (int r = 0; r < R; ++r)
			tpx_put(t, xg, offset + g * R + r, xr[r] + acc[r]);
	}
	__device__ __forceinline__ void finish_all(int g, const float *acc) const {
#pragma unroll
		for (int r = 0; r < R; ++r)
			tpx_put(t, xg, offset + g * R + r, (base ? base[g * R + r] : 0.0f) + acc[r]);
	}
	__device__ __forceinline__ void finish(int g, const float *acc, int lane) const { // gemv_kernel
		if (lane < R)
			tpx_put(t, xg, offset + g * R + lane, (base ? base[g * R + lane] : 0.0f) + acc[lane]);
	}
};

// Virtual row space [wq | wk | wv]; a wave owns the RoPE pair (2g, 2g+1).
template <class WT>
struct PQKV {
	static constexpr int R = 2;
	const char *wq, *wk, *wv;
	int n, q_dim, kv_dim, head_dim, n_groups;
	float qkv_clip;
	const float *inv_freq; // (head_dim/2) 1/theta^(2j/rotary_dim), 0 past rotary_dim
	const StepState *step;
	float *q_out;
	uint16_t *kcache, *vcache;
	// the attention sinks' one-position rotation (infer.cpp:303-317, infer.cu:679-697), spread over
	// the launch: each thread of every workgroup loads its pair of rows < KV_SINKS BEFORE the weight
	// stream (early, unconditionally: step->kv_sink is not known yet) and rotates it after the stream
	// (late), so no wave waits on a dependent round trip; rows < kv_sink never alias the kv_pos
	// row the epilogue writes (kv_pos >= kv_sink)
	static constexpr bool EARLY = true;
	static constexpr int KV_SINKS = 2; // model.h:12
	struct Early {
		uint32_t kv; // the pair (fp16 x 2) of pair index pi below
		int pi;
	};
	__device__ __forceinline__ Early early() const {
		Early e;
		e.pi = (int)(threadIdx.x * gridDim.x + blockIdx.x);
		const int half = kv_dim >> 1;
		e.kv = e.pi < KV_SINKS * half ? *(const uint32_t *)(kcache + (size_t)(e.pi / half) * kv_dim + 2 * (e.pi % half))
		                              : 0u;
		return e;
	}
	__device__ __forceinline__ void rotate_pair(int pi, uint32_t kv) const {
		const int half = kv_dim >> 1;
		const int r = pi / half, i = 2 * (pi % half);
		float v0 = h2f((uint16_t)(kv & 0xFFFF)), v1 = h2f((uint16_t)(kv >> 16));
		const int j = (i % head_dim) >> 1;
		float fcr = step->rope_sink[2 * j], fci = step->rope_sink[2 * j + 1];
		const uint32_t o0 = f2h(v0 * fcr - v1 * fci), o1 = f2h(v0 * fci + v1 * fcr);
		*(uint32_t *)(kcache + (size_t)r * kv_dim + i) = o0 | (o1 << 16);
	}
	__device__ __forceinline__ void late(const Early &e) const {
		const int half = kv_dim >> 1, npairs = step->kv_sink * half;
		const int stride = (int)(blockDim.x * gridDim.x);
		for (int pi = e.pi; pi < npairs; pi += stride) { // past KV_SINKS rows (not in the reference's schedule): loaded here
			const uint32_t kv = pi == e.pi && pi < KV_SINKS * half
			                        ? e.kv
			                        : *(const uint32_t *)(kcache + (size_t)(pi / half) * kv_dim + 2 * (pi % half));
			rotate_pair(pi, kv);
		}
	}
	__device__ __forceinline__ void prologue() const { late(early()); } // gemv_kernel
	__device__ __forceinline__ const char *row(int g, int r) const {
		int vr = 2 * g + r;
		if (vr < q_dim)
			return wq + (size_t)vr * n * WT::BYTES;
		vr -= q_dim;
		if (vr < kv_dim)
			return wk + (size_t)vr * n * WT::BYTES;
		vr -= kv_dim;
		return wv + (size_t)vr * n * WT::BYTES;
	}
	__device__ __forceinline__ void finish(int g, const float *acc, int lane) const {
		if (lane != 0)
			return;
		// infer.cpp:280-288 clip; infer.cpp:291-301 rope; infer.cu:642-677 cache write
		float v0 = acc[0] < -qkv_clip ? -qkv_clip : (acc[0] > qkv_clip ? qkv_clip : acc[0]);
		float v1 = acc[1] < -qkv_clip ? -qkv_clip : (acc[1] > qkv_clip ? qkv_clip : acc[1]);
		int vr = 2 * g;
		if (vr >= q_dim + kv_dim) { // V: no rotation
			size_t o = (size_t)step->kv_pos * kv_dim + (vr - q_dim - kv_dim);
			vcache[o] = f2h(v0);
			vcache[o + 1] = f2h(v1);
			return;
		}
		int i = vr < q_dim ? vr : vr - q_dim;
		const int j = (i % head_dim) >> 1; // cos / sin of pos * inv_freq[j]: the step kernel's table
		float fcr = step->rope[2 * j];
		float fci = step->rope[2 * j + 1];
		float r0 = v0 * fcr - v1 * fci;
		float r1 = v0 * fci + v1 * fcr;
		if (vr < q_dim) {
			q_out[i] = r0;
			q_out[i + 1] = r1;
		} else {
			size_t o = (size_t)step->kv_pos * kv_dim + i;
			kcache[o] = f2h(r0);
			kcache[o + 1] = f2h(r1);
		}
	}
	__device__ __forceinline__ void finish_all(int g, const float *acc) const { finish(g, acc, 0); }
};

template <class WT, int ACT>
struct PGlu {
	static constexpr int R = 2;
	const char *w1, *w3;
	int n;
	float *out;
	int n_groups;
	__device__ __forceinline__ void prologue() const {}
	__device__ __forceinline__ const char *row(int g, int r) const {
		return (r == 0 ? w1 : w3) + (size_t)g * n * WT::BYTES;
	}
	__device__ __forceinline__ void finish(int g, const float *acc, int lane) const {
		if (lane == 0)
			out[g] = act_fn<ACT>(acc[0]) * acc[1];
	}
	__device__ __forceinline__ void finish_all(int g, const float *acc) const { finish(g, acc, 0); }
};

// Stage x (n floats) into LDS, optionally as rmsnorm(x) * w (infer.cpp:134-144
// statement order: scale = 1/sqrt(sum/n + eps); o = x * scale * w).
template <bool NORM>
__device__ __forceinline__ void stage_x(float *xs, const float *__restrict__ x, const float *__restrict__ normw, int n,
                                        float eps) {
	const int tid = threadIdx.x;
	const int nthreads = blockDim.x;
	float scale = 1.0f;
	if constexpr (NORM) {
		float *red = xs + ((n + 3) & ~3); // scratch after x (one aligned LDS region, G17)
		float ss = 0.0f;
		for (int i = tid * 4; i < n; i += nthreads * 4) {
			float4_t v = *(const float4_t *)(x + i);
			ss = sumsq4(ss, v);
		}
		ss = wave_sum(ss);
		if ((tid & 63) == 0)
			red[tid >> 6] = ss;
		__syncthreads();
		float tot = 0.0f;
		for (int w = 0; w < nthreads / YALM_WAVE; ++w)
			tot += red[w];
		float rms = sqrtf(tot / n + eps);
		scale = 1.0f / rms;
	}
	for (int i = tid * 4; i < n; i += nthreads * 4) {
		float4_t v = *(const float4_t *)(x + i);
		if constexpr (NORM) {
			float4_t w = *(const float4_t *)(normw + i);
			v[0] = v[0] * scale * w[0];
			v[1] = v[1] * scale * w[1];
			v[2] = v[2] * scale * w[2];
			v[3] = v[3] * scale * w[3];
		}
		*(float4_t *)(xs + i) = v;
	}
	__syncthreads();
}

// x (and the norm weights) loaded into registers BEFORE the weight stream is
// issued, so the staging does not wait behind the weight loads (vmcnt is in
// order): xpre_n float4 per thread (2 with the norm weights, 4 without:
// n <= 4 * xpre_n * blockDim.x); finished by stage_x_regs.
// Without the norm at 512 threads: 7 float4 = n 14336 (W2's hb for Mistral; round 3: the fp8
// W2 at {512, 4, 1} staged its 57 KB x from global AFTER its first weight loads, so the first
// FMA waited for both round trips in vmcnt order).
template <bool NORM, int THREADS>
constexpr int xpre_n() {
	return NORM ? 2 : (THREADS == 512 ? 7 : 4);
}
template <bool NORM, int THREADS>
struct XPre {
	float4_t x[xpre_n<NORM, THREADS>()], w[NORM ? xpre_n<NORM, THREADS>() : 1];
};
template <bool NORM, int THREADS>
__device__ __forceinline__ void prefetch_x(XPre<NORM, THREADS> &r, const float *__restrict__ x,
                                           const float *__restrict__ normw, int n) {
	const int nthreads = blockDim.x;
#pragma unroll
	for (int k = 0; k < xpre_n<NORM, THREADS>(); ++k) {
		int i = (threadIdx.x + k * nthreads) * 4;
		i = i < n ? i : n - 4; // unconditional (clamped) loads: no branch for hipcc to wait at
		r.x[k] = *(const float4_t *)(x + i);
		if constexpr (NORM)
			r.w[k] = *(const float4_t *)(normw + i);
	}
}
// infer.cpp:134-144 statement order, as stage_x
template <bool NORM, int THREADS>
__device__ __forceinline__ void stage_x_regs(float *xs, const XPre<NORM, THREADS> &r, int n, float eps) {
	const int tid = threadIdx.x;
	const int nthreads = blockDim.x;
	float scale = 1.0f;
	if constexpr (NORM) {
		float *red = xs + ((n + 3) & ~3);
		float ss = 0.0f;
#pragma unroll
		for (int k = 0; k < xpre_n<NORM, THREADS>(); ++k) {
			if ((tid + k * nthreads) * 4 < n) {
				const float4_t v = r.x[k];
				ss = sumsq4(ss, v);
			}
		}
		ss = wave_sum(ss);
		if ((tid & 63) == 0)
			red[tid >> 6] = ss;
		__syncthreads();
		float tot = 0.0f;
		for (int w = 0; w < nthreads / YALM_WAVE; ++w)
			tot += red[w];
		float rms = sqrtf(tot / n + eps);
		scale = 1.0f / rms;
	}
#pragma unroll
	for (int k = 0; k < xpre_n<NORM, THREADS>(); ++k) {
		const int i = (tid + k * nthreads) * 4;
		if (i < n) {
			float4_t v = r.x[k];
			if constexpr (NORM) {
				const float4_t w = r.w[k];
				v[0] = v[0] * scale * w[0];
				v[1] = v[1] * scale * w[1];
				v[2] = v[2] * scale * w[2];
				v[3] = v[3] * scale * w[3];
			}
			*(float4_t *)(xs + i) = v;
		}
	}
	__syncthreads();
}

template <class WT, int R>
__device__ __forceinline__ void fma_chunk(float (&acc)[R], const u32x4_t (&w)[R], const float *xs_lane) {
	constexpr int EPL = WT::EPL;
	float xv[EPL];
#pragma unroll
	for (int e = 0; e < EPL; e += 4) {
		float4_t t = *(const float4_t *)(xs_lane + e);
		xv[e] = t[0];
		xv[e + 1] = t[1];
		xv[e + 2] = t[2];
		xv[e + 3] = t[3];
	}
#pragma unroll
	for (int r = 0; r < R; ++r) {
		float wf[EPL];
		WT::unpack(w[r], wf);
#pragma unroll
		for (int e = 0; e < EPL; ++e)
			acc[r] = fmaf(wf[e], xv[e], acc[r]);
	}
}

// n must be a multiple of WT::EPL (the reference asserts n % 16 == 0,
// infer.cpp:66) and of 4. Each wave processes `gpw` consecutive row groups.
template <class WT, class P, int U, bool NORM>
__global__ __launch_bounds__(GEMV_THREADS) void gemv_kernel(P p, const float *__restrict__ x,
                                                            const float *__restrict__ normw, float eps, int gpw) {
	extern __shared__ __attribute__((aligned(16))) float xs[];
	constexpr int R = P::R;
	constexpr int EPL = WT::EPL;
	constexpr int CH = YALM_WAVE * EPL; // elements per wave-wide chunk
	const int n = p.n;
	p.prologue();
	stage_x<NORM>(xs, x, normw, n, eps);

	const int lane = threadIdx.x & 63;
	const int wave = threadIdx.x >> 6;
	const int waves = blockDim.x >> 6;
	const int g0 = (blockIdx.x * waves + wave) * gpw;
	const int nfull = n / CH;
	const int rem = n - nfull * CH;

	for (int gi = 0; gi < gpw; ++gi) {
		const int g = g0 + gi;
		if (g >= p.n_groups)
			break;
		const char *rp[R];
#pragma unroll
		for (int r = 0; r < R; ++r)
			rp[r] = p.row(g, r) + (size_t)lane * EPL * WT::BYTES;
		float acc[R];
#pragma unroll
		for (int r = 0; r < R; ++r)
			acc[r] = 0.0f;

		int c = 0;
		for (; c + U <= nfull; c += U) {
			u32x4_t w[U][R];
#pragma unroll
			for (int u = 0; u < U; ++u)
#pragma unroll
				for (int r = 0; r < R; ++r)
					w[u][r] = load_nt16(rp[r] + (size_t)(c + u) * CH * WT::BYTES);
#pragma unroll
			for (int u = 0; u < U; ++u)
				fma_chunk<WT, R>(acc, w[u], xs + (c + u) * CH + lane * EPL);
		}
		for (; c < nfull; ++c) {
			u32x4_t w[R];
#pragma unroll
			for (int r = 0; r < R; ++r)
				w[r] = load_nt16(rp[r] + (size_t)c * CH * WT::BYTES);
			fma_chunk<WT, R>(acc, w, xs + c * CH + lane * EPL);
		}
		if (rem > 0 && lane * EPL < rem) {
			u32x4_t w[R];
#pragma unroll
			for (int r = 0; r < R; ++r)
				w[r] = load_nt16(rp[r] + (size_t)nfull * CH * WT::BYTES);
			fma_chunk<WT, R>(acc, w, xs + nfull * CH + lane * EPL);
		}
#pragma unroll
		for (int r = 0; r < R; ++r)
			acc[r] = wave_sum(acc[r]);
		p.finish(g, acc, lane);
	}
}

// Row-block GEMV — the production path (n % (64 * EPL) == 0).
//
// One workgroup per CU (gridDim.x = NB ~ CU count): row group g belongs to
// workgroup g % NB, so at every moment the chip streams ONE contiguous window
// of rows (giving each CU a contiguous slice instead puts every CU on the same
// HBM channels at once: tools/persist_bench.hip measured 3.2 vs 6.4 TB/s).
// Inside the workgroup the (virtual row, 1-KB chunk) items of its groups are
// dealt round-robin over the waves — balanced to one item whatever n is — and
// each wave streams its items with U loads in flight. The refill of slot u is
// issued unconditionally (past the end it re-reads a line of x, an L2 hit) so
// hipcc's vmcnt bookkeeping stays static: with a conditional refill it emits
// vmcnt(0) before every load and the pipeline collapses. x is staged (and
// rmsnorm'ed) once per CU instead of once per small workgroup (1792 x 32 KB
// of L2 reads for W1/W3 before). Row partials are wave-reduced (DPP), parked
// in LDS per (row, wave) and summed in wave order by one thread per group,
// which runs the policy epilogue (finish_all).
//
// ROWS (chosen by the launcher when every workgroup's virtual rows divide evenly over its
// waves: W1|W3, W2): whole rows are dealt round-robin instead, each wave streaming all
// chunks of its rows, so the wave reduction runs once per row instead of once per 1-KB
// chunk (W1|W3 at n 4096: 8 reductions per row -> 1; tools/pattern_bench.hip: the chunk
// order with its per-chunk work ran 10-25% below the streaming envelope, whole rows at it).
//
// TIN (tensor parallelism over IPC, tp_exchange.h): this launch is the consumer of exchange
// tin -- x is the rank-order sum of every rank's pushed partial. The granules of the first
// passes are loaded BEFORE the weight stream (as x is otherwise, XPre), waited for and summed
// after it is issued, so the exchange latency runs under the weight stream's start instead
// of in a launch of its own.
template <class WT, class P, int U, bool NORM, int THREADS, bool ROWS = false, bool TIN = false>
__global__ __launch_bounds__(THREADS) void gemv_rb_kernel(P p, const float *__restrict__ x,
                                                          const float *__restrict__ normw, float eps, TpX tin) {
	extern __shared__ __attribute__((aligned(16))) float xs[];
	constexpr int R = P::R;
	constexpr int EPL = WT::EPL;
	constexpr int CH = YALM_WAVE * EPL;
	constexpr size_t CHB = (size_t)CH * WT::BYTES;
	constexpr int W = THREADS / YALM_WAVE;
	const int n = p.n;
	const int nch = n / CH;
	const int NB = gridDim.x;
	const int b = blockIdx.x;
	const int lane = threadIdx.x & 63;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int ngl = b < p.n_groups ? (p.n_groups - 1 - b) / NB + 1 : 0; // groups of this workgroup
	const int items = ngl * R * nch;
	const int mine = ROWS ? (ngl * R > wave ? ((ngl * R - 1 - wave) / W + 1) * nch : 0) // rows wave, wave + W, ...
	                      : (items > wave ? (items - 1 - wave) / W + 1 : 0);            // items wave, wave + W, ...
	float *part = xs + ((n + 3) & ~3) + 64;                         // [ngl * R][W]
	const size_t lane_off = (size_t)lane * EPL * WT::BYTES;
	const char *dummy = (const char *)x + lane * 16;
#ifdef YALM_WG_TRACE
	const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif

	auto advance = [&](int &vr, int &c) {
		if constexpr (ROWS) {
			if (++c == nch) {
				c = 0;
				vr += W;
			}
		} else {
			c += W;
			while (c >= nch) {
				c -= nch;
				++vr;
			}
		}
	};
	auto iaddr = [&](int vr, int c) {
		const int gl = vr / R, r = vr - gl * R;
		return p.row(b + gl * NB, r) + (size_t)c * CHB + lane_off;
	};
	auto pslot = [&](int vr) { return vr * W + wave; }; // LDS partial slot of item row vr

	int ivr = ROWS ? wave : wave / nch, ic = ROWS ? 0 : wave - (wave / nch) * nch; // issue cursor
	const int vr0 = ivr, c0 = ic;
	const bool xregs = !TIN && n <= 4 * xpre_n<NORM, THREADS>() * THREADS; // x (+ norm weights) fit the registers
	XPre<NORM, THREADS> xp;
	// exchange passes loaded ahead (n <= 4 * TPRE * THREADS: 4096 at 512 or 1024 threads)
	constexpr int TPRE = TIN ? (THREADS >= 1024 ? 1 : 2) : 0;
	TpxPre<TPRE ? TPRE : 1> tpre;
	TpxView tview;
	if constexpr (TIN) {
		tview = tpx_view(tin, tin.g());
		tpx_prefetch<NORM, THREADS, TPRE>(tpre, tview, tin, normw, n); // ahead of the weight stream in vmcnt order
	} else if (xregs) {
		prefetch_x<NORM, THREADS>(xp, x, normw, n); // ahead of the weight stream in vmcnt order
	}
	float xr[R] = {}; // PRE policies: the epilogue's rows of group threadIdx.x (clamped, unconditional)
	if constexpr (gemv_pre<P>::value) {
		const int g0 = min(b + min((int)threadIdx.x, max(ngl - 1, 0)) * NB, p.n_groups - 1);
#pragma unroll
		for (int r = 0; r < R; ++r)
			xr[r] = p.pre(g0, r);
	}
	typename early_of<P>::type ek{}; // PQKV: the sink pairs, loaded ahead of the weight stream
	if constexpr (gemv_early<P>::value)
		ek = p.early();
	u32x4_t buf[U];
#pragma unroll
	for (int u = 0; u < U; ++u) {
		buf[u] = load_nt16(u < mine ? iaddr(ivr, ic) : dummy);
		advance(ivr, ic);
	}
	if constexpr (!gemv_early<P>::value)
		p.prologue();
	for (int i = threadIdx.x; i < ngl * R * W; i += THREADS)
		part[i] = 0.0f;
	if constexpr (TIN)
		tpx_stage_x<NORM, THREADS, TPRE>(xs, tin, tview, tpre, normw, n, eps);
	else if (xregs)
		stage_x_regs<NORM, THREADS>(xs, xp, n, eps);
	else
		stage_x<NORM>(xs, x, normw, n, eps);

	if (mine > 0) {
		int cvr = vr0, cc = c0, cur = vr0; // consume cursor, row being accumulated
		float acc[1] = {0.0f};
		for (int k = 0; k < mine; k += U) {
#pragma unroll
			for (int u = 0; u < U; ++u) {
				const int j = k + u;
				if (j < mine) {
					if (cvr != cur) {
						const float s = wave_sum(acc[0]);
						if (lane == 0)
							part[pslot(cur)] = s;
						acc[0] = 0.0f;
						cur = cvr;
					}
					const u32x4_t wv[1] = {buf[u]};
					fma_chunk<WT, 1>(acc, wv, xs + cc * CH + lane * EPL);
					advance(cvr, cc);
				}
				buf[u] = load_nt16(j + U < mine ? iaddr(ivr, ic) : dummy);
				advance(ivr, ic);
			}
		}
		const float s = wave_sum(acc[0]);
		if (lane == 0)
			part[pslot(cur)] = s;
	}
	if constexpr (gemv_early<P>::value) // after the stream: its loads (and step's) have long landed
		p.late(ek);
	__syncthreads();
	for (int gl = threadIdx.x; gl < ngl; gl += THREADS) {
		float a[R];
#pragma unroll
		for (int r = 0; r < R; ++r) {
			float t = 0.0f;
#pragma unroll
			for (int w = 0; w < W; ++w)
				t += part[(gl * R + r) * W + w];
			a[r] = t;
		}
		if constexpr (gemv_pre<P>::value) {
			if (gl == (int)threadIdx.x)
				p.finish_pre(b + gl * NB, a, xr);
			else
				p.finish_all(b + gl * NB, a);
		} else {
			p.finish_all(b + gl * NB, a);
		}
	}
#ifdef YALM_WG_TRACE // tools/wg_timeline.hip: per-workgroup start/end (s_memrealtime, 100 MHz)
	if (threadIdx.x == 0) {
		yalm_wg_trace[2 * b] = t_start;
		yalm_wg_trace[2 * b + 1] = __builtin_amdgcn_s_memrealtime();
	}
#endif
}

