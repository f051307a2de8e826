// prefill.h — batched prefill / perplexity path on the matrix cores (MFMA).
//
// The reference has no batched prefill: `-m perplexity` (main.cpp:128-200)
// and prompt hydration run the single-token forward once per position. Here
// the T positions of a prompt go through each layer together, so every weight
// matrix is read once per prompt instead of once per token and the work is
// dense GEMMs on the gfx950 MFMA units:
//   X[T, dim] f32 residual stream (infer.cpp:443-523 semantics per row)
//   Xn = f16(rmsnorm(X) * w)                         (A operand of the GEMMs)
//   [Q | K | V] = Xn · [Wq | Wk | Wv]^T   + clip + RoPE; K, V -> the fp16 cache
//   O = causal GQA attention(Q, Kcache, Vcache)      (flash-style, MFMA)
//   X += O · Wo^T
//   H = f16(silu(Xn · W1^T) * (Xn · W3^T))           (one GEMM, two B operands)
//   X += H · W2^T
//   logits = f16(rmsnorm(X)) · Wcls^T -> per-row (max, sum exp, target logit)
// Weights stay in the .yalm layout ([out][in] f16, row-major): C = A · W^T is
// an "NT" GEMM whose two operands are both K-contiguous, so every MFMA operand
// fragment is a 16-byte row read (no transposes); the GEMMs are in
// prefill_gemm.h. Accumulation is f32; the activations are rounded to f16 for
// the MFMA inputs, except the K / V columns of the QKV GEMM, whose A operand is
// the normalised x split as f16 hi + lo (round 4: the K / V cache rows then carry
// one f16 rounding, as infer.cpp:299's, not two).
#pragma once

#include <float.h>

#include "device_common.h"

typedef float f32x16_t __attribute__((ext_vector_type(16)));
#define YALM_LDS __attribute__((address_space(3)))

namespace pf {

constexpr int BN = 128, BK = 64; // prefill dims must be multiples of BN (and of BK for K)
constexpr int THREADS = 256;      // attention prefill: 4 waves x 32 queries

__device__ __forceinline__ uint16_t f2h_bits(float x) {
	_Float16 h = (_Float16)x;
	uint16_t u;
	__builtin_memcpy(&u, &h, 2);
	return u;
}

// Range guard of the f16 MFMA operands: the reference keeps every
// activation in f32 (infer.cpp:360-375), the prefill rounds them to f16, which is inf past
// 65504. A lane whose largest |stored value| reaches that (or is NaN) records its largest
// |unscaled value| in `slot` (float bits; atomicMax orders non-negative floats, NaN above
// inf). No atomics while everything fits; the host reads the slots after the pass
// (prefill.hip run_prefill): the GLU output gets an exact power-of-two scale and the pass
// runs again, any other operand out of range is YALM_ERR_UNSUPPORTED.
__device__ __forceinline__ void range_note(unsigned *slot, float stored_absmax, float raw_absmax) {
	if (slot && !(stored_absmax < 65504.0f))
		atomicMax(slot, __float_as_uint(raw_absmax));
}

// C/D map of v_mfma_f32_32x32x16: column = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
__device__ __forceinline__ int crow(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

// B operand rows n = 0..N-1 drawn from up to 3 row-major [rows][K] matrices
// laid end to end (wq | wk | wv). Every 128-row tile lies inside one segment.
struct BSrc {
	const uint16_t *p[3];
	int end[3]; // exclusive row end of each segment (cumulative)
	__device__ __forceinline__ void tile(int col0, const uint16_t *&base, int &r0, int &rows) const {
		int s = col0 < end[0] ? 0 : (col0 < end[1] ? 1 : 2);
		const int start = s == 0 ? 0 : end[s - 1];
		base = p[s];
		r0 = col0 - start;
		rows = end[s] - start;
	}
};

__device__ __forceinline__ void raw_barrier() {
	asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------- attention
// Causal GQA attention for the prompt rows (flash-style, online softmax),
// infer.cpp:216-248 per (position, head): s_t = q·k_t / sqrt(D) over keys
// t <= pos, softmax, o = sum_t p_t v_t. Keys/values come from the fp16 cache
// rows 0 .. pos0 + T - 1 (written by the QKV epilogue). Grid (query blocks of
// 128, q heads), 4 waves x 32 queries. Per 64-key tile:
//   S = Q K^T   (A = Q fragments kept in registers, B = K rows from LDS)
//   online softmax in the C layout (key on the lane: row reductions are
//   DPP/permlane over 32 lanes, rows = registers)
//   O += P V    (P via a per-wave LDS transpose; V staged transposed in LDS so
//   its B fragments are row reads)
constexpr int AQ = 128, AKT = 64; // queries per workgroup, keys per tile

// Dynamic LDS of attn_prefill_kernel<D, KT>: K[2][KT][D], V[2][KT][D] (f16).
template <int D, int KT = AKT>
constexpr size_t attn_prefill_lds() {
	return (size_t)(4 * KT * D) * 2;
}

// Stage one 64-key tile of K or V (rows key0.., kv head g) by LDS-DMA. Row r of
// the lane-linear image holds source chunk c ^ sw(r): sw = r % (D/8) for K
// (row reads of 16 B, conflict-spread over 16 rows) and (r & 3) << 1 for V
// (ds_read_b64_tr_b16 reads 4 rows x 32 B: the 4 rows land on distinct banks).
template <int D, bool ISV, int KT = AKT>
__device__ __forceinline__ void stage_kv(uint16_t *dst, const uint16_t *__restrict__ src, int key0, int kv_rows,
                                         int kv_dim, int g, int wave, int lane) {
	constexpr int DCH = D / 8;
	constexpr int RPI = 1024 / (D * 2); // rows per 1-KB wave-instruction
	constexpr int NI = KT / RPI / 4;    // instructions per wave
#pragma unroll
	for (int i = 0; i < NI; ++i) {
		const int rb = wave * NI + i;
		const int r = rb * RPI + lane / DCH;
		const int c = lane % DCH;
		const int sw = ISV ? ((r & 3) << 1) : (r % DCH);
		const uint16_t *p = src + (size_t)min(key0 + r, kv_rows - 1) * kv_dim + g * D + 8 * (c ^ sw);
		__builtin_amdgcn_global_load_lds((const void *)p, (YALM_LDS void *)(dst + rb * RPI * D), 16, 0, 0);
	}
}

typedef short short4_t __attribute__((ext_vector_type(4)));

// "Swapped" formulation (cdna_hip_programming.md §3, accumulator as the next
// operand; Appendix B fused attention): S^T = K Q^T puts the query on the
// lane and 32 of the tile's 64 keys in registers, so the softmax row max / sum
// are register folds plus one permlane32 swap (no per-key cross-lane
// reductions, no LDS transpose of P), and O^T += V^T P^T takes P^T straight
// from the S^T accumulators (k order permuted: element e of lane half h is key
// 16 s + 8 (e >> 2) + 4 h + (e & 3) of the 32-key block) with V^T fragments
// from hardware-transposed LDS reads. O^T keeps the query on the lane too, so
// the online-softmax rescale is one per-lane factor.
//
// SPLIT (the split-operand precision form, yalm_set_prefill_precision): Q rows are [hi | lo]
// (2 q_dim wide), S^T = K hi^T + K lo^T; P^T is split too (P = hi + lo, both f16) so
// O^T += V^T hi^T + V^T lo^T; O is stored as [hi | lo] rows (2 q_dim wide) for the Wo
// GEMM's split A operand: the f16 roundings of q, P and o are gone, the
// matrix work doubles.
template <int D, int KT = AKT, bool SPLIT = false>
__global__ __launch_bounds__(THREADS) void attn_prefill_kernel(const uint16_t *__restrict__ Q,
                                                               const uint16_t *__restrict__ kc,
                                                               const uint16_t *__restrict__ vc, int T, int pos0,
                                                               int n_heads, int n_kv, uint16_t *__restrict__ O) {
	static_assert(D == 64 || D == 128, "head_dim");
	static_assert(KT == 32 || KT == 64, "keys per tile");
	constexpr int NJ = KT / 32; // 32-key blocks per tile
	constexpr int DCH = D / 8;
	extern __shared__ __attribute__((aligned(16))) uint16_t asmem[];
	uint16_t *const Kb = asmem;               // [2][KT * D]
	uint16_t *const Vb = asmem + 2 * KT * D; // [2][KT * D]
	const int lane = threadIdx.x & 63, l32 = lane & 31, hh = lane >> 5;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	// grid (heads, query blocks), x fastest: every head's heaviest (latest) query block
	// is dispatched before any lighter one (longest-first over the whole causal grid)
	const int qb = gridDim.y - 1 - blockIdx.y;
	const int h = blockIdx.x, g = h / (n_heads / n_kv);
	const int q_dim = n_heads * D, kv_dim = n_kv * D;
	const int qw0 = qb * AQ + wave * 32; // this wave's first query row
	const int qrow = qw0 + l32;          // this lane's query
	const int qpos = pos0 + qrow;
	// scores in log2 units: exp2(s * log2(e) / sqrt(D) - m)
	const float sl2 = 1.4426950408889634f / sqrtf((float)D);
	const int kv_rows = pos0 + T; // valid cache rows (masked keys past a query are never used)

	constexpr int QS = SPLIT ? 2 : 1; // Q / O row width in q_dim units
	half8_t qf[D / 16]; // B operand of S^T = K Q^T: Q[query = l32][d = 16 s + 8 h ..]
	half8_t ql[SPLIT ? D / 16 : 1]; // SPLIT: the lo half of Q
	{
		const uint16_t *qp = Q + (size_t)min(qrow, T - 1) * q_dim * QS + h * D + 8 * hh;
#pragma unroll
		for (int s = 0; s < D / 16; ++s) {
			qf[s] = *(const half8_t *)(qp + 16 * s);
			if constexpr (SPLIT)
				ql[s] = *(const half8_t *)(qp + q_dim + 16 * s);
		}
	}
	f32x16_t o[D / 32]; // O^T tiles: rows = d (32 jd + crow), column = query
#pragma unroll
	for (int jd = 0; jd < D / 32; ++jd)
		o[jd] = f32x16_t{};
	float m = -FLT_MAX, l = 0.0f;
	const int qmax_blk = min(qb * AQ + AQ, T) - 1; // last query row of the block
	const int ntile = (pos0 + qmax_blk) / KT + 1; // key tiles up to its position
	// transposed-read lane geometry (ds_read_b64_tr_b16: 16-lane groups, 4 rows x 16 columns)
	const int gi = lane & 15, gq = gi >> 2, gp = gi & 3;
	const int dgrp = 16 * ((lane >> 4) & 1);

	stage_kv<D, false, KT>(Kb, kc, 0, kv_rows, kv_dim, g, wave, lane);
	stage_kv<D, true, KT>(Vb, vc, 0, kv_rows, kv_dim, g, wave, lane);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	int cur = 0;
	for (int kt = 0; kt < ntile; ++kt) {
		const int key0 = kt * KT;
		if (kt + 1 < ntile) { // next tile's LDS-DMA overlaps this tile's math
			stage_kv<D, false, KT>(Kb + (cur ^ 1) * KT * D, kc, key0 + KT, kv_rows, kv_dim, g, wave, lane);
			stage_kv<D, true, KT>(Vb + (cur ^ 1) * KT * D, vc, key0 + KT, kv_rows, kv_dim, g, wave, lane);
		}
		const uint16_t *Ks = Kb + cur * KT * D;
		const uint16_t *Vs = Vb + cur * KT * D;

		// a tile wholly past this wave's last query (the block's second diagonal tile for
		// its first waves) adds nothing: skip its math (the wave still stages and syncs)
		const bool live = key0 <= pos0 + qw0 + 31;
		// ---- S^T = K Q^T: two 32-key blocks; register r of block j is key key0 + 32 j + crow(r, lane)
		f32x16_t st[NJ];
		half8_t pb[NJ][2]; // P^T fragments: [block j][k-step s]
		half8_t pl[SPLIT ? NJ : 1][2]; // SPLIT: P - f16(P)
		if (live) {
#pragma unroll
			for (int j = 0; j < NJ; ++j) {
				st[j] = f32x16_t{};
				const int kr = 32 * j + l32;
#pragma unroll
				for (int s = 0; s < D / 16; ++s) {
					const int kcnk = 2 * s + hh;
					const half8_t ka = *(const half8_t *)(Ks + kr * D + 8 * (kcnk ^ (kr % DCH)));
					st[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ka, qf[s], st[j], 0, 0, 0);
					if constexpr (SPLIT)
						st[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ka, ql[s], st[j], 0, 0, 0);
				}
			}
			// ---- online softmax for this lane's query. Raw scores; the 1/sqrt(D) log2(e)
			// scale is folded into the exponent's FMA (sl2 > 0: the max commutes with it).
			// Causal mask only on diagonal tiles (a uniform branch).
			if (key0 + KT - 1 > pos0 + qw0) {
#pragma unroll
				for (int j = 0; j < NJ; ++j)
#pragma unroll
					for (int r = 0; r < 16; ++r)
						if (key0 + 32 * j + crow(r, lane) > qpos)
							st[j][r] = -INFINITY;
			}
			float mx = st[0][0];
#pragma unroll
			for (int j = 0; j < NJ; ++j)
#pragma unroll
				for (int r = (j == 0 ? 1 : 0); r < 16; ++r)
					mx = fmaxf(mx, st[j][r]);
			mx = fmaxf(mx, xor32(mx)) * sl2; // the other lane half holds the other keys of each block
			// deferred rescale (cdna_hip_programming.md T13): while no query's max grows by
			// more than 2^RESCALE_LOG2 the old max stays the reference (P <= 2^8, exact
			// enough in f16; l and O are f32); otherwise every lane moves to its new max.
			// The decision precedes this tile's exponentials, so nothing is scaled twice.
			if (!__all(mx - m <= 8.0f)) {
				const float mn = fmaxf(m, mx);
				const float alpha = __builtin_amdgcn_exp2f(m - mn);
				m = mn;
				l *= alpha;
#pragma unroll
				for (int jd = 0; jd < D / 32; ++jd)
					o[jd] *= alpha;
			}
			float ls = 0.0f;
#pragma unroll
			for (int j = 0; j < NJ; ++j)
#pragma unroll
				for (int r = 0; r < 16; ++r) {
					const float p = __builtin_amdgcn_exp2f(fmaf(st[j][r], sl2, -m));
					ls += p;
					pb[j][r >> 3][r & 7] = (_Float16)p;
					if constexpr (SPLIT)
						pl[j][r >> 3][r & 7] = (_Float16)(p - (float)pb[j][r >> 3][r & 7]);
				}
			ls += xor32(ls);
			l += ls;
		}
		// ---- O^T += V^T P^T
		if (live) {
#pragma unroll
			for (int j = 0; j < NJ; ++j)
#pragma unroll
				for (int s = 0; s < 2; ++s) {
					const int klo = 32 * j + 16 * s + 4 * hh + gq; // keys of elements 0..3 (row gq of the 4-row block)
#pragma unroll
					for (int jd = 0; jd < D / 32; ++jd) {
						const int d = 32 * jd + dgrp + 4 * gp;
						const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
						    (YALM_LDS short4_t *)(Vs + klo * D + 8 * ((d >> 3) ^ ((klo & 3) << 1)) + (d & 7)));
						const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((YALM_LDS short4_t *)(
						    Vs + (klo + 8) * D + 8 * ((d >> 3) ^ (((klo + 8) & 3) << 1)) + (d & 7)));
						half8_t va;
#pragma unroll
						for (int e = 0; e < 4; ++e) {
							va[e] = __builtin_bit_cast(_Float16, (short)lo[e]);
							va[4 + e] = __builtin_bit_cast(_Float16, (short)hi[e]);
						}
						o[jd] = __builtin_amdgcn_mfma_f32_32x32x16_f16(va, pb[j][s], o[jd], 0, 0, 0);
						if constexpr (SPLIT)
							o[jd] = __builtin_amdgcn_mfma_f32_32x32x16_f16(va, pl[j][s], o[jd], 0, 0, 0);
					}
				}
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads(); // next tile landed; this tile's K / V reads are done
		cur ^= 1;
	}
	// ---- normalise and store O[query][h * D + d] (f16, the Wo GEMM's A operand); d = 32 jd + crow(r)
	if (qrow < T) {
		const float inv = 1.0f / l;
		uint16_t *op = O + (size_t)qrow * q_dim * QS + h * D;
#pragma unroll
		for (int jd = 0; jd < D / 32; ++jd)
#pragma unroll
			for (int r4 = 0; r4 < 4; ++r4) { // registers 4 r4 .. 4 r4 + 3 are 4 consecutive d
				const int d = 32 * jd + 8 * r4 + 4 * hh;
				float v[4];
				uint16_t hb[4];
#pragma unroll
				for (int e = 0; e < 4; ++e) {
					v[e] = o[jd][4 * r4 + e] * inv;
					hb[e] = f2h_bits(v[e]);
				}
				*(uint2 *)(op + d) = make_uint2(hb[0] | ((uint32_t)hb[1] << 16), hb[2] | ((uint32_t)hb[3] << 16));
				if constexpr (SPLIT) {
					uint16_t lb[4];
#pragma unroll
					for (int e = 0; e < 4; ++e)
						lb[e] = f2h_bits(v[e] - h2f(hb[e]));
					*(uint2 *)(op + q_dim + d) =
						make_uint2(lb[0] | ((uint32_t)lb[1] << 16), lb[2] | ((uint32_t)lb[3] << 16));
				}
			}
	}
}

// ---------------------------------------------------------------- row kernels
// X[t] = f32(E[token[t]])  (copy_embedding, infer.cu:632-640)
template <class WT>
__global__ __launch_bounds__(256) void embed_rows_kernel(const int *__restrict__ tokens, const void *__restrict__ emb,
                                                         int dim, float *__restrict__ X) {
	const int t = blockIdx.x;
	const char *row = (const char *)emb + (size_t)tokens[t] * dim * WT::BYTES;
	for (int i = threadIdx.x * WT::EPL; i < dim; i += blockDim.x * WT::EPL) {
		float f[WT::EPL];
		WT::unpack(load16(row + (size_t)i * WT::BYTES), f);
#pragma unroll
		for (int e = 0; e < WT::EPL; ++e)
			X[(size_t)t * dim + i + e] = f[e];
	}
}

// E5M2 weights -> f16 for the prefill of an fp8 model: the byte b is the f16 with bits
// b << 8 (the decode path's exact upcast), so the f16 MFMA GEMMs over the
// dequantised copy compute exactly what they compute for the f16 twin model. Up to 8
// tensors per launch (one launch per layer); 16 bytes in, 32 out per thread step.
struct DqSegs {
	const uint8_t *src[8];
	uint16_t *dst[8];
	size_t end[8]; // cumulative 16-byte pieces
	int n;
};
__global__ __launch_bounds__(256) void e5m2_to_f16_kernel(DqSegs s) {
	const size_t total = s.end[s.n - 1];
	for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
		const uint8_t *sp = s.src[0];
		uint16_t *dp = s.dst[0];
		size_t base = 0;
#pragma unroll
		for (int m = 1; m < 8; ++m) // constant indices: the kernel-argument arrays stay in SGPRs
			if (m < s.n && i >= s.end[m - 1]) {
				sp = s.src[m];
				dp = s.dst[m];
				base = s.end[m - 1];
			}
		const size_t j = i - base;
		const u32x4_t v = load_nt16(sp + 16 * j);
		u32x4_t o[2];
#pragma unroll
		for (int q = 0; q < 4; ++q) {
			const uint32_t w = v[q];
			o[q >> 1][2 * (q & 1) + 0] = ((w & 0xffu) << 8) | ((w & 0xff00u) << 16);
			o[q >> 1][2 * (q & 1) + 1] = ((w & 0xff0000u) >> 8) | (w & 0xff000000u);
		}
		u32x4_t *d = (u32x4_t *)(dp + 16 * j);
		d[0] = o[0];
		d[1] = o[1];
	}
}

// Xn[t] = f16(rmsnorm(X[t]) * w)  (rmsnorm, infer.cpp:134-144 statement order).
// SPLIT: row t of Xn is [hi | lo], 2 dim wide: hi = f16(v), lo = f16(v - hi), so
// hi + lo carries v to ~22 bits (the K / V columns of the QKV GEMM run over both
// halves against the same weight row; prefill_gemm.h BWrap).
template <bool SPLIT>
__global__ __launch_bounds__(256) void rmsnorm_rows_kernel(const float *__restrict__ X, const float *__restrict__ w,
                                                           int dim, float eps, uint16_t *__restrict__ Xn,
                                                           unsigned *range = nullptr) {
	__shared__ float red[4];
	const int t = blockIdx.x;
	const float *x = X + (size_t)t * dim;
	float ss = 0.0f;
	for (int i = threadIdx.x * 4; i < dim; i += 256 * 4) {
		const float4_t v = *(const float4_t *)(x + i);
		ss += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
	}
	ss = wave_sum(ss);
	if ((threadIdx.x & 63) == 0)
		red[threadIdx.x >> 6] = ss;
	__syncthreads();
	const float tot = red[0] + red[1] + red[2] + red[3];
	const float scale = 1.0f / sqrtf(tot / dim + eps);
	uint16_t *row = Xn + (size_t)t * dim * (SPLIT ? 2 : 1);
	float ymax = 0.0f;
	for (int i = threadIdx.x * 4; i < dim; i += 256 * 4) {
		const float4_t v = *(const float4_t *)(x + i);
		const float4_t g = *(const float4_t *)(w + i);
		float y[4];
		uint16_t hb[4];
#pragma unroll
		for (int e = 0; e < 4; ++e) {
			y[e] = v[e] * scale * g[e];
			hb[e] = f2h_bits(y[e]);
			ymax = fmaxf(ymax, y[e] != y[e] ? __builtin_inff() : fabsf(y[e])); // NaN counts as inf
		}
		*(uint2 *)(row + i) = make_uint2(hb[0] | ((uint32_t)hb[1] << 16), hb[2] | ((uint32_t)hb[3] << 16));
		if constexpr (SPLIT) {
			uint16_t lb[4];
#pragma unroll
			for (int e = 0; e < 4; ++e)
				lb[e] = f2h_bits(y[e] - h2f(hb[e]));
			*(uint2 *)(row + dim + i) =
			    make_uint2(lb[0] | ((uint32_t)lb[1] << 16), lb[2] | ((uint32_t)lb[3] << 16));
		}
	}
	range_note(range, ymax, ymax);
}

// The same row norm with ONE WAVE per row and the whole row in registers (NV float4 per
// lane, dim <= 256 NV): every load of the row issued at once, x read once, no LDS and no
// barrier (round 6: the workgroup-per-row form above reads x twice and pays a load round
// trip, a barrier and a second round trip per row; 15.7 / 20.1 us at Llama-3B T 4096 for
// 75 / 100 MB). Sum order: per lane over its float4s, then the wave's DPP sum.
template <bool SPLIT, int NV>
__global__ __launch_bounds__(256) void rmsnorm_rows_wave_kernel(const float *__restrict__ X,
                                                                const float *__restrict__ w, int dim, int T,
                                                                float eps, uint16_t *__restrict__ Xn,
                                                                unsigned *range = nullptr) {
	const int lane = threadIdx.x & 63;
	const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
	if (t >= T)
		return;
	const float *x = X + (size_t)t * dim;
	float4_t v[NV];
	float ss = 0.0f;
#pragma unroll
	for (int k = 0; k < NV; ++k) {
		const int i = (lane + 64 * k) * 4;
		v[k] = i < dim ? *(const float4_t *)(x + i) : float4_t{0.0f, 0.0f, 0.0f, 0.0f};
	}
#pragma unroll
	for (int k = 0; k < NV; ++k)
		ss += v[k][0] * v[k][0] + v[k][1] * v[k][1] + v[k][2] * v[k][2] + v[k][3] * v[k][3];
	ss = wave_sum(ss);
	const float scale = 1.0f / sqrtf(ss / dim + eps);
	uint16_t *row = Xn + (size_t)t * dim * (SPLIT ? 2 : 1);
	float ymax = 0.0f;
#pragma unroll
	for (int k = 0; k < NV; ++k) {
		const int i = (lane + 64 * k) * 4;
		if (i >= dim)
			break;
		const float4_t g = *(const float4_t *)(w + i);
		float y[4];
		uint16_t hb[4];
#pragma unroll
		for (int e = 0; e < 4; ++e) {
			y[e] = v[k][e] * scale * g[e];
			hb[e] = f2h_bits(y[e]);
			ymax = fmaxf(ymax, y[e] != y[e] ? __builtin_inff() : fabsf(y[e])); // NaN counts as inf
		}
		*(uint2 *)(row + i) = make_uint2(hb[0] | ((uint32_t)hb[1] << 16), hb[2] | ((uint32_t)hb[3] << 16));
		if constexpr (SPLIT) {
			uint16_t lb[4];
#pragma unroll
			for (int e = 0; e < 4; ++e)
				lb[e] = f2h_bits(y[e] - h2f(hb[e]));
			*(uint2 *)(row + dim + i) = make_uint2(lb[0] | ((uint32_t)lb[1] << 16), lb[2] | ((uint32_t)lb[3] << 16));
		}
	}
	range_note(range, ymax, ymax);
}

// RoPE (cos, sin) per prompt row and frequency, the decode path's exact
// formula (angle = (float)pos * inv_freq[j]; cosf / sinf, infer.cpp:291-301):
// computed once per prefill instead of 2 x 64 transcendentals per QKV element.
__global__ __launch_bounds__(256) void rope_table_kernel(const float *__restrict__ inv_freq, int half_dim, int T,
                                                         int pos0, float *__restrict__ rope) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= T * half_dim)
		return;
	const int m = i / half_dim, j = i % half_dim;
	const float val = (float)(pos0 + m) * inv_freq[j];
	rope[2 * i] = cosf(val);
	rope[2 * i + 1] = sinf(val);
}

// log p(target) per row from the vocab-tile partials: M = max, S = sum_i s_i e^(m_i - M)
__global__ __launch_bounds__(256) void logprob_kernel(const float *__restrict__ pmax, const float *__restrict__ psum,
                                                      const float *__restrict__ tgt_logit,
                                                      const int *__restrict__ targets, int M, int ntiles,
                                                      float *__restrict__ out) {
	__shared__ float red[4];
	const int m = blockIdx.x;
	float mx = -FLT_MAX;
	for (int i = threadIdx.x; i < ntiles; i += 256)
		mx = fmaxf(mx, pmax[(size_t)m * ntiles + i]);
	mx = wave_max(mx);
	if ((threadIdx.x & 63) == 0)
		red[threadIdx.x >> 6] = mx;
	__syncthreads();
	mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
	__syncthreads();
	float s = 0.0f;
	for (int i = threadIdx.x; i < ntiles; i += 256)
		s += psum[(size_t)m * ntiles + i] * expf(pmax[(size_t)m * ntiles + i] - mx);
	s = wave_sum(s);
	if ((threadIdx.x & 63) == 0)
		red[threadIdx.x >> 6] = s;
	__syncthreads();
	if (threadIdx.x == 0) {
		const float tot = red[0] + red[1] + red[2] + red[3];
		out[m] = targets[m] >= 0 ? tgt_logit[m] - mx - logf(tot) : 0.0f;
	}
}

} // namespace pf
