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
// fragment is a 16-byte row read (no transposes). Accumulation is f32; the
// activations are rounded to f16 for the MFMA inputs (the parity tolerance of
// tests/test_gpu_prefill.py covers exactly that).
#pragma once

#include <float.h>

#include "device_common.h"

typedef float f32x16_t __attribute__((ext_vector_type(16)));
#define YALM_LDS __attribute__((address_space(3)))

namespace pf {

constexpr int BM = 128, BN = 128, BK = 64; // block tile; BK = 64 f16 = 128-byte rows
constexpr int THREADS = 256;               // 4 waves as 2 (M) x 2 (N), 64 x 64 each
constexpr int TILE = BM * BK;              // f16 elements per staged operand tile (16 KB)

__device__ __forceinline__ uint16_t f2h_bits(float x) {
	_Float16 h = (_Float16)x;
	uint16_t u;
	__builtin_memcpy(&u, &h, 2);
	return u;
}

// Stage a 128-row x 64-k f16 tile global -> LDS with 16-byte LDS-DMA
// (global_load_lds_dwordx4): wave-instruction = 1 KB = 8 rows. The LDS image
// is lane-linear; the XOR swizzle (chunk ^ (row & 7)) goes on the per-lane
// SOURCE address, the matching read is frag_addr below. Rows past `rows`
// re-read the last valid row (never stored).
__device__ __forceinline__ void stage_tile(uint16_t *lds_tile, const uint16_t *__restrict__ g, int ld, int row0,
                                           int rows, int k0, int wave, int lane) {
#pragma unroll
	for (int i = 0; i < BM / 8 / (THREADS / 64); ++i) {
		const int rb = wave * (BM / 8 / (THREADS / 64)) + i;
		const int r = rb * 8 + (lane >> 3);
		const int c = lane & 7;
		const int gr = min(row0 + r, rows - 1);
		const uint16_t *src = g + (size_t)gr * ld + k0 + 8 * (c ^ (r & 7));
		__builtin_amdgcn_global_load_lds((const void *)src, (YALM_LDS void *)(lds_tile + rb * 8 * BK), 16, 0, 0);
	}
}

// 32x32x16 f16 operand fragment of tile row r, k-step s (16 deep): lane half h
// holds k = 16 s + 8 h .. +7 (cdna_hip_programming.md §3 A/B lane maps).
__device__ __forceinline__ half8_t frag(const uint16_t *lds_tile, int r, int s, int h) {
	const int kc = 2 * s + h;
	return *(const half8_t *)(lds_tile + r * BK + 8 * (kc ^ (r & 7)));
}

// C/D map of v_mfma_f32_32x32x16: column = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
__device__ __forceinline__ int crow(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

// ---------------------------------------------------------------- epilogues
// Each gets the wave's accumulators acc[NB][2][2] (32x32 tiles, rows m0 + 32 i,
// columns n0 + 32 j) after the K loop.

struct EpiStoreF32 { // C -> f32 (tests)
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	float *c;
	int ldc, M;
	template <int NB>
	__device__ __forceinline__ void apply(f32x16_t (&acc)[NB][2][2], int m0, int n0, int lane) const {
#pragma unroll
		for (int i = 0; i < 2; ++i)
#pragma unroll
			for (int j = 0; j < 2; ++j)
#pragma unroll
				for (int r = 0; r < 16; ++r) {
					const int m = m0 + 32 * i + crow(r, lane), n = n0 + 32 * j + (lane & 31);
					if (m < M)
						c[(size_t)m * ldc + n] = acc[0][i][j][r];
				}
	}
};

struct EpiResidual { // X[m][n] += C  (fused_matmul_add_residuals, per row)
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	float *x;
	int ldx, M;
	template <int NB>
	__device__ __forceinline__ void apply(f32x16_t (&acc)[NB][2][2], int m0, int n0, int lane) const {
#pragma unroll
		for (int i = 0; i < 2; ++i)
#pragma unroll
			for (int j = 0; j < 2; ++j)
#pragma unroll
				for (int r = 0; r < 16; ++r) {
					const int m = m0 + 32 * i + crow(r, lane), n = n0 + 32 * j + (lane & 31);
					if (m < M)
						x[(size_t)m * ldx + n] += acc[0][i][j][r];
				}
	}
};

template <int ACT>
struct EpiGlu { // H = f16(act(X W1^T) * (X W3^T))  (fused_ffn_w1_w3_glu_act)
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	uint16_t *h;
	int ldh, M;
	template <int NB>
	__device__ __forceinline__ void apply(f32x16_t (&acc)[NB][2][2], int m0, int n0, int lane) const {
#pragma unroll
		for (int i = 0; i < 2; ++i)
#pragma unroll
			for (int j = 0; j < 2; ++j)
#pragma unroll
				for (int r = 0; r < 16; ++r) {
					const int m = m0 + 32 * i + crow(r, lane), n = n0 + 32 * j + (lane & 31);
					if (m < M)
						h[(size_t)m * ldh + n] = f2h_bits(act_fn<ACT>(acc[0][i][j][r]) * acc[NB - 1][i][j][r]);
				}
	}
};

// [q | k | v] columns: clip (infer.cpp:280-288), RoPE on (even, odd) column
// pairs = lanes (l, l ^ 1) via DPP (infer.cpp:291-301, angle = pos * freq),
// q -> f16 Q[T][q_dim], k / v -> the fp16 KV cache rows pos0 + m
// (fused_rope_and_cache_update, infer.cu:642-677).
struct EpiQKV {
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	uint16_t *q;
	uint16_t *kc, *vc;
	const float *rope; // [M][head_dim / 2][2] (cos, sin) of pos * inv_freq (rope_table_kernel)
	int M, q_dim, kv_dim, head_dim, pos0;
	float clip;
	template <int NB>
	__device__ __forceinline__ void apply(f32x16_t (&acc)[NB][2][2], int m0, int n0, int lane) const {
		const bool odd = lane & 1;
#pragma unroll
		for (int i = 0; i < 2; ++i)
#pragma unroll
			for (int j = 0; j < 2; ++j) {
				const int n = n0 + 32 * j + (lane & 31);
				const bool is_v = n >= q_dim + kv_dim;
				const int nn = n < q_dim ? n : (n < q_dim + kv_dim ? n - q_dim : n - q_dim - kv_dim);
				const int fj = (nn % head_dim) >> 1;
#pragma unroll
				for (int r = 0; r < 16; ++r) {
					float v = acc[0][i][j][r];
					v = v < -clip ? -clip : (v > clip ? clip : v);
					const float p = dpp<0xB1>(v); // partner column (n ^ 1)
					const int m = m0 + 32 * i + crow(r, lane);
					if (m >= M)
						continue;
					const int pos = pos0 + m;
					float o = v;
					if (!is_v) {
						const float2_t cs = *(const float2_t *)(rope + ((size_t)m * (head_dim >> 1) + fj) * 2);
						o = odd ? p * cs[1] + v * cs[0] : v * cs[0] - p * cs[1];
					}
					if (n < q_dim)
						q[(size_t)m * q_dim + n] = f2h_bits(o);
					else if (!is_v)
						kc[(size_t)pos * kv_dim + nn] = f2h(o);
					else
						vc[(size_t)pos * kv_dim + nn] = f2h(o);
				}
			}
	}
};

// Per (row, 128-column tile): max and sum of exp over the tile's logits, and
// the target token's logit when it falls in the tile (sample_prob,
// sampler.cpp:11-25, split over vocab tiles; combined by logprob_kernel).
struct EpiLogits {
	static constexpr bool NEEDS_LDS = true;
	float *pmax, *psum, *tgt_logit;
	const int *targets; // target token of row m (-1: none)
	int M, ntiles;
	float *red; // LDS scratch [2 waves (N)][128 rows][2]
	template <int NB>
	__device__ __forceinline__ void apply(f32x16_t (&acc)[NB][2][2], int m0, int n0, int lane) const {
		const int wave = threadIdx.x >> 6;
		const int wn = wave & 1, wm = wave >> 1;
#pragma unroll
		for (int i = 0; i < 2; ++i) {
#pragma unroll
			for (int r = 0; r < 16; ++r) {
				const int ml = 32 * i + crow(r, lane); // row within the wave's 64
				const int m = m0 + ml;
				const int tgt = m < M ? targets[m] : -1;
				float mx = fmaxf(acc[0][i][0][r], acc[0][i][1][r]);
				mx = row16_max(mx);
				mx = fmaxf(mx, xor16(mx)); // 32 columns of this lane half
#pragma unroll
				for (int j = 0; j < 2; ++j) {
					const int n = n0 + 32 * j + (lane & 31);
					if (n == tgt)
						tgt_logit[m] = acc[0][i][j][r];
				}
				float s = expf(acc[0][i][0][r] - mx) + expf(acc[0][i][1][r] - mx);
				s = row16_sum(s);
				s += xor16(s);
				if ((lane & 31) == 0) {
					red[(wn * BM + wm * 64 + ml) * 2 + 0] = mx;
					red[(wn * BM + wm * 64 + ml) * 2 + 1] = s;
				}
			}
		}
		__syncthreads();
		for (int row = threadIdx.x; row < BM; row += THREADS) {
			const int m = m0 - (m0 % BM) + row; // block's row
			if (m >= M)
				continue;
			const float a = red[row * 2], sa = red[row * 2 + 1];
			const float b = red[(BM + row) * 2], sb = red[(BM + row) * 2 + 1];
			const float mx = fmaxf(a, b);
			const int tile = (n0 - (n0 % BN)) / BN;
			pmax[(size_t)m * ntiles + tile] = mx;
			psum[(size_t)m * ntiles + tile] = sa * expf(a - mx) + sb * expf(b - mx);
		}
	}
};

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

// C[M, N] (epilogue) = A[M, K] · W_b[N, K]^T for b < NB (NB = 2: W1 and W3
// share the A tile). N % 128 == 0, K % 64 == 0, any M.
//   NS = 2: two LDS buffers; the next K tile's LDS-DMA is issued before the
//     current tile's MFMAs and drained (vmcnt(0) + barrier) after them (the
//     2-phase structure of cdna_hip_programming.md §5.5 T3+T4, minimum form).
//   NS = 3: three LDS buffers, ONE tile kept in flight across every barrier
//     (cdna_hip_programming.md §5 "Pipelining across barriers": counted
//     vmcnt(N) — N = this thread's LDS-DMA instructions per tile — and a raw
//     s_barrier with lgkmcnt(0) only; __syncthreads() would drain the DMA).
//     Per K step: wait for tile kt (tile kt + 1 may stay in flight) -> barrier
//     (every wave's tile kt landed; every wave done reading tile kt - 1) ->
//     issue tile kt + 2 into tile kt - 1's buffer -> MFMAs on tile kt.
template <int NB>
constexpr int gemm_lds_per_tile() {
	return (1 + NB) * BM / 8 / (THREADS / 64); // LDS-DMA instructions per thread per K tile
}
__device__ __forceinline__ void raw_barrier() {
	asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt_wait() {
	asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// WIDE: a 128 x 256 output tile for a single weight matrix, run as NB = 2 with
// the two B tiles = columns [col0, col0 + 128) and [col0 + 128, col0 + 256) of
// the same B: twice the MFMAs per A fragment read from LDS (the GLU kernel's
// shape, ~1 PF/s where the 128 x 128 tile reached 0.55-0.75); the narrow
// epilogue runs once per column half.
template <class EPI, int NB, int NS, bool WIDE = false>
__global__ __launch_bounds__(THREADS) void gemm_nt_kernel(const uint16_t *__restrict__ A, int M, int K, BSrc B0,
                                                          BSrc B1, int N, EPI epi) {
	extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
	constexpr int BUF = (1 + NB) * TILE; // f16 per buffer
	const int lane = threadIdx.x & 63;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int wm = wave >> 1, wn = wave & 1;
	const int h = lane >> 5, l32 = lane & 31;

	// tile index: XCD-aware (blocks b, b+8, ... share an XCD's L2): consecutive
	// tiles of one XCD walk down M for a fixed N panel (the W panel is reused)
	static_assert(!WIDE || NB == 2, "the wide tile runs as two B tiles");
	constexpr int TBN = WIDE ? 2 * BN : BN; // output columns per tile
	const int tiles_m = (M + BM - 1) / BM, tiles_n = N / TBN;
	const int nwg = tiles_m * tiles_n;
	int wg = blockIdx.x;
	{
		const int q = nwg / 8, rr = nwg % 8, xcd = wg % 8, idx = wg / 8;
		wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
	}
	const int tm = wg % tiles_m, tn = wg / tiles_m;
	const int row0 = tm * BM, col0 = tn * TBN;

	f32x16_t acc[NB][2][2];
#pragma unroll
	for (int b = 0; b < NB; ++b)
#pragma unroll
		for (int i = 0; i < 2; ++i)
#pragma unroll
			for (int j = 0; j < 2; ++j)
				acc[b][i][j] = f32x16_t{};

	const int nk = K / BK;
	const uint16_t *w0, *w1 = nullptr;
	int w0r, w0n, w1r = 0, w1n = 1;
	B0.tile(col0, w0, w0r, w0n);
	if constexpr (NB == 2)
		B1.tile(WIDE ? col0 + BN : col0, w1, w1r, w1n);
	auto stage = [&](int buf, int kt) {
		uint16_t *base = smem + buf * BUF;
		stage_tile(base, A, K, row0, M, kt * BK, wave, lane);
		stage_tile(base + TILE, w0, K, w0r, w0n, kt * BK, wave, lane);
		if constexpr (NB == 2)
			stage_tile(base + 2 * TILE, w1, K, w1r, w1n, kt * BK, wave, lane);
	};
	auto compute = [&](const uint16_t *a_t) {
#pragma unroll
		for (int s = 0; s < BK / 16; ++s) {
			half8_t af[2], bf[NB][2];
#pragma unroll
			for (int i = 0; i < 2; ++i)
				af[i] = frag(a_t, wm * 64 + 32 * i + l32, s, h);
#pragma unroll
			for (int b = 0; b < NB; ++b)
#pragma unroll
				for (int j = 0; j < 2; ++j)
					bf[b][j] = frag(a_t + (1 + b) * TILE, wn * 64 + 32 * j + l32, s, h);
#pragma unroll
			for (int b = 0; b < NB; ++b)
#pragma unroll
				for (int i = 0; i < 2; ++i)
#pragma unroll
					for (int j = 0; j < 2; ++j)
						acc[b][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[b][j], acc[b][i][j], 0, 0, 0);
		}
	};
	if constexpr (NS == 2) {
		stage(0, 0);
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads();
		int cur = 0;
		for (int kt = 0; kt < nk; ++kt) {
			if (kt + 1 < nk)
				stage(cur ^ 1, kt + 1);
			compute(smem + cur * BUF);
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			__syncthreads();
			cur ^= 1;
		}
	} else {
		constexpr int L = gemm_lds_per_tile<NB>();
		stage(0, 0);
		if (nk > 1)
			stage(1, 1);
		int cur = 0; // buffer of tile kt
		for (int kt = 0; kt < nk; ++kt) {
			if (kt + 1 < nk)
				vmcnt_wait<L>(); // tile kt landed (this thread's DMAs); tile kt + 1 may stay in flight
			else
				vmcnt_wait<0>();
			raw_barrier();
			if (kt + 2 < nk)
				stage(cur == 0 ? 2 : cur - 1, kt + 2); // tile kt - 1's buffer: every wave is past reading it
			compute(smem + cur * BUF);
			cur = cur == 2 ? 0 : cur + 1;
		}
		raw_barrier(); // the epilogue may reuse the staging buffers (EpiLogits)
	}
	EPI e = epi;
	if constexpr (EPI::NEEDS_LDS)
		e.red = (float *)smem; // the staging buffers are free after the K loop's last barrier
	if constexpr (WIDE) {
		typedef f32x16_t half_acc_t[1][2][2];
		e.template apply<1>(*reinterpret_cast<half_acc_t *>(&acc[0]), row0 + wm * 64, col0 + wn * 64, lane);
		if constexpr (EPI::NEEDS_LDS)
			__syncthreads(); // the first half's readers are done with e.red
		e.template apply<1>(*reinterpret_cast<half_acc_t *>(&acc[1]), row0 + wm * 64, col0 + BN + wn * 64, lane);
	} else {
		e.template apply<NB>(acc, row0 + wm * 64, col0 + wn * 64, lane);
	}
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
template <int D, int KT = AKT>
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

	half8_t qf[D / 16]; // B operand of S^T = K Q^T: Q[query = l32][d = 16 s + 8 h ..]
	{
		const uint16_t *qp = Q + (size_t)min(qrow, T - 1) * q_dim + h * D + 8 * hh;
#pragma unroll
		for (int s = 0; s < D / 16; ++s)
			qf[s] = *(const half8_t *)(qp + 16 * s);
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
		uint16_t *op = O + (size_t)qrow * q_dim + h * D;
#pragma unroll
		for (int jd = 0; jd < D / 32; ++jd)
#pragma unroll
			for (int r4 = 0; r4 < 4; ++r4) { // registers 4 r4 .. 4 r4 + 3 are 4 consecutive d
				const int d = 32 * jd + 8 * r4 + 4 * hh;
				uint32_t w0 = (uint32_t)f2h_bits(o[jd][4 * r4 + 0] * inv) | ((uint32_t)f2h_bits(o[jd][4 * r4 + 1] * inv) << 16);
				uint32_t w1 = (uint32_t)f2h_bits(o[jd][4 * r4 + 2] * inv) | ((uint32_t)f2h_bits(o[jd][4 * r4 + 3] * inv) << 16);
				*(uint2 *)(op + d) = make_uint2(w0, w1);
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

// Xn[t] = f16(rmsnorm(X[t]) * w)  (rmsnorm, infer.cpp:134-144 statement order)
__global__ __launch_bounds__(256) void rmsnorm_rows_kernel(const float *__restrict__ X, const float *__restrict__ w,
                                                           int dim, float eps, uint16_t *__restrict__ Xn) {
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
	for (int i = threadIdx.x * 4; i < dim; i += 256 * 4) {
		const float4_t v = *(const float4_t *)(x + i);
		const float4_t g = *(const float4_t *)(w + i);
		uint16_t *o = Xn + (size_t)t * dim + i;
		o[0] = f2h_bits(v[0] * scale * g[0]);
		o[1] = f2h_bits(v[1] * scale * g[1]);
		o[2] = f2h_bits(v[2] * scale * g[2]);
		o[3] = f2h_bits(v[3] * scale * g[3]);
	}
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
