// prefill_gemm.h — the prefill's MFMA GEMMs: C = A · W^T with a 256-row output
// tile per workgroup and 8 waves (the round-2 128 x 128 tile, bound by LDS
// traffic, was removed in round 4).
//
// A is [M][lda] f16 and the GEMM runs over K of its columns; B rows are K_b = kb
// wide and column k >= kb of the product reads B column k - kb ("B wrap"): with
// A = [hi | lo] (2 kb wide) that is C = hi W^T + lo W^T, the split-f16 A operand of
// the QKV GEMM's K / V columns (prefill.h rmsnorm_rows_kernel<true>).
//
// Why a big tile: an MFMA needs its A and B fragments read from LDS. With
// the 128 x 128 tile of round 2 each of the 4 waves owned 64 x 64 outputs and read one
// 1-KB fragment per 32x32x16 MFMA (4 reads per 4 MFMAs); the LDS-DMA fill of
// the next K tile added 32 KB per 64-deep step. Here each of the 8 waves owns
// 128 x 64 (BN 256) or 64 x 64 (BN 128) outputs of a 256 x BN tile and issues
// v_mfma_f32_16x16x32_f16: 12 fragment reads per 32 MFMAs (BN 256), and the
// per-flop LDS-DMA traffic halves (cdna_hip_programming.md §5: the 256² tile is
// the one that gets past the 128²-tile ceiling).
//
// Pipeline: two LDS buffers of one 64-deep K tile (A 32 KB + B BN x 128 B);
// the LDS-DMA of tile kt + 1 (global_load_lds_dwordx4, XOR-swizzled source,
// lane-linear LDS image) is issued before tile kt's MFMAs and waited for
// (counted vmcnt(0), raw s_barrier) after them, so it has a whole tile of MFMA
// time (2048 SIMD cycles at BN 256) to land from L2 / MALL. Two waves per SIMD:
// one wave's fragment reads overlap the other's MFMAs.
//
// Operands: A [M][K] f16 (activations), W [N][K] f16 (.yalm [out][in] layout):
// both K-contiguous, every fragment a 16-byte row read. B rows come from a
// policy (BRowsPlain: up to 3 matrices end to end, the wq | wk | wv QKV;
// BRowsGlu: W1 and W3 rows interleaved per wave so one wave holds W1 and W3
// columns of the same 32 outputs). Accumulation f32; epilogues in the 16x16
// C layout (column = lane & 15, row = 4 (lane >> 4) + reg).
#pragma once

#include "prefill.h"

namespace pf {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int G_BM = 256, G_BK = 64, G_THREADS = 512;

// C/D map of v_mfma_f32_16x16x32: column = lane & 15, row = 4 (lane >> 4) + reg.
__device__ __forceinline__ int crow16(int reg, int lane) { return 4 * (lane >> 4) + reg; }

// ---------------------------------------------------------------- B row policies
struct BRowsPlain { // W rows n0 + r from up to 3 row-major [rows][K] matrices laid end to end
	BSrc src;
	static constexpr int COLS_PER_TILE_DIV = 1; // output columns per tile = BN
	__device__ __forceinline__ const uint16_t *row(int n0, int r, int K) const {
		const int n = n0 + r;
		const int s = n < src.end[0] ? 0 : (n < src.end[1] ? 1 : 2);
		const int start = s == 0 ? 0 : src.end[s - 1];
		return src.p[s] + (size_t)(n - start) * K;
	}
};

// GLU: a tile covers BN / 2 hidden columns h0 .. ; wave column wc's TN B rows are
// TN / 2 W1 rows then the same TN / 2 W3 rows (h0 + wc * TN / 2 + ..).
template <int TN>
struct BRowsGlu {
	const uint16_t *w1, *w3;
	static constexpr int COLS_PER_TILE_DIV = 2;
	__device__ __forceinline__ const uint16_t *row(int h0, int r, int K) const {
		const int wc = r / TN, within = r % TN;
		const int mat = within / (TN / 2);
		const int hc = h0 + wc * (TN / 2) + within % (TN / 2);
		return (mat ? w3 : w1) + (size_t)hc * K;
	}
};

// ---------------------------------------------------------------- epilogues (16x16 layout)
// apply(acc, m0, n0, lane): acc[FI][FJ] f32x4; element (i, j, r) is row
// m0 + 16 i + crow16(r), column n0 + 16 j + (lane & 15) of the tile-local output.

struct E16StoreF32 {
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	float *c;
	int ldc, M;
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(f32x4_t (&acc)[FI][FJ], int m0, int n0, int lane, int, int) const {
#pragma unroll
		for (int i = 0; i < FI; ++i)
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const int m = m0 + 16 * i + crow16(r, lane);
				if (m >= M)
					continue;
#pragma unroll
				for (int j = 0; j < FJ; ++j)
					c[(size_t)m * ldc + n0 + 16 * j + (lane & 15)] = acc[i][j][r];
			}
	}
};

struct E16Residual { // X[m][n] += scale C  (fused_matmul_add_residuals, per row)
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	float *x;
	int ldx, M;
	float scale = 1.0f; // 2^e: undoes the exact power-of-two scale of an f16 A operand (E16Glu::hscale)
	// per row fragment: all 4 FJ loads of x issued (rows clamped) before any add, the stores
	// predicated on the row (a per-element branch around the load made hipcc wait for each
	// load separately: E16QKV below)
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(f32x4_t (&acc)[FI][FJ], int m0, int n0, int lane, int, int) const {
#pragma unroll
		for (int i = 0; i < FI; ++i) {
			float xv[4][FJ];
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const int m = min(m0 + 16 * i + crow16(r, lane), M - 1);
#pragma unroll
				for (int j = 0; j < FJ; ++j)
					xv[r][j] = x[(size_t)m * ldx + n0 + 16 * j + (lane & 15)];
			}
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const int m = m0 + 16 * i + crow16(r, lane);
				if (m < M)
#pragma unroll
					for (int j = 0; j < FJ; ++j)
						x[(size_t)m * ldx + n0 + 16 * j + (lane & 15)] = xv[r][j] + acc[i][j][r] * scale;
			}
		}
	}
};

// SiLU / GELU-tanh (infer.cu:586-596) with the hardware exp2 / reciprocal (1 ulp each)
// instead of the libm-accurate expf, tanhf and IEEE division: the result is rounded to
// f16 for the next GEMM anyway (its rounding error, 2^-11, is ~1000x these ulps), and
// the accurate forms made the GLU epilogue ~10% of the GEMM (tools/gemm_epi_bench.hip).
// The decode path keeps act_fn (parity bars of 1e-4 there).
template <int ACT>
__device__ __forceinline__ float act_fast(float x) {
	if constexpr (ACT == 1) {
		return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
	} else {
		const float y = 0.797885f * (x + 0.044715f * x * x * x);
		// tanh(y) = 1 - 2 / (e^(2y) + 1); e^(2y) overflows to inf for large y -> 1
		const float t = 1.0f - 2.0f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(2.8853900817779268f * y) + 1.0f);
		return 0.5f * x * (1.0f + t);
	}
}

// H = f16(act(X W1^T) * (X W3^T)) (fused_ffn_w1_w3_glu_act): columns j < FJ / 2 of a
// wave are W1 outputs, j >= FJ / 2 the W3 outputs of the same hidden columns.
// n0 here is the wave's first HIDDEN column (BRowsGlu).
// hscale: an exact power of two 2^-e (default 1) applied before the f16 rounding when the
// layer's GLU products exceed the f16 range (prefill.hip: found by range_note, the pass
// re-run with the scale, the W2 epilogue multiplying by 2^e); values below 2^-14 * 2^e then
// lose relative precision as f16 subnormals, far under the W2 sum's own rounding.
// The range check is one v_max with an |abs| modifier per element: finite operands give a
// finite or overflowing (inf, caught) product, and a NaN needs an inf or NaN upstream,
// which the row norms' checks catch. SPLIT (the split-operand form): H rows [hi | lo], lo
// `hidden` columns after hi (ldh = 2 hidden).
template <int ACT, bool SPLIT = false>
struct E16Glu {
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	uint16_t *h;
	int ldh, M;
	float hscale = 1.0f;
	unsigned *range = nullptr;
	int lo_off = 0; // SPLIT: columns from hi to lo
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(f32x4_t (&acc)[FI][FJ], int m0, int n0, int lane, int, int) const {
		float vmax = 0.0f;
#pragma unroll
		for (int i = 0; i < FI; ++i)
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const int m = m0 + 16 * i + crow16(r, lane);
				if (m >= M)
					continue;
#pragma unroll
				for (int j = 0; j < FJ / 2; ++j) {
					const float v = act_fast<ACT>(acc[i][j][r]) * acc[i][j + FJ / 2][r];
					vmax = fmaxf(vmax, fabsf(v));
					const float vs = v * hscale;
					const uint16_t hb = f2h_bits(vs);
					uint16_t *const hp = h + (size_t)m * ldh + n0 + 16 * j + (lane & 15);
					hp[0] = hb;
					if constexpr (SPLIT)
						hp[lo_off] = f2h_bits(vs - h2f(hb));
				}
			}
		range_note(range, vmax * hscale, vmax);
	}
};

// [q | k | v] columns: clip (infer.cpp:280-288), RoPE on (even, odd) column pairs =
// lanes (l, l ^ 1) via DPP (infer.cpp:291-301), q -> f16 Q, k / v -> the fp16 cache
// rows pos0 + m (fused_rope_and_cache_update, infer.cu:642-677); as EpiQKV.
// A 16-column block never straddles q / k / v (multiples of head_dim), so the region is
// wave-uniform per block j (a scalar branch), and a block's 4 FI (cos, sin) pairs per
// lane are loaded unconditionally (rows clamped) before any use: with per-element
// region / row branches hipcc waited for each table load separately (the epilogue cost
// 71 of 172 us at Llama-3B T 4096, tools/gemm_epi_bench.hip).
// SPLITQ (the split-operand form): Q rows [hi | lo], lo q_lo (= q_dim) columns after hi.
template <bool SPLITQ = false>
struct E16QKVt {
	static constexpr bool NEEDS_LDS = false;
	float *red = nullptr;
	uint16_t *q;
	uint16_t *kc, *vc;
	const float *rope;
	int M, q_dim, kv_dim, head_dim, pos0;
	float clip;
	unsigned *range = nullptr; // the f16 Q operand out of range (range_note, |max| only: see
							   // E16Glu); K / V are the f16 cache rows of the reference too
							   // (infer.cpp:299)
	int q_lo = 0;
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(f32x4_t (&acc)[FI][FJ], int m0, int n0, int lane, int, int) const {
		const bool odd = lane & 1;
		float qmax = 0.0f;
#pragma unroll
		for (int j = 0; j < FJ; ++j) {
			const int nb = __builtin_amdgcn_readfirstlane(n0 + 16 * j); // block's first column
			const int region = nb < q_dim ? 0 : (nb < q_dim + kv_dim ? 1 : 2);
			const int base = region == 0 ? 0 : (region == 1 ? q_dim : q_dim + kv_dim);
			const int nn = nb - base + (lane & 15); // column inside q / k / v
			const int fj = (nn % head_dim) >> 1;
			const bool rot = region != 2;
			uint16_t *const dst = (region == 0 ? q : (region == 1 ? kc : vc)) + nn;
			const int ld = region == 0 ? (SPLITQ ? 2 * q_dim : q_dim) : kv_dim, roff = region == 0 ? 0 : pos0;
			constexpr int IB = FI < 4 ? FI : 4; // row fragments per batch of table loads
#pragma unroll
			for (int i0 = 0; i0 < FI; i0 += IB) {
				float2_t cs[IB][4];
#pragma unroll
				for (int i = 0; i < IB; ++i)
#pragma unroll
					for (int r = 0; r < 4; ++r) {
						const int m = min(m0 + 16 * (i0 + i) + crow16(r, lane), M - 1);
						cs[i][r] = *(const float2_t *)(rope + ((size_t)m * (head_dim >> 1) + fj) * 2);
					}
#pragma unroll
				for (int i = 0; i < IB; ++i)
#pragma unroll
					for (int r = 0; r < 4; ++r) {
						float v = acc[i0 + i][j][r];
						v = v < -clip ? -clip : (v > clip ? clip : v);
						const float p = dpp<0xB1>(v); // partner column (n ^ 1)
						const float ro = odd ? p * cs[i][r][1] + v * cs[i][r][0] : v * cs[i][r][0] - p * cs[i][r][1];
						const int m = m0 + 16 * (i0 + i) + crow16(r, lane);
						const float o = rot ? ro : v;
						if (m < M) {
							const uint16_t ob = f2h(o);
							dst[(size_t)(roff + m) * ld] = ob;
							if (region == 0) {
								qmax = fmaxf(qmax, fabsf(o));
								if constexpr (SPLITQ)
									dst[(size_t)m * ld + q_lo] = f2h(o - h2f(ob));
							}
						}
					}
			}
		}
		range_note(range, qmax, qmax);
	}
};
using E16QKV = E16QKVt<false>;

// Per (row, BN-column tile): max and sum of exp over the tile's logits, and the
// target token's logit when it falls in the tile (sample_prob, sampler.cpp:11-25,
// split over vocab tiles; combined by logprob_kernel). Wave partials meet in LDS.
struct E16Logits {
	static constexpr bool NEEDS_LDS = true;
	float *pmax, *psum, *tgt_logit;
	const int *targets;
	int M, ntiles;
	float *red; // LDS scratch [WN][256 rows][2]
	// The targets of a row fragment's 4 rows are loaded together (rows clamped, the store
	// predicated: no load inside a per-element branch, see E16QKV), and exp(l - max) is the
	// hardware exp2 on a log2(e)-scaled FMA (1 ulp, far inside the perplexity bar).
	template <int FI, int FJ>
	__device__ __forceinline__ void apply(f32x4_t (&acc)[FI][FJ], int m0, int n0, int lane, int wc, int wn) const {
		const int tm0 = m0 - (m0 % G_BM); // tile's first row
		constexpr float L2E = 1.4426950408889634f;
#pragma unroll
		for (int i = 0; i < FI; ++i) {
			int tg[4];
#pragma unroll
			for (int r = 0; r < 4; ++r)
				tg[r] = targets[min(m0 + 16 * i + crow16(r, lane), M - 1)];
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const int m = m0 + 16 * i + crow16(r, lane);
				float mx = acc[i][0][r];
#pragma unroll
				for (int j = 1; j < FJ; ++j)
					mx = fmaxf(mx, acc[i][j][r]);
				mx = row16_max(mx); // the 16 lanes of this row group hold its 16 columns
#pragma unroll
				for (int j = 0; j < FJ; ++j)
					if (m < M && n0 + 16 * j + (lane & 15) == tg[r])
						tgt_logit[m] = acc[i][j][r];
				const float mxs = mx * L2E;
				float s = 0.0f;
#pragma unroll
				for (int j = 0; j < FJ; ++j)
					s += __builtin_amdgcn_exp2f(fmaf(acc[i][j][r], L2E, -mxs));
				s = row16_sum(s);
				if ((lane & 15) == 0) {
					const int rl = m - tm0;
					red[(wc * G_BM + rl) * 2 + 0] = mx;
					red[(wc * G_BM + rl) * 2 + 1] = s;
				}
			}
		}
		__syncthreads();
		for (int row = threadIdx.x; row < G_BM; row += G_THREADS) {
			const int m = tm0 + row;
			if (m >= M)
				continue;
			float mx = -FLT_MAX;
			for (int w = 0; w < wn; ++w)
				mx = fmaxf(mx, red[(w * G_BM + row) * 2]);
			float s = 0.0f;
			for (int w = 0; w < wn; ++w)
				s += red[(w * G_BM + row) * 2 + 1] * expf(red[(w * G_BM + row) * 2] - mx);
			const int tile = n0 / (16 * FJ * wn); // n0 of wave 0 ... any wave: tile = column tile index
			pmax[(size_t)m * ntiles + tile] = mx;
			psum[(size_t)m * ntiles + tile] = s;
		}
	}
};

// ---------------------------------------------------------------- the kernel
// Stage ROWS x 64 f16 of one operand into a lane-linear LDS image by LDS-DMA: wave
// instruction = 8 rows x 128 B; lane l writes row 8 rb + (l >> 3), chunk l & 7 and
// reads source chunk (l & 7) ^ (row & 7) (the swizzle lives on the source address;
// g16frag applies the same involution on the read). rowp[i]: this lane's row base of
// instruction i (already clamped / mapped).
template <int NI>
__device__ __forceinline__ void g16stage(uint16_t *lds, const uint16_t *const (&rowp)[NI], int k0, int wave, int lane) {
#pragma unroll
	for (int i = 0; i < NI; ++i) {
		const int rb = wave * NI + i;
		const int r = rb * 8 + (lane >> 3);
		const int c = lane & 7;
		__builtin_amdgcn_global_load_lds((const void *)(rowp[i] + k0 + 8 * (c ^ (r & 7))),
		                                 (YALM_LDS void *)(lds + rb * 8 * G_BK), 16, 0, 0);
	}
}

// 16x16x32 operand fragment: tile row r, k-step s (32 deep): lane group q = lane >> 4
// holds k = 32 s + 8 q .. + 7 (cdna_hip_programming.md §3 16x16x32 A/B maps).
__device__ __forceinline__ half8_t g16frag(const uint16_t *lds, int r, int s, int lane) {
	const int kc = 4 * s + (lane >> 4);
	return *(const half8_t *)(lds + r * G_BK + 8 * (kc ^ (r & 7)));
}

// C tile [256][BN] of C = A · B^T, B rows through BMAP. 8 waves as WM x (8 / WM).
template <class EPI, class BMAP, int BN, int WM>
__global__ __launch_bounds__(G_THREADS, 1) void gemm16_kernel(const uint16_t *__restrict__ A, int lda, int M, int K,
                                                             int kb, BMAP bm, int N, EPI epi, int c0) {
	constexpr int WN = 8 / WM;
	constexpr int TM = G_BM / WM, TN = BN / WN; // per-wave output
	constexpr int FI = TM / 16, FJ = TN / 16;
	constexpr int NIA = G_BM / 8 / 8, NIB = BN / 8 / 8; // LDS-DMA instructions per thread and operand
	constexpr int TA = G_BM * G_BK, TB = BN * G_BK;    // f16 per operand tile
	constexpr int BUF = TA + TB;
	extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
	const int lane = threadIdx.x & 63;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int wr = wave / WN, wc = wave % WN;

	// XCD-aware tile order (bijective remap, cdna_hip_programming.md §5 'XCD swizzle'):
	// the workgroups sharing an XCD walk down M for fixed column panels (B reused in L2)
	const int tiles_m = (M + G_BM - 1) / G_BM, tiles_n = N / BN;
	const int nwg = tiles_m * tiles_n;
	int wg = blockIdx.x;
	{
		const int q = nwg / 8, rr = nwg % 8, xcd = wg % 8, idx = wg / 8;
		wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
	}
	const int tm = wg % tiles_m, tn = wg / tiles_m;
	const int row0 = tm * G_BM;
	const int colB = c0 + tn * (BN / BMAP::COLS_PER_TILE_DIV); // first B column (plain) / hidden column (GLU)

	const uint16_t *ap[NIA], *bp[NIB];
#pragma unroll
	for (int i = 0; i < NIA; ++i)
		ap[i] = A + (size_t)min(row0 + (wave * NIA + i) * 8 + (lane >> 3), M - 1) * lda;
#pragma unroll
	for (int i = 0; i < NIB; ++i)
		bp[i] = bm.row(colB, (wave * NIB + i) * 8 + (lane >> 3), kb);

	f32x4_t acc[FI][FJ];
#pragma unroll
	for (int i = 0; i < FI; ++i)
#pragma unroll
		for (int j = 0; j < FJ; ++j)
			acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

	const int nk = K / G_BK;
	auto stage = [&](int buf, int kt) {
		uint16_t *base = smem + buf * BUF;
		const int k0 = kt * G_BK;
		g16stage<NIA>(base, ap, k0, wave, lane);
		g16stage<NIB>(base + TA, bp, k0 < kb ? k0 : k0 - kb, wave, lane); // B wrap
	};
	stage(0, 0);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	raw_barrier();
	for (int kt = 0; kt < nk; ++kt) {
		if (kt + 1 < nk)
			stage((kt + 1) & 1, kt + 1); // that buffer's last readers passed the previous barrier
		const uint16_t *sa = smem + (kt & 1) * BUF;
		const uint16_t *sb = sa + TA;
#pragma unroll
		for (int s = 0; s < G_BK / 32; ++s) {
			half8_t af[FI], bf[FJ];
#pragma unroll
			for (int j = 0; j < FJ; ++j)
				bf[j] = g16frag(sb, wc * TN + 16 * j + (lane & 15), s, lane);
#pragma unroll
			for (int i = 0; i < FI; ++i)
				af[i] = g16frag(sa, wr * TM + 16 * i + (lane & 15), s, lane);
			__builtin_amdgcn_s_setprio(1);
#pragma unroll
			for (int i = 0; i < FI; ++i)
#pragma unroll
				for (int j = 0; j < FJ; ++j)
					acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
			__builtin_amdgcn_s_setprio(0);
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // tile kt + 1 landed (this thread's DMAs)
		raw_barrier();                                     // ... everyone's; everyone done reading tile kt
	}
	EPI e = epi;
	if constexpr (EPI::NEEDS_LDS)
		e.red = (float *)smem; // the staging buffers are free after the last barrier
	const int n0 = BMAP::COLS_PER_TILE_DIV == 1 ? colB + wc * TN : colB + wc * (TN / 2);
	e.template apply<FI, FJ>(acc, row0 + wr * TM, n0, lane, wc, WN);
}

template <int BN>
constexpr size_t gemm16_lds() {
	return (size_t)2 * (G_BM + BN) * G_BK * sizeof(uint16_t);
}

// ---------------------------------------------------------------- 8-phase 256 x 256 GEMM
// The same C = A · B^T tile as gemm16_kernel<BN 256, WM 2> (8 waves as 2 M x 4 N, each
// wave 128 x 64 outputs, v_mfma_f32_16x16x32_f16), with the K loop cut into PHASES
// (cdna_hip_programming.md §5 "The 256² 8-phase template", T3+T4) instead of one
// stage / read / MFMA / drain / barrier step per K tile:
//
// * LDS: 2 buffers (E, O) x 4 HALF-TILES of 128 rows x 64 k (16 KB each) = 128 KB:
//     Am0 = the first 64 rows of each wave row's 128 (tile rows 0-63, 128-191),
//     Am1 = the other 64 (64-127, 192-255),
//     Bn0 = the first 32 B rows of each wave column's 64 (0-31, 64-95, 128-159, 192-223),
//     Bn1 = the other 32.
// * A K tile is 4 phases, one output quadrant each (16 MFMAs per wave):
//     q1 (m0, n0): read Am0 -> a, Bn0 -> b0     q2 (m0, n1): read Bn1 -> b1
//     q3 (m1, n1): read Am1 -> a                q4 (m1, n0): no read (a, b0 held)
//   so a half-tile's last LDS read in a K tile is q1 (Am0, Bn0), q2 (Bn1) or q3 (Am1).
// * Every phase stages ONE half-tile (2 LDS-DMAs per thread) and waits vmcnt(8): the
//   half-tile issued 4 phases earlier has landed, 4 stay in flight across the barriers
//   (no vmcnt(0) in the loop). Iteration = 8 phases = K tiles 2i (E) and 2i + 1 (O);
//   stage order: p1 Bn1 O(2i+1), p2 Am1 O(2i+1), p3 Am0 E(2i+2), p4 Bn0 E(2i+2),
//   p5 Bn1 E(2i+2), p6 Am1 E(2i+2), p7 Am0 O(2i+3), p8 Bn0 O(2i+3).
// * The two wave rows run one barrier apart (wave row 1 passes one extra barrier
//   first): each phase is {reads, stage, vmcnt} barrier {MFMAs} barrier, so on every
//   SIMD one wave's MFMAs run while the other's LDS reads and DMA issue do.
// * Hazards, with barrier intervals I_k (between barriers k and k + 1 of an iteration;
//   wave row 0 reads / stages phase p in I_{2p-2}, row 1 in I_{2p-1}; a ds_read issued
//   in I_k is complete before its wave reaches barrier k + 2):
//     WAR: a half-tile is restaged at phase s only when its last reader's interval is
//       <= 2s - 4 (Am0/Bn0 of E read last in I_1, restaged from I_4; Bn1 I_3 -> I_8;
//       Am1 I_5 -> I_10; O: I_9 -> I_12 / I_14, I_11 -> I_16, I_13 -> I_18).
//     RAW: the half-tile staged at phase s is retired by both rows' vmcnt(8) at phase
//       s + 4 (row 1: before barrier 2s + 8) and first read at phase >= s + 5 (row 0:
//       after barrier 2s + 8).
// * Tail: phases whose K tile is past the end stage nothing and wait vmcnt(0).
// * Tile widths: a wave's TN = 16 (FJ0 + FJ1) columns are split into the quadrant
//   column halves n0 (16 FJ0) and n1 (16 FJ1): BN = 4 TN = 256 (2, 2), 192 (2, 1),
//   128 (1, 1) (320 = (3, 2) would spill: 256 registers + scratch). A launch covers N
//   columns from column c0 (the QKV GEMM runs as a q launch and a k | v launch). Bn0 / Bn1 are 64 FJ0 / 64 FJ1 rows (FJ0 / FJ1 LDS-DMAs per thread); a
//   window of 4 consecutive phases always holds one stage of each half-tile, so the
//   count left in flight is the same at every phase: FJ0 + FJ1 + 4.
constexpr int P8_HT = 128 * G_BK; // f16 per A half-tile (128 rows)

// Two K depths in one launch (the QKV GEMM, §4b split-f16): columns [c_split, N) of the
// launch run K2 (> K, the B rows wrapping at kb), columns [0, c_split) run K. Their tiles
// (twice the work) come first in dispatch order, each class keeping its own XCD-aware
// order: with one workgroup per tile the hardware then hands the K tiles to the CUs the
// K2 tiles leave free (longest first).
template <class EPI, class BMAP, int FJ0 = 2, int FJ1 = 2>
__global__ __launch_bounds__(G_THREADS, 1) void gemm8p_kernel(const uint16_t *__restrict__ A, int lda, int M, int K,
                                                             int kb, BMAP bm, int N, EPI epi, int c0, int c_split,
                                                             int K2) {
	constexpr int FI = 8, FJ = FJ0 + FJ1, TM = 128, TN = 16 * FJ, BN = 4 * TN;
	constexpr int HB0 = 64 * FJ0 * G_BK, HB1 = 64 * FJ1 * G_BK; // f16 per B half-tile
	constexpr int OFF[4] = {0, P8_HT, 2 * P8_HT, 2 * P8_HT + HB0}; // Am0, Am1, Bn0, Bn1 in a buffer
	constexpr int BUFE = 2 * P8_HT + HB0 + HB1;
	constexpr int INFLIGHT = FJ0 + FJ1 + 4;
	static_assert(FJ0 >= 1 && FJ1 >= 1 && FJ0 <= 3 && FJ1 <= 3, "quadrant widths");
	extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
	const int lane = threadIdx.x & 63;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int wr = wave >> 2, wc = wave & 3;

	const int tiles_m = (M + G_BM - 1) / G_BM, tiles_n = N / BN;
	const int nwg = tiles_m * tiles_n;
	const int tn_split = c_split / BN;             // column tiles with depth K
	const int nwg2 = tiles_m * (tiles_n - tn_split); // tiles with depth K2, dispatched first
	// one tile per workgroup, or (grid smaller than the tile count) a persistent loop over
	// tiles b, b + grid, ...: the next tile's LDS-DMA prologue follows this tile's epilogue
	// stores without a workgroup exit and dispatch in between
	for (int t = blockIdx.x; t < nwg; t += gridDim.x) {
		if (EPI::NEEDS_LDS && t != (int)blockIdx.x) // the previous tile's epilogue is done with LDS
			asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); // (stores may stay in flight)
		const bool deep = t < nwg2;
		int wg = deep ? t : t - nwg2;
		{ // XCD-aware order inside the class: consecutive tiles of one XCD share A rows
			const int n = deep ? nwg2 : nwg - nwg2;
			const int q = n / 8, rr = n % 8, xcd = wg % 8, idx = wg / 8;
			wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
		}
		const int tm = wg % tiles_m, tn = wg / tiles_m + (deep ? tn_split : 0);
		const int Kt = deep ? K2 : K;
		const int row0 = tm * G_BM;
		const int colB = c0 + tn * (BN / BMAP::COLS_PER_TILE_DIV); // c0: first column of this launch

		// staging sources: instruction i of a half-tile covers its rows lr = (NI wave + i) * 8
		// + (lane >> 3), 16-byte chunk lane & 7 read from source chunk (lane & 7) ^ (lr & 7)
		// (the swizzle g16frag undoes)
		uint32_t aoff[2][2]; // [m half][i]: element offset into A
		const uint16_t *bp[2][3];
	#pragma unroll
		for (int i = 0; i < 2; ++i) {
			const int lr = (2 * wave + i) * 8 + (lane >> 3);
			const int sw = 8 * ((lane & 7) ^ (lr & 7));
			const int ra = lr < 64 ? lr : lr + 64; // Am0 tile row; Am1 = + 64
			aoff[0][i] = (uint32_t)min(row0 + ra, M - 1) * lda + sw;
			aoff[1][i] = (uint32_t)min(row0 + ra + 64, M - 1) * lda + sw;
		}
	#pragma unroll
		for (int i = 0; i < FJ0; ++i) {
			const int lr = (FJ0 * wave + i) * 8 + (lane >> 3);
			const int sw = 8 * ((lane & 7) ^ (lr & 7));
			bp[0][i] = bm.row(colB, (lr / (16 * FJ0)) * TN + lr % (16 * FJ0), kb) + sw;
		}
	#pragma unroll
		for (int i = 0; i < FJ1; ++i) {
			const int lr = (FJ1 * wave + i) * 8 + (lane >> 3);
			const int sw = 8 * ((lane & 7) ^ (lr & 7));
			bp[1][i] = bm.row(colB, (lr / (16 * FJ1)) * TN + 16 * FJ0 + lr % (16 * FJ1), kb) + sw;
		}
		// half-tile h (0 Am0, 1 Am1, 2 Bn0, 3 Bn1) of K tile kt into buffer buf
		auto stage = [&](int buf, int h, int kt) {
			const int k0 = kt * G_BK;
			const int kw = k0 < kb ? k0 : k0 - kb; // B wrap
			uint16_t *base = smem + buf * BUFE + OFF[h];
			if (h < 2) {
	#pragma unroll
				for (int i = 0; i < 2; ++i)
					__builtin_amdgcn_global_load_lds((const void *)(A + aoff[h][i] + k0),
					                                 (YALM_LDS void *)(base + (2 * wave + i) * 8 * G_BK), 16, 0, 0);
			} else if (h == 2) {
	#pragma unroll
				for (int i = 0; i < FJ0; ++i)
					__builtin_amdgcn_global_load_lds((const void *)(bp[0][i] + kw),
					                                 (YALM_LDS void *)(base + (FJ0 * wave + i) * 8 * G_BK), 16, 0, 0);
			} else {
	#pragma unroll
				for (int i = 0; i < FJ1; ++i)
					__builtin_amdgcn_global_load_lds((const void *)(bp[1][i] + kw),
					                                 (YALM_LDS void *)(base + (FJ1 * wave + i) * 8 * G_BK), 16, 0, 0);
			}
		};

		f32x4_t acc[FI][FJ];
	#pragma unroll
		for (int i = 0; i < FI; ++i)
	#pragma unroll
			for (int j = 0; j < FJ; ++j)
				acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
		half8_t a[4][2], b0[FJ0][2], b1[FJ1][2];

		const int nk = Kt / G_BK;
		// prologue = the previous iteration's stages p3 .. p8 for K tiles 0 (E) and 1 (O)
		const int k1 = nk > 1 ? 1 : 0;
		stage(0, 0, 0);
		stage(0, 2, 0);
		stage(0, 3, 0);
		stage(0, 1, 0);
		stage(1, 0, k1);
		stage(1, 2, k1);
		asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory"); // Am0, Bn0 of K tile 0
		asm volatile("s_barrier" ::: "memory");
		if (wr == 1)
			asm volatile("s_barrier" ::: "memory"); // wave row 1 runs one barrier behind

		auto rd_a = [&](int buf, int mh) {
			const uint16_t *s = smem + buf * BUFE + OFF[mh];
	#pragma unroll
			for (int i = 0; i < 4; ++i)
	#pragma unroll
				for (int ks = 0; ks < 2; ++ks)
					a[i][ks] = g16frag(s, wr * 64 + 16 * i + (lane & 15), ks, lane);
		};
		auto rd_b0 = [&](int buf) {
			const uint16_t *s = smem + buf * BUFE + OFF[2];
	#pragma unroll
			for (int j = 0; j < FJ0; ++j)
	#pragma unroll
				for (int ks = 0; ks < 2; ++ks)
					b0[j][ks] = g16frag(s, wc * 16 * FJ0 + 16 * j + (lane & 15), ks, lane);
		};
		auto rd_b1 = [&](int buf) {
			const uint16_t *s = smem + buf * BUFE + OFF[3];
	#pragma unroll
			for (int j = 0; j < FJ1; ++j)
	#pragma unroll
				for (int ks = 0; ks < 2; ++ks)
					b1[j][ks] = g16frag(s, wc * 16 * FJ1 + 16 * j + (lane & 15), ks, lane);
		};
		// {stage (or drain), barrier, MFMAs on quadrant (mh, nh), barrier}
		auto sync_stage = [&](int sbuf, int sh, int skt) {
			if (skt < nk) {
				stage(sbuf, sh, skt);
				asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
			} else {
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			}
			asm volatile("s_barrier" ::: "memory");
			__builtin_amdgcn_sched_barrier(0);
			__builtin_amdgcn_s_setprio(1);
		};
		auto sync_end = [&]() {
			__builtin_amdgcn_s_setprio(0);
			__builtin_amdgcn_sched_barrier(0);
			asm volatile("s_barrier" ::: "memory");
		};
		auto mfma_n0 = [&](int mh) {
	#pragma unroll
			for (int i = 0; i < 4; ++i)
	#pragma unroll
				for (int j = 0; j < FJ0; ++j)
	#pragma unroll
					for (int ks = 0; ks < 2; ++ks)
						acc[4 * mh + i][j] =
						    __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][ks], b0[j][ks], acc[4 * mh + i][j], 0, 0, 0);
		};
		auto mfma_n1 = [&](int mh) {
	#pragma unroll
			for (int i = 0; i < 4; ++i)
	#pragma unroll
				for (int j = 0; j < FJ1; ++j)
	#pragma unroll
					for (int ks = 0; ks < 2; ++ks)
						acc[4 * mh + i][FJ0 + j] =
						    __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][ks], b1[j][ks], acc[4 * mh + i][FJ0 + j], 0, 0, 0);
		};

		for (int it = 0;; ++it) {
			const int ke = 2 * it, ko = 2 * it + 1;
			// K tile ke from E
			rd_a(0, 0);
			rd_b0(0);
			sync_stage(1, 3, ko); // p1: Bn1 O(2i+1)
			mfma_n0(0);
			sync_end();
			rd_b1(0);
			sync_stage(1, 1, ko); // p2: Am1 O(2i+1)
			mfma_n1(0);
			sync_end();
			rd_a(0, 1);
			sync_stage(0, 0, ke + 2); // p3: Am0 E(2i+2)
			mfma_n1(1);
			sync_end();
			sync_stage(0, 2, ke + 2); // p4: Bn0 E(2i+2)
			mfma_n0(1);
			sync_end();
			if (ko >= nk)
				break;
			// K tile ko from O
			rd_a(1, 0);
			rd_b0(1);
			sync_stage(0, 3, ke + 2); // p5: Bn1 E(2i+2)
			mfma_n0(0);
			sync_end();
			rd_b1(1);
			sync_stage(0, 1, ke + 2); // p6: Am1 E(2i+2)
			mfma_n1(0);
			sync_end();
			rd_a(1, 1);
			sync_stage(1, 0, ko + 2); // p7: Am0 O(2i+3)
			mfma_n1(1);
			sync_end();
			sync_stage(1, 2, ko + 2); // p8: Bn0 O(2i+3)
			mfma_n0(1);
			sync_end();
			if (ke + 2 >= nk)
				break;
		}
		if (wr == 0)
			asm volatile("s_barrier" ::: "memory"); // rows back in step
		asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
		EPI e = epi;
		if constexpr (EPI::NEEDS_LDS)
			e.red = (float *)smem;
		const int n0 = BMAP::COLS_PER_TILE_DIV == 1 ? colB + wc * TN : colB + wc * (TN / 2);
		e.template apply<FI, FJ>(acc, row0 + wr * TM, n0, lane, wc, 4);
	}
}

template <int FJ0 = 2, int FJ1 = 2>
constexpr size_t gemm8p_lds() {
	return (size_t)2 * (2 * P8_HT + 64 * (FJ0 + FJ1) * G_BK) * sizeof(uint16_t);
}

} // namespace pf
