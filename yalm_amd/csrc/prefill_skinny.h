// prefill_skinny.h — the prefill's GEMMs for a SHORT prompt (T <= 64 rows: the
// CLI's prompt hydration, main.cpp:91-97 in the reference, runs T one-token
// forwards there). At small T the 256-row tiles of prefill_gemm.h leave most CUs
// idle (Llama-3B Wo / W2, N 3072: 12-16 tiles) and the GEMM is a weight stream, not
// MFMA work: every weight byte is read once, for T <= 64 rows.
//
//   skinny_gemm_kernel: split-K. Workgroup = 4 waves x 16 weight rows (64 rows of
//     B) x KC columns of K; the A rows of its K chunk (T padded to 16 MT) are staged
//     once in LDS (XOR-swizzled 16-byte chunks), the weight rows stream straight
//     into registers (lane (row r, group q) reads 16 B at k + 8 q: 16 rows x 64 B per
//     wave-instruction, U of them in flight) and feed v_mfma_f32_16x16x32_f16 with the
//     TOKENS as the A operand and the weight rows as B. Each wave leaves its f32
//     [16 MT][16] partial in part[ks][row][col].
//   skinny_reduce_kernel: per (16 rows x 16 FJ columns) wave block, the KS partials
//     summed in ks order (deterministic) into the 16x16 MFMA C layout, then the same
//     epilogue object as the large-tile GEMM (prefill_gemm.h E16*: RoPE + cache
//     write, residual add, GLU).
// Columns k >= kb of A wrap to B column k - kb (the split-f16 K / V operand); a K chunk
// never straddles kb (the host splits the k | v GEMM in 2 KS chunks of the q GEMM's size).
#pragma once

#include "prefill_gemm.h"

namespace pf {

constexpr int SK_ROWS = 64;    // B rows per workgroup (16 per wave)
constexpr int SK_U = 8;        // weight loads in flight per lane (8 x 32 k)
constexpr int SK_KSTEP = 32 * SK_U;

// lds: [16 MT][KC] f16, 16-byte chunk c of row r stored at chunk c ^ (r & 15)
template <int MT>
__device__ __forceinline__ half8_t sk_afrag(const uint16_t *lds, int KC, int row, int k) {
	const int c = (k >> 3) ^ (row & 15);
	return *(const half8_t *)(lds + (size_t)row * KC + 8 * c);
}

// A rows [0, TP) x columns [k0, k0 + KC) into LDS, 16-byte chunk c of row r at c ^ (r & 15)
// (rows past T are zeros). TP * KC <= 16384 f16 (32 KB: the host's K split) = at most
// SK_AMAX chunks per thread, all loaded before any is stored: one memory round trip.
// (A loop of load -> LDS store per chunk waited vmcnt(0) per chunk -- and for the weight
// loads issued before it: 8 serial round trips per workgroup.)
constexpr int SK_AMAX = 8;
template <int MT>
__device__ __forceinline__ void sk_stage_a(uint16_t *as, const uint16_t *__restrict__ A, int lda, int T, int k0,
                                           int KC) {
	constexpr int TP = 16 * MT;
	const int cpr = KC / 8, nch = TP * cpr, tid = threadIdx.x;
	u32x4_t v[SK_AMAX];
#pragma unroll
	for (int u = 0; u < SK_AMAX; ++u) {
		const int i = min(tid + 256 * u, nch - 1);
		const int r = i / cpr, c = i % cpr;
		v[u] = *(const u32x4_t *)(A + (size_t)min(r, T - 1) * lda + k0 + 8 * c);
	}
#pragma unroll
	for (int u = 0; u < SK_AMAX; ++u) {
		const int i = tid + 256 * u;
		if (i < nch) {
			const int r = i / cpr, c = i % cpr;
			*(u32x4_t *)(as + (size_t)r * KC + 8 * (c ^ (r & 15))) = r < T ? v[u] : u32x4_t{0u, 0u, 0u, 0u};
		}
	}
}

// C[:, c0 .. c0 + N) partials over K columns of A (row stride lda; B rows kb wide,
// wrapping), K chunks of KC: part[ks][row][c] with row stride Np (c absolute).
template <int MT, class BMAP>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(const uint16_t *__restrict__ A, int lda, int T, int K,
                                                          int kb, BMAP bm, int N, int KC, int c0, int Np,
                                                          float *__restrict__ part) {
	extern __shared__ __attribute__((aligned(16))) uint16_t as[];
	const int nblk = N / SK_ROWS;
	const int nb = blockIdx.x % nblk, ks = blockIdx.x / nblk;
	const int k0 = ks * KC;
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	constexpr int TP = 16 * MT;
	// ---- this wave's 16 weight rows (through the row policy: plain / QKV segments / GLU)
	const int cb = c0 + nb * SK_ROWS;           // the workgroup's first B row index (output column)
	const int col = cb + 16 * wave;              // the wave's
	const int kw0 = k0 < kb ? k0 : k0 - kb;      // B wrap (a K chunk never straddles kb)
	// row policy: tile base = first output column (plain) or first hidden column (GLU:
	// 64 B rows = 32 W1 rows then the same 32 W3 rows, BRowsGlu<64>)
	const uint16_t *wrow =
	    bm.row(cb / BMAP::COLS_PER_TILE_DIV, 16 * wave + (lane & 15), kb) + kw0 + 8 * (lane >> 4);
	// ---- the weight stream: a ring of SK_U 16-byte loads per lane (32 K columns each),
	// the first SK_U issued before the A chunk is staged; every consumed slot is refilled
	// SK_U steps ahead, unconditionally (past the chunk it re-reads step 0, an L2 hit:
	// a conditional refill makes hipcc drain vmcnt to 0 before every load). Round 4's
	// first cut loaded SK_U steps, waited, computed, loaded the next SK_U: one full
	// memory latency per 256 K columns (Mistral T = 1 prefill: 3.8 TB/s).
	const int nst = KC / 32;
	half8_t b[SK_U];
#pragma unroll
	for (int u = 0; u < SK_U; ++u)
		b[u] = __builtin_bit_cast(half8_t, load_nt16(wrow + 32 * (u < nst ? u : 0)));
	sk_stage_a<MT>(as, A, lda, T, k0, KC);
	__syncthreads();
	f32x4_t acc[MT];
#pragma unroll
	for (int m = 0; m < MT; ++m)
		acc[m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
	for (int j0 = 0; j0 < nst; j0 += SK_U) {
#pragma unroll
		for (int u = 0; u < SK_U; ++u) {
			const int j = j0 + u;
			if (j < nst) {
#pragma unroll
				for (int m = 0; m < MT; ++m) {
					const half8_t a = sk_afrag<MT>(as, KC, 16 * m + (lane & 15), 32 * j + 8 * (lane >> 4));
					acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[u], acc[m], 0, 0, 0);
				}
			}
			b[u] = __builtin_bit_cast(half8_t, load_nt16(wrow + 32 * (j + SK_U < nst ? j + SK_U : 0)));
		}
	}
	// ---- partial: element r of acc[m] is row 16 m + 4 (lane >> 4) + r, column col + (lane & 15)
	float *pp = part + (size_t)ks * TP * Np;
#pragma unroll
	for (int m = 0; m < MT; ++m)
#pragma unroll
		for (int r = 0; r < 4; ++r)
			pp[(size_t)(16 * m + crow16(r, lane)) * Np + col + (lane & 15)] = acc[m][r];
}

// The same partials with the weight rows staged through LDS by LDS-DMA, so every
// wave-instruction reads 4 rows x 256 contiguous bytes (skinny_gemm_kernel's register
// loads read 16 rows x 64 B per instruction: half cache lines, 16 DRAM rows at once).
// Each wave owns its 16 weight rows in a 3-stage ring of 128-column stages (4 KB per
// wave per stage): no workgroup barrier in the loop, one counted vmcnt per stage. The
// 16-byte chunks of a row are XOR-swizzled by the row (source side of the DMA) so the
// MFMA B-fragment reads (16 rows x one chunk) spread over the banks. LDS: the A chunk
// (<= 32 KB) + 48 KB of ring: two workgroups per CU.
constexpr int SKL_KS = 128;                    // K columns per stage
constexpr int SKL_NS = 3;                      // ring stages
constexpr int SKL_STAGE = SK_ROWS * SKL_KS;    // f16 per stage (16 KB)
constexpr size_t SKL_RING_BYTES = (size_t)SKL_NS * SKL_STAGE * 2;

template <int MT, class BMAP>
__global__ __launch_bounds__(256) void skinny_gemm_lds_kernel(const uint16_t *__restrict__ A, int lda, int T, int K,
                                                              int kb, BMAP bm, int N, int KC, int c0, int Np,
                                                              float *__restrict__ part) {
	extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
	constexpr int TP = 16 * MT;
	uint16_t *const as = sm;                                      // [TP][KC], swizzled as skinny_gemm_kernel
	uint16_t *const ring = sm + (size_t)TP * KC;                  // [SKL_NS][64 rows][SKL_KS]
	const int nblk = N / SK_ROWS;
	const int nb = blockIdx.x % nblk, ks = blockIdx.x / nblk;
	const int k0 = ks * KC;
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
	const int cb = c0 + nb * SK_ROWS;      // the workgroup's first B row (output column)
	const int col = cb + 16 * wave;        // the wave's
	const int kw0 = k0 < kb ? k0 : k0 - kb; // B wrap (a K chunk never straddles kb)
	const int nst = KC / SKL_KS;
	// DMA geometry: instruction i of a stage covers the wave's rows 4 i .. 4 i + 3, lane
	// l row 4 i + (l >> 4), LDS slot l & 15 <- source chunk (l & 15) ^ row
	const uint16_t *src[4];
#pragma unroll
	for (int i = 0; i < 4; ++i) {
		const int rr = 4 * i + (lane >> 4);
		src[i] = bm.row(cb / BMAP::COLS_PER_TILE_DIV, 16 * wave + rr, kb) + kw0 + 8 * ((lane & 15) ^ rr);
	}
	uint16_t *const wring = ring + wave * 16 * SKL_KS; // this wave's rows in every stage
	auto issue = [&](int st) { // stage st (clamped: past the chunk it re-reads the last stage, an L2 hit)
		const int sc = st < nst ? st : nst - 1;
		uint16_t *dst = wring + (st % SKL_NS) * SKL_STAGE;
#pragma unroll
		for (int i = 0; i < 4; ++i)
			__builtin_amdgcn_global_load_lds((const void *)(src[i] + sc * SKL_KS),
			                                 (YALM_LDS void *)(dst + 4 * i * SKL_KS), 16, 0, 0);
	};
	issue(0);
	issue(1);
	sk_stage_a<MT>(as, A, lda, T, k0, KC);
	__syncthreads();
	f32x4_t acc[MT];
#pragma unroll
	for (int m = 0; m < MT; ++m)
		acc[m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
	const int n = lane & 15, q = lane >> 4;
	for (int st = 0; st < nst; ++st) {
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // stage st - 1's B reads are done...
		issue(st + 2); // ...before its slot is re-staged
		asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); // stage st landed (2 stages x 4 behind it)
		const uint16_t *bst = wring + (st % SKL_NS) * SKL_STAGE + n * SKL_KS;
#pragma unroll
		for (int j = 0; j < SKL_KS / 32; ++j) {
			const half8_t b = *(const half8_t *)(bst + 8 * ((4 * j + q) ^ n));
#pragma unroll
			for (int m = 0; m < MT; ++m) {
				const half8_t a = sk_afrag<MT>(as, KC, 16 * m + n, st * SKL_KS + 32 * j + 8 * q);
				acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[m], 0, 0, 0);
			}
		}
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the clamped tail stages, before the wave exits
	float *pp = part + (size_t)ks * TP * Np;
#pragma unroll
	for (int m = 0; m < MT; ++m)
#pragma unroll
		for (int r = 0; r < 4; ++r)
			pp[(size_t)(16 * m + crow16(r, lane)) * Np + col + n] = acc[m][r];
}

// One wave per (16 rows, 16 FJ columns) block of C: the KS partials summed
// in ks order, then epi.apply<1, FJ>(acc, row0, n0, ...) exactly as the large-tile GEMM's
// epilogue sees its fragments. n0: the block's first output column, or (GLU) its first
// hidden column (BRowsGlu: 16 FJ B rows = 8 FJ W1 rows then the same 8 FJ W3 rows).
// Columns < c_split sum KS partial slots, the others KS2 (the QKV buffer: the k | v
// GEMM ran 2 KS K chunks).
template <int FJ, bool GLU, class EPI>
__global__ __launch_bounds__(256) void skinny_reduce_kernel(const float *__restrict__ part, int KS, int KS2,
                                                            int c_split, int TP, int T, int N, EPI epi) {
	const int lane = threadIdx.x & 63;
	const int gw = blockIdx.x * 4 + (threadIdx.x >> 6); // global wave = block (row tile, col block)
	const int ncb = N / (16 * FJ);
	const int rt = gw / ncb, cb = gw % ncb;
	if (rt * 16 >= T)
		return;
	const int nks = cb * 16 * FJ < c_split ? KS : KS2;
	// the KS partials of this lane's 4 FJ values: all 4 FJ loads of 4 consecutive ks in
	// flight at once, summed in ks order (deterministic; round 4's first cut ran one serial
	// chain of KS dependent loads per value: 27 us per Wo / W2 reduce at T = 1)
	f32x4_t acc[1][FJ];
	size_t off[FJ][4];
#pragma unroll
	for (int j = 0; j < FJ; ++j) {
		acc[0][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
		for (int r = 0; r < 4; ++r)
			off[j][r] = (size_t)(16 * rt + crow16(r, lane)) * N + cb * 16 * FJ + 16 * j + (lane & 15);
	}
	const size_t kstride = (size_t)TP * N;
	int ks = 0;
	for (; ks + 4 <= nks; ks += 4) {
		float v[4][FJ][4];
#pragma unroll
		for (int q = 0; q < 4; ++q)
#pragma unroll
			for (int j = 0; j < FJ; ++j)
#pragma unroll
				for (int r = 0; r < 4; ++r)
					v[q][j][r] = part[(size_t)(ks + q) * kstride + off[j][r]];
#pragma unroll
		for (int q = 0; q < 4; ++q)
#pragma unroll
			for (int j = 0; j < FJ; ++j)
#pragma unroll
				for (int r = 0; r < 4; ++r)
					acc[0][j][r] += v[q][j][r];
	}
	for (; ks < nks; ++ks) {
#pragma unroll
		for (int j = 0; j < FJ; ++j)
#pragma unroll
			for (int r = 0; r < 4; ++r)
				acc[0][j][r] += part[(size_t)ks * kstride + off[j][r]];
	}
	const int n0 = GLU ? cb * 8 * FJ : cb * 16 * FJ;
	epi.template apply<1, FJ>(acc, 16 * rt, n0, lane, 0, 1);
}

} // namespace pf
