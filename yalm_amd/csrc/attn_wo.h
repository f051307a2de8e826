// attn_wo.h — decode attention and the attention output projection (Wo +
// residual) as ONE launch, with the Wo weight stream running under the attention.
//
// In the launch path the attention kernel reads no weights: for its ~5 us HBM
// carries only the (small) KV read, and the Wo GEMV that follows starts its
// 33.5 MB stream (Mistral-7B fp16) from a cold pipe. Here one grid holds two
// kinds of workgroups:
//   * ATTENTION workgroups [0, n_kv * S): attn_decode_body (attention.h) with
//     write-through (sc1) head outputs; the workgroup that finishes kv head g
//     (single-chunk writer or last arriver) drains its stores (vmcnt(0)), joins
//     a workgroup barrier and adds 1 to every replica of kv head g's done
//     counter (one wave instruction, 8 lanes). They issue no weight loads: a
//     weight stream queued in front of the merge's loads (vmcnt is in order)
//     would hold the whole hand-off behind it.
//   * Wo workgroups [n_kv * S, grid): each owns AWO_RPW contiguous Wo rows and
//     issues them as register loads at once, so the 33.5 MB stream runs while
//     the attention works. Each WAVE then takes its input pieces in turn: its
//     lane 0 polls the XCD replica of the done counter of every kv head the
//     piece's columns cover (sc1 loads, bounded), the wave gathers the piece
//     with 4-byte sc1 loads and dots it into every resident row
//     (MI355X_MICROARCH.md §visibility, "Valid forms" row 2: counters kept in
//     R = 8 replicas on lines of their own), so a wave works as soon as ITS
//     heads are done; then the rows are reduced across the workgroup in a
//     fixed order and added to the residual (fused_matmul_add_residuals,
//     infer.cu:270).
// Workgroups dispatch in index order, so every attention workgroup is resident
// before any Wo workgroup spins, and attention never waits on Wo: no deadlock
// even when the grid is not co-resident. Counters: one slot of n_kv x 8
// replicas per layer; layer l's launch zeroes layer l - 1's slot (finished, next used one
// token later; n_layers >= 2), so there is no in-launch reset ticket (a
// returning atomic from every workgroup costs ~6 us of serialised fan-in,
// MI355X_MICROARCH.md row fanin). Every spin is bounded and reports in *err.
//
// Geometry: Wo rows are q_dim * BYTES = XS * 4 KB (XS in {1, 2}); Wo workgroup
// j owns rows [j * AWO_RPW, j * AWO_RPW + AWO_RPW) and thread t loads 16-byte
// pieces i * 256 + t of that contiguous slice (LPT = AWO_RPW * XS loads).
#pragma once

#include "attention.h"
#include "engine.h"

#define AWO_RPW 16                   // Wo rows per Wo workgroup (256 of them for Mistral-7B)
#define AWO_TIMEOUT 200000000ull     // 2 s of s_memrealtime (100 MHz)
#define AWO_REPL 8                   // done-counter replicas (one per XCD)
#define AWO_REPL_STRIDE 32           // words between replicas (128-B lines of their own)
#define AWO_HEAD (AWO_REPL * AWO_REPL_STRIDE) // words per kv head's counter; a layer slot is n_kv of them

struct AttnWoArgs {
	int n_heads, n_kv, max_seq_len, nsplit, S; // S = key-chunk splits per kv head: n_kv * S attention workgroups
	int q_dim, dim;
	float *part;        // attention chunk partials (n_heads, nsplit, D + 2)
	unsigned *counters; // per-kv-head arrival tickets (attention.h)
	float *att;         // attention output (q_dim), written sc1
	const char *wo;     // Wo (dim, q_dim)
	float *x;           // residual stream (dim)
	unsigned *done;     // this layer's per-kv-head counters: [n_kv][AWO_REPL replicas, AWO_REPL_STRIDE words apart]
	unsigned *prev;     // the previous layer's counters (zeroed here)
	unsigned *err;      // error bits (bounded spin gave up)
	unsigned long long *trace; // [grid][4] s_memrealtime stamps (YALM_ATTN_WO_TRACE=1) or null
};

template <class WT, int GT, int XS>
__global__ __launch_bounds__(ATTN_THREADS) void attn_wo_kernel(const float *__restrict__ q,
                                                               const uint16_t *__restrict__ kc,
                                                               const uint16_t *__restrict__ vc,
                                                               const StepState *__restrict__ step, AttnWoArgs p) {
	constexpr int D = 128;
	constexpr int EPL = WT::EPL;
	constexpr int LPT = AWO_RPW * XS;
	static_assert(ATTN_THREADS == 256 && ATTN_WAVES == 4, "4-wave workgroups: one 4-row reduction per wave");
	const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int units = p.n_kv * p.S;
	unsigned long long *tr = p.trace && tid == 0 ? p.trace + (size_t)b * 4 : nullptr;
	if (tr) // [0] start, [1] hand-off signalled / Wo slice issued, [2] poll passed, [3] end
		tr[0] = __builtin_amdgcn_s_memrealtime(), tr[1] = tr[2] = tr[3] = 0;

	if (b < units) { // ---- attention workgroup
		const bool wrote = attn_decode_body<D, GT, true>(true, b % p.n_kv, b / p.n_kv, p.S, q, kc, vc, step,
		                                                 p.n_heads, p.n_kv, p.max_seq_len, p.nsplit, p.part,
		                                                 p.counters, p.att, nullptr, [] {});
		if (wrote) {
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // every storing wave drains its sc1 stores
			__syncthreads();
			if (tid < AWO_REPL) // kv head b % n_kv done: one wave instruction, one lane per replica
				__hip_atomic_fetch_add(&p.done[(b % p.n_kv) * AWO_HEAD + tid * AWO_REPL_STRIDE], 1u,
				                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			if (tr)
				tr[1] = __builtin_amdgcn_s_memrealtime();
		}
		if (tr)
			tr[3] = __builtin_amdgcn_s_memrealtime();
		return;
	}

	// ---- Wo workgroup j
	__shared__ float rowpart[AWO_RPW][ATTN_WAVES];
	const int j = b - units;
	const int row0 = j * AWO_RPW;
	// the last slice may run past the matrix: shifted back so every load stays in
	// bounds (unconditional loads); rows below row0 belong to workgroup j - 1
	const int lrow0 = min(row0, p.dim - AWO_RPW);
	const char *wbase = p.wo + (size_t)lrow0 * p.q_dim * WT::BYTES;
	u32x4_t wr[LPT];
#pragma unroll
	for (int i = 0; i < LPT; ++i)
		wr[i] = load_nt16(wbase + ((size_t)i * ATTN_THREADS + tid) * 16);
	if (j == 0 && tid < p.n_kv * AWO_REPL) // previous layer's counters: done, next used one token later
		p.prev[tid * AWO_REPL_STRIDE] = 0u;
	if (tr)
		tr[1] = __builtin_amdgcn_s_memrealtime();

	// ---- per wave and input piece k: wait for the kv heads whose outputs the piece covers
	// (its 64 * EPL columns span q heads e0 / D .. and kv groups / G), gather it with
	// 4-byte sc1 loads, dot it into every resident row. The polling lane's wave loads
	// only after the poll matched (MI355X_MICROARCH.md §visibility "Valid forms" row 2).
	const int G = p.n_heads / p.n_kv;
	const int rep = (b % AWO_REPL) * AWO_REPL_STRIDE;
	float a0[AWO_RPW], a1[AWO_RPW];
#pragma unroll
	for (int r = 0; r < AWO_RPW; ++r)
		a0[r] = a1[r] = 0.0f;
#pragma unroll
	for (int k = 0; k < XS; ++k) {
		const int e0 = (k * ATTN_THREADS + 64 * wave) * EPL;
		const int g_lo = e0 / D / G, g_hi = (e0 + 64 * EPL - 1) / D / G;
		if (lane == 0) {
			for (int g = g_lo; g <= g_hi; ++g) {
				const unsigned *c = p.done + g * AWO_HEAD + rep;
				const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
				while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
					__builtin_amdgcn_s_sleep(1);
					if (__builtin_amdgcn_s_memrealtime() - t0 > AWO_TIMEOUT) {
						__hip_atomic_fetch_or(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
						break;
					}
				}
			}
		}
		if (tr && k == XS - 1)
			tr[2] = __builtin_amdgcn_s_memrealtime();
		float xk[EPL];
		const float *src = p.att + (size_t)(k * ATTN_THREADS + tid) * EPL;
#pragma unroll
		for (int e = 0; e < EPL; ++e)
			xk[e] = eng_ld_sc1(src + e);
#pragma unroll
		for (int r = 0; r < AWO_RPW; ++r)
			eng_dot16<WT>(a0[r], a1[r], wr[r * XS + k], xk);
	}
	// ---- resident rows . slice; 4-row transposed wave reductions; fixed-order workgroup sum
#pragma unroll
	for (int r0 = 0; r0 < AWO_RPW; r0 += 4) {
		float acc[4];
#pragma unroll
		for (int t = 0; t < 4; ++t)
			acc[t] = a0[r0 + t] + a1[r0 + t];
		const float tot = eng_sum4_t(acc); // lanes 16 g .. 16 g + 15: row r0 + g
		if ((lane & 15) == 0)
			rowpart[r0 + (lane >> 4)][wave] = tot;
	}
	__syncthreads();
	const int row = lrow0 + tid;
	if (tid < AWO_RPW && row >= row0) {
		const float s = (rowpart[tid][0] + rowpart[tid][1]) + (rowpart[tid][2] + rowpart[tid][3]);
		p.x[row] += s;
	}
	if (tr)
		tr[3] = __builtin_amdgcn_s_memrealtime();
}
