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
//     a workgroup barrier and stores the launch epoch (StepState::epoch) into
//     every replica of kv head g's done flag (one wave instruction, 8 lanes, sc1
//     stores). They issue no weight loads: a
//     weight stream queued in front of the merge's loads (vmcnt is in order)
//     would hold the whole hand-off behind it.
//   * Wo workgroups [n_kv * S, grid): each owns AWO_RPW contiguous Wo rows and
//     issues them as register loads at once, so the 33.5 MB stream runs while
//     the attention works. Each WAVE then takes its input pieces in turn: its
//     lane 0 polls the XCD replica of the done flag of every kv head the
//     piece's columns cover until it holds this launch's epoch (sc1 loads,
//     bounded), the wave gathers the piece with 16-byte sc1 loads and dots it
//     into every resident row (MI355X_MICROARCH.md §visibility, "Valid forms"
//     row 1: one flag per producer, kept in R = 8 replicas on lines of their
//     own), so a wave works as soon as ITS
//     heads are done; then the rows are reduced across the workgroup in a
//     fixed order and added to the residual (fused_matmul_add_residuals,
//     infer.cu:270).
// Workgroups dispatch in index order, so every attention workgroup is resident
// before any Wo workgroup spins, and attention never waits on Wo: no deadlock
// even when the grid is not co-resident. Flags: one slot of n_kv x 8 replicas
// per layer, each holding the epoch of the last launch that finished that kv
// head. The epoch grows by one per forward and per yalm_block call, so a flag
// is never reset and any order of layer launches (one layer repeated, a forward
// stopped part-way) stays correct; there is no in-launch reset ticket either (a
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
	unsigned *done;     // this layer's per-kv-head done flags: [n_kv][AWO_REPL replicas, AWO_REPL_STRIDE words apart]
	unsigned *err;      // error bits (bounded spin gave up)
	unsigned long long *trace; // [grid][4] s_memrealtime stamps (YALM_ATTN_WO_TRACE=1) or null
	int win;            // Wo loads in flight per lane: 0 = all at once, 8 / 16 / 24 (YALM_ATTN_WO_WIN);
	                    // -1 = no weight loads (YALM_ABLATE bit 32, timing only: results wrong)
	int delay;          // s_memrealtime ticks (10 ns) the Wo workgroups wait before their slice loads
	                    // (YALM_ATTN_WO_DELAY, tuning knob: lets the attention chain start alone)
};

// Gather this lane's XS pieces of the attention output (EPL floats each, pieces
// 256 * EPL floats apart) with 16-byte sc1 loads -- the hand-off's load form
// (4- or 16-byte sc1 loads). 4-byte loads at a 32-byte lane stride made every
// wave instruction request 16 lines for 256 useful bytes, 8 times over, from all
// 256 Wo workgroups at once. hipcc does not track asm loads: one statement issues
// them all and drains vmcnt (the weight slice has landed by then anyway).
template <int EPL, int XS>
__device__ __forceinline__ void awo_gather(float (&xs)[XS][EPL], const float *src) {
	constexpr int NL = XS * EPL / 4; // 16-byte loads per lane: 2, 4 or 8
	static_assert(NL == 2 || NL == 4 || NL == 8, "EPL * XS in {8, 16, 32}");
	constexpr int LPP = EPL / 4;      // loads per piece
	const float *a[8];
#pragma unroll
	for (int i = 0; i < NL; ++i)
		a[i] = src + (size_t)(i / LPP) * ATTN_THREADS * EPL + (i % LPP) * 4;
	u32x4_t v[8];
	if constexpr (NL == 2) {
		asm volatile("global_load_dwordx4 %0, %2, off sc1\n\t"
		             "global_load_dwordx4 %1, %3, off sc1\n\t"
		             "s_waitcnt vmcnt(0)"
		             : "=&v"(v[0]), "=&v"(v[1])
		             : "v"(a[0]), "v"(a[1])
		             : "memory");
	} else if constexpr (NL == 4) {
		asm volatile("global_load_dwordx4 %0, %4, off sc1\n\t"
		             "global_load_dwordx4 %1, %5, off sc1\n\t"
		             "global_load_dwordx4 %2, %6, off sc1\n\t"
		             "global_load_dwordx4 %3, %7, off sc1\n\t"
		             "s_waitcnt vmcnt(0)"
		             : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
		             : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
		             : "memory");
	} else {
		asm volatile("global_load_dwordx4 %0, %8, off sc1\n\t"
		             "global_load_dwordx4 %1, %9, off sc1\n\t"
		             "global_load_dwordx4 %2, %10, off sc1\n\t"
		             "global_load_dwordx4 %3, %11, off sc1\n\t"
		             "global_load_dwordx4 %4, %12, off sc1\n\t"
		             "global_load_dwordx4 %5, %13, off sc1\n\t"
		             "global_load_dwordx4 %6, %14, off sc1\n\t"
		             "global_load_dwordx4 %7, %15, off sc1\n\t"
		             "s_waitcnt vmcnt(0)"
		             : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
		               "=&v"(v[7])
		             : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7])
		             : "memory");
	}
#pragma unroll
	for (int i = 0; i < NL * 4; ++i) {
		const uint32_t w = v[i / 4][i % 4];
		xs[i / EPL][i % EPL] = __uint_as_float(w);
	}
}

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
	if (tr) // [0] start, [1] hand-off signalled / Wo slice landed, [2] poll passed, [3] end
		tr[0] = __builtin_amdgcn_s_memrealtime(), tr[1] = tr[2] = tr[3] = 0;

	const unsigned epoch = step->epoch; // this launch's tag (step_begin_kernel / set_step_full_kernel)
	if (b < units) { // ---- attention workgroup
		const bool wrote = attn_decode_body<D, GT, true>(true, b % p.n_kv, b / p.n_kv, p.S, q, kc, vc, step,
		                                                 p.n_heads, p.n_kv, p.max_seq_len, p.nsplit, p.part,
		                                                 p.counters, p.att, nullptr, [] {});
		if (wrote) {
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // every storing wave drains its sc1 stores
			__syncthreads();
			if (tid < AWO_REPL) // kv head b % n_kv done: one wave instruction, one lane per replica
				__hip_atomic_store(&p.done[(b % p.n_kv) * AWO_HEAD + tid * AWO_REPL_STRIDE], epoch, __ATOMIC_RELAXED,
				                   __HIP_MEMORY_SCOPE_AGENT);
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
	if (p.delay > 0) {
		const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
		while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)p.delay)
			__builtin_amdgcn_s_sleep(2);
	}
	u32x4_t wr[LPT];
	// p.win > 0: at most win loads in flight per lane (a sliding window), so the
	// slice does not fill the CU's memory queues ahead of the attention's loads
#pragma unroll
	for (int i = 0; i < LPT; ++i) {
		if (i >= 8) {
			if (p.win == 8)
				asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
			else if (p.win == 16 && i >= 16)
				asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
			else if (p.win == 24 && i >= 24)
				asm volatile("s_waitcnt vmcnt(23)" ::: "memory");
		}
		wr[i] = p.win >= 0 ? load_nt16(wbase + ((size_t)i * ATTN_THREADS + tid) * 16) : u32x4_t{0u, 0u, 0u, 0u};
	}
	if (tr) { // tracing only: when the whole slice has landed
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		tr[1] = __builtin_amdgcn_s_memrealtime();
	}

	// ---- per wave: wait for every kv head its input pieces cover (piece k's 64 * EPL
	// columns span q heads e0 / D .. and kv groups / G), then gather all pieces at
	// once with 16-byte sc1 loads (one round trip) and dot them into every resident
	// row. The polling lane's wave loads only after its polls matched
	// (MI355X_MICROARCH.md §visibility "Valid forms" row 2).
	const int G = p.n_heads / p.n_kv;
	const int rep = (b % AWO_REPL) * AWO_REPL_STRIDE;
	if (lane == 0) {
		const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
		bool dead = false;
#pragma unroll
		for (int k = 0; k < XS; ++k) {
			const int e0 = (k * ATTN_THREADS + 64 * wave) * EPL;
			const int g_lo = e0 / D / G, g_hi = (e0 + 64 * EPL - 1) / D / G;
			for (int g = g_lo; g <= g_hi && !dead; ++g) {
				const unsigned *c = p.done + g * AWO_HEAD + rep;
				while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
					__builtin_amdgcn_s_sleep(1);
					if (__builtin_amdgcn_s_memrealtime() - t0 > AWO_TIMEOUT) {
						__hip_atomic_fetch_or(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
						dead = true;
						break;
					}
				}
			}
		}
	}
	if (tr)
		tr[2] = __builtin_amdgcn_s_memrealtime();
	float xs[XS][EPL];
	awo_gather<EPL, XS>(xs, p.att + (size_t)tid * EPL);
	float a0[AWO_RPW], a1[AWO_RPW];
#pragma unroll
	for (int r = 0; r < AWO_RPW; ++r) {
		a0[r] = a1[r] = 0.0f;
#pragma unroll
		for (int k = 0; k < XS; ++k)
			eng_dot16<WT>(a0[r], a1[r], wr[r * XS + k], xs[k]);
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
