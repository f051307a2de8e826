// attn_wo.h — decode attention and the attention output projection (Wo +
// residual) as ONE launch, with the Wo weight stream running under the attention.
//
// In the launch path the attention kernel reads no weights: for its ~5 us HBM
// carries only the (small) KV read, and the Wo GEMV that follows starts its
// 33.5 MB stream (Mistral-7B fp16) from a cold pipe. Here one grid holds two
// kinds of workgroups:
//   * ATTENTION workgroups [0, n_kv * (S + G - 1)): attn_decode_body (attention.h), then
//     n_kv * G MERGER workgroups (attn_merge_body); the workgroup that finishes
//     a head (the single attention workgroup holding keys, or the head's merger)
//     writes each head-output element as an 8-byte
//     {value, epoch} GRANULE with ONE sc1 store into this layer's granule buffer:
//     the data is its own ready flag (MI355X_MICROARCH.md §visibility, R2
//     granule), so there is no drain (vmcnt(0)) and no separate flag store.
//     They issue no weight loads: a weight stream queued in front of the merge's
//     loads (vmcnt is in order) would hold the whole hand-off behind it.
//   * Wo workgroups [n_kv * (S + G), grid): each owns AWO_RPW contiguous Wo rows and
//     issues them as register loads at once, so the 33.5 MB stream runs while
//     the attention works. Each WAVE then gathers its input columns' granules
//     with 16-byte sc1 loads (two granules each), re-reading a batch until every
//     tag in the wave holds this launch's epoch (bounded), so a wave works as
//     soon as ITS heads are done; it dots the columns into every resident row;
//     the rows are reduced across the workgroup in a fixed order and added to
//     the residual (fused_matmul_add_residuals, infer.cu:270).
// Round 1 handed off through per-kv-head done flags (writer: drain, barrier,
// flag; reader: poll, then gather): two more serialised memory round trips.
// Workgroups dispatch in index order, so every attention workgroup is resident
// before any Wo workgroup spins, and attention never waits on Wo: no deadlock
// even when the grid is not co-resident. Tags: the epoch grows by one per
// forward and per yalm_block call and each layer has its own buffer, so a
// granule is never reset and any order of layer launches (one layer repeated, a
// forward stopped part-way) stays correct. Every spin is bounded and reports in
// *err.
//
// Geometry: Wo rows are q_dim * BYTES = KB KiB (KB in {1, 2, 4, 8}: 4 and 8 on one GPU
// at Mistral / Llama shapes, 2 and 1 for the per-rank Wo of tensor parallelism); Wo
// workgroup j owns rows [j * AWO_RPW, j * AWO_RPW + AWO_RPW) and thread t loads 16-byte
// pieces i * 256 + t of that contiguous slice (LPT = AWO_RPW * KB / 4 loads). KB >= 4: a
// thread's pieces cover every row of the slice, KB / 4 column pieces each; KB < 4: a
// 4-KiB load instruction covers RPL = 4 / KB rows, so a thread covers every RPL-th row
// at ONE column piece (256 / RPL threads per row).
//
// Outputs (round 5): x[row] = x + Wo v on one GPU; under tensor parallelism over RCCL
// the partial (+ x on rank 0) goes to out = xs for the all-reduce; over IPC each row is
// pushed to every rank's exchange slot as a {value, tag} granule (tp_exchange.h) -- the
// attention + Wo launch IS the exchange's producer, and the GLU GEMV after it the consumer.
// (Round 5 measured a CU-paired workgroup order, attention units sharing CUs with attention
// units and Wo with Wo, against this index order: the Wo stream from half the CUs lands
// later and the launch lost 1.6-2.7 us at kv 31 / 4091, profiles/r5h_awo_cu_pairing_ab.txt.)
#pragma once

#include "attention.h"
#include "device_common.h"
#include "tp_exchange.h"

#define AWO_RPW 16                   // Wo rows per Wo workgroup (256 of them for Mistral-7B)
#define AWO_TIMEOUT 200000000ull     // 2 s of s_memrealtime (100 MHz)
#define AWO_REPL_STRIDE 32           // words of the error slot (a 128-B line of its own)
#define AWO_SHORT_KV 64             // kv_len up to which fp8 decoders start the Wo slice loads at once (decoder.h)
#define AWO_TRACE_N 16               // s_memrealtime + s_memtime stamps per workgroup (yalm_attn_wo_trace)

struct AttnWoArgs {
	int n_heads, n_kv, max_seq_len, nsplit, S; // S = key splits per kv head: n_kv * (S + G - 1) attention workgroups
	int head_max;                              // head mode up to this many 64-key chunks (attention.h)
	int q_dim, dim;
	unsigned long long *part; // attention chunk partials (n_heads, nsplit, D + 2) as tagged granules
	int layer, n_layers;      // partial tag = epoch * n_layers + layer (attention.h)
	const unsigned long long *gran; // this layer's attention output (q_dim) as {value, epoch} granules
	const char *wo;     // Wo (dim, q_dim)
	float *x;           // residual stream (dim): read for the residual when add_base
	float *out;         // x (one GPU), xs (RCCL partial) -- unused when push.n > 0
	int add_base;       // out = x + Wo v (one GPU, TP rank 0) or Wo v (other TP ranks)
	TpX push;           // IPC tensor parallelism: push.n > 0 pushes the rows (tp_exchange.h)
	unsigned *err;      // error bits (bounded spin gave up)
	unsigned long long *trace; // [grid][AWO_TRACE_N] s_memrealtime stamps (YALM_ATTN_WO_TRACE=1) or null
	int delay;          // s_memrealtime ticks (10 ns) the Wo workgroups wait before their slice loads
	                    // (lets the attention's K/V and q loads reach HBM first)
};

// Eight 16-byte sc1 loads from arbitrary addresses in one statement, one vmcnt(0)
// (hipcc does not track asm loads: the statement drains its own).
// Single-copy atomicity assumption: each 16-byte load covers two 8-byte granules,
// each written by ONE 64-bit atomic store of {value, tag}. Correctness needs the
// load to see each granule whole (never the new tag with the old value). The HIP
// memory model does not promise this for a plain asm load racing an atomic store;
// gfx950 delivers it (MI355X_MICROARCH.md:190, "observed untorn on gfx950 / ROCm
// 7.2, also for 16-B sc1"), and tests/test_gpu_attn_wo.py::test_attn_wo_stress
// replays many forwards at high split counts against the separate-launch path.
__device__ __forceinline__ void awo_ld8_sc1(u32x4_t (&v)[8], const void *const (&a)[8]) {
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

// This lane's XS pieces of the attention output (EPL columns each, pieces
// ATTN_THREADS * EPL columns apart) as {value, tag} granules, gathered with
// 16-byte sc1 loads (two granules each) in batches of 8, each batch re-read until
// all its tags equal `tag` across the wave (the check that makes it correct).
// Nothing is issued before this wave's Wo slice has landed: a load samples memory
// when the memory system executes it, so one issued at launch start (behind the
// slice in the CU's queue, its result usable only once the slice is in, vmcnt
// being in order) would return a stale sample and cost a second round trip.
// First the cheap sentinel poll (one 8-byte load per lane: the last element of
// each covered head), then the gather. Round 3 measured a combined first attempt
// (gather + sentinels in one round trip) slower: 1024 waves gathering the same
// 32 KB of granules as the slices land is a burst the poll avoids
// (profiles/r3_ab_awo.txt); round 4 measured gathering first (sentinels only after a
// stale tag) slower again: fp8 kv 17 7.40 -> 8.49 us, kv 100 8.86 -> 11.68
// (profiles/r4k_decode_ab.txt). False if the bounded spin gave up (deadline,
// s_memrealtime).
// XS pieces of EPL columns each: piece k of this thread starts at column
// (piece0 + 256 k) * EPL; wpiece0 = piece0 of the wave's lane 0 (the sentinel heads).
template <int EPL, int XS>
__device__ __forceinline__ bool awo_gather_gran(float (&xs)[XS][EPL], const unsigned long long *gran, int piece0,
                                                int wpiece0, unsigned tag, unsigned long long deadline) {
	constexpr int LPP = EPL / 2;   // 16-byte loads per piece
	constexpr int NL = XS * LPP;   // 4, 8 or 16
	constexpr int NB = (NL + 7) / 8;
	constexpr int D = 128;
	constexpr int HPP = 64 * EPL / D; // heads per piece (4 or 8)
	bool alive = true;
	const int lane = threadIdx.x & 63;
	const unsigned long long *sent;
	{
		const int l = lane < XS * HPP ? lane : 0;
		const int k = l / HPP;
		const int h = (k * ATTN_THREADS + wpiece0) * EPL / D + l % HPP;
		sent = gran + (size_t)h * D + (D - 1);
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the slice has landed
	for (;;) {
		const unsigned long long g = __hip_atomic_load(sent, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (__all((unsigned)(g >> 32) == tag))
			break;
		__builtin_amdgcn_s_sleep(1);
		if (__builtin_amdgcn_s_memrealtime() > deadline) {
			alive = false;
			break;
		}
	}
#pragma unroll
	for (int bt = 0; bt < NB; ++bt) {
		const void *a[8];
#pragma unroll
		for (int i = 0; i < 8; ++i) {
			const int l = bt * 8 + (i < NL - bt * 8 ? i : 0); // pad a short batch with a repeat
			const int k = l / LPP, e = (l % LPP) * 2;
			a[i] = gran + (size_t)(k * ATTN_THREADS + piece0) * EPL + e;
		}
		u32x4_t v[8];
		for (;;) {
			awo_ld8_sc1(v, a);
			bool ok = true;
#pragma unroll
			for (int i = 0; i < 8; ++i)
				ok = ok && v[i][1] == tag && v[i][3] == tag;
			if (__all(ok) || !alive)
				break;
			__builtin_amdgcn_s_sleep(1);
			if (__builtin_amdgcn_s_memrealtime() > deadline)
				alive = false; // one more pass, then give up (results wrong, reported)
		}
#pragma unroll
		for (int i = 0; i < 8; ++i) {
			if (i < NL - bt * 8) {
				const int l = bt * 8 + i;
				const int k = l / LPP, e = (l % LPP) * 2;
				const uint32_t w0 = v[i][0], w1 = v[i][2];
				xs[k][e] = __uint_as_float(w0);
				xs[k][e + 1] = __uint_as_float(w1);
			}
		}
	}
	return alive;
}

template <class WT, int GT, int KB>
__global__ __launch_bounds__(ATTN_THREADS) void attn_wo_kernel(const float *__restrict__ q,
                                                               const uint16_t *__restrict__ kc,
                                                               const uint16_t *__restrict__ vc,
                                                               const StepState *__restrict__ step, AttnWoArgs p) {
	constexpr int D = 128;
	constexpr int EPL = WT::EPL;
	constexpr int XS = KB >= 4 ? KB / 4 : 1;   // column pieces per thread
	constexpr int RPL = KB >= 4 ? 1 : 4 / KB;  // rows per 4-KiB load instruction
	constexpr int TPR = ATTN_THREADS / RPL;    // threads per row (KB < 4)
	constexpr int LPT = AWO_RPW * KB / 4;      // 16-byte loads per thread
	static_assert(ATTN_THREADS == 256 && ATTN_WAVES == 4, "4-wave workgroups: one 4-row reduction per wave");
	static_assert(KB == 1 || KB == 2 || KB == 4 || KB == 8, "Wo rows of 1, 2, 4 or 8 KiB");
	const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int G = p.n_heads / p.n_kv;
	const int units = p.n_kv * (p.S + G - 1); // attention workgroups (head units + split units)
	const int munits = units + p.n_heads;     // + one merger per query head
	// include/yalm_hip.h yalm_attn_wo_trace: [0] start, [1] hand-off signalled / Wo slice landed, ...
	// (kept in registers, stored when the workgroup is done: see attention.h `stamp`)
	unsigned long long *tr = p.trace && tid == 0 ? p.trace + (size_t)b * AWO_TRACE_N : nullptr;
	unsigned long long t_start = 0, c_start = 0;
	if (tr) { // slot 8 (the start's shader clock) carries where the workgroup runs: HW_ID | XCC_ID << 32
		t_start = __builtin_amdgcn_s_memrealtime();
		c_start = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
		          ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
	}

	const unsigned epoch = step->epoch; // this launch's tag (step_begin_kernel / set_step_full_kernel)
	if (b < munits) { // ---- attention or merger workgroup
		const unsigned ptag = epoch * (unsigned)p.n_layers + (unsigned)p.layer;
		if (tr) { // phases this workgroup never reaches read 0, not an earlier launch's stamps
			tr[2] = tr[10] = 0;
			for (int k = 4; k < 8; ++k)
				tr[k] = tr[8 + k] = 0;
		}
		const bool wrote =
		    b < units ? attn_decode_body<D, GT, true>(b % p.n_kv, b / p.n_kv, p.S, p.head_max, q, kc, vc, step,
		                                               p.n_heads, p.n_kv, p.max_seq_len, p.nsplit, p.part, ptag,
		                                               (float *)p.gran, nullptr, epoch, tr, p.trace != nullptr)
		              : attn_merge_body<D, true>((b - units) % p.n_kv, (b - units) / p.n_kv, p.S, p.head_max, step,
		                                         p.n_heads, p.n_kv, p.max_seq_len, p.nsplit, p.part, ptag, p.err,
		                                         (float *)p.gran, nullptr, epoch, tr);
		if (tr) { // the head outputs are their own ready flags: nothing to drain or signal
			const unsigned long long t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
			tr[0] = t_start, tr[8] = c_start;
			tr[1] = wrote ? t1 : 0, tr[9] = wrote ? c1 : 0;
			tr[3] = t1, tr[11] = c1;
		}
		return;
	}

	// ---- Wo workgroup j
	__shared__ float rowpart[AWO_RPW][ATTN_WAVES];
	const int j = b - munits;
	const int row0 = j * AWO_RPW;
	// the last slice may run past the matrix: shifted back so every load stays in
	// bounds (unconditional loads); rows below row0 belong to workgroup j - 1
	const int lrow0 = min(row0, p.dim - AWO_RPW);
	const char *wbase = p.wo + (size_t)lrow0 * p.q_dim * WT::BYTES;
	// the residual rows this workgroup adds to, loaded first (nothing else in the launch
	// writes x): the read-modify-write at the end costs no load round trip
	const float xres = p.add_base ? p.x[lrow0 + (tid & (AWO_RPW - 1))] : 0.0f;
	const bool push = p.push.n > 0;
	const unsigned xg = push ? p.push.g() : 0u; // exchange index, read ahead of the stream
	if (p.delay > 0) {
		const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
		while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)p.delay)
			__builtin_amdgcn_s_sleep(2);
	}
	u32x4_t wr[LPT];
#pragma unroll
	for (int i = 0; i < LPT; ++i)
		wr[i] = load_nt16(wbase + ((size_t)i * ATTN_THREADS + tid) * 16);
	unsigned long long t_slice = 0, c_slice = 0, t_poll = 0, c_poll = 0;
	if (tr) { // tracing only: when the whole slice has landed
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		t_slice = __builtin_amdgcn_s_memrealtime(), c_slice = __builtin_amdgcn_s_memtime();
	}

	// ---- per wave: gather this lane's input columns as {value, tag} granules with
	// 16-byte sc1 loads until every tag holds this launch's epoch (each wave waits
	// only for the heads its columns cover), then dot them into every resident row.
	const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
	float xs[XS][EPL];
	const int piece0 = KB >= 4 ? tid : tid % TPR, wpiece0 = KB >= 4 ? 64 * wave : (64 * wave) % TPR;
	if (!awo_gather_gran<EPL, XS>(xs, p.gran, piece0, wpiece0, epoch, t0 + AWO_TIMEOUT) && lane == 0)
		__hip_atomic_fetch_or(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	if (tr)
		t_poll = __builtin_amdgcn_s_memrealtime(), c_poll = __builtin_amdgcn_s_memtime();
	if constexpr (KB >= 4) {
		float a0[AWO_RPW], a1[AWO_RPW];
#pragma unroll
		for (int r = 0; r < AWO_RPW; ++r) {
			a0[r] = a1[r] = 0.0f;
#pragma unroll
			for (int k = 0; k < XS; ++k)
				dot16_mix<WT>(a0[r], a1[r], wr[r * XS + k], xs[k]);
		}
		// ---- resident rows . slice; 4-row transposed wave reductions; fixed-order workgroup sum
#pragma unroll
		for (int r0 = 0; r0 < AWO_RPW; r0 += 4) {
			float acc[4];
#pragma unroll
			for (int t = 0; t < 4; ++t)
				acc[t] = a0[r0 + t] + a1[r0 + t];
			const float tot = sum4_t(acc); // lanes 16 g .. 16 g + 15: row r0 + g
			if ((lane & 15) == 0)
				rowpart[r0 + (lane >> 4)][wave] = tot;
		}
	} else {
		// load i holds row i * RPL + tid / TPR at column piece tid % TPR: per-wave totals of 4
		// loads at a time (sum4_t), then (RPL 2: two waves per row) the waves of a row in LDS
#pragma unroll
		for (int i0 = 0; i0 < LPT; i0 += 4) {
			float acc[4];
#pragma unroll
			for (int t = 0; t < 4; ++t) {
				float a0 = 0.0f, a1 = 0.0f;
				dot16_mix<WT>(a0, a1, wr[i0 + t], xs[0]);
				acc[t] = a0 + a1;
			}
			const float tot = sum4_t(acc); // lanes 16 g .. 16 g + 15: load i0 + g
			if ((lane & 15) == 0) {
				const int i = i0 + (lane >> 4);
				rowpart[i * RPL + tid / TPR][RPL == 4 ? 0 : (wave & 1)] = tot;
			}
		}
	}
	__syncthreads();
	const int row = lrow0 + tid;
	if (tid < AWO_RPW && row >= row0) {
		const float s = KB >= 4 ? (rowpart[tid][0] + rowpart[tid][1]) + (rowpart[tid][2] + rowpart[tid][3])
		                        : (RPL == 4 ? rowpart[tid][0] : rowpart[tid][0] + rowpart[tid][1]);
		if (push)
			tpx_put(p.push, xg, row, xres + s);
		else
			p.out[row] = xres + s;
	}
	if (tr) {
		tr[3] = __builtin_amdgcn_s_memrealtime(), tr[11] = __builtin_amdgcn_s_memtime();
		tr[0] = t_start, tr[8] = c_start, tr[1] = t_slice, tr[9] = c_slice, tr[2] = t_poll, tr[10] = c_poll;
		for (int k = 4; k < 8; ++k)
			tr[k] = tr[8 + k] = 0;
	}
}
