// attention.h — split-KV ("flash-decode") grouped-query attention for one
// token over the fp16 sliding-window KV cache, wave64-native, one launch.
//
// Replaces attn_dot / attn_softmax / att_mix (infer.cu:338-524: three launches,
// 32-lane layout, each K/V row re-read once per query head). One workgroup
// (4 waves) owns (kv head g, key chunk s of CHUNK rows): every K and V row of
// the chunk is read from HBM exactly once and serves all G = n_heads /
// n_kv_heads query heads of the group. Semantics follow the CPU oracle attn
// (infer.cpp:216-248):  s_t = (q . k_t) / sqrt(head_dim);  p = softmax(s);
// out = sum_t p_t v_t.
//
// Decode attention is latency-bound, so the kernel is built around round
// trips: K/V rows are read as 16-byte pieces (D/8 lanes per row); the
// cross-lane sums go through LDS (shuffles lower to serialised ds_bpermute
// round trips on gfx950) and the softmax reductions use DPP; chunks are
// small (64 keys) so the KV read spreads over many CUs, and the q and first
// K/V chunk loads of the per-head workgroups are issued speculatively before
// kv_len is known (rows past kv_len are read but masked), overlapping the
// step-state load.
//  * Short contexts (<= ATTN_HEAD_MAX chunks, "head mode"): one workgroup per
//    query head runs all the keys and writes the head directly.
//  * Longer contexts ("key mode"): the keys are split over S key splits per kv
//    head; each split publishes per head (max, sum, unnormalised out) as 8-byte
//    {value, tag} granules (one sc1 store each: the data is its own ready flag,
//    MI355X_MICROARCH.md §visibility R2), and one MERGER workgroup per query head,
//    dispatched after every attention workgroup of the launch, gathers them,
//    re-reading until every tag holds this launch's tag, and folds them in a
//    fixed order (deterministic). Tags: epoch * n_layers + layer, unique per
//    (forward, layer), so the one partial buffer serves every layer and is never
//    reset. Round 2 used a drained write + agent-scope arrival ticket +
//    last-arriver merge: three serialised round trips instead of one.
#pragma once

#include <float.h>

#include <type_traits>

#include "device_common.h"

#define ATTN_THREADS 256
#define ATTN_SPLITS 32     // key-chunk splits (workgroups) per kv head
#define ATTN_MAX_SPLITS 64 // the merger gathers one partial per lane
#define ATTN_HEAD_MAX 4    // head mode up to this many 64-key chunks (attn_decode_body)
#define ATTN_WAVES (ATTN_THREADS / YALM_WAVE)

// Keys per workgroup. Small on purpose: one CU streams only ~50-100 GB/s, so
// a decode-size KV read must be spread over many CUs to be fast (kv 4096 ->
// 64 chunks x n_kv_heads workgroups); the merge is a cheap sc1 hand-off.
template <int D>
constexpr int attn_chunk() {
	return 64;
}

// K / V rows per lane per chunk: lane (row group, piece) covers 8 dims of every
// (4 waves x 64 / (D / 8))-th row of the chunk
template <int D>
constexpr int attn_nk() {
	return attn_chunk<D>() / (ATTN_WAVES * (64 / (D / 8))) > 0 ? attn_chunk<D>() / (ATTN_WAVES * (64 / (D / 8))) : 1;
}

// One lane's K / V rows of a 64-key chunk through buffer resources: the per-lane byte
// offsets (row group, piece) are fixed voffsets; each chunk gets its OWN descriptor pair,
// built in SGPRs: base = the cache + t0 rows, num_records = the chunk's rows inside the
// cache (0 when the chunk is not live), so a dead load moves no data and the rows of a
// partial final chunk past max_seq_len read as zeros through voffset alone. Round 4 put
// the chunk in soffset of one whole-cache descriptor and relied on the range check
// covering soffset; tools/soffset_probe.hip shows gfx950 does check voffset + soffset
// (profiles/r5_soffset_probe.txt: soffset = num_records reads zero), so that form read
// nothing past the allocation either -- but its num_records (max_seq_len x row bytes)
// wrapped at 4 GiB, and the per-chunk descriptor needs neither the
// undocumented rule nor 32-bit cache sizes: num_records covers at most 64 rows.
// Round 4 first used flat loads at per-chunk 64-bit addresses: their address temporaries
// re-used the registers of the previous chunk's loads, and hipcc drained vmcnt to 0 at
// every chunk-loop iteration -- the next chunk's loads waited for the prefetch (one load
// latency per two chunks). The descriptors are scalar, so that does not come back.
template <int D>
struct KvRows {
	static constexpr int LPK = D / 8, KPW = 64 / LPK, RSTEP = (ATTN_THREADS / 64) * KPW;
	static constexpr int NK = attn_nk<D>();
	const char *kb, *vb;
	uint32_t rowb, msl; // bytes per cache row, rows per layer (max_seq_len)
	uint32_t voff[NK];
	__device__ __forceinline__ KvRows(const uint16_t *kc, const uint16_t *vc, int n_kv_heads, int max_seq_len, int g) {
		const int lane = threadIdx.x & 63;
		const int tl0 = (threadIdx.x >> 6) * KPW + lane / LPK, piece = lane % LPK;
		// descriptor inputs made provably wave-uniform (readfirstlane): otherwise hipcc wraps
		// each buffer load in a waterfall loop (cdna_hip_programming.md T20)
		auto uni = [](const uint16_t *p) {
			const uint64_t a = (uint64_t)p;
			const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
			const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
			return (const char *)(((uint64_t)hi << 32) | lo);
		};
		rowb = (uint32_t)__builtin_amdgcn_readfirstlane(n_kv_heads * D * 2);
		msl = (uint32_t)__builtin_amdgcn_readfirstlane(max_seq_len);
		kb = uni(kc);
		vb = uni(vc);
#pragma unroll
		for (int i = 0; i < NK; ++i)
			voff[i] = (uint32_t)(tl0 + i * RSTEP) * rowb + (uint32_t)(g * D + piece * 8) * 2;
	}
	// the chunk at row t0 (nothing when !live)
	__device__ __forceinline__ void load(int t0, bool live, u32x4_t (&kw)[NK], u32x4_t (&vw)[NK]) const {
		// wave-uniform (T20); t0 and live must come from scalar values (attn_core keeps its
		// chunk loop in SGPRs): a VALU select here took a register of the previous chunk's
		// loads and cost a vmcnt(0) per chunk. Branch-free scalar arithmetic: a 64-bit compare
		// here became scalar branches, and hipcc then drained vmcnt(0) at the join.
		const uint32_t t = (uint32_t)t0;
		// rows of the cache from t0 on, at most one chunk (a live chunk has t0 < kv_len <=
		// max_seq_len). Only s_min / s_cselect: a clamp became v_med3 and an unsigned
		// saturating subtract v_sub clamp -- VALU temporaries that re-used a register of the
		// previous chunk's loads (a vmcnt(0) per chunk) or forced a waterfall loop
		const int rows = min((int)msl - t0, attn_chunk<D>());
		const int nrec = live ? rows * (int)rowb : 0;
		const uint64_t o = (uint64_t)t * rowb;
		const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc((void *)(kb + o), (short)0, nrec, 0x00020000);
		const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc((void *)(vb + o), (short)0, nrec, 0x00020000);
#pragma unroll
		for (int i = 0; i < NK; ++i) {
			kw[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(kr, voff[i], 0, 0));
			vw[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(vr, voff[i], 0, 0));
		}
	}
};

__device__ __forceinline__ void st_sc1(float *p, float v) {
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float *p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// head outputs: plain stores for the next launch (GRAN = false), or, when other
// workgroups of the same launch consume them (attn_wo.h), one 8-byte {value, tag}
// granule per element written by ONE sc1 store, so that the data is its own
// ready flag (MI355X_MICROARCH.md §visibility, R2 granules: no drain, no flag).
template <bool GRAN>
__device__ __forceinline__ void attn_out(float *out, size_t i, float v, unsigned tag) {
	if constexpr (GRAN) {
		const unsigned long long g = (unsigned long long)__float_as_uint(v) | ((unsigned long long)tag << 32);
		__hip_atomic_store((unsigned long long *)out + i, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	} else {
		out[i] = v;
	}
}

#define ATTN_TIMEOUT 200000000ull // 2 s of s_memrealtime (100 MHz): a merger that never sees a chunk gives up

__device__ __forceinline__ unsigned long long gran_ld(const unsigned long long *p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Tag of one attention launch's chunk partials: unique per (forward, layer).
__device__ __forceinline__ unsigned attn_part_tag(const StepState *step, int layer, int n_layers) {
	return step->epoch * (unsigned)n_layers + (unsigned)layer;
}

// Sum over each aligned group of LPK lanes (one K row's pieces, LPK = head_dim / 8
// in 2..32), result in every lane of the group: xor-butterfly of DPP quad_perm
// [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror, then a lane swap across rows.
template <int LPK>
__device__ __forceinline__ float attn_row_sum(float v) {
	if constexpr (LPK >= 2)
		v += dpp<0xB1>(v);
	if constexpr (LPK >= 4)
		v += dpp<0x4E>(v);
	if constexpr (LPK >= 8)
		v += dpp<0x141>(v);
	if constexpr (LPK >= 16)
		v += dpp<0x140>(v);
	if constexpr (LPK >= 32)
		v += xor16(v);
	return v;
}
// Sum / max over the row groups inside each DPP row, lane by lane (a lane meets
// the lanes of the same piece, or of the same head when LPK is the head count):
// row_ror by LPK, 2 LPK, .. 8.
template <int LPK, bool MAX>
__device__ __forceinline__ float attn_fold_row(float v) {
	auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
	if constexpr (LPK <= 1)
		v = op(v, dpp<0x121>(v));
	if constexpr (LPK <= 2)
		v = op(v, dpp<0x122>(v));
	if constexpr (LPK <= 4)
		v = op(v, dpp<0x124>(v));
	if constexpr (LPK <= 8)
		v = op(v, dpp<0x128>(v));
	return v;
}
// One halving step of a 16-lane reduce-scatter over J groups of R values: the lane
// keeps the upper or lower half of each group and adds its partner's copy of it
// (CTRL: a DPP involution pairing lanes with opposite `upper`).
template <int CTRL, int J, int R>
__device__ __forceinline__ void attn_rs_step(const float (&in)[J * R], float (&out)[J * R / 2], bool upper) {
	constexpr int H = R / 2;
#pragma unroll
	for (int j = 0; j < J; ++j)
#pragma unroll
		for (int k = 0; k < H; ++k) {
			const float lo = in[j * R + k], hi = in[j * R + H + k];
			out[j * H + k] = (upper ? hi : lo) + dpp<CTRL>(upper ? lo : hi);
		}
}
// Lane r's value broadcast to its whole DPP row (row_newbcast:r, gfx90a+); r must
// fold to a constant once the caller's loops are unrolled.
__device__ __forceinline__ float row_bcast16(float v, int r) {
	switch (r) {
	case 0: return dpp<0x150>(v);
	case 1: return dpp<0x151>(v);
	case 2: return dpp<0x152>(v);
	case 3: return dpp<0x153>(v);
	case 4: return dpp<0x154>(v);
	case 5: return dpp<0x155>(v);
	case 6: return dpp<0x156>(v);
	case 7: return dpp<0x157>(v);
	case 8: return dpp<0x158>(v);
	case 9: return dpp<0x159>(v);
	case 10: return dpp<0x15A>(v);
	case 11: return dpp<0x15B>(v);
	case 12: return dpp<0x15C>(v);
	case 13: return dpp<0x15D>(v);
	case 14: return dpp<0x15E>(v);
	default: return dpp<0x15F>(v);
	}
}
// Max / sum over all the wave's row groups of a value every lane of a group holds.
template <int LPK, bool MAX>
__device__ __forceinline__ float attn_wave_red(float v) {
	auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
	v = attn_fold_row<LPK, MAX>(v);
	if constexpr (LPK <= 16)
		v = op(v, xor16(v));
	return op(v, xor32(v));
}

// Work of one attention workgroup on kv head g, after its speculative loads (q of
// the group's G heads in qv, the first chunk's K/V rows in kA / vA): query heads
// hq0 .. hq0 + Gh - 1 of the group (Gh <= GT) over the key chunks c_first,
// c_first + cstride, ... < ns. final_out: these are all the keys of those heads --
// normalise and write the head outputs (returns true); otherwise publish ONE partial
// per head (unnormalised o[D], max M, sum L) as granules tagged ptag into part
// [n_heads][nsplit][D + 2] at split s_part, folded by the MERGER workgroups
// (attn_merge_body). D = head_dim (16 .. 256, a power of two).
// GRAN: outputs as {value, gtag} granules into `out` read as unsigned long long[].
// ts / trace_on: attn_wo.h's timeline stamps (thread 0) and the trace-only waits.
//
// Layout: each wave runs its 16 keys of every chunk to the end WITHOUT a workgroup
// barrier -- lane (row group, piece) holds 8 dims of NK K/V rows; the scores are
// reduced across the row's pieces with DPP, the softmax statistics are per wave
// (max / sum across row groups with DPP and lane swaps), P is never stored, and the
// P.V sums stay in registers. Across the workgroup's chunks the wave keeps a running
// (max, sum, P.V) with the flash-decoding rescaling, and the next chunk's K/V rows
// are loaded before the current one is computed, so a workgroup with several chunks
// pays one load latency, not one per chunk. One barrier at the end combines the 4
// waves. Round 3 published one partial per 64-key chunk and the last attention
// workgroup merged them in serial batches of 8 (kv 4096: 64 partials, 8 dependent
// round trips, 20 us standalone).
template <int D, int GT, int GQ, bool GRAN>
// (no __restrict__ here: the standalone kernel keeps it on its arguments)
__device__ __forceinline__ bool attn_core(int g, int hq0, int Gh, int c_first, int cstride, int ns, bool final_out,
                                          int s_part, const float4_t (&qv)[(GQ * D + 255) / 256],
                                          u32x4_t (&kA)[attn_nk<D>()], u32x4_t (&vA)[attn_nk<D>()],
                                          int kv_len, const uint16_t *kc, const uint16_t *vc, int n_heads,
                                          int n_kv_heads, int max_seq_len, int nsplit, unsigned long long *part,
                                          unsigned ptag, float *out, float *att_dbg, unsigned gtag,
                                          unsigned long long *ts, bool trace_on) {
	constexpr int CHUNK = attn_chunk<D>();
	// the chunk loop's values in SGPRs (KvRows::load's descriptors are computed from them)
	c_first = __builtin_amdgcn_readfirstlane(c_first);
	cstride = __builtin_amdgcn_readfirstlane(cstride);
	ns = __builtin_amdgcn_readfirstlane(ns);
	kv_len = __builtin_amdgcn_readfirstlane(kv_len);
	constexpr int LPK = D / 8;                      // lanes per K/V row, 16 B each
	static_assert(LPK >= 2 && LPK <= 32 && (LPK & (LPK - 1)) == 0, "head_dim 16 .. 256, a power of two");
	constexpr int KPW = 64 / LPK;                   // row groups per wave (rows per wave-instruction)
	constexpr int RSTEP = ATTN_WAVES * KPW;         // rows per workgroup-instruction
	constexpr int NK = CHUNK / RSTEP > 0 ? CHUNK / RSTEP : 1; // rows per lane (D 16: half the rows masked)
	constexpr int QL = (GQ * D + 255) / 256;        // 16-byte q loads per lane (wave-private copy)
	__shared__ __attribute__((aligned(16))) float qs[ATTN_WAVES][GQ * D];
	__shared__ float wsum[ATTN_WAVES][GT][D]; // per-wave P.V sums
	__shared__ float wml[ATTN_WAVES][GT][2];  // per-wave (max, sum of exp)

	const int G = n_heads / n_kv_heads;
	const int hb = g * G + hq0; // first query head computed here
	const int lane = threadIdx.x & 63;
	const int wave = threadIdx.x >> 6;
	const int tid = threadIdx.x;
	const int sub = lane / LPK;
	const int piece = lane % LPK;
	const int tl0 = wave * KPW + sub;

	const KvRows<D> rows(kc, vc, n_kv_heads, max_seq_len, g);
	auto load_kv = [&](int t0, u32x4_t (&kw)[NK], u32x4_t (&vw)[NK]) { rows.load(t0, t0 < kv_len, kw, vw); };
	// trace (attn_wo.h, thread 0 only): s_memrealtime + shader clock (s_memtime) at
	// checkpoint k, kept in LDS and stored at the end -- a store issued mid-way would
	// queue behind the co-resident Wo workgroup's weight loads and stall the wave, and
	// 16 64-bit stamps kept in registers cost the fused kernel its second workgroup per CU
	__shared__ unsigned long long tss[16];
	auto stamp = [&](int k) {
		if (ts) {
			tss[k] = __builtin_amdgcn_s_memrealtime();
			tss[8 + k] = __builtin_amdgcn_s_memtime();
		}
	};
	auto flush = [&]() {
		if (ts) {
#pragma unroll
			for (int k = 2; k < 8; ++k)
				if (k != 3)
					ts[k] = tss[k], ts[8 + k] = tss[8 + k];
		}
	};
	if (trace_on) { // tracing only: when the first chunk's loads have landed in every wave
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads();
		stamp(2);
	}
	// q through this wave's own LDS copy: lane (row group, piece) needs dims piece*8..+8
	// of every head (LDS reads from one wave are ordered after its writes: no barrier)
	const int gq = G * D;
#pragma unroll
	for (int j = 0; j < QL; ++j)
		if ((j * 64 + lane) * 4 < gq)
			*(float4_t *)&qs[wave][(j * 64 + lane) * 4] = qv[j];
	float qr[GT][8];
#pragma unroll
	for (int h = 0; h < GT; ++h) {
		const float *qp = &qs[wave][(hq0 + (h < Gh ? h : 0)) * D + piece * 8];
		const float4_t a = *(const float4_t *)qp;
		const float4_t b = *(const float4_t *)(qp + 4);
		qr[h][0] = a[0], qr[h][1] = a[1], qr[h][2] = a[2], qr[h][3] = a[3];
		qr[h][4] = b[0], qr[h][5] = b[1], qr[h][6] = b[2], qr[h][7] = b[3];
	}
	const float sq = sqrtf((float)D);

	// running state of this wave over its chunks: P.V sums (element e of head h at dim
	// piece * 8 + e, not yet reduced across row groups), and per head the running max and
	// sum of exponentials (head_dim 128: lane p of each 16-lane row holds head p % GT's;
	// otherwise every lane holds all heads')
	float acc[GT * 8];
#pragma unroll
	for (int k = 0; k < GT * 8; ++k)
		acc[k] = 0.0f;
	float Mr = -FLT_MAX, Lr = 0.0f, mw[GT], lw[GT];
#pragma unroll
	for (int h = 0; h < GT; ++h)
		mw[h] = -FLT_MAX, lw[h] = 0.0f;

	// FIRST: the workgroup's first chunk (nothing to rescale yet)
	auto chunk = [&](auto first, const u32x4_t (&kw)[NK], const u32x4_t (&vw)[NK], int t0) {
		constexpr bool FIRST = decltype(first)::value;
		const int nt = min(CHUNK, kv_len - t0);
		if constexpr (LPK == 16) {
			// ---- head_dim 128: the row's 16 lanes share out its NK * GT scores (V values,
			// padded to 16 J): a 4-step reduce-scatter of the partial dots leaves lane p of
			// the row with score f = 16 j + p (key row i = f / GT, head h = f % GT), so
			// the exp, max and sum run once per score, not once per lane
			constexpr int V = NK * GT, J = V >= 16 ? V / 16 : 1;
			float d16[J * 16];
			{
				float kf[NK][8];
#pragma unroll
				for (int i = 0; i < NK; ++i)
					WF16::unpack(kw[i], kf[i]);
#pragma unroll
				for (int f = 0; f < J * 16; ++f) {
					float d = 0.0f;
					if (f < V) {
#pragma unroll
						for (int e = 0; e < 8; ++e)
							d = fmaf(qr[f % GT][e], kf[f / GT][e], d);
					}
					d16[f] = d;
				}
			}
			float r8[J * 8], r4[J * 4], r2[J * 2], sc[J];
			attn_rs_step<0x140, J, 16>(d16, r8, lane & 8); // row_mirror: lanes p, 15 - p
			attn_rs_step<0x141, J, 8>(r8, r4, lane & 4);   // row_half_mirror: p, p ^ 7
			attn_rs_step<0x4E, J, 4>(r4, r2, lane & 2);    // quad_perm xor 2
			attn_rs_step<0xB1, J, 2>(r2, sc, lane & 1);    // quad_perm xor 1
			const int p = lane & 15, h = p % GT;
			bool ok[J];
			float m = -FLT_MAX;
#pragma unroll
			for (int j = 0; j < J; ++j) {
				const int f = j * 16 + p, i = f / GT;
				ok[j] = f < V && tl0 + i * RSTEP < nt;
				sc[j] = sc[j] / sq;
				m = ok[j] ? fmaxf(m, sc[j]) : m;
				if (att_dbg && ok[j] && h < Gh) // test hook: raw scores (normalised by the writer)
					st_sc1(att_dbg + (size_t)(hb + h) * max_seq_len + t0 + tl0 + i * RSTEP, sc[j]);
			}
			stamp(4);
			// ---- per-wave softmax statistics of head h over the row's lanes of the same
			// head (row_ror by GT, 2 GT, ..) and the 4 rows, folded into the running ones
			m = attn_wave_red<GT, true>(m);
			const float Mn = FIRST ? m : fmaxf(Mr, m);
			float pj[J], l = 0.0f;
#pragma unroll
			for (int j = 0; j < J; ++j) {
				pj[j] = ok[j] ? expf(sc[j] - Mn) : 0.0f;
				l += pj[j];
			}
			l = attn_wave_red<GT, false>(l);
			if constexpr (FIRST) {
				Lr = l;
			} else {
				const float corr = expf(Mr - Mn);
				Lr = fmaf(Lr, corr, l);
#pragma unroll
				for (int hh = 0; hh < GT; ++hh) { // head hh's factor from lane hh of the row
					const float c = row_bcast16(corr, hh);
#pragma unroll
					for (int e = 0; e < 8; ++e)
						acc[hh * 8 + e] *= c;
				}
			}
			Mr = Mn;
			stamp(5);
			// ---- P.V: probability f is broadcast from lane f % 16 of each row (row_newbcast)
#pragma unroll
			for (int i = 0; i < NK; ++i) {
				float vf[8];
				const bool valid = tl0 + i * RSTEP < nt;
				WF16::unpack(valid ? vw[i] : u32x4_t{0u, 0u, 0u, 0u}, vf); // rows past kv_len may hold anything
#pragma unroll
				for (int hh = 0; hh < GT; ++hh) {
					const int f = i * GT + hh;
					const float pv = row_bcast16(pj[f / 16], f % 16);
#pragma unroll
					for (int e = 0; e < 8; ++e)
						acc[hh * 8 + e] = fmaf(pv, vf[e], acc[hh * 8 + e]);
				}
			}
		} else {
			// ---- other head dims: every lane of a row group reduces all its rows' scores
			float sv[NK][GT];
			bool valid[NK];
#pragma unroll
			for (int i = 0; i < NK; ++i) {
				valid[i] = tl0 + i * RSTEP < nt;
				float kf[8];
				WF16::unpack(kw[i], kf);
#pragma unroll
				for (int h = 0; h < GT; ++h) {
					float d = 0.0f;
#pragma unroll
					for (int e = 0; e < 8; ++e)
						d = fmaf(qr[h][e], kf[e], d);
					sv[i][h] = attn_row_sum<LPK>(d) / sq;
				}
			}
			if (att_dbg && piece == 0) { // test hook: raw scores (normalised by the writer)
#pragma unroll
				for (int i = 0; i < NK; ++i)
#pragma unroll
					for (int h = 0; h < GT; ++h)
						if (valid[i] && h < Gh)
							st_sc1(att_dbg + (size_t)(hb + h) * max_seq_len + t0 + tl0 + i * RSTEP, sv[i][h]);
			}
			stamp(4);
#pragma unroll
			for (int h = 0; h < GT; ++h) {
				float m = -FLT_MAX;
#pragma unroll
				for (int i = 0; i < NK; ++i)
					m = valid[i] ? fmaxf(m, sv[i][h]) : m;
				m = attn_wave_red<LPK, true>(m);
				const float Mn = FIRST ? m : fmaxf(mw[h], m);
				float l = 0.0f;
#pragma unroll
				for (int i = 0; i < NK; ++i) {
					sv[i][h] = valid[i] ? expf(sv[i][h] - Mn) : 0.0f;
					l += sv[i][h];
				}
				l = attn_wave_red<LPK, false>(l);
				if constexpr (FIRST) {
					lw[h] = l;
				} else {
					const float corr = expf(mw[h] - Mn);
					lw[h] = fmaf(lw[h], corr, l);
#pragma unroll
					for (int e = 0; e < 8; ++e)
						acc[h * 8 + e] *= corr;
				}
				mw[h] = Mn;
			}
			stamp(5);
#pragma unroll
			for (int i = 0; i < NK; ++i) {
				float vf[8];
				WF16::unpack(valid[i] ? vw[i] : u32x4_t{0u, 0u, 0u, 0u}, vf); // rows past kv_len may hold anything
#pragma unroll
				for (int h = 0; h < GT; ++h)
#pragma unroll
					for (int e = 0; e < 8; ++e)
						acc[h * 8 + e] = fmaf(sv[i][h], vf[e], acc[h * 8 + e]);
			}
		}
	};

	// chunks c_first, c_first + cstride, ...: straight-line loads for one chunk; beyond
	// it the next chunk's rows are loaded before the current one is computed (the prefetch
	// past the last chunk is issued with a zero-record descriptor and moves no data,
	// KvRows: unconditional loads keep hipcc's vmcnt counting exact, a conditional one
	// would drain to 0 before every load)
	using T_ = std::true_type;
	using F_ = std::false_type;
	if (c_first + cstride >= ns) {
		chunk(T_{}, kA, vA, c_first * CHUNK);
	} else {
		u32x4_t kB[NK], vB[NK];
		load_kv((c_first + cstride) * CHUNK, kB, vB);
		chunk(T_{}, kA, vA, c_first * CHUNK);
		for (int c = c_first + cstride;; c += 2 * cstride) { // kB / vB hold chunk c
			load_kv((c + cstride) * CHUNK, kA, vA);
			chunk(F_{}, kB, vB, c * CHUNK);
			if (c + cstride >= ns)
				break;
			load_kv((c + 2 * cstride) * CHUNK, kB, vB);
			chunk(F_{}, kA, vA, (c + cstride) * CHUNK);
			if (c + 2 * cstride >= ns)
				break;
		}
	}

	// ---- this wave's running (max, sum) and P.V sums over its row groups, into LDS
	if constexpr (LPK == 16) {
		if (lane < GT && lane < Gh) {
			wml[wave][lane][0] = Mr;
			wml[wave][lane][1] = Lr;
		}
	} else if (lane < Gh) {
		float m = mw[0], l = lw[0];
#pragma unroll
		for (int h = 1; h < GT; ++h)
			if (lane == h)
				m = mw[h], l = lw[h];
		wml[wave][lane][0] = m;
		wml[wave][lane][1] = l;
	}
	if constexpr (LPK <= 16) {
		// the row groups inside each DPP row first (LPK < 16), then across the 4 DPP
		// rows transposed: for value group k, lane `piece` of DPP row r holds value
		// 4k + r of that piece summed over the wave (element e of head h: dim piece * 8 + e)
#pragma unroll
		for (int k = 0; k < GT * 8; ++k)
			acc[k] = attn_fold_row<LPK, false>(acc[k]);
#pragma unroll
		for (int k = 0; k < GT * 2; ++k) {
			const float v4[4] = {acc[4 * k], acc[4 * k + 1], acc[4 * k + 2], acc[4 * k + 3]};
			const float s = sum4_rows(v4);
			const int idx = 4 * k + (lane >> 4), h = idx >> 3, e = idx & 7;
			if (h < Gh && (lane & 15) < LPK)
				wsum[wave][h][(lane & 15) * 8 + e] = s;
		}
	} else { // LPK 32: two row groups, the wave's halves
#pragma unroll
		for (int k = 0; k < GT * 8; ++k)
			acc[k] += xor32(acc[k]);
		if (lane < 32) {
#pragma unroll
			for (int h = 0; h < GT; ++h)
#pragma unroll
				for (int e = 0; e < 8; ++e)
					if (h < Gh)
						wsum[wave][h][lane * 8 + e] = acc[h * 8 + e];
		}
	}
	if (att_dbg) // test hook: every wave's raw scores visible before the barrier / the partials
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	stamp(6);

	// ---- combine the waves (fixed order): o = sum_w e^(m_w - M) o_w, L likewise
	for (int i = tid; i < Gh * D; i += ATTN_THREADS) {
		const int h = i / D, d = i % D;
		float M = wml[0][h][0];
#pragma unroll
		for (int w = 1; w < ATTN_WAVES; ++w)
			M = fmaxf(M, wml[w][h][0]);
		float o = 0.0f, L = 0.0f;
#pragma unroll
		for (int w = 0; w < ATTN_WAVES; ++w) {
			const float c = expf(wml[w][h][0] - M); // 0 for a wave without valid rows (m_w = -FLT_MAX)
			o = fmaf(wsum[w][h][d], c, o);
			L = fmaf(wml[w][h][1], c, L);
		}
		if (final_out) { // all keys of these heads: normalise and write the head outputs
			attn_out<GRAN>(out, (size_t)(hb + h) * D + d, o / L, gtag);
		} else { // this workgroup's partial (o[D], M, L per head) as tagged granules
			const size_t pp = ((size_t)(hb + h) * nsplit + s_part) * (D + 2);
			attn_out<true>((float *)part, pp + d, o, ptag);
			if (d == 0) {
				attn_out<true>((float *)part, pp + D, M, ptag);
				attn_out<true>((float *)part, pp + D + 1, L, ptag);
			}
		}
	}
	stamp(7); // this workgroup's head outputs / partials issued
	if (final_out && att_dbg) { // test hook: raw scores -> probabilities
		const int nt = kv_len;
		for (int i = tid; i < Gh * nt; i += ATTN_THREADS) {
			const int h = i / nt, t = i % nt;
			float M = wml[0][h][0];
#pragma unroll
			for (int w = 1; w < ATTN_WAVES; ++w)
				M = fmaxf(M, wml[w][h][0]);
			float L = 0.0f;
#pragma unroll
			for (int w = 0; w < ATTN_WAVES; ++w)
				L = fmaf(wml[w][h][1], expf(wml[w][h][0] - M), L);
			float *a = att_dbg + (size_t)(hb + h) * max_seq_len + t;
			*a = expf(ld_sc1(a) - M) / L;
		}
	}
	flush();
	return final_out;
}

// One attention workgroup: unit u of kv head g's S + G - 1 units. Units u < G are HEAD
// units (query head u of the group), units u >= G are SPLIT units (every query head of
// the group, key split s = u - G + 1). Speculative loads first (q; a head unit's first
// chunk, chunk 0 in both modes), then one of
//   * HEAD mode (kv_len <= head_max chunks): head unit u runs query head u over ALL
//     the chunks and writes it directly -- no partial, no merger hop, and a quarter of
//     the per-wave arithmetic of a 4-head chunk (Mistral: G = 4). The G head units of a
//     kv head read the same K/V rows (dispatched to the same XCD: the 2nd .. Gth from L2).
//   * KEY mode (longer contexts): key split 0 (chunks 0, S, 2S, ...) is run by the G head
//     units, one query head each; split s >= 1 (chunks s, s + S, ...) by split unit
//     s + G - 1 for every head; one partial per (head, split) for the mergers (or, with
//     only split 0 holding keys, the head outputs).
// Round 4's first cut made units s0 < G both the head-mode units and key-mode split s0:
// they speculated on chunk 0, so key-mode units 1 .. G-1 re-issued their own chunk
// after kv_len (a load latency: Mistral kv 501 attention 7.0 us), and loading both
// guesses cost the short contexts 0.5 us.
// Returns true on a workgroup that wrote head outputs.
template <int D, int GT, bool GRAN>
__device__ __forceinline__ bool attn_decode_body(int g, int u, int S, int head_max, const float *q,
                                                 const uint16_t *kc, const uint16_t *vc, const StepState *step,
                                                 int n_heads, int n_kv_heads, int max_seq_len, int nsplit,
                                                 unsigned long long *part, unsigned ptag, float *out, float *att_dbg,
                                                 unsigned gtag = 0, unsigned long long *ts = nullptr,
                                                 bool trace_on = false) {
	constexpr int CHUNK = attn_chunk<D>();
	constexpr int LPK = D / 8;
	constexpr int KPW = 64 / LPK;
	constexpr int RSTEP = ATTN_WAVES * KPW;
	constexpr int NK = CHUNK / RSTEP > 0 ? CHUNK / RSTEP : 1;
	constexpr int QL = (GT * D + 255) / 256;
	const int G = n_heads / n_kv_heads;
	const int lane = threadIdx.x & 63;
	const bool hu = u < G;             // head unit (query head u)
	const int s = hu ? 0 : u - G + 1; // key split
	// ---- speculative loads: q of the group's G heads (G * D contiguous floats, QL
	// 16-byte pieces per lane), the unit's first chunk's K/V rows (zeros past the cache)
	const int gq = G * D;
	float4_t qv[QL];
#pragma unroll
	for (int j = 0; j < QL; ++j)
		qv[j] = *(const float4_t *)(q + (size_t)g * gq + min((j * 64 + lane) * 4, gq - 4));
	// head units: chunk 0, speculatively; split units load their chunk once kv_len says it
	// holds keys (their speculative loads were 6.3 MB of dead reads per layer at short
	// contexts, 192 units x 32 KB: fused fp8 kv 17 8.3 -> 7.9 us, fp16 bench +0.9%, long
	// context -0.2%, profiles/r4q_split_spec.txt). The instruction stays unconditional
	// (a split unit's gets a zero-record descriptor and moves no data): hipcc's vmcnt
	// counting stays static.
	u32x4_t kA[NK], vA[NK];
	const KvRows<D> rows(kc, vc, n_kv_heads, max_seq_len, g);
	rows.load(0, hu, kA, vA);
	const int kv_len = step->kv_len;
	const int ns = (kv_len + CHUNK - 1) / CHUNK;
	if (ns <= head_max) { // (the host passes head_max >= 1, and >= every ns when S = 1)
		if (!hu)
			return false; // whole workgroup leaves before any barrier
		return attn_core<D, 1, GT, GRAN>(g, u, 1, 0, 1, ns, true, 0, qv, kA, vA, kv_len, kc, vc, n_heads, n_kv_heads,
		                                 max_seq_len, nsplit, part, ptag, out, att_dbg, gtag, ts, trace_on);
	}
	if (s * CHUNK >= kv_len)
		return false;
	if (!hu)
		rows.load(s * CHUNK, true, kA, vA);
	// key mode: ns >= 2 and S >= 2, so every head has at least two partials and the
	// mergers write the heads
	if (hu)
		return attn_core<D, 1, GT, GRAN>(g, u, 1, 0, S, ns, false, 0, qv, kA, vA, kv_len, kc, vc, n_heads, n_kv_heads,
		                                 max_seq_len, nsplit, part, ptag, out, att_dbg, gtag, ts, trace_on);
	return attn_core<D, GT, GT, GRAN>(g, 0, G, s, S, ns, false, s, qv, kA, vA, kv_len, kc, vc, n_heads, n_kv_heads,
	                                  max_seq_len, nsplit, part, ptag, out, att_dbg, gtag, ts, trace_on);
}

// MERGER workgroup of (kv head g, query head h = g * G + hq): in key mode with
// nact > 1 attention workgroups holding keys, gathers their nact partials of head h and
// writes the normalised head output. Mergers are dispatched after every attention
// workgroup of the launch, so they only wait on earlier ones (no deadlock however
// few workgroups are resident). Wave w takes splits w, w + 4, ...: all its granule
// loads (per lane 2 dims of each of its splits, and lane j the (M, L) of its j-th
// split) are issued at once and re-read until every tag holds ptag; the waves'
// (max, sum, o) meet in LDS and are folded in wave order (deterministic). One head
// per workgroup: a merger gathers (D + 2) x 8 B per split (33 KB at kv 4096), where
// the round-4 first cut merged all G heads of a kv head in ONE workgroup (131 KB
// through one CU). Returns true if it wrote the head (nact > 1).
template <int D, bool GRAN>
__device__ __forceinline__ bool attn_merge_body(int g, int hq, int S, int head_max, const StepState *step, int n_heads,
                                                int n_kv_heads, int max_seq_len, int nsplit,
                                                const unsigned long long *part, unsigned ptag, unsigned *err,
                                                float *out, float *att_dbg, unsigned gtag = 0,
                                                unsigned long long *ts = nullptr) {
	constexpr int CHUNK = attn_chunk<D>();
	constexpr int SPW = ATTN_MAX_SPLITS / ATTN_WAVES; // splits per wave, at most
	constexpr int E = D >= 64 ? D / 64 : 1;           // dims per lane: lane + 64 k
	__shared__ float mml[ATTN_WAVES][2];
	__shared__ float mo[ATTN_WAVES][D];
	const int G = n_heads / n_kv_heads;
	const int h = g * G + hq;
	const int kv_len = step->kv_len;
	const int ns = (kv_len + CHUNK - 1) / CHUNK;
	const int nact = min(ns, S);
	if (ns <= head_max || hq >= G)
		return false; // head mode (attn_decode_body): nothing to merge
	const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
	const int nsw = (nact - wave + ATTN_WAVES - 1) / ATTN_WAVES; // this wave's splits: wave + 4 j, j < nsw
	const int dl = lane < D ? lane : 0; // lanes past D (D < 64) re-read dim 0 and only follow along
	const unsigned long long *ph = part + (size_t)h * nsplit * (D + 2);
	const unsigned long long *pl = ph + (size_t)(wave + ATTN_WAVES * min(lane, max(nsw - 1, 0))) * (D + 2);
	const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + ATTN_TIMEOUT;
	if (ts) // trace (attn_wo.h, thread 0): [5] gather issued, [7] every partial seen (merger rows keep [2] = 0)
		ts[5] = __builtin_amdgcn_s_memrealtime(), ts[13] = __builtin_amdgcn_s_memtime();
	bool alive = true;
	float ms = -FLT_MAX, ls = 0.0f, ob[SPW][E];
	for (;;) {
		unsigned long long gm = 0, gl = 0, go[SPW][E];
		if (nsw > 0) {
			gm = gran_ld(pl + D);
			gl = gran_ld(pl + D + 1);
		}
#pragma unroll
		for (int j = 0; j < SPW; ++j) {
			if (j < nsw) {
				const unsigned long long *pc = ph + (size_t)(wave + ATTN_WAVES * j) * (D + 2);
#pragma unroll
				for (int k = 0; k < E; ++k)
					go[j][k] = gran_ld(pc + dl + 64 * k);
			}
		}
		bool ok = lane >= nsw || ((unsigned)(gm >> 32) == ptag && (unsigned)(gl >> 32) == ptag);
#pragma unroll
		for (int j = 0; j < SPW; ++j) {
			if (j < nsw) {
#pragma unroll
				for (int k = 0; k < E; ++k) {
					ok = ok && (unsigned)(go[j][k] >> 32) == ptag;
					ob[j][k] = __uint_as_float((unsigned)go[j][k]);
				}
			}
		}
		if (lane < nsw) {
			ms = __uint_as_float((unsigned)gm);
			ls = __uint_as_float((unsigned)gl);
		}
		if (__all(ok) || !alive)
			break;
		__builtin_amdgcn_s_sleep(1);
		if (__builtin_amdgcn_s_memrealtime() > deadline) {
			alive = false; // one more pass, then give up (results wrong, reported)
			if (err && lane == 0)
				__hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
	}
	// this wave's max, then the workgroup's (LDS), the weights e^(m_s - M) on lane j
	const float mw = wave_max(ms);
	if (lane == 0)
		mml[wave][0] = mw;
	__syncthreads();
	if (ts) // every wave's partials in registers
		ts[7] = __builtin_amdgcn_s_memrealtime(), ts[15] = __builtin_amdgcn_s_memtime();
	const float M = fmaxf(fmaxf(mml[0][0], mml[1][0]), fmaxf(mml[2][0], mml[3][0]));
	const float ws = lane < nsw ? expf(ms - M) : 0.0f;
	const float lw = wave_sum(ws * ls);
	float o[E];
#pragma unroll
	for (int k = 0; k < E; ++k)
		o[k] = 0.0f;
#pragma unroll
	for (int j = 0; j < SPW; ++j) {
		if (j < nsw) {
			const float w = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ws), j));
#pragma unroll
			for (int k = 0; k < E; ++k)
				o[k] = fmaf(w, ob[j][k], o[k]);
		}
	}
	if (lane < D) {
#pragma unroll
		for (int k = 0; k < E; ++k)
			mo[wave][lane + 64 * k] = o[k];
	}
	if (lane == 0)
		mml[wave][1] = lw;
	__syncthreads();
	const float L = (mml[0][1] + mml[1][1]) + (mml[2][1] + mml[3][1]);
	for (int d = tid; d < D; d += ATTN_THREADS)
		attn_out<GRAN>(out, (size_t)h * D + d, ((mo[0][d] + mo[1][d]) + (mo[2][d] + mo[3][d])) / L, gtag);
	if (att_dbg) {
		for (int t = tid; t < kv_len; t += ATTN_THREADS) {
			float *a = att_dbg + (size_t)h * max_seq_len + t;
			*a = expf(ld_sc1(a) - M) / L;
		}
	}
	return true;
}

// Grid: n_kv * (S + G - 1) attention workgroups (b = g + n_kv * u: unit u of kv head g;
// with n_kv a multiple of 8 a kv head's units share an XCD), then n_kv * G merger
// workgroups (g, hq), dispatched after every attention workgroup.
template <int D, int GT>
__global__ __launch_bounds__(ATTN_THREADS) void attn_decode_kernel(
    const float *__restrict__ q, const uint16_t *__restrict__ kc, const uint16_t *__restrict__ vc,
    const StepState *__restrict__ step, int n_heads, int n_kv_heads, int max_seq_len, int nsplit, int S,
    int head_max, unsigned long long *__restrict__ part, int layer, int n_layers, unsigned *__restrict__ err,
    float *__restrict__ out, float *__restrict__ att_dbg) {
	const int b = blockIdx.x, units = n_kv_heads * (S + n_heads / n_kv_heads - 1);
	const unsigned ptag = attn_part_tag(step, layer, n_layers);
	if (b < units)
		attn_decode_body<D, GT, false>(b % n_kv_heads, b / n_kv_heads, S, head_max, q, kc, vc, step, n_heads,
		                               n_kv_heads, max_seq_len, nsplit, part, ptag, out, att_dbg);
	else
		attn_merge_body<D, false>((b - units) % n_kv_heads, (b - units) / n_kv_heads, S, head_max, step, n_heads,
		                          n_kv_heads, max_seq_len, nsplit, part, ptag, err, out, att_dbg);
}
