// attn_wo_local.h — the short-context form of the fused attention + Wo launch
// (attn_wo.h): no cross-CU hand-off, every Wo workgroup recomputes the attention.
#pragma once

#include <float.h>

#include "attn_wo.h"

// ---------------------------------------------------------------------------
// Short-context form (kv_len <= a threshold the host picks, default 64): NO
// hand-off at all. Every Wo workgroup computes the whole attention itself from
// the L2-resident K/V cache while its Wo slice streams in, then dots the slice.
//
// Why: above, the attention output crosses CUs (granule store -> poll -> gather:
// ~3 us of round trips on top of the 33.5 MB Wo stream, MI355X_MICROARCH.md row
// handoff-1to1). At decode-size contexts the whole attention input is small
// (kv_len x 8 kv heads x 2 x 256 B = 152 KB at kv_len 38), served from each
// XCD's L2 after the first touch, so recomputing it in each of the 256 Wo
// workgroups costs ~1 us of L2 reads + ALU that run UNDER the Wo stream,
// instead of a serial hand-off after it. The host picks this kernel per token
// from the position it tracks (two captured graphs); the kernel itself is
// correct at any kv_len (64-key blocks with the online-softmax rescale).
//
// One workgroup = 16 waves (1024 threads) per 16 Wo rows, in two roles so that no
// wave's K/V loads sit behind Wo loads in its (in-order) vmcnt queue:
//   * waves 0-7 hold the 128 KB Wo slice (16 KB per wave, issued at launch), then
//     dot it with the attention output from LDS;
//   * waves 8-15 each own kv head w - 8 (+ 8, ... when n_kv > 8): 32-key blocks,
//     lanes t and t + 32 hold the two halves of key t's K row for the scores (one
//     permlane32 swap completes the dot; q broadcast from LDS), lane = 2 output dims
//     for P.V (one V dword per key and lane; p broadcast from LDS).
// Semantics: infer.cpp:216-248 (softmax(q.k / sqrt(D)) . V), then
// fused_matmul_add_residuals (infer.cu:270).
#define AWL_THREADS 1024
#define AWL_WO_WAVES 8
#define AWL_AT_WAVES 8
#define AWL_KB 32 // keys per block

// Workgroup barrier for LDS hand-offs only. __syncthreads() is a workgroup-scope
// release + acquire, which hipcc lowers with s_waitcnt vmcnt(0): the Wo waves would
// wait for their whole slice at the first barrier and hold the attention waves
// behind it. Only LDS is shared here, so: drain this wave's LDS ops, then s_barrier
// (one asm statement with a memory clobber: no memory op moves across it).
__device__ __forceinline__ void awl_barrier() {
	asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

struct AttnWoLocalArgs {
	int n_heads, n_kv, max_seq_len, q_dim, dim;
	const char *wo; // Wo (dim, q_dim)
	float *x;       // residual stream (dim)
	unsigned long long *trace; // [grid][4] s_memrealtime stamps or null
	int kv_first; // Wo waves issue their slice only after the attention waves issued their first K/V block
	int ablate;   // timing only (YALM_AWL_ABLATE, results wrong): 1 = no attention, 2 = no Wo loads
};

// one 32-key block of kv head g, read in whole cache lines: K rows as 16 lanes x
// 16 B per row, 4 rows per wave instruction (lane l holds piece l % 16 of rows
// tb + 4 i + l / 16, i < 8); V dims 2 l, 2 l + 1 of rows tb .. tb + 31 as buffer
// loads whose row offset is a uniform SGPR soffset (one 256-B row per
// instruction, no per-row VGPR address). Rows are clamped into the cache and
// masked by kv_len. (A first version gave each lane a whole K row: 64 lines per
// instruction, every CU of an XCD hitting the same two L2 channels: 13 us per block.)
template <int D>
__device__ __forceinline__ void awl_load_block(const uint16_t *kc, const uint16_t *vc, int g, int tb, int kv_dim,
                                               int max_seq_len, u32x4_t (&kw)[AWL_KB / 4], uint32_t (&vw)[AWL_KB]) {
	static_assert(D == 128, "16 lanes x 8 halves per K row");
	const int lane = threadIdx.x & 63;
#pragma unroll
	for (int i = 0; i < AWL_KB / 4; ++i) {
		const int t = min(tb + 4 * i + (lane >> 4), max_seq_len - 1);
		kw[i] = load16(kc + (size_t)t * kv_dim + g * D + (lane & 15) * 8);
	}
	const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
	    (void *)(vc + g * D), (short)0, max_seq_len * kv_dim * 2 - g * D * 2, 0x00020000);
#pragma unroll
	for (int tt = 0; tt < AWL_KB; ++tt) {
		const int r = min(tb + tt, max_seq_len - 1);
		vw[tt] = __builtin_amdgcn_raw_buffer_load_b32(vr, lane * 4, r * kv_dim * 2, 0);
	}
}

// scores, online softmax and P.V of one block for the GT (>= G) query heads of kv head g
template <int D, int GT>
__device__ __forceinline__ void awl_block(const float *qs, float (*pbw)[AWL_KB], int g, int G, int tb, int kv_len,
                                          const u32x4_t (&kw)[AWL_KB / 4], const uint32_t (&vw)[AWL_KB],
                                          float (&m)[GT], float (&l)[GT], float (&o)[GT][2]) {
	constexpr int NS = AWL_KB / 4; // row slots per lane
	const int lane = threadIdx.x & 63;
	const int rg = lane >> 4, piece = lane & 15;
	const float sq = sqrtf((float)D);
	// one head at a time (registers): its q piece (dims piece * 8 .. + 8) from LDS,
	// the scores s[i] of keys tb + 4 i + rg (the 16 lanes of a row group end
	// equal), the block's softmax statistics and p into LDS
#pragma unroll
	for (int h = 0; h < GT; ++h) {
		if (h < G) {
			const float *qh = qs + (size_t)(g * G + h) * D + piece * 8;
			const float4_t qa = *(const float4_t *)qh, qb = *(const float4_t *)(qh + 4);
			float sv[NS];
#pragma unroll
			for (int i = 0; i < NS; ++i) {
				float kf[8];
				WF16::unpack(kw[i], kf);
				float d = qa[0] * kf[0];
				d = fmaf(qa[1], kf[1], d);
				d = fmaf(qa[2], kf[2], d);
				d = fmaf(qa[3], kf[3], d);
				d = fmaf(qb[0], kf[4], d);
				d = fmaf(qb[1], kf[5], d);
				d = fmaf(qb[2], kf[6], d);
				d = fmaf(qb[3], kf[7], d);
				d = row16_sum(d);
				sv[i] = tb + 4 * i + rg < kv_len ? d / sq : -FLT_MAX;
			}
			float bm = sv[0];
#pragma unroll
			for (int i = 1; i < NS; ++i)
				bm = fmaxf(bm, sv[i]);
			bm = fmaxf(bm, xor16(bm));
			bm = fmaxf(bm, xor32(bm));
			const float mn = fmaxf(m[h], bm);
			float ls = 0.0f;
#pragma unroll
			for (int i = 0; i < NS; ++i) {
				const float pr = tb + 4 * i + rg < kv_len ? expf(sv[i] - mn) : 0.0f;
				ls += pr;
				if (piece == 0)
					pbw[h][4 * i + rg] = pr;
			}
			ls += xor16(ls);
			ls += xor32(ls);
			const float r = expf(m[h] - mn); // 0 on the first block (m = -FLT_MAX)
			l[h] = l[h] * r + ls;
			o[h][0] *= r;
			o[h][1] *= r;
			m[h] = mn;
		}
	}
	asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // this wave's p row is in LDS before any lane reads it
#pragma unroll
	for (int t4 = 0; t4 < AWL_KB; t4 += 4) {
#pragma unroll
		for (int h = 0; h < GT; ++h) {
			if (h < G) {
				const float4_t pv = *(const float4_t *)&pbw[h][t4];
#pragma unroll
				for (int u = 0; u < 4; ++u) {
					const half2_t hv = __builtin_bit_cast(half2_t, vw[t4 + u]);
					const bool ok = tb + t4 + u < kv_len; // p is 0 there; zero v too (stale rows may be inf/nan)
					o[h][0] = fmaf(pv[u], ok ? (float)hv[0] : 0.0f, o[h][0]);
					o[h][1] = fmaf(pv[u], ok ? (float)hv[1] : 0.0f, o[h][1]);
				}
			}
		}
	}
}

template <class WT, int GT, int XS>
__global__ __launch_bounds__(AWL_THREADS) void attn_wo_local_kernel(const float *q, const uint16_t *kc,
                                                                    const uint16_t *vc, const StepState *step,
                                                                    AttnWoLocalArgs p) {
	constexpr int D = 128;
	constexpr int EPL = WT::EPL;
	constexpr int WOT = AWL_WO_WAVES * 64;     // Wo threads
	constexpr int LPT = 8 * XS;                // 16-byte Wo loads per Wo thread (16 rows x XS * 4 KB / 8 KB)
	constexpr int QD = 4096 * XS / WT::BYTES;  // q_dim: Wo rows are XS * 4 KB
	constexpr int QPT = QD / (4 * AWL_AT_WAVES * 64); // q float4 per attention thread
	static_assert(AWO_RPW == 16 && QPT >= 1, "16 Wo rows per workgroup, q_dim >= 2048");
	__shared__ __attribute__((aligned(16))) float qs[QD];
	__shared__ __attribute__((aligned(16))) float os[QD];
	__shared__ __attribute__((aligned(16))) float pb[AWL_AT_WAVES][GT][AWL_KB];
	__shared__ float rowpart[AWO_RPW][AWL_WO_WAVES];
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
	const bool wo_wave = wave < AWL_WO_WAVES;
	const int G = p.n_heads / p.n_kv;
	const int kv_dim = p.n_kv * D;
	unsigned long long *tr = p.trace && tid == 0 ? p.trace + (size_t)blockIdx.x * 4 : nullptr;
	if (tr) // [0] start, [1] attention in LDS, [2] Wo slice landed, [3] end
		tr[0] = __builtin_amdgcn_s_memrealtime();
	const int row0 = blockIdx.x * AWO_RPW;
	const int lrow0 = min(row0, p.dim - AWO_RPW); // last slice shifted back: unconditional loads

	// The two roles run as separate code paths, each with its own three workgroup
	// barriers (the role is wave-uniform), so that the Wo slice's registers are not
	// live across the attention code and vice versa.
	if (wo_wave) { // ---- the Wo slice, at once
		if (p.kv_first)
			awl_barrier(); // (0) the attention waves' K/V loads are ahead of the slice in the CU's queue
		u32x4_t wr[LPT];
		const char *wbase = p.wo + (size_t)lrow0 * p.q_dim * WT::BYTES;
#pragma unroll
		for (int i = 0; i < LPT; ++i)
			wr[i] = p.ablate & 2 ? u32x4_t{0u, 0u, 0u, 0u} : load_nt16(wbase + ((size_t)i * WOT + tid) * 16);
		if (tid < AWO_RPW * AWL_WO_WAVES)
			(&rowpart[0][0])[tid] = 0.0f;
		awl_barrier(); // (1) q staged
		awl_barrier(); // (2) attention output in os
		if (tr)
			tr[1] = __builtin_amdgcn_s_memrealtime();
		// thread tid holds column piece cp of rows i (XS = 2) or 2 i + tid / 256 (XS = 1)
		const int cp = XS == 2 ? tid : (tid & 255);
		float xv[EPL];
#pragma unroll
		for (int e = 0; e < EPL; e += 4) {
			const float4_t t4 = *(const float4_t *)(os + cp * EPL + e);
			xv[e] = t4[0], xv[e + 1] = t4[1], xv[e + 2] = t4[2], xv[e + 3] = t4[3];
		}
		if (tr) {
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			tr[2] = __builtin_amdgcn_s_memrealtime();
		}
		float a[LPT];
#pragma unroll
		for (int i = 0; i < LPT; ++i) {
			float a0 = 0.0f, a1 = 0.0f;
			eng_dot16<WT>(a0, a1, wr[i], xv);
			a[i] = a0 + a1;
		}
#pragma unroll
		for (int i0 = 0; i0 < LPT; i0 += 4) {
			const float acc[4] = {a[i0], a[i0 + 1], a[i0 + 2], a[i0 + 3]};
			const float tot = eng_sum4_t(acc); // lanes 16 k .. 16 k + 15: value i0 + k
			if ((lane & 15) == 0) {
				const int i = i0 + (lane >> 4);
				const int r = XS == 2 ? i : 2 * i + (wave >= AWL_WO_WAVES / 2 ? 1 : 0);
				rowpart[r][wave] = tot;
			}
		}
		awl_barrier(); // (3) row partials
	} else { // ---- q, this wave's first K/V block, then the attention of kv head aw (+ 8 k)
		const int aw = wave - AWL_WO_WAVES;
		const int at = tid - WOT;
		float4_t qv[QPT];
#pragma unroll
		for (int k = 0; k < QPT; ++k)
			qv[k] = *(const float4_t *)(q + (size_t)(k * AWL_AT_WAVES * 64 + at) * 4);
		const int kv_len = p.ablate & 1 ? 0 : step->kv_len;
		u32x4_t kw[AWL_KB / 4];
		uint32_t vw[AWL_KB];
		awl_load_block<D>(kc, vc, min(aw, p.n_kv - 1), 0, kv_dim, p.max_seq_len, kw, vw);
		if (p.kv_first)
			awl_barrier(); // (0)
#pragma unroll
		for (int k = 0; k < QPT; ++k)
			*(float4_t *)(qs + (size_t)(k * AWL_AT_WAVES * 64 + at) * 4) = qv[k];
		awl_barrier(); // (1)
		for (int g = aw; g < p.n_kv; g += AWL_AT_WAVES) {
			float m[GT], l[GT], o[GT][2];
#pragma unroll
			for (int h = 0; h < GT; ++h)
				m[h] = -FLT_MAX, l[h] = 0.0f, o[h][0] = o[h][1] = 0.0f;
			for (int tb = 0; tb < kv_len; tb += AWL_KB) {
				if (g != aw || tb != 0)
					awl_load_block<D>(kc, vc, g, tb, kv_dim, p.max_seq_len, kw, vw);
				awl_block<D, GT>(qs, pb[aw], g, G, tb, kv_len, kw, vw, m, l, o);
			}
#pragma unroll
			for (int h = 0; h < GT; ++h) {
				if (h < G) {
					float *op = os + (size_t)(g * G + h) * D + 2 * lane;
					op[0] = o[h][0] / l[h];
					op[1] = o[h][1] / l[h];
				}
			}
		}
		awl_barrier(); // (2)
		awl_barrier(); // (3)
	}
	const int row = lrow0 + tid;
	if (tid < AWO_RPW && row >= row0) {
		float s = 0.0f;
#pragma unroll
		for (int w = 0; w < AWL_WO_WAVES; w += 2)
			s += rowpart[tid][w] + rowpart[tid][w + 1];
		p.x[row] += s;
	}
	if (tr)
		tr[3] = __builtin_amdgcn_s_memrealtime();
}
