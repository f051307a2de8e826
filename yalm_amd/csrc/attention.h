// attention.h — split-KV ("flash-decode") grouped-query attention for one
// token over the fp16 sliding-window KV cache, wave64-native, one launch.
//
// Replaces attn_dot / attn_softmax / att_mix (infer.cu:338-524: three launches,
// 32-lane layout, each K/V row re-read once per query head). Here one
// workgroup owns (kv head g, key chunk s): every K and V row of the chunk is
// read from HBM exactly once — K and V loads are issued together up front —
// and serves all G = n_heads / n_kv_heads query heads of the group.
// Semantics follow the CPU oracle attn (infer.cpp:216-248):
//   s_t = (q . k_t) / sqrt(head_dim);  p = softmax(s);  out = sum_t p_t v_t.
// Chunks are merged inside the same launch: each workgroup publishes its
// (max, sum, unnormalised out) partial, takes an arrival ticket, and the last
// workgroup of kv head g combines all chunks in chunk order (deterministic,
// independent of arrival order) — the agent-scope release/acquire hand-off of
// cdna_hip_programming.md Guideline 16 / "In-launch split-K reduction".
#pragma once

#include <float.h>

#include "device_common.h"

#define ATTN_THREADS 256
#define ATTN_WAVES (ATTN_THREADS / YALM_WAVE)
#define ATTN_CHUNK 128

// D = head_dim (multiple of 8, D/8 a power of two <= 64); GT >= G.
template <int D, int GT>
__global__ __launch_bounds__(ATTN_THREADS) void attn_decode_kernel(
    const float *__restrict__ q, const uint16_t *__restrict__ kc, const uint16_t *__restrict__ vc,
    const StepState *__restrict__ step, int n_heads, int n_kv_heads, int max_seq_len, int nsplit,
    float *__restrict__ part, unsigned *__restrict__ counters, float *__restrict__ out, float *__restrict__ att_dbg) {
	constexpr int LPK = D / 8;                       // lanes per K/V row, 16 B each
	constexpr int KPW = 64 / LPK;                    // rows per wave-instruction
	constexpr int RSTEP = ATTN_WAVES * KPW;          // rows per workgroup-instruction
	constexpr int NK = (ATTN_CHUNK + RSTEP - 1) / RSTEP; // rows per lane
	__shared__ float sc[GT][ATTN_CHUNK];
	__shared__ float red[ATTN_WAVES][GT][D];
	__shared__ float ml[GT][2];
	__shared__ int last_flag;

	const int g = blockIdx.x;
	const int s = blockIdx.y;
	const int kv_len = step->kv_len;
	const int t0 = s * ATTN_CHUNK;
	if (t0 >= kv_len)
		return; // whole workgroup exits before any barrier
	const int nt = min(ATTN_CHUNK, kv_len - t0);
	const int ns = (kv_len + ATTN_CHUNK - 1) / ATTN_CHUNK;
	const int G = n_heads / n_kv_heads;
	const int kv_dim = n_kv_heads * D;
	const int lane = threadIdx.x & 63;
	const int wave = threadIdx.x >> 6;
	const int sub = lane / LPK;
	const int piece = lane % LPK;
	const int tl0 = wave * KPW + sub;

	// issue every K and V load of this lane first (one HBM round trip)
	// (rows past the chunk end re-load the last valid row: unconditional loads
	// keep hipcc from branching around each one with a vmcnt(0) wait)
	u32x4_t kw[NK], vw[NK];
#pragma unroll
	for (int i = 0; i < NK; ++i) {
		const int tl = min(tl0 + i * RSTEP, nt - 1);
		const size_t off = (size_t)(t0 + tl) * kv_dim + g * D + piece * 8;
		kw[i] = load16(kc + off);
		vw[i] = load16(vc + off);
	}
	float qr[GT][8];
#pragma unroll
	for (int h = 0; h < GT; ++h) {
		if (h < G) {
			const float *qp = q + (size_t)(g * G + h) * D + piece * 8;
			float4_t a = *(const float4_t *)qp;
			float4_t b = *(const float4_t *)(qp + 4);
			qr[h][0] = a[0], qr[h][1] = a[1], qr[h][2] = a[2], qr[h][3] = a[3];
			qr[h][4] = b[0], qr[h][5] = b[1], qr[h][6] = b[2], qr[h][7] = b[3];
		}
	}
	const float sq = sqrtf((float)D);

	// scores
#pragma unroll
	for (int i = 0; i < NK; ++i) {
		const int tl = tl0 + i * RSTEP;
		if (tl < nt) {
			float kf[8];
			WF16::unpack(kw[i], kf);
#pragma unroll
			for (int h = 0; h < GT; ++h) {
				if (h < G) {
					float d = 0.0f;
#pragma unroll
					for (int e = 0; e < 8; ++e)
						d = fmaf(qr[h][e], kf[e], d);
					d = group_sum(d, LPK);
					if (piece == 0)
						sc[h][tl] = d / sq;
				}
			}
		}
	}
	__syncthreads();

	// chunk-local softmax statistics; wave w owns heads w, w+4, ...
	for (int h = wave; h < G; h += ATTN_WAVES) {
		float m = -FLT_MAX;
		for (int t = lane; t < nt; t += 64)
			m = fmaxf(m, sc[h][t]);
		m = wave_max(m);
		float l = 0.0f;
		for (int t = lane; t < nt; t += 64) {
			const float sv = sc[h][t];
			if (att_dbg)
				att_dbg[(size_t)(g * G + h) * max_seq_len + t0 + t] = sv;
			const float p = expf(sv - m);
			sc[h][t] = p;
			l += p;
		}
		l = wave_sum(l);
		if (lane == 0) {
			ml[h][0] = m;
			ml[h][1] = l;
		}
	}
	__syncthreads();

	// P.V from the prefetched V rows
	float acc[GT][8];
#pragma unroll
	for (int h = 0; h < GT; ++h)
#pragma unroll
		for (int e = 0; e < 8; ++e)
			acc[h][e] = 0.0f;
#pragma unroll
	for (int i = 0; i < NK; ++i) {
		const int tl = tl0 + i * RSTEP;
		if (tl < nt) {
			float vf[8];
			WF16::unpack(vw[i], vf);
#pragma unroll
			for (int h = 0; h < GT; ++h) {
				if (h < G) {
					const float p = sc[h][tl];
#pragma unroll
					for (int e = 0; e < 8; ++e)
						acc[h][e] = fmaf(p, vf[e], acc[h][e]);
				}
			}
		}
	}
#pragma unroll
	for (int off = LPK; off < 64; off <<= 1)
#pragma unroll
		for (int h = 0; h < GT; ++h)
#pragma unroll
			for (int e = 0; e < 8; ++e)
				acc[h][e] += __shfl_xor(acc[h][e], off, 64);
	if (sub == 0) {
#pragma unroll
		for (int h = 0; h < GT; ++h)
			if (h < G)
#pragma unroll
				for (int e = 0; e < 8; ++e)
					red[wave][h][piece * 8 + e] = acc[h][e];
	}
	__syncthreads();

	if (ns == 1) { // single chunk: normalise and write the head outputs directly
		for (int i = threadIdx.x; i < G * D; i += ATTN_THREADS) {
			const int h = i / D, d = i % D;
			float o = 0.0f;
#pragma unroll
			for (int w = 0; w < ATTN_WAVES; ++w)
				o += red[w][h][d];
			out[(size_t)(g * G + h) * D + d] = o / ml[h][1];
		}
		if (att_dbg) {
			for (int i = threadIdx.x; i < G * nt; i += ATTN_THREADS) {
				const int h = i / nt, t = i % nt;
				float *a = att_dbg + (size_t)(g * G + h) * max_seq_len + t;
				*a = sc[h][t] / ml[h][1];
			}
		}
		return;
	}

	// publish this chunk's partial: o[D], m, l per head
	for (int i = threadIdx.x; i < G * D; i += ATTN_THREADS) {
		const int h = i / D, d = i % D;
		float o = 0.0f;
#pragma unroll
		for (int w = 0; w < ATTN_WAVES; ++w)
			o += red[w][h][d];
		part[((size_t)(g * G + h) * nsplit + s) * (D + 2) + d] = o;
	}
	if (threadIdx.x < G) {
		float *pp = part + ((size_t)(g * G + threadIdx.x) * nsplit + s) * (D + 2);
		pp[D] = ml[threadIdx.x][0];
		pp[D + 1] = ml[threadIdx.x][1];
	}
	// release: every storing wave drains, barrier, one agent-scope release, ticket
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if (threadIdx.x == 0) {
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		const unsigned ticket = __hip_atomic_fetch_add(&counters[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const int last = ticket == (unsigned)(ns - 1);
		if (last) {
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			// reset for the next launch (kernel boundary orders it before reuse)
			__hip_atomic_store(&counters[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		last_flag = last;
	}
	__syncthreads();
	if (!last_flag)
		return;

	// last arriver: merge the ns chunk partials of heads g*G .. g*G+G-1 in chunk order
	for (int h = wave; h < G; h += ATTN_WAVES) {
		const float *ph = part + (size_t)(g * G + h) * nsplit * (D + 2);
		float M = -FLT_MAX;
		for (int c = 0; c < ns; ++c)
			M = fmaxf(M, ph[c * (D + 2) + D]);
		float L = 0.0f;
		for (int c = 0; c < ns; ++c)
			L += expf(ph[c * (D + 2) + D] - M) * ph[c * (D + 2) + D + 1];
		for (int d = lane; d < D; d += 64) {
			float o = 0.0f;
			for (int c = 0; c < ns; ++c)
				o += expf(ph[c * (D + 2) + D] - M) * ph[c * (D + 2) + d];
			out[(size_t)(g * G + h) * D + d] = o / L;
		}
		if (att_dbg) {
			// raw scores were written by every chunk's workgroup before its release
			for (int t = lane; t < kv_len; t += 64) {
				float *a = att_dbg + (size_t)(g * G + h) * max_seq_len + t;
				*a = expf(*a - M) / L;
			}
		}
	}
}
