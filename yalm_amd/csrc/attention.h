// attention.h — split-KV ("flash-decode") grouped-query attention for one
// token over the fp16 sliding-window KV cache, wave64-native.
//
// Replaces attn_dot / attn_softmax / att_mix (infer.cu:338-524), whose
// 32-lane layout re-reads each K/V row once per query head. Here one
// workgroup owns (kv head g, key chunk s): every K and V row of the chunk is
// read from HBM exactly once and serves all G = n_heads / n_kv_heads query
// heads of the group. Semantics follow the CPU oracle attn (infer.cpp:216-248):
// s_t = (q . k_t) / sqrt(head_dim); p = softmax(s); out = sum_t p_t v_t.
// The per-chunk (max, sum, unnormalised out) partials are merged by
// attn_combine_kernel with the usual rescaling.
#pragma once

#include <float.h>

#include "device_common.h"

#define ATTN_THREADS 256
#define ATTN_WAVES (ATTN_THREADS / YALM_WAVE)
#define ATTN_MAXCHUNK 256

// D = head_dim (multiple of 8, D/8 a power of two <= 64); GT >= G.
template <int D, int GT>
__global__ __launch_bounds__(ATTN_THREADS) void attn_split_kernel(const float *__restrict__ q,
                                                                  const uint16_t *__restrict__ kc,
                                                                  const uint16_t *__restrict__ vc,
                                                                  const StepState *__restrict__ step, int n_heads,
                                                                  int n_kv_heads, int max_seq_len, int chunk,
                                                                  int nsplit, float *__restrict__ part,
                                                                  float *__restrict__ att_dbg) {
	constexpr int LPK = D / 8;    // lanes per K/V row, 16 B each
	constexpr int KPW = 64 / LPK; // rows per wave-instruction
	__shared__ float sc[GT][ATTN_MAXCHUNK];
	__shared__ float red[ATTN_WAVES][GT][D];
	__shared__ float ml[GT][2];

	const int g = blockIdx.x;
	const int s = blockIdx.y;
	const int kv_len = step->kv_len;
	const int t0 = s * chunk;
	if (t0 >= kv_len)
		return; // whole workgroup exits: no barrier is reached
	const int nt = min(chunk, kv_len - t0);
	const int G = n_heads / n_kv_heads;
	const int kv_dim = n_kv_heads * D;
	const int lane = threadIdx.x & 63;
	const int wave = threadIdx.x >> 6;
	const int sub = lane / LPK;
	const int piece = lane % LPK;
	const float sq = sqrtf((float)D);

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

	// scores
	for (int tl = wave * KPW + sub; tl < nt; tl += ATTN_WAVES * KPW) {
		u32x4_t kw = load16(kc + (size_t)(t0 + tl) * kv_dim + g * D + piece * 8);
		float kf[8];
		WF16::unpack(kw, kf);
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
	__syncthreads();

	// chunk-local softmax statistics; wave w owns heads w, w+4, ...
	for (int h = wave; h < G; h += ATTN_WAVES) {
		float m = -FLT_MAX;
		for (int t = lane; t < nt; t += 64)
			m = fmaxf(m, sc[h][t]);
		m = wave_max(m);
		float l = 0.0f;
		for (int t = lane; t < nt; t += 64) {
			float sv = sc[h][t];
			if (att_dbg)
				att_dbg[(size_t)(g * G + h) * max_seq_len + t0 + t] = sv;
			float p = expf(sv - m);
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

	// P.V
	float acc[GT][8];
#pragma unroll
	for (int h = 0; h < GT; ++h)
#pragma unroll
		for (int e = 0; e < 8; ++e)
			acc[h][e] = 0.0f;
	for (int tl = wave * KPW + sub; tl < nt; tl += ATTN_WAVES * KPW) {
		u32x4_t vw = load16(vc + (size_t)(t0 + tl) * kv_dim + g * D + piece * 8);
		float vf[8];
		WF16::unpack(vw, vf);
#pragma unroll
		for (int h = 0; h < GT; ++h) {
			if (h < G) {
				float p = sc[h][tl];
#pragma unroll
				for (int e = 0; e < 8; ++e)
					acc[h][e] = fmaf(p, vf[e], acc[h][e]);
			}
		}
	}
	// reduce over the KPW row slots of the wave (lanes with equal `piece`)
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
}

// Merge the per-chunk partials of head h = blockIdx.x into out[h*D .. +D].
// With att_dbg, also turns the raw scores into softmax probabilities
// (the reference's mha_cuda returns them, infer.cu:890-935).
template <int D>
__global__ __launch_bounds__(128) void attn_combine_kernel(const float *__restrict__ part,
                                                           const StepState *__restrict__ step, int chunk, int nsplit,
                                                           int max_seq_len, float *__restrict__ out,
                                                           float *__restrict__ att_dbg) {
	const int h = blockIdx.x;
	const int kv_len = step->kv_len;
	const int ns = (kv_len + chunk - 1) / chunk;
	const float *ph = part + (size_t)h * nsplit * (D + 2);
	float M = -FLT_MAX;
	for (int s = 0; s < ns; ++s)
		M = fmaxf(M, ph[s * (D + 2) + D]);
	float L = 0.0f;
	for (int s = 0; s < ns; ++s)
		L += expf(ph[s * (D + 2) + D] - M) * ph[s * (D + 2) + D + 1];
	for (int d = threadIdx.x; d < D; d += blockDim.x) {
		float o = 0.0f;
		for (int s = 0; s < ns; ++s)
			o += expf(ph[s * (D + 2) + D] - M) * ph[s * (D + 2) + d];
		out[(size_t)h * D + d] = o / L;
	}
	if (att_dbg) {
		for (int t = threadIdx.x; t < kv_len; t += blockDim.x) {
			float *a = att_dbg + (size_t)h * max_seq_len + t;
			*a = expf(*a - M) / L;
		}
	}
}
