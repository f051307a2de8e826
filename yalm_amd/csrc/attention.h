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
// small (64 keys) so the KV read spreads over many CUs, and all K, V and q
// loads are issued speculatively before kv_len is known (rows past kv_len are
// read but masked), overlapping the step-state load.
//  * kv_len <= CHUNK: the workgroup normalises and writes the heads directly.
//    Longer contexts publish (max, sum, unnormalised out) per chunk as 8-byte
//    {value, tag} granules (one sc1 store each: the data is its own ready flag,
//    MI355X_MICROARCH.md §visibility R2); the MERGER -- the highest-index
//    workgroup with work for kv head g, so every workgroup it waits for was
//    dispatched before it -- gathers all chunks' granules, re-reading until
//    every tag holds this launch's tag, and merges them in chunk order
//    (deterministic). Round 2 used a drained write + agent-scope arrival ticket
//    + last-arriver merge: three serialised round trips instead of one.
//    Tags: epoch * n_layers + layer, unique per (forward, layer), so the one
//    partial buffer serves every layer and is never reset.
#pragma once

#include <float.h>

#include "device_common.h"

#define ATTN_THREADS 256
#define ATTN_WAVES (ATTN_THREADS / YALM_WAVE)

// Keys per workgroup. Small on purpose: one CU streams only ~50-100 GB/s, so
// a decode-size KV read must be spread over many CUs to be fast (kv 4096 ->
// 64 chunks x n_kv_heads workgroups); the merge is a cheap sc1 hand-off.
template <int D>
constexpr int attn_chunk() {
	return 64;
}

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

// Head outputs of the fused launch: `reps` copies, `stride` granules apart (one per
// XCD-group of consumers, attn_wo.h AWO_GR), so the 256 consumer workgroups' reads
// spread over `reps` x the addresses.
template <bool GRAN>
__device__ __forceinline__ void attn_out_rep(float *out, size_t i, float v, unsigned tag, int reps, size_t stride) {
	if constexpr (GRAN) {
		for (int r = 0; r < reps; ++r)
			attn_out<true>(out, i + (size_t)r * stride, v, tag);
	} else {
		out[i] = v;
	}
}

// One workgroup's share of the split-KV attention: kv head g, key chunks s0,
// s0 + S, ... `hook()` runs right after the speculative K/V and q loads are
// issued (attn_wo.h issues its weight stream there, behind them in vmcnt order).
// Returns true on the workgroup that wrote the final head outputs of kv head g
// (the single-chunk writer or the merger); the result is workgroup-uniform.
// D = head_dim (multiple of 8, D/8 a power of two <= 64); GT >= G.
// GRAN: outputs as {value, gtag} granules into `out` read as unsigned long long[].
// part: [n_heads][nsplit][D + 2] granules tagged ptag (attn_part_tag); err: bit 2
// set if the merger's bounded wait gave up (results wrong, reported).
template <int D, int GT, bool GRAN, class Hook>
// (no __restrict__ here: with it the K/V and q loads may legally sink below the
// hook's asm barrier once inlined; the standalone kernel keeps it on its arguments)
__device__ __forceinline__ bool attn_decode_body(bool active, int g, int s0, int S, const float *q, const uint16_t *kc,
                                                 const uint16_t *vc, const StepState *step, int n_heads,
                                                 int n_kv_heads, int max_seq_len, int nsplit, unsigned long long *part,
                                                 unsigned ptag, unsigned *err, float *out, float *att_dbg,
                                                 Hook &&hook, unsigned gtag = 0, int greps = 1) {
	constexpr int CHUNK = attn_chunk<D>();
	constexpr int LPK = D / 8;                     // lanes per K/V row, 16 B each
	constexpr int KPW = 64 / LPK;                  // rows per wave-instruction
	constexpr int RSTEP = ATTN_WAVES * KPW;        // rows per workgroup-instruction
	constexpr int NK = (CHUNK + RSTEP - 1) / RSTEP; // rows per lane
	__shared__ __attribute__((aligned(16))) float sp[GT * CHUNK * LPK]; // per-lane partial dots
	__shared__ float sc[GT][CHUNK];
	__shared__ __attribute__((aligned(16))) float red[ATTN_WAVES * KPW][GT][D]; // per-row-slot P.V partials
	__shared__ float ml[GT][2];

	const int G = n_heads / n_kv_heads;
	const int kv_dim = n_kv_heads * D;
	const int lane = threadIdx.x & 63;
	const int wave = threadIdx.x >> 6;
	const int tid = threadIdx.x;
	const int sub = lane / LPK;
	const int piece = lane % LPK;
	const int tl0 = wave * KPW + sub;

	auto load_kv = [&](int t0, u32x4_t (&kw)[NK], u32x4_t (&vw)[NK]) {
#pragma unroll
		for (int i = 0; i < NK; ++i) {
			const int t = min(t0 + tl0 + i * RSTEP, max_seq_len - 1);
			const size_t off = (size_t)t * kv_dim + g * D + piece * 8;
			kw[i] = load16(kc + off);
			vw[i] = load16(vc + off);
		}
	};
	// ---- speculative loads of the first chunk (rows clamped to the cache), q and step in flight together
	u32x4_t kw[NK], vw[NK];
	load_kv(s0 * CHUNK, kw, vw);
	float qr[GT][8];
#pragma unroll
	for (int h = 0; h < GT; ++h) {
		const int hh = h < G ? h : 0; // unconditional loads (no branch around each)
		const float *qp = q + (size_t)(g * G + hh) * D + piece * 8;
		const float4_t a = *(const float4_t *)qp;
		const float4_t b = *(const float4_t *)(qp + 4);
		qr[h][0] = a[0], qr[h][1] = a[1], qr[h][2] = a[2], qr[h][3] = a[3];
		qr[h][4] = b[0], qr[h][5] = b[1], qr[h][6] = b[2], qr[h][7] = b[3];
	}
	const int kv_len = step->kv_len; // issued before the hook's loads: its wait must not cover them
	hook();
	if (!active || s0 * CHUNK >= kv_len)
		return false; // whole workgroup leaves before any barrier
	const int ns = (kv_len + CHUNK - 1) / CHUNK;
	const float sq = sqrtf((float)D);

	// chunks s0, s0 + S, ... (S = gridDim.y splits; one pass for kv_len <= S * CHUNK)
	for (int cidx = s0; cidx < ns; cidx += S) {
		const int t0 = cidx * CHUNK;
		if (cidx != s0)
			load_kv(t0, kw, vw);
		const int nt = min(CHUNK, kv_len - t0);

		// ---- scores: each lane's 8-element partial dots go to LDS; one thread per
		// (head, key) then sums the D/8 partials in piece order (no shuffles)
#pragma unroll
		for (int i = 0; i < NK; ++i) {
			const int tl = tl0 + i * RSTEP;
			float kf[8];
			WF16::unpack(kw[i], kf);
#pragma unroll
			for (int h = 0; h < GT; ++h) {
				float d = 0.0f;
#pragma unroll
				for (int e = 0; e < 8; ++e)
					d = fmaf(qr[h][e], kf[e], d);
				if (h < G && tl < CHUNK)
					sp[(h * CHUNK + tl) * LPK + piece] = d;
			}
		}
		__syncthreads();
		for (int i = tid; i < G * CHUNK; i += ATTN_THREADS) {
			const int h = i / CHUNK, t = i % CHUNK;
			const float *pp = &sp[(h * CHUNK + t) * LPK];
			float d = 0.0f;
			if constexpr (LPK >= 4) {
#pragma unroll
				for (int j = 0; j < LPK; j += 4) {
					const float4_t v = *(const float4_t *)(pp + j);
					d += v[0] + v[1] + v[2] + v[3];
				}
			} else {
#pragma unroll
				for (int j = 0; j < LPK; ++j)
					d += pp[j];
			}
			sc[h][t] = d / sq;
		}
		__syncthreads();

		// ---- chunk-local softmax statistics; wave w owns heads w, w+4, ... (DPP reductions)
		for (int h = wave; h < G; h += ATTN_WAVES) {
			float m = -FLT_MAX;
			for (int t = lane; t < nt; t += 64)
				m = fmaxf(m, sc[h][t]);
			m = wave_max(m);
			float l = 0.0f;
			for (int t = lane; t < nt; t += 64) {
				const float sv = sc[h][t];
				if (att_dbg)
					st_sc1(att_dbg + (size_t)(g * G + h) * max_seq_len + t0 + t, sv);
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

		// ---- P.V from the loaded V rows; per-row-slot partials to LDS
		float acc[GT][8];
#pragma unroll
		for (int h = 0; h < GT; ++h)
#pragma unroll
			for (int e = 0; e < 8; ++e)
				acc[h][e] = 0.0f;
#pragma unroll
		for (int i = 0; i < NK; ++i) {
			const int tl = tl0 + i * RSTEP;
			const float pv = tl < nt ? 1.0f : 0.0f;
			float vf[8];
			WF16::unpack(vw[i], vf);
#pragma unroll
			for (int h = 0; h < GT; ++h) {
				const float p = tl < nt ? sc[h < G ? h : 0][tl < CHUNK ? tl : 0] : 0.0f;
#pragma unroll
				for (int e = 0; e < 8; ++e)
					acc[h][e] = fmaf(p, vf[e] * pv, acc[h][e]);
			}
		}
		{
			const int slot = wave * KPW + sub;
#pragma unroll
			for (int h = 0; h < GT; ++h) {
				if (h < G) {
					float *rp = &red[slot][h][piece * 8];
					*(float4_t *)rp = float4_t{acc[h][0], acc[h][1], acc[h][2], acc[h][3]};
					*(float4_t *)(rp + 4) = float4_t{acc[h][4], acc[h][5], acc[h][6], acc[h][7]};
				}
			}
		}
		__syncthreads();

		if (ns == 1) { // single chunk: normalise and write the head outputs directly
			for (int i = tid; i < G * D; i += ATTN_THREADS) {
				const int h = i / D, d = i % D;
				float o = 0.0f;
#pragma unroll
				for (int w = 0; w < ATTN_WAVES * KPW; ++w)
					o += red[w][h][d];
				attn_out_rep<GRAN>(out, (size_t)(g * G + h) * D + d, o / ml[h][1], gtag, greps, (size_t)n_heads * D);
			}
			if (att_dbg) {
				for (int i = tid; i < G * nt; i += ATTN_THREADS) {
					const int h = i / nt, t = i % nt;
					att_dbg[(size_t)(g * G + h) * max_seq_len + t] = sc[h][t] / ml[h][1];
				}
			}
			return true;
		}

		// ---- publish this chunk's partial (o[D], m, l per head) as tagged granules
		if (att_dbg) // test hook: the raw scores must be visible before the merger sees the tags
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		for (int i = tid; i < G * D; i += ATTN_THREADS) {
			const int h = i / D, d = i % D;
			float o = 0.0f;
#pragma unroll
			for (int w = 0; w < ATTN_WAVES * KPW; ++w)
				o += red[w][h][d];
			attn_out<true>((float *)part, ((size_t)(g * G + h) * nsplit + cidx) * (D + 2) + d, o, ptag);
		}
		if (tid < G) {
			const size_t pp = ((size_t)(g * G + tid) * nsplit + cidx) * (D + 2);
			attn_out<true>((float *)part, pp + D, ml[tid][0], ptag);
			attn_out<true>((float *)part, pp + D + 1, ml[tid][1], ptag);
		}
		__syncthreads(); // LDS (sp, sc, ml, red) reused by the next chunk
	}
	if (s0 != min(ns, S) - 1)
		return false; // not the merger: nothing to wait for

	// ---- merger: gather the ns chunk partials of heads g*G .. as granules, re-reading
	// a batch of MB chunks until every tag holds ptag (one round trip when the other
	// workgroups are done, which they usually are: they started together), then merge
	// in chunk order with the online rescaling of flash-decoding.
	constexpr int MB = 8;
	constexpr int DPL = D >= 64 ? D / 64 : 1; // dims per lane
	const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + ATTN_TIMEOUT;
	bool alive = true;
	for (int h = wave; h < G; h += ATTN_WAVES) {
		const unsigned long long *ph = part + (size_t)(g * G + h) * nsplit * (D + 2);
		float M = -FLT_MAX, L = 0.0f, o[DPL];
#pragma unroll
		for (int k = 0; k < DPL; ++k)
			o[k] = 0.0f;
		const int dl = lane < D ? lane : 0; // lanes past D (D < 64) re-read dim 0 and only follow along
		for (int c0 = 0; c0 < ns; c0 += MB) {
			float mb[MB], lb[MB], ob[MB][DPL];
			for (;;) {
				unsigned long long gm[MB], gl[MB], go[MB][DPL];
#pragma unroll
				for (int j = 0; j < MB; ++j) {
					const int c = min(c0 + j, ns - 1);
					const unsigned long long *pc = ph + (size_t)c * (D + 2);
					gm[j] = gran_ld(pc + D);
					gl[j] = gran_ld(pc + D + 1);
#pragma unroll
					for (int k = 0; k < DPL; ++k)
						go[j][k] = gran_ld(pc + dl + 64 * k);
				}
				bool ok = true;
#pragma unroll
				for (int j = 0; j < MB; ++j) {
					ok = ok && (unsigned)(gm[j] >> 32) == ptag && (unsigned)(gl[j] >> 32) == ptag;
#pragma unroll
					for (int k = 0; k < DPL; ++k)
						ok = ok && (unsigned)(go[j][k] >> 32) == ptag;
					mb[j] = __uint_as_float((unsigned)gm[j]);
					lb[j] = __uint_as_float((unsigned)gl[j]);
#pragma unroll
					for (int k = 0; k < DPL; ++k)
						ob[j][k] = __uint_as_float((unsigned)go[j][k]);
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
			float Mn = M;
#pragma unroll
			for (int j = 0; j < MB; ++j)
				if (c0 + j < ns)
					Mn = fmaxf(Mn, mb[j]);
			const float r = expf(M - Mn); // 0 on the first batch (M = -FLT_MAX)
			L *= r;
#pragma unroll
			for (int k = 0; k < DPL; ++k)
				o[k] *= r;
#pragma unroll
			for (int j = 0; j < MB; ++j) {
				if (c0 + j < ns) {
					const float w = expf(mb[j] - Mn);
					L += w * lb[j];
#pragma unroll
					for (int k = 0; k < DPL; ++k)
						o[k] += w * ob[j][k];
				}
			}
			M = Mn;
		}
		if (lane < D) {
#pragma unroll
			for (int k = 0; k < DPL; ++k)
				attn_out_rep<GRAN>(out, (size_t)(g * G + h) * D + lane + 64 * k, o[k] / L, gtag, greps,
				                   (size_t)n_heads * D);
		}
		if (att_dbg) {
			for (int t = lane; t < kv_len; t += 64) {
				float *a = att_dbg + (size_t)(g * G + h) * max_seq_len + t;
				*a = expf(ld_sc1(a) - M) / L;
			}
		}
	}
	return true;
}

// grid (n_kv_heads, S): workgroup (g, s) is dispatched after (g', s') for every
// s' < s, so the merger (the highest s with work) only waits on earlier ones.
template <int D, int GT>
__global__ __launch_bounds__(ATTN_THREADS) void attn_decode_kernel(
    const float *__restrict__ q, const uint16_t *__restrict__ kc, const uint16_t *__restrict__ vc,
    const StepState *__restrict__ step, int n_heads, int n_kv_heads, int max_seq_len, int nsplit,
    unsigned long long *__restrict__ part, int layer, int n_layers, unsigned *__restrict__ err,
    float *__restrict__ out, float *__restrict__ att_dbg) {
	attn_decode_body<D, GT, false>(true, blockIdx.x, blockIdx.y, gridDim.y, q, kc, vc, step, n_heads, n_kv_heads,
	                               max_seq_len, nsplit, part, attn_part_tag(step, layer, n_layers), err, out, att_dbg,
	                               [] {});
}
