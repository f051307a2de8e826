// ffn.h — the whole feed-forward half of a decode block as ONE launch:
// rmsnorm → W1/W3 + SiLU/GELU-GLU → W2 + residual (infer.cpp:339-384,
// infer.cu:598-620 + 270-288; the reference launches rmsnorm, the GLU GEMV and
// the W2 GEMV separately).
//
// Why: at batch 1 each weight-streaming launch pays a fixed ~3-5 us (kernel
// boundary, first-byte latency of a cold pipe, the last workgroup's tail) on
// top of its bytes. Between the GLU GEMV and the W2 GEMV that gap is pure
// dependency (W2 needs every hb value), not data: the W2 weights can be in
// flight while the last GLU rows finish. Here one grid of NB workgroups (one
// per CU, all co-resident) runs both phases back to back:
//
//   1. GLU phase (8 streaming waves): the gemv_rb_kernel item stream over hidden
//      rows b, b + NB, ... (rows interleaved over workgroups so the chip reads
//      one contiguous window at a time); per-(row, wave) partials in LDS.
//      Near the end of its GLU items every streaming wave's refills run on into
//      its first W2 items, and P more are issued on top: U + P KB of W2 weights
//      per wave are in flight across the seam below.
//   2. Seam (control waves, which hold no weight loads, so their memory ops do
//      not queue behind the stream: vmcnt is in order): one control wave sums
//      the partials, applies act(W1 row) * (W3 row) and publishes this
//      workgroup's hb values with write-through (sc1) 4-byte stores, drains them
//      (vmcnt(0)) and stores the launch epoch into its flag (sc1). It then polls
//      all NB flags (sc1 loads, bounded spin). After a workgroup barrier the
//      control waves gather the whole hb vector (hidden floats) with 16-byte sc1
//      loads into LDS — MI355X_MICROARCH.md §visibility "Valid forms" row 1
//      (one flag per producer workgroup, sc1 stores and loads both sides).
//   3. W2 phase (streaming waves): gemv_rb items over output rows b, b + NB, ...
//      with hb from LDS; per-row partials summed in fixed wave order; the row's
//      owner adds it to x (fused_matmul_add_residuals). Deterministic: every
//      output row has one owner and a fixed summation order.
//
// x is read (rmsnorm staging) by every workgroup before its GLU phase and
// written only after the seam, i.e. after every workgroup has published hb and
// therefore finished staging: no read/write race on x.
//
// Residency: the seam waits on every workgroup of the grid, so all NB must be
// resident at once (NB = CU count, one 1024-thread workgroup per CU; checked
// with the occupancy query at decoder creation). Every spin is bounded (2 s)
// and reports through *err -> engine_check -> YALM_ERR_HIP.
// Flags: one slot of NB words per layer holding the epoch of the last launch
// (StepState::epoch grows per forward and per yalm_block): never reset.
#pragma once

#include "gemv.h"

#define FFN_TIMEOUT 200000000ull // 2 s of s_memrealtime (100 MHz)
#define FFN_W 8                  // streaming waves
#define FFN_C 8                  // control waves (publish, poll, hb gather)
#define FFN_THREADS ((FFN_W + FFN_C) * 64)
#define FFN_TRACE_WORDS 8

struct FfnArgs {
	const char *w1, *w3, *w2; // W1, W3 (hidden, dim); W2 (dim, hidden) — the .yalm layout, untouched
	const float *normw;       // rms_ffn (dim)
	float eps;
	float *x;                 // residual stream (dim)
	float *hb;                // GLU output (hidden), published sc1 by its owner workgroup
	unsigned *flags;          // this layer's per-workgroup epoch flags [NB]
	unsigned *err;            // error bits (bounded spin gave up)
	const StepState *step;    // epoch of this launch
	int dim, hidden;
	unsigned long long *trace; // [NB][FFN_TRACE_WORDS] s_memrealtime stamps or null
};

// Eight 16-byte sc1 loads in one statement, one vmcnt(0) (hipcc does not track
// asm loads: the statement drains its own).
__device__ __forceinline__ void ffn_ld8_sc1(u32x4_t (&v)[8], const float *const (&a)[8]) {
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

// LDS floats: x staging (dim + 64 scratch) | hb (hidden) | GLU partials | W2 partials
__host__ __device__ inline size_t ffn_lds_floats(int dim, int hidden, int NB) {
	const int ngl1 = (hidden + NB - 1) / NB, ngl2 = (dim + NB - 1) / NB;
	return (size_t)dim + 64 + hidden + (size_t)ngl1 * 2 * FFN_W + (size_t)ngl2 * FFN_W;
}

// dim and hidden multiples of 64 * EPL (one 1-KB chunk per wave instruction).
template <class WT, int ACT, int U, int P>
__global__ __launch_bounds__(FFN_THREADS) void ffn_kernel(FfnArgs p) {
	constexpr int W = FFN_W;
	constexpr int EPL = WT::EPL;
	constexpr int CH = YALM_WAVE * EPL;
	constexpr size_t CHB = (size_t)CH * WT::BYTES;
	constexpr int NS = U + P; // W2 pipeline depth
	extern __shared__ __attribute__((aligned(16))) float lds[];
	const int dim = p.dim, hidden = p.hidden;
	const int nch = dim / CH, nch2 = hidden / CH;
	const int NB = gridDim.x, b = blockIdx.x;
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
	const bool ctl = wave >= W;
	const int ngl1 = b < hidden ? (hidden - 1 - b) / NB + 1 : 0; // hidden rows b + gl * NB
	const int ngl2 = b < dim ? (dim - 1 - b) / NB + 1 : 0;       // output rows b + gl * NB
	const int items1 = ngl1 * 2 * nch, items2 = ngl2 * nch2;
	const int mine1 = ctl ? 0 : (items1 > wave ? (items1 - 1 - wave) / W + 1 : 0);
	const int mine2 = ctl ? 0 : (items2 > wave ? (items2 - 1 - wave) / W + 1 : 0);
	const int mine1p = (mine1 + U - 1) / U * U; // GLU items padded to whole slot rounds
	float *xs = lds;
	float *hbs = xs + dim + 64;
	float *part1 = hbs + hidden;           // [ngl1 * 2][W]
	float *part2 = part1 + ngl1 * 2 * W;   // [ngl2][W]
	const size_t lane_off = (size_t)lane * EPL * WT::BYTES;
	const char *dummy = (const char *)p.x + lane * 16; // past-the-end refills: an L2-resident line
	const unsigned epoch = p.step->epoch;
	// stamps: [0] start, [1] GLU partials done, [2] hb published, [3] every flag seen,
	// [4] hb in LDS, [5] end, [6] GLU | W2 items of wave 0
	unsigned long long *tr = p.trace && tid == 0 ? p.trace + (size_t)b * FFN_TRACE_WORDS : nullptr;
	unsigned long long *trc = p.trace && tid == W * 64 ? p.trace + (size_t)b * FFN_TRACE_WORDS : nullptr;
	if (tr)
		tr[0] = __builtin_amdgcn_s_memrealtime();

	// ---- issue cursor over [GLU items | pad | W2 items | dummies] (wave-uniform)
	int ii = 0;
	int ivr = wave / nch, ic = wave - (wave / nch) * nch;     // GLU: virtual row (2 gl + {W1, W3}), chunk
	int jg = wave / nch2, jc = wave - (wave / nch2) * nch2;   // W2: row group, chunk
	auto issue = [&]() -> u32x4_t {
		const char *a = dummy;
		if (ii < mine1) {
			a = ((ivr & 1) ? p.w3 : p.w1) + (size_t)(b + (ivr >> 1) * NB) * dim * WT::BYTES + (size_t)ic * CHB +
			    lane_off;
			ic += W;
			while (ic >= nch) {
				ic -= nch;
				++ivr;
			}
		} else if (ii >= mine1p && ii - mine1p < mine2) {
			a = p.w2 + (size_t)(b + jg * NB) * hidden * WT::BYTES + (size_t)jc * CHB + lane_off;
			jc += W;
			while (jc >= nch2) {
				jc -= nch2;
				++jg;
			}
		}
		++ii;
		return load_nt16(a);
	};

	u32x4_t s[NS];
	if (!ctl) {
#pragma unroll
		for (int u = 0; u < U; ++u)
			s[u] = issue();
	}
	for (int i = tid; i < ngl1 * 2 * W + ngl2 * W; i += FFN_THREADS)
		part1[i] = 0.0f;
	stage_x<true>(xs, p.x, p.normw, dim, p.eps); // rmsnorm(x) * rms_ffn (infer.cpp:341)

	// ---- 1. GLU phase
	if (!ctl) {
		int cvr = wave / nch, cc = wave - (wave / nch) * nch, cur = cvr;
		float acc[1] = {0.0f};
		for (int k = 0; k < mine1p; k += U) {
#pragma unroll
			for (int u = 0; u < U; ++u) {
				if (k + u < mine1) {
					if (cvr != cur) {
						const float t = wave_sum(acc[0]);
						if (lane == 0)
							part1[cur * W + wave] = t;
						acc[0] = 0.0f;
						cur = cvr;
					}
					const u32x4_t wv[1] = {s[u]};
					fma_chunk<WT, 1>(acc, wv, xs + cc * CH + lane * EPL);
					cc += W;
					while (cc >= nch) {
						cc -= nch;
						++cvr;
					}
				}
				s[u] = issue();
			}
		}
		if (mine1 > 0) {
			const float t = wave_sum(acc[0]);
			if (lane == 0)
				part1[cur * W + wave] = t;
		}
		// deepen the W2 stream across the seam
#pragma unroll
		for (int q = 0; q < P; ++q)
			s[U + q] = issue();
	}
	__syncthreads(); // GLU partials complete
	if (tr)
		tr[1] = __builtin_amdgcn_s_memrealtime();

	// ---- 2. seam: publish hb, wait for every workgroup's, gather it into LDS
	if (wave == W) {
		for (int gl = lane; gl < ngl1; gl += 64) {
			float a = 0.0f, c = 0.0f;
			for (int w = 0; w < W; ++w)
				a += part1[(2 * gl) * W + w];
			for (int w = 0; w < W; ++w)
				c += part1[(2 * gl + 1) * W + w];
			__hip_atomic_store(p.hb + b + gl * NB, act_fn<ACT>(a) * c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the publishing wave drains its sc1 stores
		if (lane == 0)
			__hip_atomic_store(p.flags + b, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (trc)
			trc[2] = __builtin_amdgcn_s_memrealtime();
		const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
		bool dead = false;
		for (int f0 = 0; f0 < NB && !dead; f0 += 256) { // flags f0 .. f0 + 255: four loads per lane at once
			const unsigned *fa[4];
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				const int f = f0 + 64 * k + lane;
				fa[k] = p.flags + (f < NB ? f : b); // past the grid: this workgroup's own (already set) flag
			}
			for (;;) {
				unsigned v[4];
#pragma unroll
				for (int k = 0; k < 4; ++k)
					v[k] = __hip_atomic_load(fa[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				if (__all(v[0] == epoch && v[1] == epoch && v[2] == epoch && v[3] == epoch))
					break;
				__builtin_amdgcn_s_sleep(1);
				if (__builtin_amdgcn_s_memrealtime() - t0 > FFN_TIMEOUT) {
					if (lane == 0)
						__hip_atomic_fetch_or(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					dead = true;
					break;
				}
			}
		}
		if (trc)
			trc[3] = __builtin_amdgcn_s_memrealtime();
	}
	__syncthreads(); // every flag seen (the polling wave joins)
	if (ctl) {
		const int ct = tid - W * 64;
		constexpr int CT = FFN_C * 64;
		const int npieces = hidden / 4;
		for (int q0 = 0; q0 < npieces; q0 += 8 * CT) {
			const float *a[8];
#pragma unroll
			for (int k = 0; k < 8; ++k) {
				const int q = q0 + k * CT + ct;
				a[k] = p.hb + 4 * (q < npieces ? q : 0);
			}
			u32x4_t v[8];
			ffn_ld8_sc1(v, a);
#pragma unroll
			for (int k = 0; k < 8; ++k) {
				const int q = q0 + k * CT + ct;
				if (q < npieces) {
					float4_t f;
					f[0] = __uint_as_float(v[k][0]);
					f[1] = __uint_as_float(v[k][1]);
					f[2] = __uint_as_float(v[k][2]);
					f[3] = __uint_as_float(v[k][3]);
					*(float4_t *)(hbs + 4 * q) = f;
				}
			}
		}
	}
	__syncthreads(); // hb in LDS
	if (tr)
		tr[4] = __builtin_amdgcn_s_memrealtime();

	// ---- 3. W2 phase: items mine1p .. mine1p + mine2 of the issue stream, NS in flight
	if (!ctl && mine2 > 0) {
		int cg = wave / nch2, cc = wave - (wave / nch2) * nch2, cur = cg;
		float acc[1] = {0.0f};
		for (int k = 0; k < mine2; k += NS) {
#pragma unroll
			for (int u = 0; u < NS; ++u) {
				if (k + u < mine2) {
					if (cg != cur) {
						const float t = wave_sum(acc[0]);
						if (lane == 0)
							part2[cur * W + wave] = t;
						acc[0] = 0.0f;
						cur = cg;
					}
					const u32x4_t wv[1] = {s[u]};
					fma_chunk<WT, 1>(acc, wv, hbs + cc * CH + lane * EPL);
					cc += W;
					while (cc >= nch2) {
						cc -= nch2;
						++cg;
					}
				}
				s[u] = issue();
			}
		}
		const float t = wave_sum(acc[0]);
		if (lane == 0)
			part2[cur * W + wave] = t;
	}
	__syncthreads();
	for (int gl = tid; gl < ngl2; gl += FFN_THREADS) {
		float t = 0.0f;
#pragma unroll
		for (int w = 0; w < W; ++w)
			t += part2[gl * W + w];
		p.x[b + gl * NB] += t;
	}
	if (tr) {
		tr[5] = __builtin_amdgcn_s_memrealtime();
		tr[6] = (unsigned long long)mine1 | ((unsigned long long)mine2 << 32);
		tr[7] = 0;
	}
}
