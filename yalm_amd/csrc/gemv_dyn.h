// gemv_dyn.h — row-block GEMV with a work-stealing tail.
//
// gemv_rb_kernel deals its row groups statically (group g to workgroup g % NB):
// every workgroup gets the same bytes, yet per-CU streaming rates differ by a
// few percent, so the last workgroup ends ~1.7-2.2 us after the median one
// (tools/wg_timeline.hip, tools/ffn_trace.py) while HBM idles. Here each
// workgroup streams a static interleaved prefix (groups b + gl * NB, gl < ks)
// and then drains a shared pool of the remaining groups one group at a time:
//   * the pool is sharded per XCD under round-robin placement (shard b % 8,
//     pool groups S + s + 8 j; speed only, never correctness) so that no counter
//     word sees more than ~50 dequeues per us (MI355X_MICROARCH.md row dequeue);
//   * a control wave (no weight loads of its own, so its returning atomics do
//     not queue behind the stream: vmcnt is in order) keeps D dequeues in
//     flight and appends the groups it wins to an LDS queue; the streaming
//     waves' issue cursors read group ids from the queue (LDS spin, no barrier);
//   * counters reset themselves: every workgroup's control wave ends with
//     exactly D failed dequeues (each returns >= the shard's pool size), so the
//     one that receives pool + D * (workgroups of the shard) - 1 made the last
//     dequeue of the launch and stores 0 (the next launch is ordered behind this
//     one by the stream).
// Each group is computed whole by one workgroup, and W (streaming waves) divides
// the group's R * nch items, so item k of every group runs on wave k % W and the
// row partials are summed in fixed wave order: the results do not depend on which
// workgroup takes a group, or when (deterministic), and equal gemv_rb_kernel's
// bit for bit at the same wave count.
#pragma once

#include "gemv.h"

#define DYN_QMAX 256   // dynamic groups one workgroup can take (LDS queue slots)
#define DYN_SHARDS 8   // counter shards (one per XCD under round-robin placement)
#define DYN_STRIDE 32  // words between shards (own 128-B line each)

struct DynArgs {
	unsigned *ctr; // DYN_SHARDS counters, DYN_STRIDE words apart (zero at rest)
	int ks;        // static groups per workgroup: groups [0, NB * ks) are dealt statically
	int pool;      // groups [NB * ks, NB * ks + pool) are dequeued; NB * ks + pool == n_groups
};

// dynamic LDS: x staging (n + 64 scratch) | partials [(ks + QMAX) * R][W]
template <int W>
__host__ __device__ inline size_t dyn_lds_floats(int n, int ks, int R) {
	return (size_t)((n + 3) & ~3) + 64 + (size_t)(ks + DYN_QMAX) * R * W;
}

// LDS queue words: relaxed workgroup-scope atomics on __shared__ arrays (ds_read /
// ds_write; a volatile access would add vmcnt(0) waits that drain the stream)
__device__ __forceinline__ int lds_ld(int *p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// LDS read for the streaming waves' spin: hand-written so that no wait on the
// wave's weight loads (vmcnt) is attached to it, only its own lgkmcnt
__device__ __forceinline__ int lds_ld_spin(int *p) {
	const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int *)p;
	int v;
	asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
	return v;
}
__device__ __forceinline__ void lds_st(int *p, int v) {
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// W streaming waves + 1 control wave. IPW = R * n / (64 * EPL) / W items per
// wave per group (W divides a group's items, so wave w's (row, chunk) pairs are
// the same in every group: their offsets are computed once); GA groups in
// flight per wave (IPW * GA 16-byte loads per lane); D dequeues in flight.
// ks >= GA (every wave's first GA groups are static: issued before the staging).
// Pool per shard <= DYN_QMAX.
template <class WT, class P, int IPW, int GA, bool NORM, int W, int D>
__global__ __launch_bounds__((W + 1) * 64) void gemv_dyn_kernel(P p, const float *__restrict__ x,
                                                                const float *__restrict__ normw, float eps,
                                                                DynArgs dy) {
	extern __shared__ __attribute__((aligned(16))) float xs[];
	constexpr int THREADS = (W + 1) * 64;
	constexpr int R = P::R;
	constexpr int EPL = WT::EPL;
	constexpr int CH = YALM_WAVE * EPL;
	constexpr size_t CHB = (size_t)CH * WT::BYTES;
	const int n = p.n;
	const int nch = n / CH;
	const int NB = gridDim.x;
	const int b = blockIdx.x;
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
	const int ks = dy.ks;
	const int S0 = NB * ks; // first pooled group
	const int shard = b % DYN_SHARDS;
	const int ps = dy.pool > shard ? (dy.pool - 1 - shard) / DYN_SHARDS + 1 : 0; // this shard's pool
	const int nwg_s = NB > shard ? (NB - 1 - shard) / DYN_SHARDS + 1 : 0;       // workgroups on this shard
	float *part = xs + ((n + 3) & ~3) + 64; // [(ks + QMAX) * R][W]
	__shared__ int queue[DYN_QMAX];          // pooled group ids, in the order this workgroup won them
	__shared__ int ctl[2];                   // [0] ids published, [1] pool exhausted at this slot
	unsigned *ctr = dy.ctr + shard * DYN_STRIDE;

	if (tid == 0) {
		lds_st(&ctl[0], 0);
		lds_st(&ctl[1], ps == 0 ? 0 : 0x7fffffff);
	}
	for (int i = tid; i < (ks + DYN_QMAX) * R * W; i += THREADS)
		part[i] = 0.0f;
	// (stage_x's barrier orders these LDS initialisations before any use)

	// this wave's items of any group: item k = wave + m * W -> row rm[m], chunk cm[m]
	int rm[IPW];
	size_t off[IPW]; // byte offset inside the row, this lane's 16 bytes
	int xo[IPW];     // x offset (floats) of the chunk, this lane's EPL elements
#pragma unroll
	for (int m = 0; m < IPW; ++m) {
		const int k = wave + m * W;
		rm[m] = k / nch;
		const int c = k - rm[m] * nch;
		off[m] = (size_t)c * CHB + (size_t)lane * EPL * WT::BYTES;
		xo[m] = c * CH + lane * EPL;
	}
	const char *dummy = (const char *)x + lane * 16;
	// slot gl -> group id (wave-uniform): static, or from the LDS queue; -1 past the pool
	auto group_of = [&](int gl) -> int {
		if (gl < ks)
			return b + gl * NB;
		const int q = gl - ks;
		for (;;) {
			if (__builtin_amdgcn_readfirstlane(lds_ld_spin(&ctl[0])) > q)
				return __builtin_amdgcn_readfirstlane(lds_ld_spin(&queue[q]));
			if (__builtin_amdgcn_readfirstlane(lds_ld_spin(&ctl[1])) <= q)
				return -1;
			__builtin_amdgcn_s_sleep(1);
		}
	};
	u32x4_t buf[GA][IPW];
	// unconditional loads (a branch around a load makes hipcc wait for it at the
	// join): past the pool the lane address selects this lane's line of x
	auto fill = [&](u32x4_t(&slot)[IPW], int g) {
		const int gg = g < 0 ? 0 : g;
#pragma unroll
		for (int m = 0; m < IPW; ++m) {
			const uintptr_t real = (uintptr_t)(p.row(gg, rm[m]) + off[m]);
			const uintptr_t dm = (uintptr_t)dummy;
			slot[m] = load_nt16((const void *)(g < 0 ? dm : real));
		}
	};
	if (wave < W) {
#pragma unroll
		for (int a = 0; a < GA; ++a)
			fill(buf[a], b + a * NB); // static groups (ks >= GA)
	}
	p.prologue();
	stage_x<NORM>(xs, x, normw, n, eps);

	if (wave == W) {
		// ---- dequeue loop (lane 0): D in flight, wins appended in order
		if (lane == 0 && ps > 0) {
			unsigned res[D];
#pragma unroll
			for (int t = 0; t < D; ++t)
				res[t] = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			int q = 0;
			bool stopped = false;
			unsigned fail_max = 0;
			while (!stopped) {
#pragma unroll
				for (int t = 0; t < D; ++t) {
					const unsigned v = res[t];
					if (stopped) {
						fail_max = v > fail_max ? v : fail_max;
					} else if (v < (unsigned)ps) {
						lds_st(&queue[q], S0 + shard + (int)v * DYN_SHARDS);
						lds_st(&ctl[0], ++q); // LDS writes of one wave land in order
						res[t] = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					} else {
						stopped = true;
						lds_st(&ctl[1], q);
						fail_max = v;
					}
				}
			}
			// the dequeues still in flight were issued after the first failure: they fail too
#pragma unroll
			for (int t = 0; t < D; ++t)
				fail_max = res[t] > fail_max ? res[t] : fail_max;
			if (fail_max == (unsigned)(ps + D * nwg_s - 1)) // this shard's last dequeue of the launch
				__hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
	} else {
		// ---- streaming waves: group slots gl = 0, 1, ...; slot gl + GA is issued as gl is consumed
		int gend = 0x7fffffff; // first invalid slot (known once the issue side reaches it)
		for (int g0 = 0; g0 < gend; g0 += GA) {
#pragma unroll
			for (int a = 0; a < GA; ++a) {
				const int gl = g0 + a;
				if (gl < gend) {
					float acc[R];
#pragma unroll
					for (int r = 0; r < R; ++r)
						acc[r] = 0.0f;
#pragma unroll
					for (int m = 0; m < IPW; ++m) {
						float t[1] = {0.0f};
						const u32x4_t wv[1] = {buf[a][m]};
						fma_chunk<WT, 1>(t, wv, xs + xo[m]);
						acc[rm[m]] += t[0];
					}
#pragma unroll
					for (int r = 0; r < R; ++r) {
						bool has = false;
#pragma unroll
						for (int m = 0; m < IPW; ++m)
							has |= rm[m] == r;
						if (has) {
							const float s = wave_sum(acc[r]);
							if (lane == 0)
								part[(gl * R + r) * W + wave] = s;
						}
					}
				}
				int gn = -1;
				if (gl + GA < gend) {
					gn = group_of(gl + GA);
					if (gn < 0)
						gend = gl + GA;
				}
				fill(buf[a], gn);
			}
		}
	}
	__syncthreads();
	const int c0 = lds_ld(&ctl[0]), c1 = lds_ld(&ctl[1]);
	const int nq = c1 < c0 ? c1 : c0;
	for (int gl = tid; gl < ks + nq; gl += THREADS) {
		const int g = gl < ks ? b + gl * NB : lds_ld(&queue[gl - ks]);
		float a[R];
#pragma unroll
		for (int r = 0; r < R; ++r) {
			float t = 0.0f;
#pragma unroll
			for (int w = 0; w < W; ++w)
				t += part[(gl * R + r) * W + w];
			a[r] = t;
		}
		p.finish_all(g, a);
	}
}
