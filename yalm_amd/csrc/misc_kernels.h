// misc_kernels.h — per-token bookkeeping kernels: step setup + embedding row,
// device argmax (greedy -t 0), and the deterministic synthetic initialiser.
#pragma once

#include <float.h>

#include "device_common.h"
#include "tp_exchange.h"

// Host-provided (token, pos) -> device StepState. Launched eagerly ahead of a
// graph replay; kernel arguments are captured at launch, so no host buffer race.
__global__ void set_step_kernel(StepState *st, int token, int pos, int reset_gen) {
	st->token = token;
	st->pos = pos;
	if (reset_gen)
		st->n_gen = 0;
}

// RoPE (cos, sin) of this step's position: the angles the QKV epilogue used to compute itself
// with cosf / sinf on one lane per row pair at its tail (infer.cpp:291-301, the same expression,
// so the same values), now once per step by the step kernel's threads.
__device__ __forceinline__ void step_rope(StepState *st, int pos, const float *__restrict__ inv_freq, int half) {
	for (int j = threadIdx.x; j < half; j += blockDim.x) {
		const float val = (float)pos * inv_freq[j];
		st->rope[2 * j] = cosf(val);
		st->rope[2 * j + 1] = sinf(val);
		const float val1 = 1.0f * inv_freq[j];
		st->rope_sink[2 * j] = cosf(val1);
		st->rope_sink[2 * j + 1] = sinf(val1);
	}
}

// Explicit indices for the per-block test hook (Block::block signature); n_ex: the IPC
// tensor-parallel exchanges the block uses (tp_exchange.h).
__global__ void set_step_full_kernel(StepState *st, int pos, int kv_sink, int kv_pos, int kv_len, int n_ex = 0,
                                     const float *__restrict__ inv_freq = nullptr, int half = 0) {
	if (inv_freq)
		step_rope(st, pos, inv_freq, half);
	if (threadIdx.x != 0)
		return;
	st->pos = pos;
	st->kv_sink = kv_sink;
	st->kv_pos = kv_pos;
	st->kv_len = kv_len;
	st->epoch = st->epoch + 1u;
	st->xbase = st->xnext;
	st->xnext = st->xnext + (unsigned)n_ex;
}

// Timing hook (yalm_time_kernel): a new launch generation, as step_begin_kernel
// starts one, so an in-launch hand-off never sees the previous launch's tags.
__global__ void epoch_bump_kernel(StepState *st, int n_ex) {
	st->epoch = st->epoch + 1u;
	st->xbase = st->xnext;
	st->xnext = st->xnext + (unsigned)n_ex;
}

// First node of every forward graph: sliding-window indices (infer.cu:1081-
// 1083; KV_SINKS = 2, model.h:12) and x = embedding[token] (infer.cu:622-640);
// n_ex: the IPC tensor-parallel exchanges this forward uses (tp_exchange.h).
template <class WT>
__global__ __launch_bounds__(256) void step_begin_kernel(StepState *st, const void *__restrict__ emb, int dim,
                                                         float *__restrict__ x, int max_seq_len, int n_ex,
                                                         const float *__restrict__ inv_freq, int half) {
	const int token = st->token;
	const int pos = st->pos;
	step_rope(st, pos, inv_freq, half);
	const char *row = (const char *)emb + (size_t)token * dim * WT::BYTES;
	for (int i = threadIdx.x * WT::EPL; i < dim; i += blockDim.x * WT::EPL) {
		float f[WT::EPL];
		WT::unpack(load16(row + (size_t)i * WT::BYTES), f);
#pragma unroll
		for (int e = 0; e < WT::EPL; ++e)
			x[i + e] = f[e];
	}
	if (threadIdx.x == 0) {
		const int kv_sink = pos >= max_seq_len ? 2 : 0;
		st->kv_sink = kv_sink;
		st->kv_pos = kv_sink + (pos - kv_sink) % (max_seq_len - kv_sink);
		st->kv_len = pos >= max_seq_len ? max_seq_len : pos + 1;
		st->epoch = st->epoch + 1u;
		st->xbase = st->xnext;
		st->xnext = st->xnext + (unsigned)n_ex;
	}
}

// Greedy sampling on the device (sampler.cpp:27-38: strict '>' scan, so the
// FIRST maximum wins). Feeds the result back as the next step's token.
// First max of logits[0, n) over one workgroup of 1024 threads: (value, index) in thread 0.
__device__ __forceinline__ void argmax_block(const float *__restrict__ logits, int n, float &best_out, int &idx_out) {
	__shared__ float sv[16];
	__shared__ int si[16];
	float best = -FLT_MAX;
	int bi = 0x7fffffff;
	// Batches of 8 independent float4 loads per thread in flight (a load-compare
	// loop serialises one L2 round trip per element: 13 us for 32000 logits).
	// Thread t owns elements [4t, 4t+4) of each 4*blockDim.x span: ascending
	// per thread, so the strict '>' keeps its first max.
	constexpr int B = 8;
	const int n4 = n & ~3;
	for (int base = 0; base < n4; base += B * 4 * (int)blockDim.x) {
		float4_t v[B];
#pragma unroll
		for (int k = 0; k < B; ++k) {
			const int i = base + (k * (int)blockDim.x + (int)threadIdx.x) * 4;
			v[k] = i < n4 ? *(const float4_t *)(logits + i) : float4_t{-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
		}
#pragma unroll
		for (int k = 0; k < B; ++k) {
			const int i = base + (k * (int)blockDim.x + (int)threadIdx.x) * 4;
#pragma unroll
			for (int e = 0; e < 4; ++e)
				if (v[k][e] > best) {
					best = v[k][e];
					bi = i + e;
				}
		}
	}
	for (int i = n4 + (int)threadIdx.x; i < n; i += blockDim.x) {
		const float v = logits[i];
		if (v > best) {
			best = v;
			bi = i;
		}
	}
	// wave reduce: larger value wins; ties -> smaller index
#pragma unroll
	for (int off = 32; off > 0; off >>= 1) {
		float ov = __shfl_xor(best, off, 64);
		int oi = __shfl_xor(bi, off, 64);
		if (ov > best || (ov == best && oi < bi)) {
			best = ov;
			bi = oi;
		}
	}
	const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
	if (lane == 0) {
		sv[wave] = best;
		si[wave] = bi;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		float b = sv[0];
		int idx = si[0];
		for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
			if (sv[w] > b || (sv[w] == b && si[w] < idx)) {
				b = sv[w];
				idx = si[w];
			}
		}
		if (idx == 0x7fffffff)
			idx = 0; // all -FLT_MAX / NaN: the reference returns 0
		best_out = b;
		idx_out = idx;
	}
}

// the device greedy loop's bookkeeping: token `idx` is the next step's input
__device__ __forceinline__ void argmax_commit(StepState *st, int idx, int *__restrict__ tokens_out, int cap) {
	const int k = st->n_gen;
	if (tokens_out && k < cap)
		tokens_out[k] = idx;
	st->n_gen = k + 1;
	st->token = idx;
	st->pos = st->pos + 1;
}

__global__ __launch_bounds__(1024) void argmax_kernel(const float *__restrict__ logits, int n, StepState *st,
                                                      int *__restrict__ tokens_out, int cap,
                                                      float *__restrict__ pair_out = nullptr, int index_offset = 0) {
	float b = 0.0f;
	int idx = 0;
	argmax_block(logits, n, b, idx);
	if (threadIdx.x == 0) {
		if (pair_out) { // tensor-parallel shard (RCCL): publish (value, global index) for argmax_pick_kernel
			pair_out[0] = b;
			pair_out[1] = __int_as_float(idx + index_offset);
			return;
		}
		argmax_commit(st, idx, tokens_out, cap);
	}
}

// Tensor parallelism over IPC (tp_exchange.h): this rank's first max over its vocabulary
// slice [rank * n, (rank + 1) * n) is pushed as a (value, global index) pair to every rank,
// then the kernel waits for every rank's pair and picks the global first max in rank order
// (ranks own ascending slices: ties resolve to the lowest index, sampler.cpp:27-38) --
// the exchange and the pick inside the argmax launch, identical on every rank.
__global__ __launch_bounds__(1024) void argmax_tp_kernel(const float *__restrict__ logits, int n, StepState *st,
                                                         int *__restrict__ tokens_out, int cap, TpX t) {
	const unsigned g = t.g();
	float b = 0.0f;
	int idx = 0;
	argmax_block(logits, n, b, idx);
	if (threadIdx.x == 0) {
		tpx_put(t, g, 0, b);
		tpx_put(t, g, 1, __int_as_float(idx + t.rank * n));
		const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + TPX_TIMEOUT;
		float bb = 0.0f;
		int bi = 0;
		for (int p = 0; p < t.n; ++p) {
			const float v = tpx_get1(t, g, p, 0, deadline);
			const int j = __float_as_int(tpx_get1(t, g, p, 1, deadline));
			if (p == 0 || v > bb || (v == bb && j < bi)) {
				bb = v;
				bi = j;
			}
		}
		argmax_commit(st, bi, tokens_out, cap);
	}
}

// Every granule of exchange g (n per rank) has arrived, checked by one wave (bounded).
__device__ __forceinline__ void tpx_wait_all(const TpX &t, unsigned g, int n) {
	const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + TPX_TIMEOUT;
	for (int p = 0; p < t.n; ++p)
		for (int i = threadIdx.x; i < n; i += blockDim.x)
			(void)tpx_get1(t, g, p, i, deadline);
}

// Tensor parallelism over IPC, ranks sharing one GPU: wait for the exchange in one wave
// before the consumer launch (yalm_hip.hip tpx_consume).
__global__ __launch_bounds__(64) void tpx_gate_kernel(TpX t, int n) {
	tpx_wait_all(t, t.g(), n);
}

// Tensor parallelism over IPC: the consumer side of one exchange as a launch of its own --
// the summed x into `out` (the collect form of many ranks, yalm_block's result, the timing
// hook), or, with gather, the n floats of every rank's slot side by side (the sharded
// logits). Any grid: element i belongs to global thread i mod the grid's threads.
__global__ __launch_bounds__(256) void tpx_collect_kernel(TpX t, int n, int gather, float *__restrict__ out) {
	const unsigned g = t.g();
	const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + TPX_TIMEOUT;
	const int i0 = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
	if (gather) {
		for (int p = 0; p < t.n; ++p)
			for (int i = i0; i < n; i += stride)
				out[(size_t)p * n + i] = tpx_get1(t, g, p, i, deadline);
		return;
	}
	for (int i = i0; i < n; i += stride) {
		float s = tpx_get1(t, g, 0, i, deadline);
		for (int p = 1; p < t.n; ++p)
			s += tpx_get1(t, g, p, i, deadline);
		out[i] = s;
	}
}

// Timing hook (yalm_time_kernel id 6 under IPC): a producer of exchange g alone -- this
// rank's x pushed to every rank's slot -- for the collect launch that follows.
__global__ __launch_bounds__(1024) void tpx_push_kernel(TpX t, int n, const float *__restrict__ x) {
	const unsigned g = t.g();
	for (int i = threadIdx.x; i < n; i += blockDim.x)
		tpx_put(t, g, i, x[i]);
}

// Tensor parallelism: pick the global first maximum from the tp_size gathered
// (value, index) pairs (ranks own ascending vocab slices, so ties resolve to the
// lowest index as in sampler.cpp:27-38) and advance the step like argmax_kernel.
__global__ void argmax_pick_kernel(const float *__restrict__ pairs, int n_pairs, StepState *st,
                                   int *__restrict__ tokens_out, int cap) {
	float b = pairs[0];
	int idx = __float_as_int(pairs[1]);
	for (int i = 1; i < n_pairs; ++i) {
		const float v = pairs[2 * i];
		const int j = __float_as_int(pairs[2 * i + 1]);
		if (v > b || (v == b && j < idx)) {
			b = v;
			idx = j;
		}
	}
	const int k = st->n_gen;
	if (tokens_out && k < cap)
		tokens_out[k] = idx;
	st->n_gen = k + 1;
	st->token = idx;
	st->pos = st->pos + 1;
}

// Deterministic synthetic initialiser — the same integer hash as the CPU
// oracle (oracle/yalm_oracle.c orc_synth_*), so a random-weight model of a
// real shape can be built in HBM and reproduced bit-exactly on the host.
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
	x += 0x9E3779B97F4A7C15ull;
	x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
	x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
	return x ^ (x >> 31);
}

__global__ void synth_kernel(void *dst, size_t n, int dtype, uint64_t seed, float scale, float offset) {
	const float k = scale * (1.0f / 8388608.0f);
	for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		uint64_t h = splitmix64(seed ^ ((uint64_t)i * 0xD1B54A32D192ED03ull));
		int32_t s = (int32_t)(h >> 40) - 8388608;
		if (dtype == 0) {
			((float *)dst)[i] = __builtin_fmaf((float)s, k, offset);
		} else {
			float v = __fmul_rn((float)s, k);
			uint32_t hb = f2h(v); // f2h keeps the f32 rounding step (no fma_mix fusion)
			if (dtype == 1)
				((uint16_t *)dst)[i] = (uint16_t)hb;
			else
				((uint8_t *)dst)[i] = (uint8_t)((hb + 0x7Fu + ((hb >> 8) & 1u)) >> 8);
		}
	}
}
