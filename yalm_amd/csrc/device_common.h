// device_common.h — gfx950 device helpers shared by the decode kernels.
//
// Wave64 everywhere (CDNA4): reductions are xor-butterflies over 64 lanes,
// never the reference's 32-lane warp idioms (infer.cu:110-214).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define YALM_WAVE 64

typedef float float4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// Step parameters resident in device memory so that the per-token hipGraph is
// fully static (no per-node SetParams, unlike infer.cu:1146-1164).
struct StepState {
	int token;   // token fed at this step
	int pos;     // sequence position
	int kv_sink; // infer.cu:1081
	int kv_pos;  // infer.cu:1082
	int kv_len;  // infer.cu:1083
	int n_gen;   // number of greedy tokens produced so far (device loop)
	unsigned epoch; // launch generation: +1 per forward (step_begin_kernel) and per test-hook block
	                // (set_step_full_kernel); in-launch hand-off flags carry it, so they never need a reset
	unsigned xbase; // IPC tensor parallelism (tp_exchange.h): this launch sequence's first exchange index
	unsigned xnext; // the next sequence's (xbase + the exchanges this one uses)
	float rope[256]; // (cos, sin) of pos * inv_freq[j], j < head_dim / 2 (infer.cpp:291-301), once per
	                 // step (step_begin_kernel / set_step_full_kernel) for the QKV GEMV's epilogue
	float rope_sink[256]; // (cos, sin) of 1 * inv_freq[j]: the sink keys' one-position rotation
	                      // (infer.cpp:303-317), written beside rope
};

// Cross-lane exchange without the LDS crossbar: __shfl_xor lowers to
// ds_bpermute_b32 + an lgkmcnt(0) wait per step (~100+ cycles each, serialised),
// which dominated the decode attention. DPP row permutations and gfx950's
// v_permlane16/32_swap are plain VALU ops.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
	return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// partner values across rows: lane ^ 16 (permlane16_swap) and lane ^ 32 (permlane32_swap)
__device__ __forceinline__ float xor16(float v) {
	const unsigned u = __builtin_bit_cast(unsigned, v);
	auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
	// r[0] holds the swapped odd rows of vdst, r[1] the swapped even rows of src:
	// for every lane exactly one of them differs from u, and r[0]+r[1]-u is the partner.
	return __builtin_bit_cast(float, (threadIdx.x & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float xor32(float v) {
	const unsigned u = __builtin_bit_cast(unsigned, v);
	auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
	return __builtin_bit_cast(float, (threadIdx.x & 32) ? r[0] : r[1]);
}
// ss + v0^2 + v1^2 + v2^2 + v3^2 as an explicit fma chain: the x staging of the GEMV
// (gemv.h) and of the tensor-parallel exchange consumer (tp_exchange.h) must round
// identically (TP1 is bit-exact vs one GPU), and hipcc contracts a written-out sum of
// products differently depending on the surrounding code.
__device__ __forceinline__ float sumsq4(float ss, const float4_t &v) {
	float t = v[0] * v[0];
	t = __builtin_fmaf(v[1], v[1], t);
	t = __builtin_fmaf(v[2], v[2], t);
	t = __builtin_fmaf(v[3], v[3], t);
	return ss + t;
}

// Sum / max over each aligned row of 16 lanes (result in every lane of the row):
// quad_perm [1,0,3,2] (xor 1), [2,3,0,1] (xor 2), row_half_mirror, row_mirror.
__device__ __forceinline__ float row16_sum(float v) {
	v += dpp<0xB1>(v);
	v += dpp<0x4E>(v);
	v += dpp<0x141>(v);
	v += dpp<0x140>(v);
	return v;
}
__device__ __forceinline__ float row16_max(float v) {
	v = fmaxf(v, dpp<0xB1>(v));
	v = fmaxf(v, dpp<0x4E>(v));
	v = fmaxf(v, dpp<0x141>(v));
	v = fmaxf(v, dpp<0x140>(v));
	return v;
}

__device__ __forceinline__ float wave_sum(float v) {
	v = row16_sum(v);
	v += xor16(v);
	v += xor32(v);
	return v;
}

__device__ __forceinline__ float wave_max(float v) {
	v = row16_max(v);
	v = fmaxf(v, xor16(v));
	v = fmaxf(v, xor32(v));
	return v;
}

// Sum over aligned groups of `width` lanes (width a power of two <= 64).
__device__ __forceinline__ float group_sum(float v, int width) {
	for (int off = width >> 1; off > 0; off >>= 1)
		v += __shfl_xor(v, off, 64);
	return v;
}

// 16-byte streaming load of weights read exactly once per token: non-temporal
// (MI355X_MICROARCH.md row nt-weights: decode layers 5-10% faster).
__device__ __forceinline__ u32x4_t load_nt16(const void *p) {
	return __builtin_nontemporal_load((const u32x4_t *)p);
}
__device__ __forceinline__ u32x4_t load16(const void *p) {
	return *(const u32x4_t *)p;
}

__device__ __forceinline__ float h2f(uint16_t h) {
	_Float16 f;
	__builtin_memcpy(&f, &h, 2);
	return (float)f;
}
__device__ __forceinline__ uint16_t f2h(float x) { // round to nearest even
	// Opaque barrier: keeps the value's own f32 rounding. Otherwise hipcc fuses a
	// producing multiply/FMA with the convert (v_fma_mix*_f16, a single rounding),
	// which differs from the CPU reference's f32-then-f16 (infer.cpp:299, 314).
	asm volatile("" : "+v"(x));
	_Float16 f = (_Float16)x;
	uint16_t h;
	__builtin_memcpy(&h, &f, 2);
	return h;
}

// Weight element types. EPL = elements per 16-byte lane load.
struct WF32 {
	static constexpr int EPL = 4;
	static constexpr int BYTES = 4;
	__device__ static __forceinline__ void unpack(const u32x4_t &w, float *o) {
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			// copy the element out first: __builtin_bit_cast on a vector-element
			// lvalue reads element 0 under hipcc 7.2 (found by the GPU parity tests)
			const uint32_t v = w[i];
			o[i] = __builtin_bit_cast(float, v);
		}
	}
};
struct WF16 {
	static constexpr int EPL = 8;
	static constexpr int BYTES = 2;
	__device__ static __forceinline__ void unpack(const u32x4_t &w, float *o) {
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t v = w[i];
			half2_t h = __builtin_bit_cast(half2_t, v);
			o[2 * i] = (float)h[0];
			o[2 * i + 1] = (float)h[1];
		}
	}
};
// OCP E5M2 (== gfx950 "bf8"): the f16 with bits (b << 8), an exact upcast.
// gfx950 converts two packed bf8 bytes to two f32 in one VALU op
// (v_cvt_pk_f32_bf8, OCP E5M2 on CDNA4), half the work of the shift + f16
// widen sequence; tests/test_gpu_kernels.py checks all 256 byte values.
typedef float float2_t __attribute__((ext_vector_type(2)));
struct WF8 {
	static constexpr int EPL = 16;
	static constexpr int BYTES = 1;
	__device__ static __forceinline__ void unpack(const u32x4_t &w, float *o) {
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t v = w[i];
			const float2_t a = __builtin_amdgcn_cvt_pk_f32_bf8((int)v, false); // bytes 0, 1
			const float2_t b = __builtin_amdgcn_cvt_pk_f32_bf8((int)v, true);  // bytes 2, 3
			o[4 * i + 0] = a[0];
			o[4 * i + 1] = a[1];
			o[4 * i + 2] = b[0];
			o[4 * i + 3] = b[1];
		}
	}
};

// acc += w . x over one 16-byte weight piece, two independent chains (a0: even
// elements, a1: odd). f16: v_fma_mix_f32 widens the f16 operand exactly and
// rounds once, so it equals cvt + fma bit for bit at half the instruction count;
// one asm statement so no compiler padding lands between the dependent ops.
template <class WT>
__device__ __forceinline__ void dot16_mix(float &a0, float &a1, const u32x4_t &w, const float (&x)[WT::EPL]) {
	if constexpr (WT::BYTES == 2) {
		asm("v_fma_mix_f32 %0, %2, %4, %0 op_sel_hi:[1,0,0]\n\t"
		    "v_fma_mix_f32 %1, %2, %5, %1 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
		    "v_fma_mix_f32 %0, %3, %6, %0 op_sel_hi:[1,0,0]\n\t"
		    "v_fma_mix_f32 %1, %3, %7, %1 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
		    : "+v"(a0), "+v"(a1)
		    : "v"(w[0]), "v"(w[1]), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));
		asm("v_fma_mix_f32 %0, %2, %4, %0 op_sel_hi:[1,0,0]\n\t"
		    "v_fma_mix_f32 %1, %2, %5, %1 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
		    "v_fma_mix_f32 %0, %3, %6, %0 op_sel_hi:[1,0,0]\n\t"
		    "v_fma_mix_f32 %1, %3, %7, %1 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
		    : "+v"(a0), "+v"(a1)
		    : "v"(w[2]), "v"(w[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]));
	} else {
		float wf[WT::EPL];
		WT::unpack(w, wf);
#pragma unroll
		for (int e = 0; e < WT::EPL; e += 2) {
			a0 = fmaf(wf[e], x[e], a0);
			a1 = fmaf(wf[e + 1], x[e + 1], a1);
		}
	}
}

// Sums of 4 per-lane values over the wave's 4 rows (16-lane groups), transposed:
// lane p of row r ends with v[r] summed over lane p of all 4 rows. Each exchange
// sends the value the partner keeps and keeps the one it sends back (2 xor-32 +
// 1 xor-16 lane swaps instead of 4 x 2).
__device__ __forceinline__ float sum4_rows(const float (&v)[4]) {
	const bool hi32 = threadIdx.x & 32, odd16 = threadIdx.x & 16;
	const float s02 = (hi32 ? v[2] : v[0]) + xor32(hi32 ? v[0] : v[2]); // lanes 0-31: v[0], 32-63: v[2]
	const float s13 = (hi32 ? v[3] : v[1]) + xor32(hi32 ? v[1] : v[3]); // v[1] / v[3]
	return (odd16 ? s13 : s02) + xor16(odd16 ? s02 : s13);              // row r: v[r]
}
// Sums of 4 per-lane values over the whole wave, transposed: lanes 16 t .. 16 t + 15
// end with the total of v[t].
__device__ __forceinline__ float sum4_t(const float (&v)[4]) {
	return row16_sum(sum4_rows(v));
}

// infer.cu:586-596 semantics (SiLU x/(1+e^-x); GELU tanh approximation).
template <int ACT>
__device__ __forceinline__ float act_fn(float x) {
	if constexpr (ACT == 1) {
		return x / (1.0f + expf(-x));
	} else {
		return 0.5f * x * (1.0f + tanhf(0.797885f * (x + 0.044715f * x * x * x)));
	}
}
