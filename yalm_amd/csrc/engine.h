// engine.h — persistent per-token decode engine for gfx950 (one launch per token).
//
// The launch path (gemv.h / attention.h) runs a token as ~160 dependent kernels
// (5 per layer). Each boundary costs ~4.5-6 us of HBM idle time (launch + ramp +
// tail), ~21 us per Mistral-7B layer against ~67 us of pure weight streaming.
// Weights never depend on activations, so this engine decouples the two:
//
//   * one workgroup per CU, 1 LOADER wave + C CONSUMER waves;
//   * the loader streams the CU's whole per-token weight sequence (its rows of
//     every GEMV of every layer, then the classifier) into an LDS ring of
//     ENG_NS x 8 KB slots with LDS-DMA (global_load_lds_dwordx4 nt), keeping
//     ENG_INFLIGHT slots in flight and publishing "slot landed" behind a counted
//     vmcnt. It only ever waits for ring space, never for an activation, so the
//     HBM stream runs on through the seams between GEMVs for as long as the ring
//     (144 KB = ~5.7 us at 25 GB/s per CU) covers them
//     (MI355X_MICROARCH.md rows ldsdma-fill, prefetch-credit, engine-vs-launches);
//   * the consumers walk the same item sequence: per phase they gather the input
//     vector slice they need into registers (their chunk columns), optionally
//     rmsnorm it, dot the ring items, and run the phase epilogue (RoPE + KV write,
//     residual add, SiLU-GLU, logits + local argmax);
//   * a phase's outputs are handed to every CU with write-through (sc1) stores,
//     a per-CU epoch flag (sc1 store) and sc1 loads on the consumer side (the
//     fence-free hand-off of MI355X_MICROARCH.md §visibility "Valid forms", row 1);
//   * attention runs between QKV and Wo as wave-sized split-KV units (32 keys per
//     chunk, 16 lanes per key row, DPP row sums, online softmax) with a
//     last-arriver merge per kv head.
//
// Semantics per phase follow the launch-path kernels (which follow infer.cpp /
// infer.cu, cited there): QKV = rmsnorm (infer.cu:526) + fused_qkv_matmul_clip
// (290) + fused_rope_and_cache_update (642) + rotate_sink_tokens (679); ATTN =
// attn_dot/softmax/att_mix (338-524); WO, W2 = fused_matmul_add_residuals (270);
// GLU = rmsnorm + fused_ffn_w1_w3_glu_act (598); LOGITS = final rmsnorm +
// matmul_wide (1096-1126) + sample_argmax (sampler.cpp:27-38, first max wins).
//
// Every spin is bounded (ENG_TIMEOUT): a CU that never arrives (e.g. the grid
// not co-resident) turns into an error code in *err, never a hang.
#pragma once

#include <float.h>

#include "device_common.h"

#define ENG_LDS __attribute__((address_space(3)))
#define ENG_CONST __attribute__((address_space(4))) // read-only for the launch: s_load (lgkmcnt only)
#define ENG_ITEM 1024                        // one wave-wide 16 B/lane load
#define ENG_IPS 8                            // items per ring slot (8 KB)
#define ENG_LD 2                             // own slots in flight per loader wave
#define ENG_LD_LOADS "16"                    // = ENG_IPS * ENG_LD, for the s_waitcnt string
#define ENG_MAXROWS 512                      // rows of one phase per CU (row partials in LDS)
#define ENG_KC 32                            // attention keys per chunk (one wave, 8 rows per lane)
#define ENG_SMAX 32                          // attention splits per kv head
#define ENG_D 128                            // head_dim supported by the engine
#define ENG_TIMEOUT 200000000ull             // 2 s of s_memrealtime (100 MHz)
#define ENG_CTL_WORDS 64
#define ENG_PF_PAD 256                       // LDS landing pad of the prefetch wave's 4-B touches
#define ENG_PF_LINE 64                       // prefetch touch stride (bytes per lane)

enum { EK_QKV = 0, EK_ATTN = 1, EK_WO = 2, EK_GLU = 3, EK_W2 = 4, EK_LOGITS = 5 };
enum { EM_HYDRATE = 0, EM_LOGITS = 1, EM_GREEDY = 2 };
enum { ENG_ERR_SEAM = 1, ENG_ERR_RING = 2, ENG_ERR_CBAR = 4, ENG_ERR_ABORT = 8 };

// control words in LDS
enum { CTL_FULL = 0 /* .. + L: own slots landed per loader */, CTL_CONS = 4 /* .. + C */, CTL_CBAR = 12,
       CTL_SEAM = 13, CTL_ABORT = 14, CTL_NRM = 16, CTL_AMAX = 32,
       CTL_LSTALL = 48 /* .. + L: ring-full ticks per loader; 52, 53: finish time lo/hi */ };

struct EngLayer {
	const char *wq, *wk, *wv, *wo, *w1, *w2, *w3;
	const float *rms_att, *rms_ffn;
	uint16_t *kc, *vc;
};

struct EngArgs {
	const EngLayer *layers;
	int n_layers, dim, hidden, q_dim, kv_dim, n_heads, n_kv, vocab, max_seq_len, act, mode, tokens_cap;
	float eps, qkv_clip;
	const float *inv_freq;
	const char *emb;
	const float *rms_final;
	const char *wcls;
	StepState *step;
	float *x, *q, *xb2, *hb, *logits, *part, *amax;
	unsigned *tickets, *flags, *gen, *err;
	int *tokens;
	unsigned long long *trace; // [NB][5 L + 2][8] s_memrealtime stamps of the last launch (null: off)
	int dbg;      // timing-only ablations (YALM_ENGINE_DBG): 1 = no FMA math, 2 = no seams, 4 = consumers skip the ring,
	              // 32 = no epilogue / publish stores, 64 = no input gather
	int ld_depth; // own slots in flight per loader wave (1..7; YALM_ENGINE_DEPTH)
	int ld_nt;    // weight stream cache policy: 1 = nt (default), 0 = default policy (YALM_ENGINE_NT)
	int ld_waves; // loader waves that stream (1..NL; YALM_ENGINE_LOADERS); the others exit
	int poll_sleep; // consumers' s_sleep between ring polls (1, 2, 4, 8, 16; YALM_ENGINE_SLEEP)
	int pf_ahead;   // items the prefetch wave (loader wave index ld_waves) runs ahead of the landed ring;
	                // 0 = no prefetch wave (YALM_ENGINE_PF, in KB)
};
// EngArgs and the EngLayer table are read-only for a launch: every read goes through
// these constant-address-space views, so it is an s_load (lgkmcnt). Read through a
// generic pointer it would be a vector load re-issued after every memory-clobbering
// asm (the ring polls and DMAs) and guarded by a vmcnt wait -- in the loader that
// wait drains the whole in-flight weight stream.
typedef const ENG_CONST EngArgs EngA;
typedef const ENG_CONST EngLayer EngL;
__device__ __forceinline__ EngLayer eng_layer(EngL &s) {
	return EngLayer{s.wq, s.wk, s.wv, s.wo, s.w1, s.w2, s.w3, s.rms_att, s.rms_ffn, s.kc, s.vc};
}

// LDS: ring | part[ENG_MAXROWS][C] | ctl[ENG_CTL_WORDS] | prefetch landing pad (256 B, never read)
template <int C>
constexpr int eng_ring_slots() {
	return (160 * 1024 - ENG_MAXROWS * C * 4 - ENG_CTL_WORDS * 4 - ENG_PF_PAD) / (ENG_IPS * ENG_ITEM);
}
template <int C>
constexpr size_t eng_lds_bytes() {
	return (size_t)eng_ring_slots<C>() * ENG_IPS * ENG_ITEM + (size_t)ENG_MAXROWS * C * 4 + ENG_CTL_WORDS * 4 +
	       ENG_PF_PAD;
}

// ---------------------------------------------------------------- memory helpers
__device__ __forceinline__ float eng_ld_sc1(const float *p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void eng_st_sc1(float *p, float v) {
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void eng_ld2_sc1(const void *p, float &a, float &b) {
	const unsigned long long v =
	    __hip_atomic_load((const unsigned long long *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	a = __uint_as_float((unsigned)v);
	b = __uint_as_float((unsigned)(v >> 32));
}
__device__ __forceinline__ void eng_st2_sc1(void *p, float a, float b) {
	const unsigned long long v = (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32);
	__hip_atomic_store((unsigned long long *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32x4_t eng_ld16_sc1(const void *p) {
	const unsigned long long a =
	    __hip_atomic_load((const unsigned long long *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	const unsigned long long b =
	    __hip_atomic_load((const unsigned long long *)p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	return u32x4_t{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
}
__device__ __forceinline__ void eng_st_u32_sc1(void *p, uint32_t v) {
	__hip_atomic_store((uint32_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t eng_ld_u32_sc1(const void *p) {
	return __hip_atomic_load((const uint32_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned eng_lds_acq(volatile ENG_LDS unsigned *p) {
	return __hip_atomic_load((ENG_LDS unsigned *)p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void eng_lds_rel(volatile ENG_LDS unsigned *p, unsigned v) {
	__hip_atomic_store((ENG_LDS unsigned *)p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// 16-byte LDS-DMA of one lane's piece (MI355X_MICROARCH / cdna_hip_programming.md §5.7
// recipe): M0 = wave-uniform LDS destination; lane i lands at M0 + 16 i. Hidden from
// hipcc's waitcnt bookkeeping on purpose: the loader counts its own vmcnt.
__device__ __forceinline__ void eng_glds16(const void *g, unsigned lds_dst, bool nt) {
	unsigned keep;
	if (nt)
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
		             : "=&s"(keep)
		             : "v"(g), "s"(lds_dst)
		             : "memory");
	else
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
		             : "=&s"(keep)
		             : "v"(g), "s"(lds_dst)
		             : "memory");
}
// wait until at most d own slots (8 loads each) of this wave are still in flight
__device__ __forceinline__ void eng_vmcnt_slots(int d) {
	switch (d) {
	case 0:
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		break;
	case 1:
		asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
		break;
	case 2:
		asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
		break;
	case 3:
		asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
		break;
	case 4:
		asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
		break;
	case 5:
		asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
		break;
	case 6:
		asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
		break;
	default:
		asm volatile("s_waitcnt vmcnt(56)" ::: "memory");
	}
}

// one element of a weight row (embedding residual of layer 0)
template <class WT>
__device__ __forceinline__ float eng_elem(const char *row, int i) {
	if constexpr (WT::BYTES == 4) {
		return ((const float *)row)[i];
	} else if constexpr (WT::BYTES == 2) {
		return h2f(((const uint16_t *)row)[i]);
	} else {
		return h2f((uint16_t)(((const uint8_t *)row)[i] << 8));
	}
}

// acc += w . x over one 16-byte weight piece (exact widening, fp32 FMA; two chains)
template <class WT>
__device__ __forceinline__ void fma_chunk_eng(float &acc, const u32x4_t &w, const float (&x)[WT::EPL]) {
	float wf[WT::EPL];
	WT::unpack(w, wf);
	float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
	for (int e = 0; e < WT::EPL; e += 2) {
		a0 = fmaf(wf[e], x[e], a0);
		a1 = fmaf(wf[e + 1], x[e + 1], a1);
	}
	acc += a0 + a1;
}

// f16 weight (lo / hi half of a dword) x f32 activation + f32 accumulator in ONE
// instruction: v_fma_mix_f32 widens the f16 operand exactly and rounds once, so it
// equals cvt + fma bit for bit at half the instruction count.
__device__ __forceinline__ float eng_fma_mix_lo(uint32_t w2, float x, float acc) {
	float d;
	asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(w2), "v"(x), "v"(acc));
	return d;
}
__device__ __forceinline__ float eng_fma_mix_hi(uint32_t w2, float x, float acc) {
	float d;
	asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(w2), "v"(x), "v"(acc));
	return d;
}
// acc += w . x over one 16-byte piece, two independent chains
template <class WT>
__device__ __forceinline__ void eng_dot16(float &a0, float &a1, const u32x4_t &w, const float (&x)[WT::EPL]) {
	if constexpr (WT::BYTES == 2) {
		// one statement: no compiler pads between the dependent (hardware-interlocked) VALU ops
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
// Sums of 4 per-lane values over the wave, transposed: lanes 16 t .. 16 t + 15 end
// with the total of v[t]. Each exchange sends the value the partner keeps and keeps
// the one it sends back (2 xor-32 + 1 xor-16 lane swaps), then one 16-lane DPP sum.
__device__ __forceinline__ float eng_sum4_t(const float (&v)[4]) {
	const bool hi32 = threadIdx.x & 32, odd16 = threadIdx.x & 16;
	const float s02 = (hi32 ? v[2] : v[0]) + xor32(hi32 ? v[0] : v[2]); // lanes 0-31: row 0, 32-63: row 2
	const float s13 = (hi32 ? v[3] : v[1]) + xor32(hi32 ? v[1] : v[3]); // row 1 / row 3
	const float u = (odd16 ? s13 : s02) + xor16(odd16 ? s02 : s13);     // 16-lane group g: row g
	return row16_sum(u);
}

// ---------------------------------------------------------------- phase geometry
__device__ __forceinline__ int eng_kind(EngA &a, int ph) {
	return ph < 5 * a.n_layers ? ph % 5 : EK_LOGITS;
}
template <class A>
__device__ __forceinline__ void eng_geo(const A &a, int kind, int &n, int &ngroups, int &R) {
	switch (kind) {
	case EK_QKV:
		n = a.dim, ngroups = (a.q_dim + 2 * a.kv_dim) / 2, R = 2;
		break;
	case EK_WO:
		n = a.q_dim, ngroups = a.dim, R = 1;
		break;
	case EK_GLU:
		n = a.dim, ngroups = a.hidden, R = 2;
		break;
	case EK_W2:
		n = a.hidden, ngroups = a.dim, R = 1;
		break;
	default:
		n = a.dim, ngroups = a.vocab, R = 1;
	}
}
// the loader's phase geometry, copied into SGPRs once
struct EngGeo {
	int dim, hidden, q_dim, kv_dim, vocab;
	const char *wcls;
};
template <class WT>
__device__ __forceinline__ const char *eng_row(const EngGeo &a, const EngLayer &L, int kind, int g, int r, int n) {
	const size_t rb = (size_t)n * WT::BYTES;
	switch (kind) {
	case EK_QKV: {
		int vr = 2 * g + r;
		if (vr < a.q_dim)
			return L.wq + (size_t)vr * rb;
		vr -= a.q_dim;
		if (vr < a.kv_dim)
			return L.wk + (size_t)vr * rb;
		return L.wv + (size_t)(vr - a.kv_dim) * rb;
	}
	case EK_WO:
		return L.wo + (size_t)g * rb;
	case EK_GLU:
		return (r == 0 ? L.w1 : L.w3) + (size_t)g * rb;
	case EK_W2:
		return L.w2 + (size_t)g * rb;
	default:
		return a.wcls + (size_t)g * rb;
	}
}
__device__ __forceinline__ int eng_ngl(int ngroups, int b, int NB) {
	return b < ngroups ? (ngroups - 1 - b) / NB + 1 : 0;
}

// ---------------------------------------------------------------- bounded spins
struct EngSpin {
	unsigned long long t0 = 0;
	unsigned n = 0;
};
// true = give up (timeout or another wave aborted)
__device__ __forceinline__ bool eng_spin(EngSpin &s, volatile ENG_LDS unsigned *ctl) {
	__builtin_amdgcn_s_sleep(1);
	if ((++s.n & 31) == 0) {
		if (ctl[CTL_ABORT])
			return true;
		const unsigned long long t = __builtin_amdgcn_s_memrealtime();
		if (s.t0 == 0)
			s.t0 = t;
		else if (t - s.t0 > ENG_TIMEOUT)
			return true;
	}
	return false;
}
__device__ __forceinline__ void eng_fail(unsigned *err, volatile ENG_LDS unsigned *ctl, unsigned code) {
	ctl[CTL_ABORT] = 1;
	if ((threadIdx.x & 63) == 0)
		__hip_atomic_fetch_or(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ring slots landed as a contiguous prefix: loader l's first missing slot is count_l * nl + l
// (the NL <= 4 counters are one 16-byte LDS read)
template <int NL>
__device__ __forceinline__ unsigned eng_landed(volatile ENG_LDS unsigned *ctl, unsigned nl) {
	static_assert(NL >= 1 && NL <= 4 && CTL_FULL % 4 == 0, "loader counters: one ds_read_b128");
	const u32x4_t f = *(volatile ENG_LDS u32x4_t *)(ctl + CTL_FULL);
	unsigned m = f[0] * nl;
#pragma unroll
	for (int l = 1; l < NL; ++l)
		if (l < (int)nl)
			m = min(m, f[l] * nl + l);
	return m;
}

// ---------------------------------------------------------------- prefetch wave
// 4-byte LDS-DMA per lane into the landing pad: the only purpose is the HBM read
// it causes (the line lands in L2 / Infinity Cache); hipcc never sees the load.
__device__ __forceinline__ void eng_touch(const void *g, unsigned pad_lds) {
	unsigned keep;
	asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
	             : "=&s"(keep)
	             : "v"(g), "s"(pad_lds)
	             : "memory");
}
// The loaders stop whenever the ring is full -- at every seam, while the consumers
// wait for the other CUs -- and HBM idles until the consumers free slots. The
// prefetch wave walks the same per-CU weight sequence up to pf_ahead items past
// the landed ring and touches every 64-B line of it, so HBM keeps streaming
// through the seams and the ring refills from on-die cache afterwards. Weights
// are read-only: the prefetch changes timing only, never a value.
template <class WT, int NL>
__device__ __forceinline__ void eng_prefetch(EngA &ca, unsigned pad_lds, volatile ENG_LDS unsigned *ctl, int nl) {
	const int b = blockIdx.x, NB = gridDim.x, lane = threadIdx.x & 63;
	const EngGeo geo{ca.dim, ca.hidden, ca.q_dim, ca.kv_dim, ca.vocab, ca.wcls};
	const int n_layers = ca.n_layers;
	EngL *layers = (EngL *)ca.layers;
	const int nph = 5 * n_layers + (ca.mode != EM_HYDRATE ? 1 : 0);
	const unsigned ahead = (unsigned)ca.pf_ahead;
	constexpr int TI = 64 * ENG_PF_LINE / ENG_ITEM; // items covered by one touch instruction
	unsigned it = 0, lim = 0;                       // items walked / allowed
	bool dead = false;
	for (int ph = 0; ph < nph && !dead; ++ph) {
		const int kind = ph < 5 * n_layers ? ph % 5 : EK_LOGITS;
		if (kind == EK_ATTN)
			continue;
		const EngLayer Ly = eng_layer(layers[ph < 5 * n_layers ? ph / 5 : 0]);
		int n, ngroups, R;
		eng_geo(geo, kind, n, ngroups, R);
		const int nch = n * WT::BYTES / ENG_ITEM;
		const int ngl = eng_ngl(ngroups, b, NB);
		for (int gl = 0; gl < ngl && !dead; ++gl) {
			for (int r = 0; r < R && !dead; ++r) {
				const char *rp = eng_row<WT>(geo, Ly, kind, b + gl * NB, r, n);
				for (int c = 0; c < nch; c += TI) {
					if (it + c >= lim) {
						EngSpin sp;
						while ((lim = eng_landed<NL>(ctl, nl) * ENG_IPS + ahead) <= it + c) {
							if (eng_spin(sp, ctl)) { // loaders gone or stuck: stop prefetching, no error
								dead = true;
								break;
							}
						}
						if (dead)
							break;
					}
					const int off = c * ENG_ITEM + lane * ENG_PF_LINE;
					if (off < nch * ENG_ITEM)
						eng_touch(rp + off, pad_lds);
					asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); // <= 33 x 4 KB in flight
				}
				it += nch;
			}
		}
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------- loader waves
// L loader waves share the CU's item stream slot-interleaved: loader l issues the
// 8 items of every slot s with s % L == l (one wave's DMA issue rate, ~8 GB/s,
// is far below the CU's 25 GB/s share of HBM) and publishes how many of ITS
// slots have landed (ctl[CTL_FULL + l]) behind its own counted vmcnt.
template <class WT, int C, int NL>
__device__ __forceinline__ void eng_loader(EngA &ca, unsigned ring_lds, volatile ENG_LDS unsigned *ctl, int l) {
	constexpr int NS = eng_ring_slots<C>();
	const int b = blockIdx.x, NB = gridDim.x, lane = threadIdx.x & 63;
	const EngGeo geo{ca.dim, ca.hidden, ca.q_dim, ca.kv_dim, ca.vocab, ca.wcls};
	const int n_layers = ca.n_layers;
	EngL *layers = (EngL *)ca.layers;
	unsigned *const err = ca.err;
	const int nph = 5 * n_layers + (ca.mode != EM_HYDRATE ? 1 : 0);
	__builtin_amdgcn_s_setprio(3);
	unsigned slot = 0, mine = 0, free_seen = NS, stall = 0, vmwait = 0;
	const unsigned long long tbeg = __builtin_amdgcn_s_memrealtime();
	const int depth = ca.ld_depth;
	const int nl = ca.ld_waves;
	if (l >= nl) {
		if (l == nl && ca.pf_ahead > 0)
			eng_prefetch<WT, NL>(ca, (unsigned)(uintptr_t)(ctl + ENG_CTL_WORDS), ctl, nl);
		return;
	}
	const bool nt = ca.ld_nt != 0;
	int k = 0; // items of the current slot already walked
	bool dead = false;
	for (int ph = 0; ph < nph && !dead; ++ph) {
		const int kind = ph < 5 * n_layers ? ph % 5 : EK_LOGITS;
		if (kind == EK_ATTN)
			continue;
		const EngLayer Ly = eng_layer(layers[ph < 5 * n_layers ? ph / 5 : 0]);
		int n, ngroups, R;
		eng_geo(geo, kind, n, ngroups, R);
		const int nch = n * WT::BYTES / ENG_ITEM;
		const int ngl = eng_ngl(ngroups, b, NB);
		for (int gl = 0; gl < ngl && !dead; ++gl) {
			for (int r = 0; r < R && !dead; ++r) {
				const char *rp = eng_row<WT>(geo, Ly, kind, b + gl * NB, r, n) + lane * 16;
				for (int c = 0; c < nch;) {
					const int take = min(nch - c, ENG_IPS - k); // this row's items in the current slot
					if ((int)(slot % nl) == l) {
						if (k == 0 && slot >= free_seen) { // ring position of slot - NS still in use
							const unsigned long long ts = __builtin_amdgcn_s_memrealtime();
							EngSpin sp;
							for (;;) {
								unsigned m = ctl[CTL_CONS];
#pragma unroll
								for (int w = 1; w < C; ++w)
									m = min(m, (unsigned)ctl[CTL_CONS + w]);
								free_seen = m + NS;
								if (slot < free_seen)
									break;
								if (eng_spin(sp, ctl)) {
									eng_fail(err, ctl, ENG_ERR_RING);
									dead = true;
									break;
								}
							}
							stall += (unsigned)(__builtin_amdgcn_s_memrealtime() - ts);
							ctl[CTL_LSTALL + l] = stall;
							if (dead)
								break;
						}
						const unsigned dst = ring_lds + ((slot % NS) * ENG_IPS + k) * ENG_ITEM;
						for (int i = 0; i < take; ++i)
							eng_glds16(rp + (size_t)(c + i) * ENG_ITEM, __builtin_amdgcn_readfirstlane(dst + i * ENG_ITEM), nt);
					}
					c += take;
					k += take;
					if (k == ENG_IPS) {
						if ((int)(slot % nl) == l && ++mine > (unsigned)depth) {
							const unsigned long long tv = __builtin_amdgcn_s_memrealtime();
							eng_vmcnt_slots(depth);
							vmwait += (unsigned)(__builtin_amdgcn_s_memrealtime() - tv);
							ctl[CTL_FULL + l] = mine - depth;
						}
						k = 0;
						++slot;
					}
				}
			}
		}
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	if (k > 0 && (int)(slot % nl) == l)
		++mine; // the partial last slot
	ctl[CTL_FULL + l] = mine;
	const unsigned long long tf = __builtin_amdgcn_s_memrealtime();
	if (l == 0) {
		ctl[52] = (unsigned)tf;
		ctl[53] = (unsigned)(tf >> 32);
		ctl[54] = vmwait;              // ticks blocked in s_waitcnt vmcnt (data latency)
		ctl[55] = (unsigned)(tf - tbeg); // loader 0 lifetime
	}
}

// ---------------------------------------------------------------- consumer context
template <class WT, int C, int NL>
struct EngCtx {
	EngA &a;
	ENG_LDS char *ring;
	ENG_LDS float *part;
	volatile ENG_LDS unsigned *ctl;
	int b, NB, lane, w, tid;
	unsigned full_seen, cbar_n, jbase, epoch0;
	int token, pos, kv_sink, kv_pos, kv_len;
	bool dead;

	__device__ EngCtx(EngA &a_) : a(a_) {}

	// consumer-only barrier (the loader never joins: an s_barrier would stall its stream)
	__device__ __forceinline__ void cbar() {
		if (dead)
			return;
		cbar_n += C;
		if (lane == 0)
			__hip_atomic_fetch_add((ENG_LDS unsigned *)&ctl[CTL_CBAR], 1u, __ATOMIC_RELEASE,
			                       __HIP_MEMORY_SCOPE_WORKGROUP);
		EngSpin sp;
		while (eng_lds_acq(&ctl[CTL_CBAR]) < cbar_n) {
			if (eng_spin(sp, ctl)) {
				eng_fail(a.err, ctl, ENG_ERR_CBAR);
				dead = true;
				return;
			}
		}
	}

	__device__ __forceinline__ unsigned landed() { return eng_landed<NL>(ctl, (unsigned)a.ld_waves); }
	// ring slot holding item j has landed
	__device__ __forceinline__ bool wait_item(unsigned j) {
		const unsigned s = j / ENG_IPS;
		if (s < full_seen) {
			asm volatile("" ::: "memory"); // no ring read may be hoisted above this check
			return true;
		}
		EngSpin sp;
		while ((full_seen = landed()) <= s) {
			switch (a.poll_sleep) { // extra back-off: every poll is an LDS op competing with the loaders' DMA issue
			case 2:
				__builtin_amdgcn_s_sleep(1);
				break;
			case 4:
				__builtin_amdgcn_s_sleep(3);
				break;
			case 8:
				__builtin_amdgcn_s_sleep(7);
				break;
			case 16:
				__builtin_amdgcn_s_sleep(15);
				break;
			default:
				break;
			}
			if (eng_spin(sp, ctl)) {
				eng_fail(a.err, ctl, ENG_ERR_RING);
				dead = true;
				return false;
			}
		}
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); // ring reads stay behind the poll
		return true;
	}
	__device__ __forceinline__ u32x4_t ring_item(unsigned j) const {
		constexpr unsigned RING = eng_ring_slots<C>() * ENG_IPS;
		return *(const ENG_LDS u32x4_t *)(ring + (size_t)(j % RING) * ENG_ITEM + lane * 16);
	}
	__device__ __forceinline__ void release(unsigned next_item) { // every lane stores the same word
		if (!(a.dbg & 128))
			eng_lds_rel(&ctl[CTL_CONS + w], next_item / ENG_IPS);
	}

	// every CU finished phase `epoch` (flags are per-CU epochs, monotonic over launches)
	__device__ __forceinline__ void seam(unsigned epoch) {
		if (dead)
			return;
		EngSpin sp;
		if (w == 0) {
			for (;;) {
				bool ok = true;
				for (int i = lane * 4; i < NB; i += 256) {
					const unsigned long long f01 = __hip_atomic_load((const unsigned long long *)(a.flags + i),
					                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					const unsigned long long f23 = __hip_atomic_load((const unsigned long long *)(a.flags + i + 2),
					                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					ok &= (int)((unsigned)f01 - epoch) >= 0 || i >= NB;
					ok &= (int)((unsigned)(f01 >> 32) - epoch) >= 0 || i + 1 >= NB;
					ok &= (int)((unsigned)f23 - epoch) >= 0 || i + 2 >= NB;
					ok &= (int)((unsigned)(f23 >> 32) - epoch) >= 0 || i + 3 >= NB;
				}
				if (__all(ok))
					break;
				if (eng_spin(sp, ctl)) {
					eng_fail(a.err, ctl, ENG_ERR_SEAM);
					dead = true;
					return;
				}
			}
			if (lane == 0)
				eng_lds_rel(&ctl[CTL_SEAM], epoch);
		} else {
			while ((int)(eng_lds_acq(&ctl[CTL_SEAM]) - epoch) < 0) {
				if (eng_spin(sp, ctl)) {
					eng_fail(a.err, ctl, ENG_ERR_SEAM);
					dead = true;
					return;
				}
			}
		}
	}

	// this CU finished phase `epoch`: every consumer wave drains its sc1 stores, then one flag store
	__device__ __forceinline__ void publish(unsigned epoch) {
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		cbar();
		if (!dead && w == 0 && lane == 0)
			__hip_atomic_store(a.flags + b, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
};

// The wave's share of a phase: for every row, its KW chunk columns (w, w + C, ...)
// dotted with the register slice xr. Rows go in tiles of 4: one transposed
// cross-lane reduction, one branch-free LDS write of the 4 row partials
// (part[row][wave]; rows past the phase land in spare rows nobody reads) and one
// ring release per tile.
template <class WT, int C, int NL, int KW, bool MATH>
__device__ __forceinline__ bool eng_rows(EngCtx<WT, C, NL> &cx, const float (&xr)[64 / WT::EPL][WT::EPL], int rows,
                                         int nch) {
	constexpr unsigned RING = eng_ring_slots<C>() * ENG_IPS;
	const int w = cx.w, lane = cx.lane;
	const unsigned lane_off = (unsigned)lane * 16;
	for (int r0 = 0; r0 < rows; r0 += 4) {
		float acc[4];
#pragma unroll
		for (int t = 0; t < 4; ++t) {
			float a0 = 0.0f, a1 = 0.0f;
			if (r0 + t < rows) {
				const unsigned j0 = cx.jbase + (unsigned)(r0 + t) * nch + w;
				// slots land in order: waiting for my last item of the row covers the others
				if (!cx.wait_item(j0 + (KW - 1) * C))
					return false;
				unsigned pos = j0 % RING;
				u32x4_t wv[KW];
#pragma unroll
				for (int k = 0; k < KW; ++k) {
					wv[k] = *(const ENG_LDS u32x4_t *)(cx.ring + pos * ENG_ITEM + lane_off);
					pos += C;
					if (pos >= RING)
						pos -= RING;
				}
				if constexpr (MATH) {
#pragma unroll
					for (int k = 0; k < KW; ++k)
						eng_dot16<WT>(a0, a1, wv[k], xr[k]);
				} else {
#pragma unroll
					for (int k = 0; k < KW; ++k)
						a0 += __uint_as_float(wv[k][0] & 0x3fffffu);
				}
				// per row, not per tile: a tile of long rows (W2: 3.5 slots each) held until its
				// end would pin more slots than the ring minus the loaders' publication lag
				cx.release(j0 - w + nch);
			}
			acc[t] = a0 + a1;
		}
		const float tot = eng_sum4_t(acc);
		if (!(cx.a.dbg & 256))
			cx.part[(r0 + (lane >> 4)) * C + w] = tot;
	}
	return true;
}

// ---------------------------------------------------------------- GEMV phase (consumers)
template <class WT, int C, int NL>
__device__ __forceinline__ void eng_gemv(EngCtx<WT, C, NL> &cx, int kind, int layer, unsigned long long *tr) {
	constexpr int EPL = WT::EPL;
	constexpr int KMAX = 64 / EPL; // x slice registers: KMAX x EPL = 64 floats per lane
	constexpr int CH = 64 * EPL;   // elements per item
	EngA &a = cx.a;
	EngL &L = ((EngL *)a.layers)[kind == EK_LOGITS ? 0 : layer];
	const int w = cx.w, lane = cx.lane;
	int n, ngroups, R;
	eng_geo(a, kind, n, ngroups, R);
	const int nch = n / CH;
	const int kw = nch > w ? (nch - 1 - w) / C + 1 : 0; // my chunk columns: w, w + C, ...

	// ---- input slice -> registers (sc1: produced in this launch by other CUs)
	float xr[KMAX][EPL];
	const bool from_emb = kind == EK_QKV && layer == 0;
	const float *xin = kind == EK_WO ? a.xb2 : (kind == EK_W2 ? a.hb : a.x);
	const char *erow = a.emb + (size_t)cx.token * a.dim * WT::BYTES;
	const bool gather = !(a.dbg & 64);
#pragma unroll
	for (int k = 0; k < KMAX; ++k) {
		if (k < kw && !gather) {
#pragma unroll
			for (int e = 0; e < EPL; ++e)
				xr[k][e] = 0.0f;
		} else if (k < kw) {
			const int i0 = (w + k * C) * CH + lane * EPL;
			if (from_emb) {
				WT::unpack(load16(erow + (size_t)i0 * WT::BYTES), xr[k]);
			} else {
#pragma unroll
				for (int e = 0; e < EPL; e += 2)
					eng_ld2_sc1(xin + i0 + e, xr[k][e], xr[k][e + 1]);
			}
		}
	}
	// ---- rmsnorm (infer.cpp:134-144: scale = 1/sqrt(ss/n + eps); o = x * scale * w)
	if (gather && (kind == EK_QKV || kind == EK_GLU || kind == EK_LOGITS)) {
		const float *nw = kind == EK_QKV ? L.rms_att : (kind == EK_GLU ? L.rms_ffn : a.rms_final);
		float ss = 0.0f;
#pragma unroll
		for (int k = 0; k < KMAX; ++k)
			if (k < kw)
#pragma unroll
				for (int e = 0; e < EPL; ++e)
					ss = fmaf(xr[k][e], xr[k][e], ss);
		ss = wave_sum(ss);
		volatile ENG_LDS float *nrm = (volatile ENG_LDS float *)(cx.ctl + CTL_NRM);
		if (lane == 0)
			nrm[w] = ss;
		cx.cbar();
		float tot = 0.0f;
#pragma unroll
		for (int v = 0; v < C; ++v)
			tot += nrm[v];
		const float scale = 1.0f / sqrtf(tot / n + a.eps);
#pragma unroll
		for (int k = 0; k < KMAX; ++k) {
			if (k < kw) {
				const int i0 = (w + k * C) * CH + lane * EPL;
#pragma unroll
				for (int e = 0; e < EPL; e += 4) {
					const float4_t g = *(const float4_t *)(nw + i0 + e);
#pragma unroll
					for (int t = 0; t < 4; ++t)
						xr[k][e + t] = xr[k][e + t] * scale * g[t];
				}
			}
		}
	}

	// ---- sinks (pos >= max_seq_len): rotate K rows < kv_sink by one position (CU 0)
	if (kind == EK_QKV && cx.kv_sink > 0 && cx.b == 0) {
		const int hd = ENG_D;
		for (int r = 0; r < cx.kv_sink; ++r) {
			for (int i = 2 * cx.tid; i < a.kv_dim; i += 2 * 64 * C) {
				uint16_t *p = L.kc + (size_t)r * a.kv_dim + i;
				const uint32_t pr = eng_ld_u32_sc1(p);
				const float v0 = h2f((uint16_t)pr), v1 = h2f((uint16_t)(pr >> 16));
				const float freq = a.inv_freq[(i % hd) >> 1];
				const float val = 1.0f * freq;
				const float fcr = cosf(val), fci = sinf(val);
				const uint32_t o = (uint32_t)f2h(v0 * fcr - v1 * fci) | ((uint32_t)f2h(v0 * fci + v1 * fcr) << 16);
				eng_st_u32_sc1(p, o);
			}
		}
	}

	if (tr)
		tr[1] = __builtin_amdgcn_s_memrealtime();
	// ---- stream the ring: row by row, my chunks of each row (count known at compile time)
	const bool math = !(a.dbg & 1);
	const int ngl = eng_ngl(ngroups, cx.b, cx.NB);
	const int rows = ngl * R;
	bool ok = true;
	switch ((a.dbg & 4) ? 0 : kw) {
#define ENG_ROWS_CASE(K)                                                                                               \
	case K:                                                                                                            \
		if constexpr (K <= KMAX)                                                                                       \
			ok = math ? eng_rows<WT, C, NL, K, true>(cx, xr, rows, nch) : eng_rows<WT, C, NL, K, false>(cx, xr, rows, nch); \
		break;
		ENG_ROWS_CASE(1)
		ENG_ROWS_CASE(2)
		ENG_ROWS_CASE(3)
		ENG_ROWS_CASE(4)
		ENG_ROWS_CASE(5)
		ENG_ROWS_CASE(6)
		ENG_ROWS_CASE(7)
		ENG_ROWS_CASE(8)
		ENG_ROWS_CASE(9)
		ENG_ROWS_CASE(10)
		ENG_ROWS_CASE(11)
		ENG_ROWS_CASE(12)
		ENG_ROWS_CASE(13)
		ENG_ROWS_CASE(14)
		ENG_ROWS_CASE(15)
		ENG_ROWS_CASE(16)
#undef ENG_ROWS_CASE
	default: // no chunk of this phase's rows: zero partials, keep releasing
		for (int rl = 0; rl < rows; ++rl) {
			if (!(a.dbg & 4))
				cx.release(cx.jbase + (unsigned)(rl + 1) * nch);
			if (lane == 0)
				cx.part[rl * C + w] = 0.0f;
		}
	}
	if (!ok)
		return;
	cx.jbase += (unsigned)rows * nch;
	if (!(a.dbg & 4))
		cx.release(cx.jbase);
	if (tr)
		tr[2] = __builtin_amdgcn_s_memrealtime();
	cx.cbar(); // row partials of every wave are in LDS

	// ---- epilogue: one thread per row group, partials summed in wave order
	const int pos = cx.pos;
	float best = -FLT_MAX;
	int bi = 0x7fffffff;
	for (int gl = cx.tid; gl < ngl && !cx.dead && !(a.dbg & 32); gl += 64 * C) {
		float acc[2];
#pragma unroll
		for (int r = 0; r < 2; ++r) {
			float t = 0.0f;
			if (r < R)
#pragma unroll
				for (int v = 0; v < C; ++v)
					t += cx.part[(gl * R + r) * C + v];
			acc[r] = t;
		}
		const int g = cx.b + gl * cx.NB;
		switch (kind) {
		case EK_QKV: { // infer.cpp:280-301 clip + rope; infer.cu:642-677 cache write
			const float c = a.qkv_clip;
			const float v0 = acc[0] < -c ? -c : (acc[0] > c ? c : acc[0]);
			const float v1 = acc[1] < -c ? -c : (acc[1] > c ? c : acc[1]);
			const int vr = 2 * g;
			if (vr >= a.q_dim + a.kv_dim) {
				const size_t o = (size_t)cx.kv_pos * a.kv_dim + (vr - a.q_dim - a.kv_dim);
				eng_st_u32_sc1(L.vc + o, (uint32_t)f2h(v0) | ((uint32_t)f2h(v1) << 16));
			} else {
				const int i = vr < a.q_dim ? vr : vr - a.q_dim;
				const float freq = a.inv_freq[(i % ENG_D) >> 1];
				const float val = (float)pos * freq;
				const float fcr = cosf(val), fci = sinf(val);
				const float r0 = v0 * fcr - v1 * fci;
				const float r1 = v0 * fci + v1 * fcr;
				if (vr < a.q_dim) {
					eng_st2_sc1(a.q + i, r0, r1);
				} else {
					const size_t o = (size_t)cx.kv_pos * a.kv_dim + i;
					eng_st_u32_sc1(L.kc + o, (uint32_t)f2h(r0) | ((uint32_t)f2h(r1) << 16));
				}
			}
			break;
		}
		case EK_WO:
		case EK_W2: {
			const float xo = (kind == EK_WO && layer == 0) ? eng_elem<WT>(erow, g) : eng_ld_sc1(a.x + g);
			eng_st_sc1(a.x + g, xo + acc[0]);
			break;
		}
		case EK_GLU:
			eng_st_sc1(a.hb + g, (a.act == 1 ? act_fn<1>(acc[0]) : act_fn<0>(acc[0])) * acc[1]);
			break;
		default: // logits; first max of this CU's (ascending) rows
			a.logits[g] = acc[0];
			if (acc[0] > best) {
				best = acc[0];
				bi = g;
			}
		}
	}
	if (kind == EK_LOGITS && a.mode == EM_GREEDY) { // this CU's (max, first index) -> amax[b]
#pragma unroll
		for (int off = 32; off > 0; off >>= 1) {
			const float ov = __shfl_xor(best, off, 64);
			const int oi = __shfl_xor(bi, off, 64);
			if (ov > best || (ov == best && oi < bi)) {
				best = ov;
				bi = oi;
			}
		}
		volatile ENG_LDS unsigned *am = cx.ctl + CTL_AMAX;
		if (lane == 0) {
			am[2 * w] = __float_as_uint(best);
			am[2 * w + 1] = (unsigned)bi;
		}
		cx.cbar();
		if (w == 0 && lane == 0) {
			float B = __uint_as_float(am[0]);
			int I = (int)am[1];
			for (int v = 1; v < C; ++v) {
				const float ov = __uint_as_float(am[2 * v]);
				const int oi = (int)am[2 * v + 1];
				if (ov > B || (ov == B && oi < I)) {
					B = ov;
					I = oi;
				}
			}
			eng_st2_sc1(a.amax + 2 * cx.b, B, __int_as_float(I));
		}
	}
}

// ---------------------------------------------------------------- attention unit (one wave)
// kv head g, split s of S: chunks s, s + S, ... of ENG_KC keys. Lane layout: 16 lanes
// per key row (8 dims each, D = 128), 4 rows per wave instruction, 8 rows per lane.
template <int GT>
__device__ __forceinline__ void eng_attn_unit(EngA &a, EngL &L, int g, int s, int S, int ns, int kv_len, int G,
                              int lane, bool &dead, volatile ENG_LDS unsigned *ctl, int layer) {
	constexpr int D = ENG_D;
	const int sub = lane >> 4, piece = lane & 15;
	const float sq = sqrtf((float)D);
	float qr[GT][8];
#pragma unroll
	for (int h = 0; h < GT; ++h) {
		const int hh = h < G ? h : 0;
		const float *qp = a.q + (size_t)(g * G + hh) * D + piece * 8;
#pragma unroll
		for (int e = 0; e < 8; e += 2)
			eng_ld2_sc1(qp + e, qr[h][e], qr[h][e + 1]);
	}
	float M[GT], Ls[GT], o[GT][8];
#pragma unroll
	for (int h = 0; h < GT; ++h) {
		M[h] = -FLT_MAX;
		Ls[h] = 0.0f;
#pragma unroll
		for (int e = 0; e < 8; ++e)
			o[h][e] = 0.0f;
	}
	for (int c = s; c < ns; c += S) {
		const int t0 = c * ENG_KC;
		u32x4_t kw[8], vw[8];
#pragma unroll
		for (int i = 0; i < 8; ++i) {
			const int t = min(t0 + sub + 4 * i, kv_len - 1);
			const size_t off = (size_t)t * a.kv_dim + g * D + piece * 8;
			kw[i] = eng_ld16_sc1(L.kc + off);
			vw[i] = eng_ld16_sc1(L.vc + off);
		}
		float sc[GT][8];
#pragma unroll
		for (int i = 0; i < 8; ++i) {
			float kf[8];
			WF16::unpack(kw[i], kf);
			const bool valid = t0 + sub + 4 * i < kv_len;
#pragma unroll
			for (int h = 0; h < GT; ++h) {
				float d = 0.0f;
#pragma unroll
				for (int e = 0; e < 8; ++e)
					d = fmaf(qr[h][e], kf[e], d);
				d = row16_sum(d);
				sc[h][i] = valid ? d / sq : -FLT_MAX;
			}
		}
#pragma unroll
		for (int h = 0; h < GT; ++h) {
			float m = sc[h][0];
#pragma unroll
			for (int i = 1; i < 8; ++i)
				m = fmaxf(m, sc[h][i]);
			m = fmaxf(m, xor16(m));
			m = fmaxf(m, xor32(m));
			const float mn = fmaxf(M[h], m);
			const float r = expf(M[h] - mn);
			float l = 0.0f;
#pragma unroll
			for (int i = 0; i < 8; ++i) {
				const float p = expf(sc[h][i] - mn);
				sc[h][i] = p;
				l += p;
			}
			l += xor16(l);
			l += xor32(l);
			Ls[h] = Ls[h] * r + l;
			M[h] = mn;
#pragma unroll
			for (int e = 0; e < 8; ++e)
				o[h][e] *= r;
		}
#pragma unroll
		for (int i = 0; i < 8; ++i) {
			float vf[8];
			WF16::unpack(vw[i], vf);
#pragma unroll
			for (int h = 0; h < GT; ++h)
#pragma unroll
				for (int e = 0; e < 8; ++e)
					o[h][e] = fmaf(sc[h][i], vf[e], o[h][e]);
		}
	}
#pragma unroll
	for (int h = 0; h < GT; ++h)
#pragma unroll
		for (int e = 0; e < 8; ++e) {
			o[h][e] += xor16(o[h][e]);
			o[h][e] += xor32(o[h][e]);
		}
	if (S == 1) { // whole context in this unit: normalise and write the heads
		if (sub == 0) {
#pragma unroll
			for (int h = 0; h < GT; ++h) {
				if (h < G) {
					float *op = a.xb2 + (size_t)(g * G + h) * D + piece * 8;
#pragma unroll
					for (int e = 0; e < 8; e += 2)
						eng_st2_sc1(op + e, o[h][e] / Ls[h], o[h][e + 1] / Ls[h]);
				}
			}
		}
		return;
	}
	// ---- publish (o, m, l) of this split, write-through; ticket; last arriver merges
#pragma unroll
	for (int h = 0; h < GT; ++h) {
		if (h < G) {
			float *pp = a.part + ((size_t)(g * G + h) * ENG_SMAX + s) * (D + 2);
			if (sub == 0) {
#pragma unroll
				for (int e = 0; e < 8; e += 2)
					eng_st2_sc1(pp + piece * 8 + e, o[h][e], o[h][e + 1]);
			}
			if (lane == 0)
				eng_st2_sc1(pp + D, M[h], Ls[h]);
		}
	}
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	unsigned ticket = 0;
	if (lane == 0)
		ticket = __hip_atomic_fetch_add(a.tickets + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	ticket = __builtin_amdgcn_readfirstlane(ticket);
	if (ticket != (unsigned)(S - 1))
		return;
	if (lane == 0) // reset for the next layer (ordered by the seams in between)
		__hip_atomic_store(a.tickets + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	// flash-decoding merge of the S splits, 8 at a time (all loads of a batch in flight)
	for (int h = 0; h < G; ++h) {
		const float *ph = a.part + (size_t)(g * G + h) * ENG_SMAX * (D + 2);
		float Mx = -FLT_MAX, Lx = 0.0f, o0 = 0.0f, o1 = 0.0f;
		for (int s0 = 0; s0 < S; s0 += 8) {
			float mb[8], lb[8], ob0[8], ob1[8];
#pragma unroll
			for (int j = 0; j < 8; ++j) {
				const float *pc = ph + (size_t)min(s0 + j, S - 1) * (D + 2);
				eng_ld2_sc1(pc + D, mb[j], lb[j]);
				ob0[j] = eng_ld_sc1(pc + lane);
				ob1[j] = eng_ld_sc1(pc + 64 + lane);
			}
			float Mn = Mx;
#pragma unroll
			for (int j = 0; j < 8; ++j)
				if (s0 + j < S)
					Mn = fmaxf(Mn, mb[j]);
			const float r = expf(Mx - Mn);
			Lx *= r;
			o0 *= r;
			o1 *= r;
#pragma unroll
			for (int j = 0; j < 8; ++j) {
				if (s0 + j < S) {
					const float wgt = expf(mb[j] - Mn);
					Lx += wgt * lb[j];
					o0 += wgt * ob0[j];
					o1 += wgt * ob1[j];
				}
			}
			Mx = Mn;
		}
		float *op = a.xb2 + (size_t)(g * G + h) * D;
		eng_st_sc1(op + lane, o0 / Lx);
		eng_st_sc1(op + 64 + lane, o1 / Lx);
	}
}

// ---------------------------------------------------------------- the kernel
template <class WT, int C, int NL, int GT>
__global__ __launch_bounds__(64 * (C + NL)) void engine_kernel(const EngArgs *__restrict__ args) {
	// Arguments live in device memory (written once per decoder and mode): a
	// by-value struct whose address is taken is copied to scratch per lane.
	EngA &a = *(EngA *)args;
	extern __shared__ __attribute__((aligned(16))) char lds_raw[];
	constexpr int NS = eng_ring_slots<C>();
	ENG_LDS char *lds = (ENG_LDS char *)lds_raw;
	ENG_LDS char *ring = lds;
	ENG_LDS float *part = (ENG_LDS float *)(lds + (size_t)NS * ENG_IPS * ENG_ITEM);
	volatile ENG_LDS unsigned *ctl = (volatile ENG_LDS unsigned *)(part + ENG_MAXROWS * C);
	if (threadIdx.x < ENG_CTL_WORDS)
		ctl[threadIdx.x] = 0;
	__syncthreads(); // the only workgroup barrier: loader and consumers split after it

	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	if (wave >= C) {
		eng_loader<WT, C, NL>(a, (unsigned)(uintptr_t)ring, ctl, wave - C);
		return;
	}

	EngCtx<WT, C, NL> cx(a);
	cx.ring = ring;
	cx.part = part;
	cx.ctl = ctl;
	cx.b = blockIdx.x;
	cx.NB = gridDim.x;
	cx.lane = threadIdx.x & 63;
	cx.w = wave;
	cx.tid = threadIdx.x;
	cx.full_seen = 0;
	cx.cbar_n = 0;
	cx.jbase = 0;
	cx.dead = false;
	const unsigned E = 5u * a.n_layers + 2u; // epochs per launch (fixed for every mode)
	cx.epoch0 = __hip_atomic_load(a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * E;
	cx.token = a.step->token;
	cx.pos = a.step->pos;
	// sliding window (infer.cu:1081-1083, KV_SINKS = 2)
	cx.kv_sink = cx.pos >= a.max_seq_len ? 2 : 0;
	cx.kv_pos = cx.kv_sink + (cx.pos - cx.kv_sink) % (a.max_seq_len - cx.kv_sink);
	cx.kv_len = cx.pos >= a.max_seq_len ? a.max_seq_len : cx.pos + 1;

	if ((a.dbg & (4 | 128)) && cx.lane == 0) // timing only: the loaders stream unthrottled
		ctl[CTL_CONS + cx.w] = 0x40000000u;
	const int nph = 5 * a.n_layers + (a.mode != EM_HYDRATE ? 1 : 0);
	unsigned long long *trb = a.trace && cx.w == 0 && cx.lane == 0 ? a.trace + (size_t)cx.b * E * 8 : nullptr;
	if (trb)
		trb[(E - 1) * 8] = __builtin_amdgcn_s_memrealtime();
	for (int ph = 0; ph < nph && !cx.dead; ++ph) {
		const int kind = eng_kind(a, ph);
		const int layer = ph < 5 * a.n_layers ? ph / 5 : 0;
		if (ph > 0 && !(a.dbg & 2))
			cx.seam(cx.epoch0 + ph); // phase ph - 1 done everywhere
		if (cx.dead)
			break;
		unsigned long long *tr = trb ? trb + (size_t)ph * 8 : nullptr;
		if (tr) {
			tr[0] = __builtin_amdgcn_s_memrealtime();
			tr[5] = cx.landed();
			tr[6] = cx.jbase;
		}
		if (kind == EK_ATTN) {
			const int G = a.n_heads / a.n_kv;
			const int ns = (cx.kv_len + ENG_KC - 1) / ENG_KC;
			const int S = min(ns, ENG_SMAX);
			EngL &L = ((EngL *)a.layers)[layer];
			for (int u = cx.b + cx.w * cx.NB; u < a.n_kv * S; u += cx.NB * C)
				eng_attn_unit<GT>(a, L, u / S, u % S, S, ns, cx.kv_len, G, cx.lane, cx.dead, ctl, layer);
			if (tr)
				tr[1] = tr[2] = __builtin_amdgcn_s_memrealtime();
		} else {
			eng_gemv<WT, C>(cx, kind, layer, tr);
		}
		cx.publish(cx.epoch0 + ph + 1);
		if (tr) {
			tr[3] = __builtin_amdgcn_s_memrealtime();
			tr[4] = ctl[CTL_LSTALL];
		}
	}
	if (trb) { // per-CU extras in the last record: start, loader stall, loader finish, end
		trb[(E - 1) * 8 + 1] = ctl[CTL_LSTALL];
		trb[(E - 1) * 8 + 2] = (unsigned long long)ctl[52] | ((unsigned long long)ctl[53] << 32);
		trb[(E - 1) * 8 + 3] = __builtin_amdgcn_s_memrealtime();
		trb[(E - 1) * 8 + 4] = ctl[54];
		trb[(E - 1) * 8 + 5] = ctl[55];
	}
	if (cx.dead)
		return;
	if (cx.b == 0 && cx.w == 0) {
		if (a.mode == EM_GREEDY) { // global first max over the per-CU pairs (sampler.cpp:27-38)
			cx.seam(cx.epoch0 + nph);
			if (cx.dead)
				return;
			float best = -FLT_MAX;
			int bi = 0x7fffffff;
			for (int i = cx.lane; i < cx.NB; i += 64) {
				float v, fi;
				eng_ld2_sc1(a.amax + 2 * i, v, fi);
				const int ii = __float_as_int(fi);
				if (v > best || (v == best && ii < bi)) {
					best = v;
					bi = ii;
				}
			}
#pragma unroll
			for (int off = 32; off > 0; off >>= 1) {
				const float ov = __shfl_xor(best, off, 64);
				const int oi = __shfl_xor(bi, off, 64);
				if (ov > best || (ov == best && oi < bi)) {
					best = ov;
					bi = oi;
				}
			}
			if (cx.lane == 0) {
				if (bi == 0x7fffffff)
					bi = 0;
				StepState *st = a.step;
				const int k = st->n_gen;
				if (a.tokens && k < a.tokens_cap)
					a.tokens[k] = bi;
				st->n_gen = k + 1;
				st->token = bi;
				st->pos = cx.pos + 1;
			}
		}
		if (cx.lane == 0) // next launch's epochs; every CU read gen before its first flag
			__hip_atomic_store(a.gen, __hip_atomic_load(a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u,
			                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
}
