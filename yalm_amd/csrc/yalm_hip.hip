// yalm_hip.hip — C ABI (include/yalm_hip.h) of the MI355X decode engine:
// device shim, decoder (graph-captured per-token forward) and the kernel-level
// test API. Replaces /root/reference/src/infer.cu:33-90 (shim), 699-888
// (_block_cuda), 890-1019 (test API), 1021-1164 (_forward_cuda + CudaGraph)
// and the device upload of model.cpp:185-211, 323-345, 380-394.
#include "../../include/yalm_hip.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "attention.h"
#include "attn_wo.h"
#include "decoder.h"
#include "device_common.h"
#include "gemv.h"
#include "misc_kernels.h"

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;

void set_err(const std::string &s) {
	g_err = s;
}

extern "C" const char *yalm_last_error(void) {
	return g_err.c_str();
}

// ------------------------------------------------------------------ shim
extern "C" int yalm_set_device(int device) {
	HIPCHK(hipSetDevice(device));
	return YALM_OK;
}

extern "C" void *yalm_upload(const void *host, size_t size) {
	void *dev = nullptr;
	if (hipMalloc(&dev, size ? size : 1) != hipSuccess) {
		set_err("hipMalloc failed in yalm_upload");
		return nullptr;
	}
	if (size && hipMemcpy(dev, host, size, hipMemcpyHostToDevice) != hipSuccess) {
		set_err("hipMemcpy H2D failed in yalm_upload");
		(void)hipFree(dev);
		return nullptr;
	}
	return dev;
}

extern "C" void *yalm_alloc(size_t size) {
	void *dev = nullptr;
	if (hipMalloc(&dev, size ? size : 1) != hipSuccess) {
		set_err("hipMalloc failed in yalm_alloc");
		return nullptr;
	}
	if (hipMemset(dev, 0, size ? size : 1) != hipSuccess) {
		set_err("hipMemset failed in yalm_alloc");
		(void)hipFree(dev);
		return nullptr;
	}
	return dev;
}

extern "C" int yalm_download(void *host, const void *device, size_t size) {
	HIPCHK(hipMemcpy(host, device, size, hipMemcpyDeviceToHost));
	return YALM_OK;
}

extern "C" int yalm_register_host(void *host, size_t size) {
	HIPCHK(hipHostRegister(host, size, hipHostRegisterDefault));
	return YALM_OK;
}

extern "C" int yalm_unregister_host(void *host) {
	HIPCHK(hipHostUnregister(host));
	return YALM_OK;
}

extern "C" int yalm_free(void *device) {
	HIPCHK(hipFree(device));
	return YALM_OK;
}

extern "C" int yalm_stream_create(yalm_stream *out) {
	ARGCHK(out, "null stream out");
	hipStream_t s;
	HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
	*out = reinterpret_cast<yalm_stream>(s);
	return YALM_OK;
}

// A stream restricted to CU block `part` of `n_parts` (hipExtStreamCreateWithCUMask):
// bits [part * ncu / n_parts, (part + 1) * ncu / n_parts). The driver spreads such a block
// evenly over the 8 XCDs (tools/cumask_probe.hip, profiles/r6a_cumask_probe.txt: 256 / N CUs
// on all 8 XCCs, disjoint between parts); an interleaved mask (bit i to part i mod N) was
// not honoured (every part ran on all 256 CUs). Used to run N tensor-parallel rank
// processes on ONE GPU as N disjoint sets of CUs (the multi-GPU rehearsal).
extern "C" int yalm_stream_create_cu_part(int part, int n_parts, yalm_stream *out) {
	ARGCHK(out && n_parts >= 1 && part >= 0 && part < n_parts, "yalm_stream_create_cu_part: bad argument");
	const int ncu = device_cu_count();
	ARGCHK(ncu % n_parts == 0 && ncu <= 32 * YALM_CU_MASK_WORDS, "yalm_stream_create_cu_part: CUs do not divide");
	uint32_t m[YALM_CU_MASK_WORDS] = {};
	for (int i = part * (ncu / n_parts); i < (part + 1) * (ncu / n_parts); ++i)
		m[i / 32] |= 1u << (i % 32);
	hipStream_t s;
	HIPCHK(hipExtStreamCreateWithCUMask(&s, (uint32_t)((ncu + 31) / 32), m));
	*out = reinterpret_cast<yalm_stream>(s);
	return YALM_OK;
}

// The CUs a stream may run on (all of them for an ordinary stream).
static int stream_cu_mask(hipStream_t s, uint32_t *m) {
	const int ncu = device_cu_count();
	for (int i = 0; i < YALM_CU_MASK_WORDS; ++i)
		m[i] = 0;
	if (!s || hipExtStreamGetCUMask(s, (uint32_t)((ncu + 31) / 32), m) != hipSuccess) {
		(void)hipGetLastError();
		for (int i = 0; i < ncu && i < 32 * YALM_CU_MASK_WORDS; ++i)
			m[i / 32] |= 1u << (i % 32);
	}
	return YALM_OK;
}

extern "C" int yalm_stream_destroy(yalm_stream s) {
	HIPCHK(hipStreamDestroy(reinterpret_cast<hipStream_t>(s)));
	return YALM_OK;
}

extern "C" int yalm_stream_sync(yalm_stream s) {
	HIPCHK(hipStreamSynchronize(reinterpret_cast<hipStream_t>(s)));
	return YALM_OK;
}

extern "C" int yalm_synth(void *device, size_t n, int dtype, uint64_t seed, float scale, float offset, yalm_stream s) {
	ARGCHK(dtype == YALM_F32 || dtype == YALM_F16 || dtype == YALM_F8E5M2, "yalm_synth: bad dtype");
	hipStream_t st = reinterpret_cast<hipStream_t>(s);
	synth_kernel<<<4096, 256, 0, st>>>(device, n, dtype, seed, scale, offset);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// ------------------------------------------------------------------ launch helpers
int device_cu_count() {
	static int n = 0;
	if (!n) {
		int dev = 0;
		if (hipGetDevice(&dev) != hipSuccess ||
		    hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
			n = 256;
	}
	return n;
}

// Row-block geometry (gemv_rb_kernel): `gpw` = workgroups per CU (default 1),
// threads 512 (8 waves), U = 8 loads in flight per wave.
// whole-row mode (gemv.h ROWS): W1|W3 (PGlu), W2 / Wo (PResidual), QKV (PQKV) when the rows divide
// evenly over the waves
template <class P>
struct RowsMode {
	static constexpr bool value = false;
};
template <class WT, int ACT>
struct RowsMode<PGlu<WT, ACT>> {
	static constexpr bool value = true;
};
template <class WT, int R>
struct RowsMode<PResidual<WT, R>> {
	static constexpr bool value = true;
};
template <class WT>
struct RowsMode<PQKV<WT>> {
	static constexpr bool value = true;
};

// One launch of gemv_rb_kernel; a consumer of an IPC exchange (tin.n > 0, always a
// normalising GEMV: QKV, W1|W3, logits) runs the TIN instantiation.
template <class WT, class P, bool NORM, int THREADS, int U, bool ROWS>
static int launch_rb_k(const P &p, const float *x, const float *normw, float eps, int nb, size_t lds, hipStream_t st,
                       const TpX &tin) {
	auto kern = gemv_rb_kernel<WT, P, U, NORM, THREADS, ROWS>;
	if constexpr (NORM) {
		if (tin.n > 0)
			kern = gemv_rb_kernel<WT, P, U, NORM, THREADS, ROWS, true>;
	} else if (tin.n > 0) {
		set_err("internal: an exchange consumer must be a normalising GEMV");
		return YALM_ERR_UNSUPPORTED;
	}
	if (lds > 65536)
		HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
	hipLaunchKernelGGL(kern, dim3(nb), dim3(THREADS), lds, st, p, x, normw, eps, tin);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

template <class WT, class P, bool NORM, int THREADS, int U>
static int launch_rb_t(const P &p, const float *x, const float *normw, float eps, int wpc, hipStream_t st,
                       const TpX &tin) {
	// an exchange consumer stages x from the exchange once per CU: one workgroup per CU
	const int nb = std::max(1, std::min(p.n_groups, device_cu_count() * (tin.n > 0 ? 1 : std::max(1, wpc))));
	const int ngl = (p.n_groups + nb - 1) / nb;
	const size_t lds = ((size_t)((p.n + 3) & ~3) + 64 + (size_t)ngl * P::R * (THREADS / YALM_WAVE)) * sizeof(float);
	if constexpr (RowsMode<P>::value) {
		// every workgroup the same number of rows and a whole number of rows, at least 2,
		// per wave (profiles/r3_gemv_rows.txt: W1|W3 fp16 39.4-40.0 -> 36.9 us, fp8 W2 13.4 ->
		// 12.7-13.0; fp16 W2 with ONE 28-KB row per wave went 20.3 -> 21.3, so it keeps the
		// chunk order); YALM_GEMV_ROWS=0 keeps the chunk order everywhere (A/B)
		const bool rows_on = !ab_env("YALM_GEMV_ROWS") || atoi(ab_env("YALM_GEMV_ROWS")) != 0;
		constexpr int W = THREADS / YALM_WAVE;
		if (rows_on && p.n_groups % nb == 0 && (ngl * P::R) % W == 0 && ngl * P::R >= 2 * W)
			return launch_rb_k<WT, P, NORM, THREADS, U, true>(p, x, normw, eps, nb, lds, st, tin);
	}
	return launch_rb_k<WT, P, NORM, THREADS, U, false>(p, x, normw, eps, nb, lds, st, tin);
}

// Per-kind, per-weight-type defaults from tools/sweep_gemv.py on MI355X
// (profiles/r1_sweep_rb*.txt): {threads, U, workgroups per CU}.
template <class WT>
static GemvCfg default_rb_cfg(int kind) {
	if constexpr (WT::BYTES == 1) { // fp8: more ALU per byte -> fewer loads in flight per lane
		switch (kind) {
		case GK_W2:
			return GemvCfg{512, 4, 1};
		case GK_GLU: // round 3, whole-row mode (14 rows per wave): 20.5 us vs 21.4-21.6 for {512, 2, 2}
			return GemvCfg{512, 4, 1};
		case GK_QKV: // round 3, whole-row mode (3 rows per wave): 7.6 us vs 8.0-8.4 for {512, 2, 2}
			return GemvCfg{512, 4, 1};
		default:
			return GemvCfg{512, 2, 2};
		}
	}
	switch (kind) {
	case GK_QKV: // one workgroup per CU: 24 rows each = 3 whole rows per wave (ROWS mode),
	             // 10.6-10.7 vs 11.2-11.4 us for {512, 2, 2} (profiles/r3_gemv_rows.txt)
		return GemvCfg{512, 4, 1};
	case GK_WO:
		return GemvCfg{1024, 2, 2};
	case GK_W2:
		return GemvCfg{1024, 2, 1};
	case GK_CLS:
		return GemvCfg{512, 4, 4};
	default:
		return GemvCfg{512, 4, 1};
	}
}

template <class WT, class P, bool NORM, int THREADS>
static int launch_rb_u(const P &p, const float *x, const float *normw, float eps, int U, int wpc, hipStream_t st,
                       const TpX &tin) {
	switch (U) {
	case 2:
		return launch_rb_t<WT, P, NORM, THREADS, 2>(p, x, normw, eps, wpc, st, tin);
	case 8:
		return launch_rb_t<WT, P, NORM, THREADS, 8>(p, x, normw, eps, wpc, st, tin);
	default:
		return launch_rb_t<WT, P, NORM, THREADS, 4>(p, x, normw, eps, wpc, st, tin);
	}
}

template <class WT, class P, bool NORM>
static int launch_rb(const P &p, const float *x, const float *normw, float eps, int kind, GemvCfg want,
                     hipStream_t st, const TpX &tin) {
	const GemvCfg def = default_rb_cfg<WT>(kind);
	const int threads = want.threads ? want.threads : def.threads;
	const int U = want.U ? want.U : def.U;
	const int wpc = want.gpw ? want.gpw : def.gpw;
	if (threads == 256)
		return launch_rb_u<WT, P, NORM, 256>(p, x, normw, eps, U, wpc, st, tin);
	if (threads == 1024)
		return launch_rb_u<WT, P, NORM, 1024>(p, x, normw, eps, U, wpc, st, tin);
	return launch_rb_u<WT, P, NORM, 512>(p, x, normw, eps, U, wpc, st, tin);
}

// tin: the exchange this launch consumes (tensor parallelism over IPC), default none
template <class WT, class P, bool NORM>
static int launch_gemv(const P &p, const float *x, const float *normw, float eps, int kind, GemvCfg want,
                       hipStream_t st, const TpX &tin = TpX{}) {
	const size_t lds = (size_t)((p.n + 3) & ~3) * sizeof(float) + 64 * sizeof(float);
	constexpr int CH = YALM_WAVE * WT::EPL;
	if (p.n % CH != 0) { // ragged K: generic kernel (tests / unusual shapes)
		if (tin.n > 0) {
			set_err("tensor parallel: dim must be a multiple of 64 x elements per 16 bytes");
			return YALM_ERR_UNSUPPORTED;
		}
		auto kern = gemv_kernel<WT, P, 4, NORM>;
		if (lds > 65536)
			HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		const int blocks = (p.n_groups + GEMV_THREADS / YALM_WAVE - 1) / (GEMV_THREADS / YALM_WAVE);
		hipLaunchKernelGGL(kern, dim3(blocks), dim3(GEMV_THREADS), lds, st, p, x, normw, eps, 1);
		HIPCHK(hipGetLastError());
		return YALM_OK;
	}
	return launch_rb<WT, P, NORM>(p, x, normw, eps, kind, want, st, tin);
}

// The decoder's weight-streaming GEMVs: gemv_rb_kernel with the geometry set
// through yalm_set_gemv_config (or the per-kind default).
template <class WT, class P, bool NORM>
static int launch_gemv_d(yalm_decoder_s *d, const P &p, const float *x, const float *normw, float eps, int kind,
                         const TpX &tin = TpX{}) {
	return launch_gemv<WT, P, NORM>(p, x, normw, eps, kind, d->gemv[kind], d->stream, tin);
}

static bool attn_supported(int head_dim, int G) {
	return (head_dim == 16 || head_dim == 32 || head_dim == 64 || head_dim == 128 || head_dim == 256) && G >= 1 &&
	       G <= 8;
}

// head mode up to this many 64-key chunks (attention.h attn_decode_body; A/B build:
// YALM_ATTN_HEADMAX). At least 1 (one chunk is key split 0 alone: the same work with a
// merger hop more), and every context with one key split (S = 1): key mode needs two.
// (A kernel-side `ns == 1 ||` cost the attention 44 VGPRs: 192 -> 236.)
static int attn_head_max(int S, int nchunks) {
	static const int h = ab_env("YALM_ATTN_HEADMAX") ? atoi(ab_env("YALM_ATTN_HEADMAX")) : ATTN_HEAD_MAX;
	return S <= 1 ? nchunks : std::max(1, h);
}

template <int D>
static void launch_attn_D(int G, const float *q, const uint16_t *kc, const uint16_t *vc, const StepState *step,
                          int n_heads, int n_kv, int max_seq_len, int nsplit, unsigned long long *part, int layer,
                          int n_layers, unsigned *err, float *att, float *out, hipStream_t st) {
	// S key-chunk splits per kv head, each workgroup looping over chunks s, s + S, ...: a grid
	// sized for max_seq_len would issue the speculative first-chunk loads of every idle
	// workgroup (15.6 MB of dead KV reads per layer at max_seq_len 4096, kv_len ~150).
	static const int splits = ab_env("YALM_ATTN_SPLITS") ? std::max(1, std::min(ATTN_MAX_SPLITS, atoi(ab_env("YALM_ATTN_SPLITS")))) : ATTN_SPLITS;
	const int nchunks = (max_seq_len + attn_chunk<D>() - 1) / attn_chunk<D>();
	const int S = std::min(nchunks, splits);
	const int grid = n_kv * (S + G - 1) + n_heads; // head + split units, then one merger per query head
	const int hmax = attn_head_max(S, nchunks);
#define YALM_ATTN(GT)                                                                                                  \
	attn_decode_kernel<D, GT><<<grid, ATTN_THREADS, 0, st>>>(q, kc, vc, step, n_heads, n_kv, max_seq_len, nsplit, S, \
	                                                         hmax, part, layer, n_layers, err, out, att)
	if (G <= 1)
		YALM_ATTN(1);
	else if (G <= 2)
		YALM_ATTN(2);
	else if (G <= 4)
		YALM_ATTN(4);
	else
		YALM_ATTN(8);
#undef YALM_ATTN
}

// partial-buffer stride: chunks per kv head (the chunk is 64 keys for every head_dim)
static int attn_nsplit(int max_seq_len) {
	return (max_seq_len + attn_chunk<128>() - 1) / attn_chunk<128>();
}

// part: (n_heads, nsplit, head_dim + 2) granules (zeroed once; tags never repeat);
// err: error word (bit 2: a merger gave up waiting).
static int launch_attn(int head_dim, int n_heads, int n_kv, const float *q, const uint16_t *kc, const uint16_t *vc,
                       const StepState *step, int max_seq_len, unsigned long long *part, int layer, int n_layers,
                       unsigned *err, float *att,
                       float *out, hipStream_t st) {
	const int G = n_heads / n_kv;
	const int nsplit = attn_nsplit(max_seq_len);
	switch (head_dim) {
	case 16:
		launch_attn_D<16>(G, q, kc, vc, step, n_heads, n_kv, max_seq_len, nsplit, part, layer, n_layers, err, att,
		                   out, st);
		break;
	case 32:
		launch_attn_D<32>(G, q, kc, vc, step, n_heads, n_kv, max_seq_len, nsplit, part, layer, n_layers, err, att,
		                   out, st);
		break;
	case 64:
		launch_attn_D<64>(G, q, kc, vc, step, n_heads, n_kv, max_seq_len, nsplit, part, layer, n_layers, err, att,
		                   out, st);
		break;
	case 128:
		launch_attn_D<128>(G, q, kc, vc, step, n_heads, n_kv, max_seq_len, nsplit, part, layer, n_layers, err, att,
		                   out, st);
		break;
	case 256:
		launch_attn_D<256>(G, q, kc, vc, step, n_heads, n_kv, max_seq_len, nsplit, part, layer, n_layers, err, att,
		                   out, st);
		break;
	default:
		set_err("unsupported head_dim");
		return YALM_ERR_UNSUPPORTED;
	}
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// ---- attention + Wo in one launch (attn_wo.h)
template <class WT, int GT, int KB>
static const void *attn_wo_fn() {
	return (const void *)attn_wo_kernel<WT, GT, KB>;
}
template <class WT, int KB>
static const void *attn_wo_fn_g(int G) {
	return G <= 1 ? attn_wo_fn<WT, 1, KB>() : G <= 2 ? attn_wo_fn<WT, 2, KB>() : G <= 4 ? attn_wo_fn<WT, 4, KB>()
	                                                                         : attn_wo_fn<WT, 8, KB>();
}
template <class WT>
static const void *attn_wo_fn_kb(int G, int KB) {
	return KB == 1 ? attn_wo_fn_g<WT, 1>(G) : KB == 2 ? attn_wo_fn_g<WT, 2>(G) : KB == 4 ? attn_wo_fn_g<WT, 4>(G)
	                                                                            : attn_wo_fn_g<WT, 8>(G);
}
static const void *attn_wo_pick(int dtype, int G, int KB) {
	return dtype == YALM_F16 ? attn_wo_fn_kb<WF16>(G, KB) : attn_wo_fn_kb<WF8>(G, KB);
}
// The fused launch's plan for a (per-rank) config: 1 with the key splits S and the grid,
// or 0 = separate attention and Wo launches. Fused needs head_dim 128, G <= 8, fp16 / fp8
// Wo rows of 1, 2, 4 or 8 KiB (one GPU: 4 / 8; a tensor-parallel rank's Wo slice: 1 / 2 too),
// and the whole grid (attention, one merger per query head, Wo)
// within the co-resident workgroup slots: a workgroup past them is dispatched only when
// an earlier one exits, and at short contexts every attention workgroup without keys
// still holds its slot for the kv_len load (S 32 at Mistral: 256 + 32 + 256 = 544 > 512
// slots put the last 32 Wo slices ~2 us late, fused launch 8.9 -> 11.2 us at kv 17). When
// fewer than 2 key splits fit (dim 8192 has 512 Wo workgroups) the fused launch
// would run every context in head mode -- one workgroup per query head over all the
// chunks -- so the separate launches (standalone attention at ATTN_SPLITS) are kept.
// Pure host arithmetic (tests/test_abi.py calls it without a GPU).
extern "C" int yalm_attn_wo_plan(const yalm_config *cp, int slots, int *splits, int *grid) {
	if (!cp || slots <= 0)
		return 0;
	const yalm_config &c = *cp;
	if (c.head_dim != 128 || c.n_kv_heads <= 0 || c.n_heads % c.n_kv_heads)
		return 0;
	const int G = c.n_heads / c.n_kv_heads;
	if (G < 1 || G > 8 || (c.weight_dtype != YALM_F16 && c.weight_dtype != YALM_F8E5M2))
		return 0;
	const int rb = c.n_heads * c.head_dim * (c.weight_dtype == YALM_F16 ? 2 : 1);
	if ((rb != 1024 && rb != 2048 && rb != 4096 && rb != 8192) || c.dim < AWO_RPW)
		return 0;
	const int nchunks = (c.max_seq_len + attn_chunk<128>() - 1) / attn_chunk<128>();
	const int n_wo = (c.dim + AWO_RPW - 1) / AWO_RPW;
	const int fit = (slots - c.n_heads - n_wo) / c.n_kv_heads - (G - 1); // key splits: S + G - 1 units per kv head
	const char *senv = ab_env("YALM_AWO_SPLITS");
	const int S = std::max(1, std::min(nchunks, senv ? std::max(1, std::min(ATTN_MAX_SPLITS, atoi(senv)))
	                                                 : std::min(ATTN_SPLITS, fit)));
	if (!senv && fit < 2 && nchunks > ATTN_HEAD_MAX)
		return 0;
	if (splits)
		*splits = S;
	if (grid)
		*grid = c.n_kv_heads * (S + G - 1) + c.n_heads + n_wo;
	return 1;
}

// Decoders whose plan (yalm_attn_wo_plan, on the per-rank config) fuses: one GPU, and
// (round 5) every tensor-parallel rank too -- the Wo workgroups then write the rank's
// partial for the all-reduce (RCCL) or push it to the exchange (IPC, tp_exchange.h).
static int attn_wo_init(yalm_decoder_s *d) {
	const yalm_config &c = d->c;
	if (c.head_dim != 128)
		return YALM_OK;
	const int G = c.n_heads / c.n_kv_heads;
	const int rb = c.n_heads * c.head_dim * (c.weight_dtype == YALM_F16 ? 2 : 1);
	if (!yalm_attn_wo_plan(&c, 1 << 30, nullptr, nullptr))
		return YALM_OK;
	int occ = 0; // the Wo workgroups spin, but only on attention workgroups dispatched before them
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, attn_wo_pick(c.weight_dtype, G, rb / 1024), ATTN_THREADS,
	                                                 0) != hipSuccess ||
	    occ < 1)
		return YALM_OK;
	if (!yalm_attn_wo_plan(&c, occ * device_cu_count(), &d->awo_S, &d->awo_nb))
		return YALM_OK;
	d->awo_slots = occ * device_cu_count();
	// per layer: the attention output as {value, epoch} granules (zero tags never match:
	// the epoch is >= 1 from the first forward / yalm_block on)
	const size_t gran = (size_t)c.n_layers * c.n_heads * c.head_dim;
	TRY(dalloc(d, (void **)&d->awo_gran, sizeof(unsigned long long) * gran));
	const char *denv = ab_env("YALM_ATTN_WO_DELAY");
	// default 0.2 us (fp16) / 0.5 us (fp8): the attention workgroups' K/V loads reach HBM
	// ahead of the Wo stream. fp16 (33.5 MB, slice lands ~5.4 us, after the heads):
	// profiles/r2_sweep_awo_delay.txt 10.6 -> 10.1 us at kv_len 17. fp8 (16.8 MB, slice lands
	// ~3.1 us, before the heads): 0.5 us gives 9.4 -> 8.4 us at kv 17, 11.3 -> 10.3 at kv 151,
	// 579 -> 586 tok/s (profiles/r3_ab_awo_delay.txt); fp16 at 0.5 us is within noise
	d->awo_delay = denv ? std::max(0, atoi(denv)) : (c.weight_dtype == YALM_F8E5M2 ? 50 : 20);
	d->awo_delay_short = denv ? -1 : (c.weight_dtype == YALM_F8E5M2 ? 0 : -1);
	// Removed in round 4 (measured losers, round 3, profiles/r3_ab_awo*.txt): the combined
	// first gather attempt (YALM_AWO_SPEC), per-XCD copies of the head outputs
	// (YALM_AWO_REPL) and a sliding window on the Wo slice loads (YALM_ATTN_WO_WIN)
	const char *tenv = ab_env("YALM_ATTN_WO_TRACE");
	if (tenv && atoi(tenv) != 0)
		TRY(dalloc(d, (void **)&d->awo_trace, sizeof(unsigned long long) * AWO_TRACE_N * d->awo_nb));
	d->attn_wo = d->attn_wo_ok = true;
	return YALM_OK;
}

// After a sync: report (once) a bounded spin that gave up -- the fused attention + Wo
// launch waiting for its heads, or an IPC exchange waiting for a peer.
int awo_check(yalm_decoder_s *d) {
	if (d->awo_err) {
		unsigned e = 0;
		HIPCHK(hipMemcpy(&e, d->awo_err, sizeof(e), hipMemcpyDeviceToHost));
		if (e) { // cleared so that later calls report only their own failures
			HIPCHK(hipMemset(d->awo_err, 0, sizeof(e)));
			// bit 1: a Wo workgroup of the fused launch gave up waiting for its head granules;
			// bit 2: a split-KV merger (fused or standalone attention) gave up waiting for a chunk
			std::string m = "bounded in-launch wait gave up (results invalid):";
			if (e & 1u)
				m += " the fused attention + Wo launch's Wo gather timed out waiting for the attention heads"
				     " (yalm_decoder_set_launch YALM_LAUNCH_SEPARATE_ATTN_WO selects separate launches);";
			if (e & 2u)
				m += " the split-KV attention merger timed out waiting for a key-chunk partial;";
			if (e & ~3u)
				m += " unknown error bits " + std::to_string(e & ~3u) + ";";
			set_err(m);
			return YALM_ERR_HIP;
		}
	}
	if (d->ipc) { // tp_exchange.h: a consumer's bounded wait for a peer's exchange gave up
		unsigned *flag = (unsigned *)((unsigned long long *)d->ipc_own + 2 * (size_t)d->tp_size * d->ipc_S); // TpX::err
		unsigned e = 0;
		HIPCHK(hipMemcpy(&e, flag, sizeof(e), hipMemcpyDeviceToHost));
		if (e) {
			HIPCHK(hipMemset(flag, 0, sizeof(e)));
			set_err("tensor-parallel IPC exchange gave up waiting for a peer rank (results invalid)");
			return YALM_ERR_HIP;
		}
	}
	return YALM_OK;
}

// The exchange descriptor of a launch taking part in exchange `ex` of the current launch
// sequence (tp_exchange.h: g = StepState.xbase + ex).
static TpX tpx_ex(const yalm_decoder_s *d, int ex) {
	TpX t = d->tpx;
	t.ex = ex;
	return t;
}

template <class WT, int GT, int KB>
static void launch_attn_wo_k(yalm_decoder_s *d, const yalm_block_weights &w, const AttnWoArgs &p) {
	attn_wo_kernel<WT, GT, KB><<<d->awo_nb, ATTN_THREADS, 0, d->stream>>>(d->q, w.key_cache, w.value_cache, d->step, p);
}
template <class WT, int KB>
static void launch_attn_wo_g(yalm_decoder_s *d, const yalm_block_weights &w, const AttnWoArgs &p, int G) {
	if (G <= 1)
		launch_attn_wo_k<WT, 1, KB>(d, w, p);
	else if (G <= 2)
		launch_attn_wo_k<WT, 2, KB>(d, w, p);
	else if (G <= 4)
		launch_attn_wo_k<WT, 4, KB>(d, w, p);
	else
		launch_attn_wo_k<WT, 8, KB>(d, w, p);
}
// The fused attention + Wo launch of one layer. One GPU: x += Wo attn(q). Tensor parallel:
// the rank's partial (+ x on rank 0) -- into xs, then the RCCL all-reduce into x; or pushed
// to the IPC exchange `ex` (consumed by the GLU GEMV's x staging, tp_exchange.h).
template <class WT>
static int launch_attn_wo(yalm_decoder_s *d, const yalm_block_weights &w, int layer, int ex) {
	const yalm_config &c = d->c;
	AttnWoArgs p;
	p.n_heads = c.n_heads;
	p.n_kv = c.n_kv_heads;
	p.max_seq_len = c.max_seq_len;
	p.nsplit = attn_nsplit(c.max_seq_len);
	p.S = d->awo_S;
	p.head_max = attn_head_max(d->awo_S, (c.max_seq_len + attn_chunk<128>() - 1) / attn_chunk<128>());
	p.q_dim = c.n_heads * c.head_dim;
	p.dim = c.dim;
	p.part = d->part;
	p.layer = layer;
	p.n_layers = c.n_layers;
	p.gran = d->awo_gran + (size_t)layer * p.q_dim;
	p.wo = (const char *)w.wo;
	p.x = d->x;
	p.out = d->comm ? d->xs : d->x;
	p.add_base = d->tp_rank == 0;
	p.push = d->ipc ? tpx_ex(d, ex) : TpX{};
	p.err = d->awo_err;
	p.trace = d->awo_trace;
	p.delay = d->awo_delay_short >= 0 && d->awo_kv_hint >= 0 && d->awo_kv_hint <= AWO_SHORT_KV ? d->awo_delay_short
	                                                                                         : d->awo_delay;
	const int G = c.n_heads / c.n_kv_heads;
	if constexpr (WT::BYTES == 2 || WT::BYTES == 1) {
		switch (p.q_dim * WT::BYTES) {
		case 1024:
			launch_attn_wo_g<WT, 1>(d, w, p, G);
			break;
		case 2048:
			launch_attn_wo_g<WT, 2>(d, w, p, G);
			break;
		case 4096:
			launch_attn_wo_g<WT, 4>(d, w, p, G);
			break;
		default:
			launch_attn_wo_g<WT, 8>(d, w, p, G);
		}
	}
	HIPCHK(hipGetLastError());
	if (d->comm && ncclAllReduce(d->xs, d->x, c.dim, ncclFloat, ncclSum, (ncclComm_t)d->comm, d->stream) != ncclSuccess) {
		set_err("ncclAllReduce failed");
		return YALM_ERR_HIP;
	}
	return YALM_OK;
}

// One tensor-parallel exchange of x alone, as launches of their own: timing hook for the
// communication cost (yalm_time_kernel id 6). RCCL: one all-reduce. IPC: x pushed to every
// rank, then the consumer side (wait for every rank + sum) -- in the forward the push is the
// producer GEMV's epilogue and the sum runs inside the next GEMV's x staging.
static int enqueue_exchange(yalm_decoder_s *d) {
	if (d->ipc) {
		tpx_push_kernel<<<1, 1024, 0, d->stream>>>(tpx_ex(d, 0), d->c.dim, d->x);
		tpx_collect_kernel<<<TPX_COLLECT_WG, 256, 0, d->stream>>>(tpx_ex(d, 0), d->c.dim, 0, d->xs);
		HIPCHK(hipGetLastError());
		return YALM_OK;
	}
	if (!d->comm) {
		set_err("kernel 6 (tensor-parallel exchange) needs a tensor-parallel decoder");
		return YALM_ERR_ARG;
	}
	if (ncclAllReduce(d->x, d->xs, d->c.dim, ncclFloat, ncclSum, (ncclComm_t)d->comm, d->stream) != ncclSuccess) {
		set_err("ncclAllReduce failed");
		return YALM_ERR_HIP;
	}
	return YALM_OK;
}

// x += W v (fused_matmul_add_residuals). Under tensor parallelism W holds this
// rank's input columns: rank 0's partial carries x. RCCL: rank 0 writes xs = x + W v, the
// others xs = W v, and one all-reduce (sum, captured in the graph) lands the sum in x on
// every rank (identical bits). IPC: the partial is pushed to every rank's exchange slot
// (PPush, exchange `ex`, tp_exchange.h); the next GEMV sums the slots while its weights
// stream in. ex < 0 under IPC: a result nothing reads (the last W2 of a hydration forward)
// stays local -- an exchange nobody consumes would break the slot-reuse order.
template <class WT>
static int enqueue_residual_gemv(yalm_decoder_s *d, const void *W, int n, const float *v, int kind, int ex) {
	const yalm_config &c = d->c;
	hipStream_t st = d->stream;
	if (d->ipc && ex >= 0) {
		PPush<WT, 1> p;
		p.W = (const char *)W;
		p.n = n;
		p.base = d->tp_rank == 0 ? d->x : nullptr;
		p.t = tpx_ex(d, ex);
		p.offset = 0;
		p.n_groups = c.dim;
		return launch_gemv<WT, PPush<WT, 1>, false>(p, v, nullptr, 0.f, kind, d->gemv[kind], st);
	}
	if (!d->comm) { // one GPU (or the unread IPC case above)
		PResidual<WT, 1> p;
		p.W = (const char *)W;
		p.n = n;
		p.out = d->x;
		p.n_groups = c.dim;
		return launch_gemv_d<WT, PResidual<WT, 1>, false>(d, p, v, nullptr, 0.f, kind);
	}
	if (d->tp_rank == 0) {
		PAddTo<WT, 1> p;
		p.W = (const char *)W;
		p.n = n;
		p.out = d->xs;
		p.base = d->x;
		p.n_groups = c.dim;
		TRY((launch_gemv<WT, PAddTo<WT, 1>, false>(p, v, nullptr, 0.f, kind, d->gemv[kind], st)));
	} else {
		PStore<WT, 1> p;
		p.W = (const char *)W;
		p.n = n;
		p.out = d->xs;
		p.n_groups = c.dim;
		TRY((launch_gemv<WT, PStore<WT, 1>, false>(p, v, nullptr, 0.f, kind, d->gemv[kind], st)));
	}
	if (ncclAllReduce(d->xs, d->x, c.dim, ncclFloat, ncclSum, (ncclComm_t)d->comm, st) != ncclSuccess) {
		set_err("ncclAllReduce failed");
		return YALM_ERR_HIP;
	}
	return YALM_OK;
}

// The exchange descriptor for a consumer launch (tp_exchange.h). Up to TPX_STAGE_MAX_RANKS
// ranks every consumer workgroup sums the ranks' granules itself; past that a collect launch
// sums x once and the consumer stages it as on one GPU (the collect form). When this rank
// shares its GPU with a peer (tests: several rank processes on one device), a 1-wave gate
// launch waits for the exchange first: a consumer whose 256 workgroups spin could otherwise
// hold every CU a peer's producer needs (a deadlock the bounded wait only reports). One GPU
// per rank (the real configuration) needs no gate: the consumer waits inside its own launch.
static TpX tpx_consume(yalm_decoder_s *d, int ex, int n) {
	if (d->tpx_collect) { // many ranks: x summed once by a collect launch, the consumer stages it as on one GPU
		tpx_collect_kernel<<<TPX_COLLECT_WG, 256, 0, d->stream>>>(tpx_ex(d, ex), n, 0, d->x);
		return TpX{};
	}
	if (d->tpx_gate)
		tpx_gate_kernel<<<1, 64, 0, d->stream>>>(tpx_ex(d, ex), n);
	return tpx_ex(d, ex);
}

// One layer. IPC tensor parallelism (tp_exchange.h): the Wo partial is exchange ex0 (the GLU
// consumes it), the W2 partial exchange ex0 + 1 (push_w2; the next QKV or the logits GEMV
// consumes it); x_exchanged: the layer's input x is exchange ex0 - 1 (the QKV GEMV consumes
// it), not a local x (the embedding of layer 0, or the x yalm_block / yalm_set_x left).
template <class WT>
static int enqueue_layer_t(yalm_decoder_s *d, int l, int ex0, bool x_exchanged, bool push_w2) {
	const yalm_config &c = d->c;
	const yalm_block_weights &w = d->b[l];
	hipStream_t st = d->stream;
	const int q_dim = c.n_heads * c.head_dim, kv_dim = c.n_kv_heads * c.head_dim;
	const TpX none{};
	{
		PQKV<WT> p;
		p.wq = (const char *)w.wq;
		p.wk = (const char *)w.wk;
		p.wv = (const char *)w.wv;
		p.n = c.dim;
		p.q_dim = q_dim;
		p.kv_dim = kv_dim;
		p.head_dim = c.head_dim;
		p.n_groups = (q_dim + 2 * kv_dim) / 2;
		p.qkv_clip = c.qkv_clip;
		p.inv_freq = d->inv_freq;
		p.step = d->step;
		p.q_out = d->q;
		p.kcache = w.key_cache;
		p.vcache = w.value_cache;
		TRY((launch_gemv_d<WT, PQKV<WT>, true>(d, p, d->x, w.rms_att, c.norm_eps, GK_QKV,
		                                         d->ipc && x_exchanged ? tpx_consume(d, ex0 - 1, c.dim) : none)));
	}
	if (d->attn_wo && WT::BYTES <= 2) {
		TRY(launch_attn_wo<WT>(d, w, l, ex0));
	} else {
		TRY(launch_attn(c.head_dim, c.n_heads, c.n_kv_heads, d->q, w.key_cache, w.value_cache, d->step, c.max_seq_len,
		                d->part, l, c.n_layers, d->awo_err, nullptr, d->xb2, st));
		TRY(enqueue_residual_gemv<WT>(d, w.wo, q_dim, d->xb2, GK_WO, ex0));
	}
	// the GLU consumes the Wo exchange under IPC tensor parallelism
	if (c.act == YALM_SILU) {
		PGlu<WT, 1> p;
		p.w1 = (const char *)w.w1;
		p.w3 = (const char *)w.w3;
		p.n = c.dim;
		p.out = d->hb;
		p.n_groups = c.hidden_dim;
		TRY((launch_gemv_d<WT, PGlu<WT, 1>, true>(d, p, d->x, w.rms_ffn, c.norm_eps, GK_GLU, d->ipc ? tpx_consume(d, ex0, c.dim) : none)));
	} else {
		PGlu<WT, 0> p;
		p.w1 = (const char *)w.w1;
		p.w3 = (const char *)w.w3;
		p.n = c.dim;
		p.out = d->hb;
		p.n_groups = c.hidden_dim;
		TRY((launch_gemv_d<WT, PGlu<WT, 0>, true>(d, p, d->x, w.rms_ffn, c.norm_eps, GK_GLU, d->ipc ? tpx_consume(d, ex0, c.dim) : none)));
	}
	return enqueue_residual_gemv<WT>(d, w.w2, c.hidden_dim, d->hb, GK_W2, push_w2 ? ex0 + 1 : -1);
}

// Final norm + classifier rows of this rank. IPC tensor parallelism: consume_ex >= 0 = the
// GEMV consumes that exchange (the last layer's W2); push_ex >= 0 (OUTPUT_LOGITS) = it also
// produces that exchange, the logits gather: this rank's vocabulary rows pushed to every rank.
template <class WT>
static int enqueue_logits_t(yalm_decoder_s *d, int consume_ex, int push_ex) {
	const yalm_config &c = d->c;
	const TpX tin = consume_ex >= 0 ? tpx_consume(d, consume_ex, c.dim) : TpX{};
	if (push_ex >= 0) {
		PPush<WT, 1> p;
		p.W = (const char *)d->wcls;
		p.n = c.dim;
		p.base = nullptr;
		p.t = tpx_ex(d, push_ex);
		p.offset = 0;
		p.n_groups = c.vocab_size;
		return launch_gemv<WT, PPush<WT, 1>, true>(p, d->x, d->rms_final, c.norm_eps, GK_CLS, d->gemv[GK_CLS],
		                                           d->stream, tin);
	}
	if (c.vocab_size % 2 == 0) {
		PStore<WT, 2> p;
		p.W = (const char *)d->wcls;
		p.n = c.dim;
		p.out = d->logits_local;
		p.n_groups = c.vocab_size / 2;
		return launch_gemv_d<WT, PStore<WT, 2>, true>(d, p, d->x, d->rms_final, c.norm_eps, GK_CLS, tin);
	}
	PStore<WT, 1> p;
	p.W = (const char *)d->wcls;
	p.n = c.dim;
	p.out = d->logits_local;
	p.n_groups = c.vocab_size;
	return launch_gemv_d<WT, PStore<WT, 1>, true>(d, p, d->x, d->rms_final, c.norm_eps, GK_CLS, tin);
}

template <class WT>
static int enqueue_begin_t(yalm_decoder_s *d, int n_ex) {
	step_begin_kernel<WT><<<1, 256, 0, d->stream>>>(d->step, d->emb, d->c.dim, d->x, d->c.max_seq_len, n_ex,
	                                                 d->inv_freq, d->c.head_dim / 2);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

#define DISPATCH_WT(dtype, FN, ...)                                                                                    \
	((dtype) == YALM_F32   ? FN<WF32>(__VA_ARGS__)                                                                     \
	 : (dtype) == YALM_F16 ? FN<WF16>(__VA_ARGS__)                                                                     \
	                       : FN<WF8>(__VA_ARGS__))

// IPC tensor parallelism (tp_exchange.h): layer l's Wo and W2 partials are exchanges 2 l and
// 2 l + 1, the logits gather / argmax pairs exchange 2 L. Every exchange of the sequence is
// consumed (the slot-reuse order relies on it), so a hydration forward keeps its last W2
// local: 2 L - 1 exchanges, 2 L + 1 with an output.
static int enqueue_forward(yalm_decoder_s *d, int which) {
	const int L = d->c.n_layers;
	const bool hyd = which == GRAPH_HYDRATE;
	TRY(DISPATCH_WT(d->c.weight_dtype, enqueue_begin_t, d, d->ipc ? (hyd ? 2 * L - 1 : 2 * L + 1) : 0));
	for (int l = 0; l < L; ++l)
		TRY(DISPATCH_WT(d->c.weight_dtype, enqueue_layer_t, d, l, 2 * l, l > 0, !(hyd && l == L - 1)));
	if (hyd)
		return YALM_OK;
	TRY(DISPATCH_WT(d->c.weight_dtype, enqueue_logits_t, d, d->ipc ? 2 * L - 1 : -1,
	                d->ipc && which == GRAPH_LOGITS ? 2 * L : -1));
	if (d->ipc) { // tp_exchange.h: no exchange launches
		if (which == GRAPH_LOGITS) { // every rank's vocabulary slice, side by side
			tpx_collect_kernel<<<TPX_COLLECT_WG, 256, 0, d->stream>>>(tpx_ex(d, 2 * L), d->c.vocab_size, 1, d->logits);
			HIPCHK(hipGetLastError());
			HIPCHK(hipMemcpyAsync(d->logits_pinned, d->logits, sizeof(float) * d->vocab_full, hipMemcpyDeviceToHost,
			                      d->stream));
		} else { // local first max, pushed; every rank's pair gathered and picked in the same launch
			argmax_tp_kernel<<<1, 1024, 0, d->stream>>>(d->logits_local, d->c.vocab_size, d->step, d->tokens,
			                                            d->tokens_cap, tpx_ex(d, 2 * L));
			HIPCHK(hipGetLastError());
		}
		return YALM_OK;
	}
	if (which == GRAPH_LOGITS) {
		if (d->comm && ncclAllGather(d->logits_local, d->logits, d->c.vocab_size, ncclFloat, (ncclComm_t)d->comm,
		                             d->stream) != ncclSuccess) {
			set_err("ncclAllGather (logits) failed");
			return YALM_ERR_HIP;
		}
		HIPCHK(hipMemcpyAsync(d->logits_pinned, d->logits, sizeof(float) * d->vocab_full, hipMemcpyDeviceToHost,
		                      d->stream));
	} else if (!d->comm) {
		argmax_kernel<<<1, 1024, 0, d->stream>>>(d->logits, d->c.vocab_size, d->step, d->tokens, d->tokens_cap);
		HIPCHK(hipGetLastError());
	} else { // sharded vocabulary: local first-max, gather (value, index) pairs, pick (identical on all ranks)
		argmax_kernel<<<1, 1024, 0, d->stream>>>(d->logits_local, d->c.vocab_size, d->step, d->tokens,
		                                         d->tokens_cap, d->amax, d->tp_rank * d->c.vocab_size);
		HIPCHK(hipGetLastError());
		if (ncclAllGather(d->amax, d->amax_all, 2, ncclFloat, (ncclComm_t)d->comm, d->stream) != ncclSuccess) {
			set_err("ncclAllGather (argmax) failed");
			return YALM_ERR_HIP;
		}
		argmax_pick_kernel<<<1, 1, 0, d->stream>>>(d->amax_all, d->tp_size, d->step, d->tokens, d->tokens_cap);
		HIPCHK(hipGetLastError());
	}
	return YALM_OK;
}

static int ensure_graph(yalm_decoder_s *d, int which) {
	if (d->exec[which] || d->eager)
		return YALM_OK;
	HIPCHK(hipStreamBeginCapture(d->stream, hipStreamCaptureModeRelaxed));
	int r = enqueue_forward(d, which);
	hipGraph_t g = nullptr;
	hipError_t e = hipStreamEndCapture(d->stream, &g);
	if (r != YALM_OK)
		return r;
	HIPCHK(e);
	d->graph[which] = g;
	HIPCHK(hipGraphInstantiate(&d->exec[which], g, nullptr, nullptr, 0));
	return YALM_OK;
}

static void drop_graphs(yalm_decoder_s *d) {
	for (int i = 0; i < N_GRAPHS; ++i) {
		if (d->exec[i])
			(void)hipGraphExecDestroy(d->exec[i]);
		if (d->graph[i])
			(void)hipGraphDestroy(d->graph[i]);
		d->exec[i] = nullptr;
		d->graph[i] = nullptr;
	}
}

static int validate_config(const yalm_config *c) {
	ARGCHK(c->dim > 0 && c->hidden_dim > 0 && c->n_layers > 0 && c->n_heads > 0 && c->n_kv_heads > 0 &&
	           c->vocab_size > 0 && c->max_seq_len > 2,
	       "config: non-positive dimension");
	ARGCHK(c->n_heads % c->n_kv_heads == 0, "config: n_heads % n_kv_heads != 0");
	ARGCHK(c->weight_dtype == YALM_F32 || c->weight_dtype == YALM_F16 || c->weight_dtype == YALM_F8E5M2,
	       "config: weight_dtype must be F32, F16 or F8E5M2");
	ARGCHK(c->dim % 16 == 0 && c->hidden_dim % 16 == 0 && (c->n_heads * c->head_dim) % 16 == 0,
	       "config: dim, hidden_dim and n_heads*head_dim must be multiples of 16 (infer.cpp:66)");
	ARGCHK(c->rotary_dim <= c->head_dim && c->rotary_dim % 2 == 0, "config: bad rotary_dim");
	if (!attn_supported(c->head_dim, c->n_heads / c->n_kv_heads)) {
		set_err("config: attention kernel needs head_dim in {16,32,64,128,256} and n_heads/n_kv_heads <= 8");
		return YALM_ERR_UNSUPPORTED;
	}
	return YALM_OK;
}

static void destroy_decoder(yalm_decoder_s *d) {
	drop_graphs(d);
	if (d->comm)
		(void)ncclCommDestroy((ncclComm_t)d->comm);
	for (void *p : d->ipc_opened)
		(void)hipIpcCloseMemHandle(p);
	if (d->ipc_own)
		(void)hipFree(d->ipc_own);
	for (void *p : d->dev_allocs)
		(void)hipFree(p);
	if (d->logits_pinned)
		(void)hipHostFree(d->logits_pinned);
	if (d->own_stream && d->stream)
		(void)hipStreamDestroy(d->stream);
	delete d;
}

int dalloc(yalm_decoder_s *d, void **p, size_t bytes) {
	HIPCHK(hipMalloc(p, bytes ? bytes : 4));
	d->dev_allocs.push_back(*p);
	HIPCHK(hipMemset(*p, 0, bytes ? bytes : 4));
	return YALM_OK;
}

// One forward of graph `which`: a graph replay, or the same kernels launched
// eagerly when d->eager.
static int replay(yalm_decoder_s *d, int which) {
	if (d->eager || (which == GRAPH_GREEDY && d->greedy_eager))
		return enqueue_forward(d, which);
	HIPCHK(hipGraphLaunch(d->exec[which], d->stream));
	if (d->graph_sync)
		HIPCHK(hipStreamSynchronize(d->stream));
	return YALM_OK;
}

// comm: an initialised ncclComm_t (tensor parallelism) or null. config holds
// the local (per-rank) dims; vocab_full the unsharded vocabulary.
static int create_decoder(const yalm_config *config, const yalm_model_weights *weights, yalm_stream s,
                          yalm_decoder *out, void *comm, int tp_rank, int tp_size, int vocab_full) {
	ARGCHK(config && weights && out && weights->blocks, "yalm_decoder_create: null argument");
	TRY(validate_config(config));
	yalm_decoder_s *d = new yalm_decoder_s();
	d->c = *config;
	d->comm = comm;
	d->tp_rank = tp_rank;
	d->tp_size = tp_size;
	d->vocab_full = vocab_full;
	d->emb = weights->token_embedding;
	d->rms_final = weights->rms_final;
	d->wcls = weights->wcls;
	d->b.assign(weights->blocks, weights->blocks + config->n_layers);
	int r = YALM_OK;
	auto fail = [&](int code) {
		destroy_decoder(d);
		return code;
	};
	if (s) {
		d->stream = reinterpret_cast<hipStream_t>(s);
	} else {
		if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) {
			set_err("hipStreamCreate failed");
			return fail(YALM_ERR_HIP);
		}
		d->own_stream = true;
	}
	const yalm_config &c = d->c;
	const int q_dim = c.n_heads * c.head_dim, kv_dim = c.n_kv_heads * c.head_dim;
	const int nsplit = attn_nsplit(c.max_seq_len);
	d->tokens_cap = 1 << 16;
	d->pf_forms = pf_forms_default();
	{
		const char *g = ab_env("YALM_GREEDY_GRAPH");
		d->greedy_eager = !(g && atoi(g) != 0);
	}
	// geometry overrides for A/B runs without a rebuild (same meaning as yalm_set_gemv_config):
	// YALM_GEMV_CFG="kind:threads:unroll:gpw[,kind:threads:unroll:gpw...]", kind 0..4
	if (const char *g = ab_env("YALM_GEMV_CFG")) {
		int k, t, u, w, n = 0;
		for (const char *p = g; sscanf(p, "%d:%d:%d:%d%n", &k, &t, &u, &w, &n) == 4; p += n + (p[n] == ',')) {
			if (k >= 0 && k < GK_N && (t == 0 || t == 256 || t == 512 || t == 1024) &&
			    (u == 0 || u == 2 || u == 4 || u == 8) && w >= 0)
				d->gemv[k] = GemvCfg{t, u, w};
			if (!p[n])
				break;
		}
	}
	if ((r = dalloc(d, (void **)&d->step, sizeof(StepState))) || (r = dalloc(d, (void **)&d->x, sizeof(float) * c.dim)) ||
	    (r = dalloc(d, (void **)&d->q, sizeof(float) * q_dim)) ||
	    (r = dalloc(d, (void **)&d->xb2, sizeof(float) * q_dim)) ||
	    (r = dalloc(d, (void **)&d->hb, sizeof(float) * c.hidden_dim)) ||
	    (r = dalloc(d, (void **)&d->part, sizeof(unsigned long long) * (size_t)c.n_heads * nsplit * (c.head_dim + 2))) ||
	    (r = dalloc(d, (void **)&d->awo_err, sizeof(unsigned) * AWO_REPL_STRIDE)) ||
	    (r = dalloc(d, (void **)&d->logits, sizeof(float) * vocab_full)) ||
	    (r = dalloc(d, (void **)&d->xs, sizeof(float) * c.dim)) ||
	    (r = dalloc(d, (void **)&d->amax, sizeof(float) * 2)) ||
	    (r = dalloc(d, (void **)&d->amax_all, sizeof(float) * 2 * tp_size)) ||
	    (r = dalloc(d, (void **)&d->inv_freq, sizeof(float) * c.head_dim / 2)) ||
	    (r = dalloc(d, (void **)&d->tokens, sizeof(int) * d->tokens_cap)))
		return fail(r);
	// RoPE frequencies on the host, bit for bit as the reference's compiled rope computes
	// them. infer.cpp:203 reads 1/powf(theta, j/rotary_dim), but under its -ffast-math
	// (Makefile:36-39) gcc emits r = 1.0f / rotary_dim; powf(theta, -(j * r)) (one scalar
	// glibc powf call; the division folded into the exponent): a freq one ulp away moves
	// the angle pos * freq by pos ulps, 2e-4 rad at pos 4095 -- tests/test_gpu_ref_glue.py
	// measured 60 f16 ulps on a K row against the reference's own rope before this form.
	std::vector<float> inv(c.head_dim / 2);
	const float rinv = 1.0f / (float)c.rotary_dim;
	for (int j = 0; j < c.head_dim; j += 2)
		inv[j / 2] = j >= c.rotary_dim ? 0.f : powf(c.rope_theta, -((float)j * rinv));
	if (hipMemcpy(d->inv_freq, inv.data(), sizeof(float) * inv.size(), hipMemcpyHostToDevice) != hipSuccess) {
		set_err("inv_freq upload failed");
		return fail(YALM_ERR_HIP);
	}
	for (auto &bw : d->b) {
		const size_t kvb = sizeof(uint16_t) * (size_t)c.max_seq_len * kv_dim;
		if (!bw.key_cache && (r = dalloc(d, (void **)&bw.key_cache, kvb)))
			return fail(r);
		if (!bw.value_cache && (r = dalloc(d, (void **)&bw.value_cache, kvb)))
			return fail(r);
	}
	d->logits_local = d->logits;
	if (tp_size > 1 && (r = dalloc(d, (void **)&d->logits_local, sizeof(float) * c.vocab_size)))
		return fail(r);
	if (hipHostMalloc((void **)&d->logits_pinned, sizeof(float) * vocab_full, hipHostMallocDefault) != hipSuccess) {
		set_err("hipHostMalloc failed");
		return fail(YALM_ERR_HIP);
	}
	if ((r = attn_wo_init(d)))
		return fail(r);
	if (hipDeviceSynchronize() != hipSuccess) {
		set_err("hipDeviceSynchronize failed after decoder allocation");
		return fail(YALM_ERR_HIP);
	}
	*out = d;
	return YALM_OK;
}

extern "C" int yalm_decoder_create(const yalm_config *config, const yalm_model_weights *weights, yalm_stream s,
                                   yalm_decoder *out) {
	ARGCHK(config, "yalm_decoder_create: null config");
	return create_decoder(config, weights, s, out, nullptr, 0, 1, config->vocab_size);
}

// ------------------------------------------------------------------ tensor parallelism
static int tp_local_config(const yalm_config &f, int tp_size, yalm_config &lc) {
	ARGCHK(f.n_kv_heads % tp_size == 0 && f.n_heads % tp_size == 0 && f.hidden_dim % tp_size == 0 &&
	           f.vocab_size % tp_size == 0,
	       "tensor parallel: n_heads, n_kv_heads, hidden_dim and vocab_size must divide by tp_size");
	lc = f;
	lc.n_heads = f.n_heads / tp_size;
	lc.n_kv_heads = f.n_kv_heads / tp_size;
	lc.hidden_dim = f.hidden_dim / tp_size;
	lc.vocab_size = f.vocab_size / tp_size;
	return YALM_OK;
}

// {value, tag} granules per (parity, source rank) slot of the IPC exchange: x, or a rank's
// vocabulary rows (tp_exchange.h)
static int ipc_slot_floats(const yalm_config &f, int tp_size) {
	const int need = std::max(f.dim, f.vocab_size / tp_size + 2);
	return (need + 63) / 64 * 64;
}
static size_t ipc_buf_bytes(const yalm_config &f, int tp_size) {
	return 2 * (size_t)tp_size * ipc_slot_floats(f, tp_size) * sizeof(unsigned long long) + TPX_CTRL_WORDS * sizeof(float);
}

extern "C" int yalm_tp_unique_id(void *id_out) {
	ARGCHK(id_out, "null id");
	ncclUniqueId id;
	if (ncclGetUniqueId(&id) != ncclSuccess) {
		set_err("ncclGetUniqueId failed");
		return YALM_ERR_HIP;
	}
	memcpy(id_out, &id, sizeof(id));
	return YALM_OK;
}

extern "C" int yalm_decoder_create_tp(const yalm_config *config, const yalm_model_weights *weights, int tp_rank,
                                      int tp_size, const void *unique_id, yalm_stream s, yalm_decoder *out) {
	ARGCHK(config && weights && unique_id && out, "yalm_decoder_create_tp: null argument");
	ARGCHK(tp_size >= 1 && tp_rank >= 0 && tp_rank < tp_size, "yalm_decoder_create_tp: bad rank / size");
	const yalm_config &f = *config;
	yalm_config lc;
	TRY(tp_local_config(f, tp_size, lc));
	ncclUniqueId id;
	memcpy(&id, unique_id, sizeof(id));
	ncclComm_t comm = nullptr;
	if (ncclCommInitRank(&comm, tp_size, id, tp_rank) != ncclSuccess) {
		set_err("ncclCommInitRank failed");
		return YALM_ERR_HIP;
	}
	const int r = create_decoder(&lc, weights, s, out, comm, tp_rank, tp_size, f.vocab_size);
	if (r != YALM_OK)
		(void)ncclCommDestroy(comm);
	return r;
}

// The rank record every rank shares (YALM_TP_HANDLE_BYTES): the IPC handle of its exchange
// buffer, then WHERE the rank runs -- its GPU's UUID and the CU mask of its decoder stream.
// Two ranks contend for compute only when both match (same GPU, overlapping CUs): ADVICE r5
// (medium) -- the round-5 test compared hipPointerGetAttributes(peer mapping).device with the
// current device, which an IPC-imported mapping need not report as the exporter's.
struct TpRankRecord {
	unsigned char ipc[64];
	unsigned char uuid[16];
	uint32_t cu_mask[YALM_CU_MASK_WORDS];
	unsigned char reserved[YALM_TP_HANDLE_BYTES - 64 - 16 - 4 * YALM_CU_MASK_WORDS];
};
static_assert(sizeof(TpRankRecord) == YALM_TP_HANDLE_BYTES, "rank record size");
static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");

extern "C" int yalm_tp_ipc_alloc(const yalm_config *config, int tp_size, yalm_stream s, void **buf,
                                 void *handle_out) {
	ARGCHK(config && buf && handle_out && tp_size >= 1 && tp_size <= 8, "yalm_tp_ipc_alloc: bad argument (1..8 ranks)");
	const size_t bytes = ipc_buf_bytes(*config, tp_size);
	// uncached (tp_exchange.h): peers push into it, so no reader's L2 may hold a stale line
	HIPCHK(hipExtMallocWithFlags(buf, bytes, hipDeviceMallocUncached));
	HIPCHK(hipMemset(*buf, 0, bytes));
	TpRankRecord rec;
	memset(&rec, 0, sizeof(rec));
	hipIpcMemHandle_t h;
	HIPCHK(hipIpcGetMemHandle(&h, *buf));
	memcpy(rec.ipc, &h, sizeof(h));
	int dev = 0;
	HIPCHK(hipGetDevice(&dev));
	hipUUID u;
	HIPCHK(hipDeviceGetUuid(&u, dev));
	memcpy(rec.uuid, &u, sizeof(rec.uuid));
	TRY(stream_cu_mask(reinterpret_cast<hipStream_t>(s), rec.cu_mask));
	memcpy(handle_out, &rec, sizeof(rec));
	HIPCHK(hipDeviceSynchronize());
	return YALM_OK;
}

extern "C" int yalm_decoder_create_tp_ipc(const yalm_config *config, const yalm_model_weights *weights, int tp_rank,
                                          int tp_size, void *own_buf, const void *handles, yalm_stream s,
                                          yalm_decoder *out) {
	ARGCHK(config && weights && own_buf && handles && out, "yalm_decoder_create_tp_ipc: null argument");
	ARGCHK(tp_size >= 1 && tp_size <= 8 && tp_rank >= 0 && tp_rank < tp_size, "bad rank / size (1..8 ranks)");
	yalm_config lc;
	TRY(tp_local_config(*config, tp_size, lc));
	ARGCHK(config->dim % (64 * (config->weight_dtype == YALM_F32 ? 4 : config->weight_dtype == YALM_F16 ? 8 : 16)) == 0,
	       "tensor parallel (IPC): dim must be a multiple of 64 x the elements of a 16-byte load");
	std::vector<TpRankRecord> recs(tp_size);
	memcpy(recs.data(), handles, sizeof(TpRankRecord) * tp_size);
	{ // this rank's record must describe the stream it decodes on
		uint32_t m[YALM_CU_MASK_WORDS];
		TRY(stream_cu_mask(reinterpret_cast<hipStream_t>(s), m));
		ARGCHK(!memcmp(m, recs[tp_rank].cu_mask, sizeof(m)),
		       "yalm_decoder_create_tp_ipc: this rank's record was made for another stream (CU mask differs)");
	}
	std::vector<float *> bases(tp_size);
	std::vector<void *> opened;
	for (int p = 0; p < tp_size; ++p) {
		if (p == tp_rank) {
			bases[p] = (float *)own_buf;
			continue;
		}
		hipIpcMemHandle_t h;
		memcpy(&h, recs[p].ipc, sizeof(h));
		void *ptr = nullptr;
		if (hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
			for (void *q : opened)
				(void)hipIpcCloseMemHandle(q);
			set_err("hipIpcOpenMemHandle failed");
			return YALM_ERR_HIP;
		}
		opened.push_back(ptr);
		bases[p] = (float *)ptr;
	}
	const int r = create_decoder(&lc, weights, s, out, nullptr, tp_rank, tp_size, config->vocab_size);
	if (r != YALM_OK) {
		for (void *q : opened)
			(void)hipIpcCloseMemHandle(q);
		return r;
	}
	yalm_decoder_s *d = *out;
	d->ipc = true;
	d->ipc_S = ipc_slot_floats(*config, tp_size);
	d->ipc_own = (float *)own_buf;
	d->ipc_opened = opened;
	void *dev_bases = nullptr;
	if (dalloc(d, &dev_bases, sizeof(float *) * tp_size) != YALM_OK ||
	    hipMemcpy(dev_bases, bases.data(), sizeof(float *) * tp_size, hipMemcpyHostToDevice) != hipSuccess) {
		destroy_decoder(d);
		*out = nullptr;
		set_err("IPC pointer table upload failed");
		return YALM_ERR_HIP;
	}
	d->ipc_bufs = (float **)dev_bases;
	// Ranks whose kernels can hold each other's CUs: the same GPU (UUID) with overlapping CU
	// masks (several rank processes on one GPU without yalm_stream_create_cu_part). One GPU
	// per rank -- or disjoint CU masks on one GPU, the rehearsal of that -- needs no gate.
	for (int p = 0; p < tp_size; ++p) {
		if (p == tp_rank || memcmp(recs[p].uuid, recs[tp_rank].uuid, sizeof(recs[p].uuid)))
			continue;
		for (int i = 0; i < YALM_CU_MASK_WORDS; ++i)
			if (recs[p].cu_mask[i] & recs[tp_rank].cu_mask[i])
				d->tpx_gate = true;
	}
	// The fused attention + Wo launch's Wo workgroups spin on attention workgroups of the
	// same launch; a workgroup only ever waits on lower-index ones, and each XCD dispatches
	// its workgroups in index order, so by induction on the index every workgroup is
	// dispatched and finishes whatever fits at once (on a CU-masked rehearsal stream the
	// production grid runs in several rounds: correct, just slower). Ranks whose grids SHARE
	// CUs break that: a workgroup dispatched on a full XCD can trail another rank's Wo
	// workgroups spinning there (measured: TP8 at Mistral dims, 8 unmasked processes on one
	// MI355X, the Wo gather timed out). Those ranks keep the separate attention and Wo launches.
	if (d->tpx_gate && d->attn_wo && d->awo_nb * tp_size > d->awo_slots)
		d->attn_wo = d->attn_wo_ok = false;
	d->tpx_collect = tp_size > TPX_STAGE_MAX_RANKS;
	d->tpx.bufs = d->ipc_bufs;
	d->tpx.rank = tp_rank;
	d->tpx.n = tp_size;
	d->tpx.S = d->ipc_S;
	d->tpx.xw = d->x;
	d->tpx.step = d->step;
	d->tpx.ex = 0;
	return YALM_OK;
}

extern "C" int yalm_copy_2d(void *dst, size_t dst_pitch, const void *src, size_t src_pitch, size_t width,
                            size_t height) {
	ARGCHK(dst && src && width <= dst_pitch && width <= src_pitch, "yalm_copy_2d: bad argument");
	HIPCHK(hipMemcpy2D(dst, dst_pitch, src, src_pitch, width, height, hipMemcpyDeviceToDevice));
	return YALM_OK;
}

extern "C" int yalm_decoder_destroy(yalm_decoder d) {
	if (!d)
		return YALM_OK;
	(void)hipStreamSynchronize(d->stream);
	destroy_decoder(d);
	return YALM_OK;
}

extern "C" int yalm_forward(yalm_decoder d, int token, int pos, int mode, float *logits_host) {
	ARGCHK(d, "null decoder");
	ARGCHK(token >= 0 && token < d->vocab_full, "token out of range");
	ARGCHK(pos >= 0, "negative pos");
	const int which = mode == YALM_HYDRATE_KV_CACHE ? GRAPH_HYDRATE : GRAPH_LOGITS;
	TRY(ensure_graph(d, which));
	set_step_kernel<<<1, 1, 0, d->stream>>>(d->step, token, pos, 0);
	HIPCHK(hipGetLastError());
	TRY(replay(d, which));
	d->host_pos = pos; // OUTPUT / HYDRATE forwards do not advance the device position
	if (which == GRAPH_LOGITS) {
		HIPCHK(hipStreamSynchronize(d->stream));
		TRY(awo_check(d));
		if (logits_host)
			memcpy(logits_host, d->logits_pinned, sizeof(float) * d->vocab_full);
	}
	return YALM_OK;
}

// n greedy forwards from position pos0 (-1: unknown); the eager path passes each forward's
// kv_len to the attention + Wo launch (awo_kv_hint), graph replays cannot
static int replay_greedy(yalm_decoder_s *d, int n, long long pos0) {
	if (!d->greedy_eager)
		TRY(ensure_graph(d, GRAPH_GREEDY));
	int r = YALM_OK;
	for (int i = 0; i < n && r == YALM_OK; ++i) {
		d->awo_kv_hint = pos0 >= 0 ? std::min<long long>(pos0 + i + 1, d->c.max_seq_len) : -1;
		r = replay(d, GRAPH_GREEDY);
	}
	d->awo_kv_hint = -1;
	return r;
}

extern "C" int yalm_enqueue_greedy(yalm_decoder d, int n_steps) {
	ARGCHK(d, "null decoder");
	ARGCHK(n_steps >= 0, "bad n_steps");
	TRY(replay_greedy(d, n_steps, d->host_pos)); // each forward advances the device position by one
	if (d->host_pos >= 0)
		d->host_pos += n_steps;
	return YALM_OK;
}

extern "C" int yalm_generate_greedy(yalm_decoder d, int token, int pos, int n_steps, int *out_tokens) {
	ARGCHK(d && out_tokens, "null argument");
	ARGCHK(token >= 0 && token < d->vocab_full && pos >= 0 && n_steps >= 0, "bad token/pos/n_steps");
	int done = 0;
	bool first = true;
	while (done < n_steps) {
		const int batch = std::min(n_steps - done, d->tokens_cap);
		if (first)
			set_step_kernel<<<1, 1, 0, d->stream>>>(d->step, token, pos, 1);
		else
			set_step_kernel<<<1, 1, 0, d->stream>>>(d->step, out_tokens[done - 1], pos + done, 1);
		HIPCHK(hipGetLastError());
		first = false;
		TRY(replay_greedy(d, batch, (long long)pos + done));
		d->host_pos = (long long)pos + done + batch;
		HIPCHK(hipMemcpyAsync(out_tokens + done, d->tokens, sizeof(int) * batch, hipMemcpyDeviceToHost, d->stream));
		HIPCHK(hipStreamSynchronize(d->stream));
		TRY(awo_check(d));
		done += batch;
	}
	return YALM_OK;
}

extern "C" int yalm_device_step(yalm_decoder d, int *token, int *pos) {
	ARGCHK(d, "null decoder");
	StepState s;
	HIPCHK(hipStreamSynchronize(d->stream));
	TRY(awo_check(d));
	HIPCHK(hipMemcpy(&s, d->step, sizeof(s), hipMemcpyDeviceToHost));
	if (token)
		*token = s.token;
	if (pos)
		*pos = s.pos;
	return YALM_OK;
}

extern "C" int yalm_device_tokens(yalm_decoder d, int *out, int cap, int *n_total) {
	ARGCHK(d && n_total && cap >= 0 && (out || cap == 0), "yalm_device_tokens: bad argument");
	StepState s;
	HIPCHK(hipStreamSynchronize(d->stream));
	TRY(awo_check(d));
	HIPCHK(hipMemcpy(&s, d->step, sizeof(s), hipMemcpyDeviceToHost));
	*n_total = s.n_gen;
	const int n = std::min(std::min(s.n_gen, d->tokens_cap), cap);
	if (n > 0)
		HIPCHK(hipMemcpy(out, d->tokens, sizeof(int) * n, hipMemcpyDeviceToHost));
	return YALM_OK;
}

extern "C" int yalm_block(yalm_decoder d, int layer, int pos, int kv_sink, int kv_pos, int kv_len) {
	ARGCHK(d && layer >= 0 && layer < d->c.n_layers, "bad layer");
	ARGCHK(kv_len >= 1 && kv_len <= d->c.max_seq_len && kv_pos >= 0 && kv_pos < d->c.max_seq_len,
	       "bad kv indices");
	set_step_full_kernel<<<1, 64, 0, d->stream>>>(d->step, pos, kv_sink, kv_pos, kv_len, d->ipc ? 2 : 0, d->inv_freq,
	                                              d->c.head_dim / 2);
	HIPCHK(hipGetLastError());
	TRY(DISPATCH_WT(d->c.weight_dtype, enqueue_layer_t, d, layer, 0, false, true));
	if (d->ipc) { // the layer's W2 pushed its partial: collect the sum into x (a forward's next GEMV would)
		tpx_collect_kernel<<<TPX_COLLECT_WG, 256, 0, d->stream>>>(tpx_ex(d, 1), d->c.dim, 0, d->x);
		HIPCHK(hipGetLastError());
	}
	HIPCHK(hipStreamSynchronize(d->stream));
	return awo_check(d);
}

extern "C" int yalm_get_x(yalm_decoder d, float *host) {
	ARGCHK(d && host, "null argument");
	HIPCHK(hipStreamSynchronize(d->stream));
	HIPCHK(hipMemcpy(host, d->x, sizeof(float) * d->c.dim, hipMemcpyDeviceToHost));
	return YALM_OK;
}

extern "C" int yalm_set_x(yalm_decoder d, const float *host) {
	ARGCHK(d && host, "null argument");
	HIPCHK(hipStreamSynchronize(d->stream));
	HIPCHK(hipMemcpy(d->x, host, sizeof(float) * d->c.dim, hipMemcpyHostToDevice));
	return YALM_OK;
}

extern "C" int yalm_get_logits(yalm_decoder d, float *host) {
	ARGCHK(d && host, "null argument");
	HIPCHK(hipStreamSynchronize(d->stream));
	HIPCHK(hipMemcpy(host, d->logits, sizeof(float) * d->vocab_full, hipMemcpyDeviceToHost));
	return YALM_OK;
}

template <class WT>
static int enqueue_one_t(yalm_decoder_s *d, int kernel_id, int l) {
	const yalm_config &c = d->c;
	const yalm_block_weights &w = d->b[l];
	const int q_dim = c.n_heads * c.head_dim;
	switch (kernel_id) {
	case 0:
	case 2:
	case 3:
	case 4: {
		// reuse the layer enqueue path for exactly one kernel
		if (kernel_id == 0) {
			PQKV<WT> p;
			p.wq = (const char *)w.wq;
			p.wk = (const char *)w.wk;
			p.wv = (const char *)w.wv;
			p.n = c.dim;
			p.q_dim = q_dim;
			p.kv_dim = c.n_kv_heads * c.head_dim;
			p.head_dim = c.head_dim;
			p.n_groups = (q_dim + 2 * p.kv_dim) / 2;
			p.qkv_clip = c.qkv_clip;
			p.inv_freq = d->inv_freq;
			p.step = d->step;
			p.q_out = d->q;
			p.kcache = w.key_cache;
			p.vcache = w.value_cache;
			return launch_gemv_d<WT, PQKV<WT>, true>(d, p, d->x, w.rms_att, c.norm_eps, GK_QKV);
		}
		if (kernel_id == 2 || kernel_id == 4) {
			PResidual<WT, 1> p;
			p.W = (const char *)(kernel_id == 2 ? w.wo : w.w2);
			p.n = kernel_id == 2 ? q_dim : c.hidden_dim;
			p.out = d->x;
			p.n_groups = c.dim;
			return launch_gemv_d<WT, PResidual<WT, 1>, false>(d, p, kernel_id == 2 ? d->xb2 : d->hb, nullptr, 0.f,
			                                                  kernel_id == 2 ? GK_WO : GK_W2);
		}
		PGlu<WT, 1> p;
		p.w1 = (const char *)w.w1;
		p.w3 = (const char *)w.w3;
		p.n = c.dim;
		p.out = d->hb;
		p.n_groups = c.hidden_dim;
		return launch_gemv_d<WT, PGlu<WT, 1>, true>(d, p, d->x, w.rms_ffn, c.norm_eps, GK_GLU);
	}
	case 1:
		return launch_attn(c.head_dim, c.n_heads, c.n_kv_heads, d->q, w.key_cache, w.value_cache, d->step,
		                   c.max_seq_len, d->part, l, c.n_layers, d->awo_err, nullptr, d->xb2, d->stream);
	case 5: // (local x: the timing hooks never take part in an exchange, except kernels 6 and 8)
		return enqueue_logits_t<WT>(d, -1, -1);
	case 6:
		return enqueue_exchange(d);
	case 8: // fused attention + Wo (IPC: pushing exchange 0 of the bumped sequence, unread)
		if constexpr (WT::BYTES <= 2)
			return launch_attn_wo<WT>(d, w, l, 0);
		break;
	}
	set_err("bad kernel_id");
	return YALM_ERR_ARG;
}

extern "C" int yalm_graph_kernels(yalm_decoder d, int mode, int *kernels, int *nodes) {
	ARGCHK(d && kernels && mode >= 0 && mode < N_GRAPHS, "yalm_graph_kernels: bad argument");
	ARGCHK(!d->eager, "yalm_graph_kernels: the decoder launches eagerly (YALM_LAUNCH_EAGER)");
	TRY(ensure_graph(d, mode));
	size_t n = 0;
	HIPCHK(hipGraphGetNodes(d->graph[mode], nullptr, &n));
	std::vector<hipGraphNode_t> v(n);
	if (n)
		HIPCHK(hipGraphGetNodes(d->graph[mode], v.data(), &n));
	int k = 0;
	for (auto node : v) {
		hipGraphNodeType t;
		HIPCHK(hipGraphNodeGetType(node, &t));
		k += t == hipGraphNodeTypeKernel;
	}
	*kernels = k;
	if (nodes)
		*nodes = (int)n;
	return YALM_OK;
}

extern "C" int yalm_decoder_set_launch(yalm_decoder d, int flags) {
	ARGCHK(d, "null decoder");
	ARGCHK(!(flags & ~(YALM_LAUNCH_EAGER | YALM_LAUNCH_SYNC | YALM_LAUNCH_SEPARATE_ATTN_WO)), "unknown launch flag");
	HIPCHK(hipStreamSynchronize(d->stream));
	drop_graphs(d); // captured graphs bake the old launch sequence
	d->eager = flags & YALM_LAUNCH_EAGER;
	d->graph_sync = flags & YALM_LAUNCH_SYNC;
	d->attn_wo = d->attn_wo_ok && !(flags & YALM_LAUNCH_SEPARATE_ATTN_WO);
	return YALM_OK;
}

extern "C" int yalm_decoder_attn_wo(yalm_decoder d) {
	return d && d->attn_wo ? 1 : 0;
}

extern "C" int yalm_attn_wo_trace(yalm_decoder d, unsigned long long *host, size_t count, int *workgroups,
                                  int *attention_workgroups) {
	ARGCHK(d && host, "null argument");
	ARGCHK(d->attn_wo && d->awo_trace, "no attn_wo trace (create the decoder with YALM_ATTN_WO_TRACE=1)");
	HIPCHK(hipStreamSynchronize(d->stream));
	const size_t total = (size_t)AWO_TRACE_N * d->awo_nb;
	HIPCHK(hipMemcpy(host, d->awo_trace, sizeof(unsigned long long) * std::min(count, total), hipMemcpyDeviceToHost));
	if (workgroups)
		*workgroups = d->awo_nb;
	if (attention_workgroups)
		*attention_workgroups = d->c.n_kv_heads * (d->awo_S + d->c.n_heads / d->c.n_kv_heads - 1) + d->c.n_heads;
	return YALM_OK;
}

// Average ms per iteration of `iters` back-to-back enqueues of kernel_id on the
// decoder stream (HIP events). With `bump`, every iteration first advances the step
// epoch (one 1-thread kernel), so a fused attention + Wo launch sees fresh tags and
// its Wo waves really wait for the heads (without it the granules of the
// previous launch already match and the hand-off is not measured).
static int time_loop(yalm_decoder_s *d, int kernel_id, int iters, bool bump, bool kernel, float *ms_out) {
	hipEvent_t e0, e1;
	HIPCHK(hipEventCreate(&e0));
	HIPCHK(hipEventCreate(&e1));
	int r = YALM_OK;
	HIPCHK(hipEventRecord(e0, d->stream));
	for (int i = 0; i < iters && r == YALM_OK; ++i) {
		if (bump)
			epoch_bump_kernel<<<1, 1, 0, d->stream>>>(d->step, 1);
		// rotate layers so weights come from HBM, not the 256 MiB Infinity Cache
		if (kernel)
			r = DISPATCH_WT(d->c.weight_dtype, enqueue_one_t, d, kernel_id, (i + 1) % d->c.n_layers);
	}
	HIPCHK(hipEventRecord(e1, d->stream));
	HIPCHK(hipEventSynchronize(e1));
	float ms = 0.f;
	HIPCHK(hipEventElapsedTime(&ms, e0, e1));
	(void)hipEventDestroy(e0);
	(void)hipEventDestroy(e1);
	*ms_out = ms / iters;
	return r;
}

extern "C" int yalm_time_kernel(yalm_decoder d, int kernel_id, int iters, float *avg_ms) {
	ARGCHK(d && avg_ms && iters > 0 && kernel_id >= 0 && kernel_id <= 8 && kernel_id != 7,
	       "bad argument (kernel ids 0-6, 8)");
	ARGCHK(kernel_id != 6 || d->comm || d->ipc, "kernel 6 (tensor-parallel exchange) needs a tensor-parallel decoder");
	ARGCHK(kernel_id != 8 || d->attn_wo, "kernel 8 (fused attention + Wo) needs yalm_decoder_attn_wo");
	// in-launch hand-offs and the IPC exchange: fresh tags per launch (one exchange per bump)
	const bool bump = kernel_id == 1 || kernel_id == 8 || (kernel_id == 6 && d->ipc);
	// the warm-up gets a fresh epoch too: under IPC it pushes exchange xbase + 0, whose slot
	// parity the previous forward's argmax exchange (2 L, even) used -- without the bump a
	// peer still reading that slot could see it overwritten (tp_exchange.h reuse rule)
	if (bump)
		epoch_bump_kernel<<<1, 1, 0, d->stream>>>(d->step, 1);
	TRY(DISPATCH_WT(d->c.weight_dtype, enqueue_one_t, d, kernel_id, 0)); // warm-up
	float ms = 0.f;
	TRY(time_loop(d, kernel_id, iters, bump, true, &ms));
	if (bump) { // minus the epoch bumps alone (one launch each), so one boundary per iteration stays in
		float mb = 0.f;
		TRY(time_loop(d, kernel_id, iters, true, false, &mb));
		ms = std::max(0.f, ms - mb);
	}
	TRY(awo_check(d));
	*avg_ms = ms;
	return YALM_OK;
}

extern "C" int yalm_set_gemv_config(yalm_decoder d, int kind, int threads, int unroll, int gpw) {
	ARGCHK(d && kind >= 0 && kind < GK_N, "bad decoder/kind");
	ARGCHK(threads == 0 || threads == 256 || threads == 512 || threads == 1024, "threads must be 0, 256, 512 or 1024");
	ARGCHK(unroll == 0 || unroll == 2 || unroll == 4 || unroll == 8, "unroll must be 0, 2, 4 or 8");
	ARGCHK(gpw >= 0, "gpw must be >= 0");
	d->gemv[kind] = GemvCfg{threads, unroll, gpw};
	// captured graphs bake the old geometry: drop them
	HIPCHK(hipStreamSynchronize(d->stream));
	drop_graphs(d);
	return YALM_OK;
}

extern "C" const char *yalm_kernel_name(yalm_decoder d, int kernel_id) {
	if (!d)
		return "";
	const char *wt = d->c.weight_dtype == YALM_F32 ? "WF32" : d->c.weight_dtype == YALM_F16 ? "WF16" : "WF8";
	const std::string gk = std::string("gemv_rb_kernel<") + wt;
	std::string s;
	switch (kernel_id) {
	case 0:
		s = gk + ", PQKV<";
		break;
	case 1:
		s = "attn_decode_kernel<";
		break;
	case 2:
	case 4:
		s = gk + ", PResidual<";
		break;
	case 3:
		s = gk + ", PGlu<";
		break;
	case 5:
		s = gk + ", PStore<";
		break;
	case 6:
		s = d->ipc ? "tpx_collect_kernel" : d->comm ? "AllReduce" : "";
		break;
	case 8:
		s = std::string("attn_wo_kernel<") + wt + ", ";
		break;
	default:
		s = "";
	}
	d->kname = s;
	return d->kname.c_str();
}

namespace {
struct DevBufT {
	void *p = nullptr;
	~DevBufT() {
		if (p)
			(void)hipFree(p);
	}
};
} // namespace

// ------------------------------------------------------------------ streaming envelope
// Pure read-only HBM stream (tools/stream_bench.hip): each wave sums `per_wave`
// contiguous 16-byte pieces with U nt loads in flight per lane; the result is
// consumed only to keep the loads alive.
template <int U>
__global__ __launch_bounds__(512) void stream_read_kernel(const u32x4_t *__restrict__ p, size_t n16, size_t per_wave,
                                                          unsigned *out) {
	const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
	const int lane = threadIdx.x & 63;
	const size_t base = wave * per_wave;
	const size_t end = base + per_wave < n16 ? base + per_wave : n16;
	unsigned acc = 0;
	for (size_t i = base + lane; i < end; i += 64 * U) {
		u32x4_t v[U];
#pragma unroll
		for (int u = 0; u < U; ++u) {
			const size_t j = i + (size_t)u * 64;
			v[u] = j < end ? load_nt16(p + j) : u32x4_t{0u, 0u, 0u, 0u};
		}
#pragma unroll
		for (int u = 0; u < U; ++u)
			acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

extern "C" int yalm_stream_envelope(size_t bytes, int iters, float *avg_ms) {
	ARGCHK(avg_ms && iters > 0 && bytes >= (1u << 20), "yalm_stream_envelope: bad argument");
	bytes &= ~(size_t)4095;
	DevBufT buf[2];
	unsigned *out = nullptr;
	for (auto &b : buf) {
		HIPCHK(hipMalloc(&b.p, bytes));
		HIPCHK(hipMemset(b.p, 1, bytes));
	}
	HIPCHK(hipMalloc((void **)&out, 64));
	hipEvent_t e0, e1;
	HIPCHK(hipEventCreate(&e0));
	HIPCHK(hipEventCreate(&e1));
	float best = 1e30f;
	const size_t n16 = bytes / 16;
	int r = YALM_OK;
	for (size_t pw_bytes : {16384ul, 32768ul, 65536ul}) {
		for (int U : {4, 8}) {
			const size_t per_wave = pw_bytes / 16;
			const size_t waves = (n16 + per_wave - 1) / per_wave;
			const int blocks = (int)((waves + 7) / 8);
			for (int pass = 0; pass < 2 && r == YALM_OK; ++pass) { // pass 0 warms up
				if (hipEventRecord(e0, nullptr) != hipSuccess)
					r = YALM_ERR_HIP;
				for (int it = 0; it < iters && r == YALM_OK; ++it) { // alternate buffers: 2x bytes > 256 MiB MALL
					const u32x4_t *src = (const u32x4_t *)buf[it & 1].p;
					if (U == 4)
						stream_read_kernel<4><<<blocks, 512>>>(src, n16, per_wave, out);
					else
						stream_read_kernel<8><<<blocks, 512>>>(src, n16, per_wave, out);
				}
				float ms = 0.f;
				if (r == YALM_OK && (hipEventRecord(e1, nullptr) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
				                     hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
					r = YALM_ERR_HIP;
				if (pass == 1 && r == YALM_OK)
					best = std::min(best, ms / iters);
			}
		}
	}
	(void)hipEventDestroy(e0);
	(void)hipEventDestroy(e1);
	(void)hipFree(out);
	if (r != YALM_OK) {
		set_err("yalm_stream_envelope: HIP call failed");
		return r;
	}
	*avg_ms = best;
	return YALM_OK;
}

// ------------------------------------------------------------------ test API (host pointers)
namespace {
struct DevBuf {
	void *p = nullptr;
	~DevBuf() {
		if (p)
			(void)hipFree(p);
	}
};
int up(DevBuf &b, const void *host, size_t bytes) {
	HIPCHK(hipMalloc(&b.p, bytes ? bytes : 4));
	if (host)
		HIPCHK(hipMemcpy(b.p, host, bytes, hipMemcpyHostToDevice));
	else
		HIPCHK(hipMemset(b.p, 0, bytes ? bytes : 4));
	return YALM_OK;
}
size_t wbytes(int dtype) {
	return dtype == YALM_F32 ? 4 : dtype == YALM_F16 ? 2 : 1;
}
} // namespace

template <class WT>
static int matmul_t(float *out, const float *x, const void *w, int n, int d) {
	PStore<WT, 1> p;
	p.W = (const char *)w;
	p.n = n;
	p.out = out;
	p.n_groups = d;
	return launch_gemv<WT, PStore<WT, 1>, false>(p, x, nullptr, 0.f, GK_GLU, GemvCfg{}, nullptr);
}

extern "C" int yalm_matmul(float *xout, const float *x, const void *w, int n, int d, int dtype) {
	ARGCHK(xout && x && w && n > 0 && d > 0, "bad argument");
	ARGCHK(dtype == YALM_F32 || dtype == YALM_F16 || dtype == YALM_F8E5M2, "bad dtype");
	ARGCHK(n % 16 == 0, "n must be a multiple of 16 (infer.cpp:66)");
	DevBuf dx, dw, dout;
	TRY(up(dx, x, sizeof(float) * n));
	TRY(up(dw, w, wbytes(dtype) * (size_t)n * d));
	TRY(up(dout, nullptr, sizeof(float) * d));
	TRY(DISPATCH_WT(dtype, matmul_t, (float *)dout.p, (const float *)dx.p, dw.p, n, d));
	HIPCHK(hipDeviceSynchronize());
	HIPCHK(hipMemcpy(xout, dout.p, sizeof(float) * d, hipMemcpyDeviceToHost));
	return YALM_OK;
}

extern "C" int yalm_mha(float *xout, float *att, const uint16_t *kb, const uint16_t *vb, const float *q, int head_dim,
                        int kv_len, int max_seq_len, int n_heads, int n_kv_heads) {
	ARGCHK(xout && kb && vb && q, "null argument");
	ARGCHK(n_kv_heads > 0 && n_heads % n_kv_heads == 0 && kv_len >= 1 && kv_len <= max_seq_len, "bad shape");
	if (!attn_supported(head_dim, n_heads / n_kv_heads)) {
		set_err("unsupported head_dim / group size");
		return YALM_ERR_UNSUPPORTED;
	}
	const size_t kvn = (size_t)max_seq_len * n_kv_heads * head_dim;
	const int nsplit = attn_nsplit(max_seq_len);
	DevBuf dk, dv, dq, dout, datt, dpart, dstep, derr;
	TRY(up(dk, kb, kvn * 2));
	TRY(up(dv, vb, kvn * 2));
	TRY(up(dq, q, sizeof(float) * n_heads * head_dim));
	TRY(up(dout, nullptr, sizeof(float) * n_heads * head_dim));
	TRY(up(datt, att, sizeof(float) * (size_t)n_heads * max_seq_len));
	TRY(up(dpart, nullptr, sizeof(unsigned long long) * (size_t)n_heads * nsplit * (head_dim + 2)));
	TRY(up(dstep, nullptr, sizeof(StepState)));
	TRY(up(derr, nullptr, sizeof(unsigned)));
	set_step_full_kernel<<<1, 1>>>((StepState *)dstep.p, kv_len - 1, 0, kv_len - 1, kv_len);
	TRY(launch_attn(head_dim, n_heads, n_kv_heads, (const float *)dq.p, (const uint16_t *)dk.p,
	                (const uint16_t *)dv.p, (const StepState *)dstep.p, max_seq_len, (unsigned long long *)dpart.p, 0, 1,
	                (unsigned *)derr.p, att ? (float *)datt.p : nullptr, (float *)dout.p, nullptr));
	HIPCHK(hipDeviceSynchronize());
	HIPCHK(hipMemcpy(xout, dout.p, sizeof(float) * n_heads * head_dim, hipMemcpyDeviceToHost));
	if (att)
		HIPCHK(hipMemcpy(att, datt.p, sizeof(float) * (size_t)n_heads * max_seq_len, hipMemcpyDeviceToHost));
	unsigned e = 0;
	HIPCHK(hipMemcpy(&e, derr.p, sizeof(e), hipMemcpyDeviceToHost));
	if (e) {
		set_err("yalm_mha: the split-KV merger gave up waiting for a chunk");
		return YALM_ERR_HIP;
	}
	return YALM_OK;
}

extern "C" int yalm_argmax(const float *logits, int n, int n_shards, int *out) {
	ARGCHK(logits && out && n > 0 && n_shards >= 1 && n_shards <= 64 && n % n_shards == 0, "yalm_argmax: bad argument");
	DevBuf dl, dst, dpairs;
	TRY(up(dl, logits, sizeof(float) * (size_t)n));
	TRY(up(dst, nullptr, sizeof(StepState)));
	TRY(up(dpairs, nullptr, sizeof(float) * 2 * n_shards));
	StepState *st = (StepState *)dst.p;
	if (n_shards == 1) {
		argmax_kernel<<<1, 1024>>>((const float *)dl.p, n, st, nullptr, 0);
	} else { // the tensor-parallel path: per-shard first max as (value, global index), then the pick
		const int ns = n / n_shards;
		for (int r = 0; r < n_shards; ++r)
			argmax_kernel<<<1, 1024>>>((const float *)dl.p + (size_t)r * ns, ns, st, nullptr, 0,
			                           (float *)dpairs.p + 2 * r, r * ns);
		argmax_pick_kernel<<<1, 1>>>((const float *)dpairs.p, n_shards, st, nullptr, 0);
	}
	HIPCHK(hipGetLastError());
	HIPCHK(hipDeviceSynchronize());
	StepState h;
	HIPCHK(hipMemcpy(&h, st, sizeof(h), hipMemcpyDeviceToHost));
	*out = h.token;
	return YALM_OK;
}

template <class WT>
static int ffn_t(float *out, const float *x, const void *w1, const void *w2, const void *w3, float *hb, int hidden,
                 int dim, int act) {
	if (act == YALM_SILU) {
		PGlu<WT, 1> p;
		p.w1 = (const char *)w1;
		p.w3 = (const char *)w3;
		p.n = dim;
		p.out = hb;
		p.n_groups = hidden;
		TRY((launch_gemv<WT, PGlu<WT, 1>, false>(p, x, nullptr, 0.f, GK_GLU, GemvCfg{}, nullptr)));
	} else {
		PGlu<WT, 0> p;
		p.w1 = (const char *)w1;
		p.w3 = (const char *)w3;
		p.n = dim;
		p.out = hb;
		p.n_groups = hidden;
		TRY((launch_gemv<WT, PGlu<WT, 0>, false>(p, x, nullptr, 0.f, GK_GLU, GemvCfg{}, nullptr)));
	}
	PStore<WT, 1> p;
	p.W = (const char *)w2;
	p.n = hidden;
	p.out = out;
	p.n_groups = dim;
	return launch_gemv<WT, PStore<WT, 1>, false>(p, hb, nullptr, 0.f, GK_GLU, GemvCfg{}, nullptr);
}

extern "C" int yalm_ffn(float *xout, const float *x, const void *w1, const void *w2, const void *w3, int hidden_dim,
                        int dim, int act, int dtype) {
	ARGCHK(xout && x && w1 && w2 && w3 && hidden_dim > 0 && dim > 0, "bad argument");
	ARGCHK(dtype == YALM_F32 || dtype == YALM_F16 || dtype == YALM_F8E5M2, "bad dtype");
	ARGCHK(dim % 16 == 0 && hidden_dim % 16 == 0, "dims must be multiples of 16");
	const size_t wb = wbytes(dtype) * (size_t)hidden_dim * dim;
	DevBuf dx, d1, d2, d3, dhb, dout;
	TRY(up(dx, x, sizeof(float) * dim));
	TRY(up(d1, w1, wb));
	TRY(up(d2, w2, wb));
	TRY(up(d3, w3, wb));
	TRY(up(dhb, nullptr, sizeof(float) * hidden_dim));
	TRY(up(dout, nullptr, sizeof(float) * dim));
	TRY(DISPATCH_WT(dtype, ffn_t, (float *)dout.p, (const float *)dx.p, d1.p, d2.p, d3.p, (float *)dhb.p, hidden_dim,
	                dim, act));
	HIPCHK(hipDeviceSynchronize());
	HIPCHK(hipMemcpy(xout, dout.p, sizeof(float) * dim, hipMemcpyDeviceToHost));
	return YALM_OK;
}
