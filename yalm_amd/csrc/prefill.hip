#include <cstdlib>
#include <cstring>
// prefill.hip — C ABI of the batched prefill / perplexity path (prefill.h):
// yalm_prefill (prompt hydration + per-position log p(next), replacing the
// reference's position-by-position loop in main.cpp:128-200 / 102-112) and
// its kernel-level test hooks (yalm_gemm_f16, yalm_attn_prefill).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <vector>

#include "decoder.h"
#include "prefill.h"
#include "prefill_gemm.h"

namespace {

int pf_alloc(yalm_decoder_s *d, void **p, size_t bytes) {
	HIPCHK(hipMalloc(p, bytes ? bytes : 4));
	d->dev_allocs.push_back(*p);
	return YALM_OK;
}

template <class EPI, int NB>
int launch_gemm(const uint16_t *A, int M, int K, pf::BSrc b0, pf::BSrc b1, int N, const EPI &epi, hipStream_t st) {
	// Form per GEMM, from per-kernel rocprofv3 times on Llama-3.2-3B at T = 4096
	// (profiles/r2_prefill_kernels.txt): the two-matrix GLU GEMM keeps one K tile in
	// flight across the barriers (3 LDS stages: 495 vs 633 us at 2); single-matrix
	// GEMMs of moderate N keep the 128 x 128 tile with 2 stages (2 workgroups per CU:
	// QKV 241 us vs 287 at 3 stages and 278 wide; Wo 154 vs 160; W2 equal); the vocab
	// GEMM (N > 16384) takes the 128 x 256 tile with 3 stages (4.77 ms vs 5.27 / 5.61).
	// YALM_PF_STAGES = 2 | 3 and YALM_PF_WIDE = 0 | 1 override (read per launch: tests
	// switch them inside one process).
	const char *se = getenv("YALM_PF_STAGES");
	const char *we = getenv("YALM_PF_WIDE");
	const bool big_n = N > 16384;
	const bool wide = NB == 1 && N % (2 * pf::BN) == 0 && (we ? atoi(we) != 0 : big_n);
	const int stages = se ? (atoi(se) == 2 ? 2 : 3) : (NB == 2 || wide ? 3 : 2);
	const void *kern = nullptr;
	size_t lds;
	if constexpr (NB == 1) {
		if (wide) {
			kern = stages == 3 ? (const void *)pf::gemm_nt_kernel<EPI, 2, 3, true>
			                   : (const void *)pf::gemm_nt_kernel<EPI, 2, 2, true>;
			b1 = b0;
		}
	}
	if (wide) {
		lds = (size_t)stages * 3 * pf::TILE * sizeof(uint16_t);
	} else {
		kern = stages == 3 ? (const void *)pf::gemm_nt_kernel<EPI, NB, 3> : (const void *)pf::gemm_nt_kernel<EPI, NB, 2>;
		lds = (size_t)stages * (1 + NB) * pf::TILE * sizeof(uint16_t);
	}
	static bool attr_set[2][2] = {}; // per template instance, form and stage count
	if (!attr_set[wide][stages - 2]) {
		HIPCHK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		attr_set[wide][stages - 2] = true;
	}
	const int nwg = ((M + pf::BM - 1) / pf::BM) * (N / (wide ? 2 * pf::BN : pf::BN));
	void *args[] = {(void *)&A, (void *)&M, (void *)&K, (void *)&b0, (void *)&b1, (void *)&N, (void *)&epi};
	HIPCHK(hipLaunchKernel(kern, dim3(nwg), dim3(pf::THREADS), args, lds, st));
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// Large-tile GEMM form per GEMM kind (prefill_gemm.h): the tile width BN of
// gemm16_kernel (256 rows x BN columns), 0 = the 128 x 128 kernel of prefill.h.
// Default: auto -- the BN dividing N that minimises rounds x (BN + 64), rounds =
// ceil(tiles / CUs): a 256-CU chip should get whole rounds of large tiles (Llama-3B
// QKV N 5120 -> 320: 256 tiles at T 4096 instead of 320; Wo / W2 N 3072 -> 192).
// YALM_PF_G16 = "qkv:256,wo:128,..." forces a width, "0" (or kind:0) the old kernel
// (read per launch: tests switch it inside one process).
enum { PG_QKV = 0, PG_WO = 1, PG_GLU = 2, PG_W2 = 3, PG_CLS = 4, PG_TEST = 5 };
int g16_form(int kind) {
	static const char *names[6] = {"qkv", "wo", "glu", "w2", "cls", "test"};
	int f = -1; // auto
	if (const char *e = getenv("YALM_PF_G16")) {
		if (!strcmp(e, "0"))
			return 0;
		const char *p = strstr(e, names[kind]);
		if (p && p[strlen(names[kind])] == ':')
			f = atoi(p + strlen(names[kind]) + 1);
	}
	return f;
}

// The 256-row tiles of width 192, 256 and 320 run the 8-phase schedule (prefill_gemm.h
// gemm8p_kernel) unless YALM_PF_8P=0 (read per launch, for A/B runs and the exactness
// tests of both forms).
bool use_8phase() {
	const char *e = getenv("YALM_PF_8P");
	return !e || atoi(e) != 0;
}

// BN for a GEMM of M x N (n_eff = B rows: 2 x hidden for the GLU); 0 = none fits
int pick_bn(int form, int M, int n_eff, bool glu, long *cost_out = nullptr) {
	static const int cands[4] = {128, 192, 256, 320};
	if (form == 0)
		return 0;
	if (form > 0) {
		const bool ok = n_eff % form == 0 && (!glu || form == 128 || form == 256) &&
		                (form == 128 || form == 192 || form == 256 || form == 320);
		return ok ? form : 0;
	}
	const long ncu = device_cu_count();
	const long tiles_m = (M + pf::G_BM - 1) / pf::G_BM;
	const bool p8 = use_8phase();
	int best = 0;
	long best_cost = 0;
	for (int bn : cands) {
		if (n_eff % bn || (glu && bn != 128 && bn != 256))
			continue;
		const long rounds = (tiles_m * (n_eff / bn) + ncu - 1) / ncu;
		// an 8-phase tile (widths 192, 256) costs 3/4 of a 2-phase tile of the same
		// width (Llama-3B T 4096, one process: Wo / W2 at 256 in the 8-phase kernel beat
		// 192 in the 2-phase one, profiles/r3_prefill_8phase.txt)
		const long cost = rounds * (bn + 64) * (p8 && (bn == 192 || bn == 256) ? 3 : 4);
		if (!best || cost < best_cost || (cost == best_cost && bn > best)) {
			best = bn;
			best_cost = cost;
		}
	}
	if (cost_out)
		*cost_out = best_cost;
	return best;
}

template <class EPI, class BMAP, int FJ0, int FJ1>
int launch_g8p(const uint16_t *A, int M, int K, const BMAP &bm, int N, const EPI &epi, hipStream_t st, int c0) {
	auto kern = pf::gemm8p_kernel<EPI, BMAP, FJ0, FJ1>;
	constexpr size_t lds = pf::gemm8p_lds<FJ0, FJ1>();
	constexpr int BN = 64 * (FJ0 + FJ1);
	static bool attr = false;
	if (!attr) {
		HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		attr = true;
	}
	const int nwg = ((M + pf::G_BM - 1) / pf::G_BM) * (N / BN);
	// more tiles than CUs: one persistent workgroup per CU walks them (YALM_PF_PERSIST=0: one
	// workgroup per tile; read per launch)
	const char *pe = getenv("YALM_PF_PERSIST");
	const int ncu = (int)device_cu_count();
	const int grid = (!pe || atoi(pe) != 0) && nwg > ncu ? ncu : nwg;
	hipLaunchKernelGGL(kern, dim3(grid), dim3(pf::G_THREADS), lds, st, A, M, K, bm, N, epi, c0);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// c0: first output column of the launch (8-phase kernel only; the 2-phase kernels start at 0)
template <class EPI, class BMAP, int BN, int WM>
int launch_g16_t(const uint16_t *A, int M, int K, const BMAP &bm, int N, const EPI &epi, hipStream_t st, int c0 = 0) {
	if (use_8phase()) { // the 8-phase schedule at the same tile width (320: spills, stays 2-phase)
		if constexpr (BN == 256 && WM == 2)
			return launch_g8p<EPI, BMAP, 2, 2>(A, M, K, bm, N, epi, st, c0);
		if constexpr (BN == 192 && WM == 2)
			return launch_g8p<EPI, BMAP, 2, 1>(A, M, K, bm, N, epi, st, c0);
		if constexpr (BN == 128 && std::is_same<BMAP, pf::BRowsPlain>::value) // GLU rows pair per 64-col wave
			return launch_g8p<EPI, BMAP, 1, 1>(A, M, K, bm, N, epi, st, c0);
	}
	if (c0 != 0) {
		set_err("prefill GEMM: a column offset needs the 8-phase kernel");
		return YALM_ERR_UNSUPPORTED;
	}
	auto kern = pf::gemm16_kernel<EPI, BMAP, BN, WM>;
	constexpr size_t lds = pf::gemm16_lds<BN>();
	static bool attr = false;
	if (!attr) {
		HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		attr = true;
	}
	const int nwg = ((M + pf::G_BM - 1) / pf::G_BM) * (N / BN);
	hipLaunchKernelGGL(kern, dim3(nwg), dim3(pf::G_THREADS), lds, st, A, M, K, bm, N, epi);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// C = A · W^T through the large-tile kernel at width bn (pick_bn); done = false
// when bn is 0 (the caller launches gemm_nt_kernel).
template <class EPI>
int launch_g16_plain(int bn, const uint16_t *A, int M, int K, const pf::BSrc &b, int N, const EPI &epi,
                     hipStream_t st, bool &done, int c0 = 0) {
	pf::BRowsPlain bm{b};
	done = true;
	switch (bn) {
	case 128:
		return launch_g16_t<EPI, pf::BRowsPlain, 128, 4>(A, M, K, bm, N, epi, st, c0);
	case 192:
		return launch_g16_t<EPI, pf::BRowsPlain, 192, 2>(A, M, K, bm, N, epi, st, c0);
	case 256:
		return launch_g16_t<EPI, pf::BRowsPlain, 256, 2>(A, M, K, bm, N, epi, st, c0);
	case 320:
		return launch_g16_t<EPI, pf::BRowsPlain, 320, 2>(A, M, K, bm, N, epi, st, c0);
	}
	done = false;
	return YALM_OK;
}

pf::BSrc one(const void *w, int rows) {
	pf::BSrc b{};
	b.p[0] = b.p[1] = b.p[2] = (const uint16_t *)w;
	b.end[0] = b.end[1] = b.end[2] = rows;
	return b;
}

int launch_attn_prefill(const uint16_t *Q, const uint16_t *kc, const uint16_t *vc, int T, int pos0, int n_heads,
                        int n_kv, int head_dim, uint16_t *O, hipStream_t st) {
	const dim3 grid(n_heads, (T + pf::AQ - 1) / pf::AQ); // heads fastest: longest-first dispatch
	static bool attr_set = false;
	if (!attr_set) {
		HIPCHK(hipFuncSetAttribute((const void *)pf::attn_prefill_kernel<128>,
		                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)pf::attn_prefill_lds<128>()));
		HIPCHK(hipFuncSetAttribute((const void *)pf::attn_prefill_kernel<64>,
		                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)pf::attn_prefill_lds<64>()));
		attr_set = true;
	}
	if (head_dim == 128)
		pf::attn_prefill_kernel<128><<<grid, pf::THREADS, pf::attn_prefill_lds<128>(), st>>>(Q, kc, vc, T, pos0,
		                                                                                       n_heads, n_kv, O);
	else if (head_dim == 64)
		pf::attn_prefill_kernel<64><<<grid, pf::THREADS, pf::attn_prefill_lds<64>(), st>>>(Q, kc, vc, T, pos0,
		                                                                                     n_heads, n_kv, O);
	else {
		set_err("prefill attention: head_dim must be 64 or 128");
		return YALM_ERR_UNSUPPORTED;
	}
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

int check_prefill_shape(const yalm_config &c) {
	const int q_dim = c.n_heads * c.head_dim, kv_dim = c.n_kv_heads * c.head_dim;
	if (c.weight_dtype != YALM_F16) {
		set_err("yalm_prefill: f16 weights only (MFMA f16 operands)");
		return YALM_ERR_UNSUPPORTED;
	}
	if (c.dim % pf::BN || c.dim % pf::BK || c.hidden_dim % pf::BN || c.hidden_dim % pf::BK || q_dim % pf::BN ||
	    q_dim % pf::BK || kv_dim % pf::BN || c.vocab_size % pf::BN || (c.head_dim != 64 && c.head_dim != 128)) {
		set_err("yalm_prefill: dims must be multiples of 128 and head_dim 64 or 128");
		return YALM_ERR_UNSUPPORTED;
	}
	return YALM_OK;
}

int ensure_bufs(yalm_decoder_s *d) {
	PrefillBufs &b = d->pf;
	if (b.cap)
		return YALM_OK;
	const yalm_config &c = d->c;
	const size_t cap = (size_t)c.max_seq_len, q_dim = (size_t)c.n_heads * c.head_dim;
	const size_t ntiles = (size_t)c.vocab_size / pf::BN;
	TRY(pf_alloc(d, (void **)&b.X, cap * c.dim * 4));
	TRY(pf_alloc(d, (void **)&b.Xn, cap * c.dim * 2));
	TRY(pf_alloc(d, (void **)&b.Q, cap * q_dim * 2));
	TRY(pf_alloc(d, (void **)&b.O, cap * q_dim * 2));
	TRY(pf_alloc(d, (void **)&b.H, cap * c.hidden_dim * 2));
	TRY(pf_alloc(d, (void **)&b.tok, cap * 4));
	TRY(pf_alloc(d, (void **)&b.tgt, cap * 4));
	TRY(pf_alloc(d, (void **)&b.pmax, cap * ntiles * 4));
	TRY(pf_alloc(d, (void **)&b.psum, cap * ntiles * 4));
	TRY(pf_alloc(d, (void **)&b.tgt_logit, cap * 4));
	TRY(pf_alloc(d, (void **)&b.lp, cap * 4));
	TRY(pf_alloc(d, (void **)&b.rope, cap * c.head_dim * 4));
	b.cap = (int)cap;
	return YALM_OK;
}

template <int ACT>
int enqueue_glu(yalm_decoder_s *d, const yalm_block_weights &w, int T) {
	const yalm_config &c = d->c;
	const int bn = pick_bn(g16_form(PG_GLU), T, 2 * c.hidden_dim, true);
	if (bn) {
		pf::E16Glu<ACT> e;
		e.h = d->pf.H;
		e.ldh = c.hidden_dim;
		e.M = T;
		pf::BRowsGlu<64> bm{(const uint16_t *)w.w1, (const uint16_t *)w.w3};
		if (bn == 256)
			return launch_g16_t<pf::E16Glu<ACT>, pf::BRowsGlu<64>, 256, 2>(d->pf.Xn, T, c.dim, bm, 2 * c.hidden_dim,
			                                                             e, d->stream);
		return launch_g16_t<pf::E16Glu<ACT>, pf::BRowsGlu<64>, 128, 4>(d->pf.Xn, T, c.dim, bm, 2 * c.hidden_dim, e,
		                                                             d->stream);
	}
	pf::EpiGlu<ACT> e;
	e.h = d->pf.H;
	e.ldh = c.hidden_dim;
	e.M = T;
	return launch_gemm<pf::EpiGlu<ACT>, 2>(d->pf.Xn, T, c.dim, one(w.w1, c.hidden_dim), one(w.w3, c.hidden_dim),
	                                       c.hidden_dim, e, d->stream);
}

// The whole prefill on d->stream: T rows at positions pos0 .. pos0 + T - 1.
int enqueue_prefill(yalm_decoder_s *d, int T, int pos0, bool want_lp) {
	const yalm_config &c = d->c;
	PrefillBufs &b = d->pf;
	hipStream_t st = d->stream;
	const int q_dim = c.n_heads * c.head_dim, kv_dim = c.n_kv_heads * c.head_dim;
	pf::embed_rows_kernel<WF16><<<T, 256, 0, st>>>(b.tok, d->emb, c.dim, b.X);
	HIPCHK(hipGetLastError());
	const int half = c.head_dim / 2;
	pf::rope_table_kernel<<<(T * half + 255) / 256, 256, 0, st>>>(d->inv_freq, half, T, pos0, b.rope);
	HIPCHK(hipGetLastError());
	for (int l = 0; l < c.n_layers; ++l) {
		const yalm_block_weights &w = d->b[l];
		pf::rmsnorm_rows_kernel<<<T, 256, 0, st>>>(b.X, w.rms_att, c.dim, c.norm_eps, b.Xn);
		HIPCHK(hipGetLastError());
		{
			pf::BSrc qkv{};
			qkv.p[0] = (const uint16_t *)w.wq;
			qkv.p[1] = (const uint16_t *)w.wk;
			qkv.p[2] = (const uint16_t *)w.wv;
			qkv.end[0] = q_dim;
			qkv.end[1] = q_dim + kv_dim;
			qkv.end[2] = q_dim + 2 * kv_dim;
			bool done = false;
			{
				pf::E16QKV e;
				e.q = b.Q;
				e.kc = w.key_cache;
				e.vc = w.value_cache;
				e.rope = b.rope;
				e.M = T;
				e.q_dim = q_dim;
				e.kv_dim = kv_dim;
				e.head_dim = c.head_dim;
				e.pos0 = pos0;
				e.clip = c.qkv_clip;
				// one launch over [q | k | v], or (8-phase, auto widths) a q launch and a k | v launch
				// when their tiles fill whole rounds better (Llama-3B T 4096: N 5120 = 16 x 320
				// 2-phase tiles, or q 16 x 192 + k | v 16 x 128 8-phase tiles); YALM_PF_QKV_SPLIT
				// = 0 | 1 forces (read per launch)
				long c_one = 0, c_q = 0, c_kv = 0;
				const int form = g16_form(PG_QKV);
				const int bn_one = pick_bn(form, T, q_dim + 2 * kv_dim, false, &c_one);
				int bn_q = 0, bn_kv = 0;
				if (use_8phase() && form < 0) {
					bn_q = pick_bn(-1, T, q_dim, false, &c_q);
					bn_kv = pick_bn(-1, T, 2 * kv_dim, false, &c_kv);
					if (bn_kv == 320)
						bn_kv = 0; // the k | v launch starts at column q_dim: 8-phase widths only
				}
				const char *se = getenv("YALM_PF_QKV_SPLIT");
				const bool split = bn_q && bn_kv && (se ? atoi(se) != 0 : c_q + c_kv < c_one);
				if (split) {
					TRY(launch_g16_plain(bn_q, b.Xn, T, c.dim, qkv, q_dim, e, st, done));
					TRY(launch_g16_plain(bn_kv, b.Xn, T, c.dim, qkv, 2 * kv_dim, e, st, done, q_dim));
				} else {
					TRY(launch_g16_plain(bn_one, b.Xn, T, c.dim, qkv, q_dim + 2 * kv_dim, e, st, done));
				}
			}
			pf::EpiQKV e;
			e.q = b.Q;
			e.kc = w.key_cache;
			e.vc = w.value_cache;
			e.rope = b.rope;
			e.M = T;
			e.q_dim = q_dim;
			e.kv_dim = kv_dim;
			e.head_dim = c.head_dim;
			e.pos0 = pos0;
			e.clip = c.qkv_clip;
			if (!done)
				TRY((launch_gemm<pf::EpiQKV, 1>(b.Xn, T, c.dim, qkv, qkv, q_dim + 2 * kv_dim, e, st)));
		}
		TRY(launch_attn_prefill(b.Q, w.key_cache, w.value_cache, T, pos0, c.n_heads, c.n_kv_heads, c.head_dim, b.O,
		                        st));
		{
			pf::EpiResidual e;
			e.x = b.X;
			e.ldx = c.dim;
			e.M = T;
			pf::E16Residual e16;
			e16.x = b.X;
			e16.ldx = c.dim;
			e16.M = T;
			bool done = false;
			TRY(launch_g16_plain(pick_bn(g16_form(PG_WO), T, c.dim, false), b.O, T, q_dim, one(w.wo, c.dim), c.dim, e16,
			                     st, done));
			if (!done)
				TRY((launch_gemm<pf::EpiResidual, 1>(b.O, T, q_dim, one(w.wo, c.dim), one(w.wo, c.dim), c.dim, e, st)));
		}
		pf::rmsnorm_rows_kernel<<<T, 256, 0, st>>>(b.X, w.rms_ffn, c.dim, c.norm_eps, b.Xn);
		HIPCHK(hipGetLastError());
		TRY(c.act == YALM_SILU ? enqueue_glu<1>(d, w, T) : enqueue_glu<0>(d, w, T));
		{
			pf::EpiResidual e;
			e.x = b.X;
			e.ldx = c.dim;
			e.M = T;
			pf::E16Residual e16;
			e16.x = b.X;
			e16.ldx = c.dim;
			e16.M = T;
			bool done = false;
			TRY(launch_g16_plain(pick_bn(g16_form(PG_W2), T, c.dim, false), b.H, T, c.hidden_dim, one(w.w2, c.dim), c.dim,
			                     e16, st, done));
			if (!done)
				TRY((launch_gemm<pf::EpiResidual, 1>(b.H, T, c.hidden_dim, one(w.w2, c.dim), one(w.w2, c.dim), c.dim, e,
				                                     st)));
		}
	}
	if (!want_lp)
		return YALM_OK;
	pf::rmsnorm_rows_kernel<<<T, 256, 0, st>>>(b.X, d->rms_final, c.dim, c.norm_eps, b.Xn);
	HIPCHK(hipGetLastError());
	const int cls_bn = pick_bn(g16_form(PG_CLS), T, c.vocab_size, false);
	const bool cls16 = cls_bn != 0;
	const int ntiles = c.vocab_size / (cls16 ? cls_bn : pf::BN);
	if (cls16) {
		pf::E16Logits e;
		e.pmax = b.pmax;
		e.psum = b.psum;
		e.tgt_logit = b.tgt_logit;
		e.targets = b.tgt;
		e.M = T;
		e.ntiles = ntiles;
		e.red = nullptr;
		bool done = false;
		TRY(launch_g16_plain(cls_bn, b.Xn, T, c.dim, one(d->wcls, c.vocab_size), c.vocab_size, e, st, done));
		pf::logprob_kernel<<<T, 256, 0, st>>>(b.pmax, b.psum, b.tgt_logit, b.tgt, T, ntiles, b.lp);
		HIPCHK(hipGetLastError());
		return YALM_OK;
	}
	pf::EpiLogits e;
	e.pmax = b.pmax;
	e.psum = b.psum;
	e.tgt_logit = b.tgt_logit;
	e.targets = b.tgt;
	e.M = T;
	e.ntiles = ntiles;
	e.red = nullptr;
	TRY((launch_gemm<pf::EpiLogits, 1>(b.Xn, T, c.dim, one(d->wcls, c.vocab_size), one(d->wcls, c.vocab_size),
	                                   c.vocab_size, e, st)));
	pf::logprob_kernel<<<T, 256, 0, st>>>(b.pmax, b.psum, b.tgt_logit, b.tgt, T, ntiles, b.lp);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

struct HostDev { // scoped device copy for the test hooks
	void *p = nullptr;
	~HostDev() {
		if (p)
			(void)hipFree(p);
	}
};
int hd(HostDev &b, const void *host, size_t bytes) {
	HIPCHK(hipMalloc(&b.p, bytes ? bytes : 4));
	if (host)
		HIPCHK(hipMemcpy(b.p, host, bytes, hipMemcpyHostToDevice));
	else
		HIPCHK(hipMemset(b.p, 0, bytes));
	return YALM_OK;
}

} // namespace

extern "C" int yalm_prefill(yalm_decoder d, const int *tokens, int n, int pos0, float *logprobs) {
	ARGCHK(d && tokens && n > 0 && pos0 >= 0, "yalm_prefill: bad argument");
	const yalm_config &c = d->c;
	ARGCHK(pos0 + n <= c.max_seq_len, "yalm_prefill: pos0 + n must be <= max_seq_len (no sliding window in prefill)");
	TRY(check_prefill_shape(c));
	TRY(ensure_bufs(d));
	PrefillBufs &b = d->pf;
	std::vector<int> tgt(n);
	for (int i = 0; i < n; ++i) {
		ARGCHK(tokens[i] >= 0 && tokens[i] < c.vocab_size, "yalm_prefill: token id out of range");
		tgt[i] = i + 1 < n ? tokens[i + 1] : -1;
	}
	HIPCHK(hipMemcpyAsync(b.tok, tokens, sizeof(int) * n, hipMemcpyHostToDevice, d->stream));
	HIPCHK(hipMemcpyAsync(b.tgt, tgt.data(), sizeof(int) * n, hipMemcpyHostToDevice, d->stream));
	TRY(enqueue_prefill(d, n, pos0, logprobs != nullptr));
	if (logprobs)
		HIPCHK(hipMemcpyAsync(logprobs, b.lp, sizeof(float) * n, hipMemcpyDeviceToHost, d->stream));
	HIPCHK(hipStreamSynchronize(d->stream));
	return YALM_OK;
}

extern "C" int yalm_prefill_time(yalm_decoder d, int n, int iters, float *avg_ms) {
	ARGCHK(d && n > 0 && iters > 0 && avg_ms, "yalm_prefill_time: bad argument");
	const yalm_config &c = d->c;
	ARGCHK(n <= c.max_seq_len, "yalm_prefill_time: n > max_seq_len");
	TRY(check_prefill_shape(c));
	TRY(ensure_bufs(d));
	std::vector<int> tok(n);
	for (int i = 0; i < n; ++i)
		tok[i] = (int)((1103515245u * (unsigned)i + 12345u) % (unsigned)c.vocab_size);
	HIPCHK(hipMemcpy(d->pf.tok, tok.data(), sizeof(int) * n, hipMemcpyHostToDevice));
	for (int i = 0; i < n; ++i)
		tok[i] = i + 1 < n ? tok[i + 1] : -1;
	HIPCHK(hipMemcpy(d->pf.tgt, tok.data(), sizeof(int) * n, hipMemcpyHostToDevice));
	TRY(enqueue_prefill(d, n, 0, true)); // warm-up
	hipEvent_t e0, e1;
	HIPCHK(hipEventCreate(&e0));
	HIPCHK(hipEventCreate(&e1));
	HIPCHK(hipEventRecord(e0, d->stream));
	for (int i = 0; i < iters; ++i)
		TRY(enqueue_prefill(d, n, 0, true));
	HIPCHK(hipEventRecord(e1, d->stream));
	HIPCHK(hipEventSynchronize(e1));
	float ms = 0;
	HIPCHK(hipEventElapsedTime(&ms, e0, e1));
	(void)hipEventDestroy(e0);
	(void)hipEventDestroy(e1);
	*avg_ms = ms / iters;
	return YALM_OK;
}

extern "C" int yalm_gemm_f16(float *c, const uint16_t *a, const uint16_t *w, int M, int N, int K) {
	ARGCHK(c && a && w && M > 0 && N > 0 && K > 0, "yalm_gemm_f16: bad argument");
	ARGCHK(N % pf::BN == 0 && K % pf::BK == 0, "yalm_gemm_f16: N % 128 and K % 64 must be 0");
	HostDev da, dw, dc;
	TRY(hd(da, a, (size_t)M * K * 2));
	TRY(hd(dw, w, (size_t)N * K * 2));
	TRY(hd(dc, nullptr, (size_t)M * N * 4));
	pf::E16StoreF32 e16;
	e16.c = (float *)dc.p;
	e16.ldc = N;
	e16.M = M;
	bool done = false;
	TRY(launch_g16_plain(pick_bn(g16_form(PG_TEST), M, N, false), (const uint16_t *)da.p, M, K, one(dw.p, N), N, e16,
	                     nullptr, done));
	pf::EpiStoreF32 e;
	e.c = (float *)dc.p;
	e.ldc = N;
	e.M = M;
	if (!done)
		TRY((launch_gemm<pf::EpiStoreF32, 1>((const uint16_t *)da.p, M, K, one(dw.p, N), one(dw.p, N), N, e, nullptr)));
	HIPCHK(hipDeviceSynchronize());
	HIPCHK(hipMemcpy(c, dc.p, (size_t)M * N * 4, hipMemcpyDeviceToHost));
	return YALM_OK;
}

extern "C" int yalm_attn_prefill(uint16_t *o, const uint16_t *q, const uint16_t *kc, const uint16_t *vc, int T,
                                 int pos0, int n_heads, int n_kv_heads, int head_dim) {
	ARGCHK(o && q && kc && vc && T > 0 && pos0 >= 0 && n_kv_heads > 0 && n_heads % n_kv_heads == 0,
	       "yalm_attn_prefill: bad argument");
	const size_t q_dim = (size_t)n_heads * head_dim, kv = (size_t)(pos0 + T) * n_kv_heads * head_dim;
	HostDev dq, dk, dv, dout;
	TRY(hd(dq, q, T * q_dim * 2));
	TRY(hd(dk, kc, kv * 2));
	TRY(hd(dv, vc, kv * 2));
	TRY(hd(dout, nullptr, T * q_dim * 2));
	TRY(launch_attn_prefill((const uint16_t *)dq.p, (const uint16_t *)dk.p, (const uint16_t *)dv.p, T, pos0, n_heads,
	                        n_kv_heads, head_dim, (uint16_t *)dout.p, nullptr));
	HIPCHK(hipDeviceSynchronize());
	HIPCHK(hipMemcpy(o, dout.p, T * q_dim * 2, hipMemcpyDeviceToHost));
	return YALM_OK;
}
