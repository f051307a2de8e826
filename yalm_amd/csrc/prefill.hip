// prefill.hip — C ABI of the batched prefill / perplexity path (prefill.h):
// yalm_prefill (prompt hydration + per-position log p(next), replacing the
// reference's position-by-position loop in main.cpp:128-200 / 91-97) and
// its kernel-level test hooks (yalm_gemm_f16, yalm_attn_prefill).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "decoder.h"
#include "prefill.h"
#include "prefill_gemm.h"
#include "prefill_skinny.h"

// Large-tile GEMM form per GEMM kind (prefill_gemm.h): the tile width BN of the
// 256-row tile. Default: auto -- the BN dividing N that minimises rounds x (BN + 64),
// rounds = ceil(tiles / CUs): a 256-CU chip should get whole rounds of large tiles
// (Llama-3B Wo / W2 N 3072 -> 192). Other exact forms (the tests, ablations) are chosen
// explicitly through yalm_set_prefill_forms: "qkv:256,wo:128,..." forces widths, 8p:0
// the 2-phase kernel, persist:0 one workgroup per tile, skinny:0 the large tiles at
// T <= 64 too (prefill_skinny.h otherwise), qkv1:0 the q and k | v GEMMs as two
// launches, skl:0 the skinny GEMMs' weights as register loads instead of LDS-DMA stages,
// wnorm:0 the workgroup-per-row norm kernel instead of one wave per row.
// The production library reads no environment for them; the A/B build (-DYALM_AB)
// takes a decoder's initial forms from YALM_PF_FORMS (same syntax).
static int parse_pf_forms(const char *spec, PfForms &f) {
	static const char *names[6] = {"qkv", "wo", "glu", "w2", "cls", "test"};
	f = PfForms{};
	if (!spec)
		return YALM_OK;
	const char *p = spec;
	while (*p) {
		char key[16];
		int val = 0, n = 0;
		if (sscanf(p, "%15[^:,]:%d%n", key, &val, &n) != 2) {
			set_err(std::string("yalm_set_prefill_forms: bad spec at '") + p + "'");
			return YALM_ERR_ARG;
		}
		bool known = false;
		for (int k = 0; k < 6; ++k)
			if (!strcmp(key, names[k])) {
				ARGCHK(val == 128 || val == 192 || val == 256 || val == 320,
				       "yalm_set_prefill_forms: a tile width is 128, 192, 256 or 320");
				f.g16[k] = val;
				known = true;
			}
		if (!strcmp(key, "8p"))
			f.p8 = val != 0, known = true;
		else if (!strcmp(key, "persist"))
			f.persist = val != 0, known = true;
		else if (!strcmp(key, "skinny"))
			f.no_skinny = val == 0, known = true;
		else if (!strcmp(key, "qkv1"))
			f.qkv1 = val != 0, known = true;
		else if (!strcmp(key, "skl"))
			f.skl = val != 0, known = true;
		else if (!strcmp(key, "split"))
			f.split = val != 0, known = true;
		else if (!strcmp(key, "wnorm"))
			f.wnorm = val != 0, known = true;
		if (!known) {
			set_err(std::string("yalm_set_prefill_forms: unknown key '") + key + "'");
			return YALM_ERR_ARG;
		}
		p += n;
		if (*p == ',')
			++p;
	}
	return YALM_OK;
}

PfForms pf_forms_default() {
	PfForms f;
	if (parse_pf_forms(ab_env("YALM_PF_FORMS"), f) != YALM_OK)
		f = PfForms{};
	return f;
}

static PfForms g_test_forms; // the forms of the yalm_gemm_f16 test hook

extern "C" int yalm_set_prefill_precision(yalm_decoder d, int mode) {
	ARGCHK(d && (mode == YALM_PREFILL_FAST || mode == YALM_PREFILL_SPLIT), "yalm_set_prefill_precision: bad argument");
	d->pf_forms.split = mode == YALM_PREFILL_SPLIT;
	return YALM_OK;
}

extern "C" int yalm_set_prefill_forms(yalm_decoder d, const char *spec) {
	PfForms f;
	TRY(parse_pf_forms(spec, f));
	if (d)
		d->pf_forms = f;
	else
		g_test_forms = f;
	return YALM_OK;
}

namespace {

enum { PG_QKV = 0, PG_WO = 1, PG_GLU = 2, PG_W2 = 3, PG_CLS = 4, PG_TEST = 5 };
// range-guard slots per layer (PrefillBufs::range), in the order the pass produces them;
// the final norm's operand is slot RG_XATT of row n_layers
enum { RG_XATT = 0, RG_Q = 1, RG_XFFN = 2, RG_H = 3, RG_N = 4 };

int pf_alloc(yalm_decoder_s *d, void **p, size_t bytes) {
	HIPCHK(hipMalloc(p, bytes ? bytes : 4));
	d->dev_allocs.push_back(*p);
	return YALM_OK;
}

// BN for a GEMM of M x N (n_eff = B rows: 2 x hidden for the GLU); 0 = none fits. A
// forced width that does not divide N falls back to the automatic choice.
int pick_bn(const PfForms &f, int kind, int M, int n_eff, bool glu) {
	static const int cands[4] = {128, 192, 256, 320};
	auto fits = [&](int bn) { return n_eff % bn == 0 && (!glu || bn == 128 || bn == 256); };
	const int form = f.g16[kind];
	if (form > 0 && fits(form) && (form == 128 || form == 192 || form == 256 || form == 320))
		return form;
	const long ncu = device_cu_count();
	const long tiles_m = (M + pf::G_BM - 1) / pf::G_BM;
	int best = 0;
	long best_cost = 0;
	for (int bn : cands) {
		if (!fits(bn))
			continue;
		const long rounds = (tiles_m * (n_eff / bn) + ncu - 1) / ncu;
		// an 8-phase tile (widths 192, 256) costs 3/4 of a 2-phase tile of the same
		// width (Llama-3B T 4096, one process: Wo / W2 at 256 in the 8-phase kernel beat
		// 192 in the 2-phase one, profiles/r3_prefill_8phase.txt)
		const long cost = rounds * (bn + 64) * (f.p8 && (bn == 192 || bn == 256) ? 3 : 4);
		if (!best || cost < best_cost || (cost == best_cost && bn > best)) {
			best = bn;
			best_cost = cost;
		}
	}
	return best;
}

// c_split / K2: columns [c_split, N) run K2 (gemm8p_kernel); c_split = N: one depth
template <class EPI, class BMAP, int FJ0, int FJ1>
int launch_g8p(const PfForms &f, const uint16_t *A, int lda, int M, int K, int kb, const BMAP &bm, int N,
               const EPI &epi, hipStream_t st, int c0, int c_split = -1, int K2 = 0) {
	auto kern = pf::gemm8p_kernel<EPI, BMAP, FJ0, FJ1>;
	constexpr size_t lds = pf::gemm8p_lds<FJ0, FJ1>();
	constexpr int BN = 64 * (FJ0 + FJ1);
	static bool attr = false;
	if (!attr) {
		HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		attr = true;
	}
	const int nwg = ((M + pf::G_BM - 1) / pf::G_BM) * (N / BN);
	// more tiles than CUs: one persistent workgroup per CU walks them
	const int ncu = (int)device_cu_count();
	// (two depths: one workgroup per tile, so the hardware balances them longest first)
	const bool two = c_split >= 0 && c_split < N;
	const int grid = f.persist && nwg > ncu && !two ? ncu : nwg;
	hipLaunchKernelGGL(kern, dim3(grid), dim3(pf::G_THREADS), lds, st, A, lda, M, K, kb, bm, N, epi, c0,
	                   two ? c_split : N, two ? K2 : K);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// C[:, c0 .. c0 + N) = A · B^T over K columns of A (row stride lda) against B rows kb
// wide (K > kb: B wrap, prefill_gemm.h), tile 256 x BN
template <class EPI, class BMAP, int BN, int WM>
int launch_g16_t(const PfForms &f, const uint16_t *A, int lda, int M, int K, int kb, const BMAP &bm, int N,
                 const EPI &epi, hipStream_t st, int c0 = 0) {
	if (f.p8) { // the 8-phase schedule at the same tile width (320: spills, stays 2-phase)
		if constexpr (BN == 256 && WM == 2)
			return launch_g8p<EPI, BMAP, 2, 2>(f, A, lda, M, K, kb, bm, N, epi, st, c0);
		if constexpr (BN == 192 && WM == 2)
			return launch_g8p<EPI, BMAP, 2, 1>(f, A, lda, M, K, kb, bm, N, epi, st, c0);
		if constexpr (BN == 128 && std::is_same<BMAP, pf::BRowsPlain>::value) // GLU rows pair per 64-col wave
			return launch_g8p<EPI, BMAP, 1, 1>(f, A, lda, M, K, kb, bm, N, epi, st, c0);
	}
	auto kern = pf::gemm16_kernel<EPI, BMAP, BN, WM>;
	constexpr size_t lds = pf::gemm16_lds<BN>();
	static bool attr = false;
	if (!attr) {
		HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		attr = true;
	}
	const int nwg = ((M + pf::G_BM - 1) / pf::G_BM) * (N / BN);
	hipLaunchKernelGGL(kern, dim3(nwg), dim3(pf::G_THREADS), lds, st, A, lda, M, K, kb, bm, N, epi, c0);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// C = A · W^T through the large-tile kernel at width bn (pick_bn; 0: no width fits)
template <class EPI>
int launch_plain(const PfForms &f, int bn, const uint16_t *A, int lda, int M, int K, int kb, const pf::BSrc &b,
                 int N, const EPI &epi, hipStream_t st, int c0 = 0) {
	pf::BRowsPlain bm{b};
	switch (bn) {
	case 128:
		return launch_g16_t<EPI, pf::BRowsPlain, 128, 4>(f, A, lda, M, K, kb, bm, N, epi, st, c0);
	case 192:
		return launch_g16_t<EPI, pf::BRowsPlain, 192, 2>(f, A, lda, M, K, kb, bm, N, epi, st, c0);
	case 256:
		return launch_g16_t<EPI, pf::BRowsPlain, 256, 2>(f, A, lda, M, K, kb, bm, N, epi, st, c0);
	case 320:
		return launch_g16_t<EPI, pf::BRowsPlain, 320, 2>(f, A, lda, M, K, kb, bm, N, epi, st, c0);
	}
	set_err("prefill GEMM: no 256-row tile width (128 / 192 / 256 / 320) divides N, or the forced one does not");
	return YALM_ERR_UNSUPPORTED;
}

// ---- short prompts (T <= SK_MAX_T): split-K skinny GEMMs (prefill_skinny.h)
constexpr int SK_MAX_T = 64;

// K splits of a skinny GEMM: every K chunk a multiple of the kernel's 256-column step
// and <= 64 KB of A rows in LDS; the fewest splits that give >= 512 workgroups (the
// weight stream needs the whole chip), else the most. kn: (N, K, mult) of each GEMM
// sharing one partial buffer, split mult x KS ways (the k | v GEMM over [hi | lo], K =
// 2 dim, takes 2 KS splits of the q GEMM's chunk size, so no chunk straddles the B
// wrap at dim).
struct SkGemm {
	int N, K, mult;
};
int sk_pick_ks(std::initializer_list<SkGemm> kn, int TP) {
	int best = -1, kmin = 1 << 30, wg1 = 0;
	for (auto &p : kn) {
		kmin = std::min(kmin, p.K / p.mult);
		wg1 += p.N / pf::SK_ROWS * p.mult;
	}
	for (int ks = 1; ks <= kmin / pf::SK_KSTEP; ++ks) {
		bool ok = true;
		for (auto &p : kn) {
			const int s = ks * p.mult;
			ok = ok && p.K % s == 0 && (p.K / s) % pf::SK_KSTEP == 0 && (size_t)TP * (p.K / s) * 2 <= 32768;
		}
		if (!ok)
			continue;
		best = ks;
		if (wg1 * ks >= 512)
			break;
	}
	return best;
}

template <int MT, class BMAP>
int launch_skinny_mt(const PfForms &f, const uint16_t *A, int lda, int T, int K, int kb, const BMAP &bm, int N,
                     int KS, int c0, int Np, float *part, hipStream_t st) {
	auto kern = f.skl ? pf::skinny_gemm_lds_kernel<MT, BMAP> : pf::skinny_gemm_kernel<MT, BMAP>;
	static bool attr[2] = {false, false};
	if (!attr[f.skl]) {
		HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
		                           32768 + (int)pf::SKL_RING_BYTES));
		attr[f.skl] = true;
	}
	const int KC = K / KS;
	const size_t lds = (size_t)16 * MT * KC * sizeof(uint16_t) + (f.skl ? pf::SKL_RING_BYTES : 0);
	hipLaunchKernelGGL(kern, dim3((N / pf::SK_ROWS) * KS), dim3(256), lds, st, A, lda, T, K, kb, bm, N, KC, c0, Np,
	                   part);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

template <class BMAP>
int launch_skinny(const PfForms &f, const uint16_t *A, int lda, int T, int K, int kb, const BMAP &bm, int N, int KS,
                  int c0, int Np, float *part, hipStream_t st) {
	switch ((T + 15) / 16) {
	case 1:
		return launch_skinny_mt<1>(f, A, lda, T, K, kb, bm, N, KS, c0, Np, part, st);
	case 2:
		return launch_skinny_mt<2>(f, A, lda, T, K, kb, bm, N, KS, c0, Np, part, st);
	case 3:
		return launch_skinny_mt<3>(f, A, lda, T, K, kb, bm, N, KS, c0, Np, part, st);
	default:
		return launch_skinny_mt<4>(f, A, lda, T, K, kb, bm, N, KS, c0, Np, part, st);
	}
}

// columns < c_split sum KS partials, the others KS2
template <bool GLU, class EPI>
int launch_skinny_reduce(const float *part, int KS, int KS2, int c_split, int T, int Np, const EPI &epi,
                         hipStream_t st) {
	const int TP = 16 * ((T + 15) / 16);
	const int waves = (TP / 16) * (Np / 64);
	pf::skinny_reduce_kernel<4, GLU, EPI><<<(waves + 3) / 4, 256, 0, st>>>(part, KS, KS2, c_split, TP, T, Np, epi);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

pf::BSrc one(const void *w, int rows) {
	pf::BSrc b{};
	b.p[0] = b.p[1] = b.p[2] = (const uint16_t *)w;
	b.end[0] = b.end[1] = b.end[2] = rows;
	return b;
}

// fp8 models: the tensors (E5M2 bytes, n elements each) dequantised to f16 into b.wdq, end
// to end; returns their f16 copies in `out` (prefill.h e5m2_to_f16_kernel)
int dequant(yalm_decoder_s *d, std::initializer_list<std::pair<const void *, size_t>> t, const uint16_t **out,
			hipStream_t st) {
	pf::DqSegs s{};
	size_t off = 0, pieces = 0;
	for (auto &p : t) {
		s.src[s.n] = (const uint8_t *)p.first;
		s.dst[s.n] = d->pf.wdq + off;
		out[s.n] = s.dst[s.n];
		pieces += p.second / 16;
		s.end[s.n] = pieces;
		off += p.second;
		++s.n;
	}
	const int grid = (int)std::min<size_t>((pieces + 255) / 256, (size_t)device_cu_count() * 8);
	pf::e5m2_to_f16_kernel<<<grid, 256, 0, st>>>(s);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// Xn = f16(rmsnorm(X) * w) rows (SPLIT: [hi | lo]): one wave per row with the row in
// registers (prefill.h rmsnorm_rows_wave_kernel) when dim <= 8192, else (or forms "wnorm:0")
// the workgroup-per-row kernel
template <bool SPLIT>
int launch_rmsnorm_t(const PfForms &f, const float *X, const float *w, int dim, int T, float eps, uint16_t *Xn,
                     unsigned *range, hipStream_t st) {
	const int nv = (dim / 4 + 63) / 64; // float4 per lane
	const int g = (T + 3) / 4;
	if (f.wnorm && nv <= 32) {
		if (nv <= 4)
			pf::rmsnorm_rows_wave_kernel<SPLIT, 4><<<g, 256, 0, st>>>(X, w, dim, T, eps, Xn, range);
		else if (nv <= 8)
			pf::rmsnorm_rows_wave_kernel<SPLIT, 8><<<g, 256, 0, st>>>(X, w, dim, T, eps, Xn, range);
		else if (nv <= 12)
			pf::rmsnorm_rows_wave_kernel<SPLIT, 12><<<g, 256, 0, st>>>(X, w, dim, T, eps, Xn, range);
		else if (nv <= 16)
			pf::rmsnorm_rows_wave_kernel<SPLIT, 16><<<g, 256, 0, st>>>(X, w, dim, T, eps, Xn, range);
		else if (nv <= 24)
			pf::rmsnorm_rows_wave_kernel<SPLIT, 24><<<g, 256, 0, st>>>(X, w, dim, T, eps, Xn, range);
		else
			pf::rmsnorm_rows_wave_kernel<SPLIT, 32><<<g, 256, 0, st>>>(X, w, dim, T, eps, Xn, range);
	} else {
		pf::rmsnorm_rows_kernel<SPLIT><<<T, 256, 0, st>>>(X, w, dim, eps, Xn, range);
	}
	HIPCHK(hipGetLastError());
	return YALM_OK;
}
int launch_rmsnorm(bool split, const PfForms &f, const float *X, const float *w, int dim, int T, float eps, uint16_t *Xn,
                   unsigned *range, hipStream_t st) {
	return split ? launch_rmsnorm_t<true>(f, X, w, dim, T, eps, Xn, range, st)
	             : launch_rmsnorm_t<false>(f, X, w, dim, T, eps, Xn, range, st);
}

template <int D, bool SPLIT>
int launch_attn_prefill_t(const uint16_t *Q, const uint16_t *kc, const uint16_t *vc, int T, int pos0, int n_heads,
						  int n_kv, uint16_t *O, hipStream_t st) {
	const dim3 grid(n_heads, (T + pf::AQ - 1) / pf::AQ); // heads fastest: longest-first dispatch
	auto kern = pf::attn_prefill_kernel<D, pf::AKT, SPLIT>;
	static bool attr_set = false;
	if (!attr_set) {
		HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
								   (int)pf::attn_prefill_lds<D>()));
		attr_set = true;
	}
	hipLaunchKernelGGL(kern, grid, dim3(pf::THREADS), pf::attn_prefill_lds<D>(), st, Q, kc, vc, T, pos0, n_heads, n_kv,
					   O);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// split: Q and O rows [hi | lo] (the split-operand form)
int launch_attn_prefill(const uint16_t *Q, const uint16_t *kc, const uint16_t *vc, int T, int pos0, int n_heads,
						int n_kv, int head_dim, uint16_t *O, hipStream_t st, bool split = false) {
	if (head_dim == 128)
		return split ? launch_attn_prefill_t<128, true>(Q, kc, vc, T, pos0, n_heads, n_kv, O, st)
					 : launch_attn_prefill_t<128, false>(Q, kc, vc, T, pos0, n_heads, n_kv, O, st);
	if (head_dim == 64)
		return split ? launch_attn_prefill_t<64, true>(Q, kc, vc, T, pos0, n_heads, n_kv, O, st)
					 : launch_attn_prefill_t<64, false>(Q, kc, vc, T, pos0, n_heads, n_kv, O, st);
	set_err("prefill attention: head_dim must be 64 or 128");
	return YALM_ERR_UNSUPPORTED;
}

int check_prefill_shape(const yalm_config &c) {
	const int q_dim = c.n_heads * c.head_dim, kv_dim = c.n_kv_heads * c.head_dim;
	if (c.weight_dtype != YALM_F16 && c.weight_dtype != YALM_F8E5M2) {
		set_err("yalm_prefill: f16 or fp8 (E5M2) weights only (MFMA f16 operands)");
		return YALM_ERR_UNSUPPORTED;
	}
	if (c.dim % pf::BN || c.hidden_dim % pf::BN || q_dim % pf::BN || kv_dim % pf::BN || c.vocab_size % pf::BN ||
	    (c.head_dim != 64 && c.head_dim != 128)) {
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
	TRY(pf_alloc(d, (void **)&b.Xn, cap * c.dim * 2 * 2));
	// Q, O, H: [hi | lo] rows in the split-operand form, 2x wide
	TRY(pf_alloc(d, (void **)&b.Q, cap * q_dim * 2 * 2));
	TRY(pf_alloc(d, (void **)&b.O, cap * q_dim * 2 * 2));
	TRY(pf_alloc(d, (void **)&b.H, cap * c.hidden_dim * 2 * 2));
	TRY(pf_alloc(d, (void **)&b.tok, cap * 4));
	TRY(pf_alloc(d, (void **)&b.tgt, cap * 4));
	TRY(pf_alloc(d, (void **)&b.pmax, cap * ntiles * 4));
	TRY(pf_alloc(d, (void **)&b.psum, cap * ntiles * 4));
	TRY(pf_alloc(d, (void **)&b.tgt_logit, cap * 4));
	TRY(pf_alloc(d, (void **)&b.lp, cap * 4));
	TRY(pf_alloc(d, (void **)&b.rope, cap * c.head_dim * 4));
	TRY(pf_alloc(d, (void **)&b.range, (size_t)(c.n_layers + 1) * RG_N * 4));
	if (c.weight_dtype == YALM_F8E5M2) { // the f16 copy of one layer's weights, or of the classifier
		const size_t layer = ((size_t)q_dim + 2 * (size_t)c.n_kv_heads * c.head_dim) * c.dim + (size_t)c.dim * q_dim +
							 3 * (size_t)c.dim * c.hidden_dim;
		TRY(pf_alloc(d, (void **)&b.wdq, 2 * std::max(layer, (size_t)c.vocab_size * c.dim)));
	}
	{ // short-prompt split-K partials: the largest [KS][64][Np] of the layer's GEMMs
		const int kv_dim = c.n_kv_heads * c.head_dim, TP = SK_MAX_T;
		const int np_qkv = (int)q_dim + 2 * kv_dim;
		// (QKV: 2 KS partial slots, the k | v GEMM's)
		const size_t sz[4] = {
		    (size_t)2 * std::max(1, sk_pick_ks({{(int)q_dim, c.dim, 1}, {2 * kv_dim, 2 * c.dim, 2}}, TP)) * np_qkv,
		    (size_t)std::max(1, sk_pick_ks({{c.dim, (int)q_dim, 1}}, TP)) * c.dim,
		    (size_t)std::max(1, sk_pick_ks({{2 * c.hidden_dim, c.dim, 1}}, TP)) * 2 * c.hidden_dim,
		    (size_t)std::max(1, sk_pick_ks({{c.dim, c.hidden_dim, 1}}, TP)) * c.dim};
		b.skp_floats = (size_t)TP * *std::max_element(sz, sz + 4);
		TRY(pf_alloc(d, (void **)&b.skp, b.skp_floats * 4));
	}
	b.cap = (int)cap;
	return YALM_OK;
}

template <int ACT, bool SPLIT>
int enqueue_glu_t(yalm_decoder_s *d, const yalm_block_weights &w, int T, float hscale, unsigned *range) {
	const yalm_config &c = d->c;
	const PfForms &f = d->pf_forms;
	const int bn = pick_bn(f, PG_GLU, T, 2 * c.hidden_dim, true);
	const int sp = SPLIT ? 2 : 1; // split-operand form: A = [hi | lo] (K = 2 dim), H rows [hi | lo]
	pf::E16Glu<ACT, SPLIT> e;
	e.h = d->pf.H;
	e.ldh = c.hidden_dim * sp;
	e.M = T;
	e.hscale = hscale;
	e.range = range;
	e.lo_off = SPLIT ? c.hidden_dim : 0;
	pf::BRowsGlu<64> bm{(const uint16_t *)w.w1, (const uint16_t *)w.w3};
	if (bn == 256)
		return launch_g16_t<pf::E16Glu<ACT, SPLIT>, pf::BRowsGlu<64>, 256, 2>(f, d->pf.Xn, sp * c.dim, T, sp * c.dim, c.dim,
                                                                     bm, 2 * c.hidden_dim, e, d->stream);
	if (bn == 128)
		return launch_g16_t<pf::E16Glu<ACT, SPLIT>, pf::BRowsGlu<64>, 128, 4>(f, d->pf.Xn, sp * c.dim, T, sp * c.dim, c.dim,
                                                                     bm, 2 * c.hidden_dim, e, d->stream);
	set_err("prefill GLU GEMM: 2 x hidden_dim must divide by 128 (or by a forced width of 128 / 256)");
	return YALM_ERR_UNSUPPORTED;
}

template <int ACT>
int enqueue_glu(yalm_decoder_s *d, const yalm_block_weights &w, int T, float hscale, unsigned *range) {
	return d->pf_forms.split ? enqueue_glu_t<ACT, true>(d, w, T, hscale, range)
	                         : enqueue_glu_t<ACT, false>(d, w, T, hscale, range);
}

// The whole prefill on d->stream: T rows at positions pos0 .. pos0 + T - 1. hexp[l] (null:
// all 0): layer l's GLU output is stored as f16(h * 2^-hexp[l]) and W2 adds 2^hexp[l] x its
// product (exact power-of-two scales; yalm_prefill chooses them from the range guard).
int enqueue_prefill(yalm_decoder_s *d, int T, int pos0, bool want_lp, const int *hexp = nullptr) {
	const yalm_config &c = d->c;
	const PfForms &f = d->pf_forms;
	PrefillBufs &b = d->pf;
	hipStream_t st = d->stream;
	const int q_dim = c.n_heads * c.head_dim, kv_dim = c.n_kv_heads * c.head_dim;
	const bool fp8 = c.weight_dtype == YALM_F8E5M2;
	if (fp8)
		pf::embed_rows_kernel<WF8><<<T, 256, 0, st>>>(b.tok, d->emb, c.dim, b.X);
	else
		pf::embed_rows_kernel<WF16><<<T, 256, 0, st>>>(b.tok, d->emb, c.dim, b.X);
	HIPCHK(hipGetLastError());
	const int half = c.head_dim / 2;
	pf::rope_table_kernel<<<(T * half + 255) / 256, 256, 0, st>>>(d->inv_freq, half, T, pos0, b.rope);
	HIPCHK(hipGetLastError());
	// GEMM widths are the same for every layer
	const int bn_q = pick_bn(f, PG_QKV, T, q_dim, false);
	const int bn_kv = pick_bn(f, PG_QKV, T, 2 * kv_dim, false);
	// q and k | v in one two-depth launch at width 256 (gemm8p_kernel): the two launches'
	// tiles balanced over the chip instead of one round each (Llama-3B at T 4096: q 82 us
	// at width 192 + k | v 115 us at 128)
	const bool qkv1 = f.qkv1 && f.p8 && f.g16[PG_QKV] < 0 && q_dim % 256 == 0 && (2 * kv_dim) % 256 == 0;
	const int bn_wo = pick_bn(f, PG_WO, T, c.dim, false);
	const int bn_w2 = pick_bn(f, PG_W2, T, c.dim, false);
	// short prompts: split-K skinny GEMMs (the 256-row tiles would leave most CUs idle)
	const int TP = 16 * ((T + 15) / 16);
	const int ks_qkv = sk_pick_ks({{q_dim, c.dim, 1}, {2 * kv_dim, 2 * c.dim, 2}}, TP);
	const int ks_wo = sk_pick_ks({{c.dim, q_dim, 1}}, TP);
	const int ks_glu = sk_pick_ks({{2 * c.hidden_dim, c.dim, 1}}, TP);
	const int ks_w2 = sk_pick_ks({{c.dim, c.hidden_dim, 1}}, TP);
	const bool small = T <= SK_MAX_T && !f.no_skinny && !f.split && ks_qkv > 0 && ks_wo > 0 && ks_glu > 0 && ks_w2 > 0;
	// the split-operand precision form (yalm_set_prefill_precision): every activation operand
	// [hi | lo] -- the normalised x of all three norms, Q, P (attention.h SPLIT), O and H --
	// each GEMM over K = 2 x its depth with the B rows wrapping (prefill_gemm.h), so no operand
	// carries an f16 rounding the reference's f32 lacks; sp = operand width factor
	const bool split = f.split;
	const int sp = split ? 2 : 1;
	const int bn_qkv_all = pick_bn(f, PG_QKV, T, q_dim + 2 * kv_dim, false);
	for (int l = 0; l < c.n_layers; ++l) {
		yalm_block_weights w = d->b[l];
		if (fp8) { // this layer's weights as f16 (exact), in the scratch the previous layer's GEMMs are done with
			const uint16_t *p[7];
			const size_t qd = (size_t)q_dim * c.dim, kd = (size_t)kv_dim * c.dim, hd = (size_t)c.hidden_dim * c.dim;
			TRY(dequant(d, {{w.wq, qd}, {w.wk, kd}, {w.wv, kd}, {w.wo, qd}, {w.w1, hd}, {w.w2, hd}, {w.w3, hd}}, p, st));
			w.wq = p[0], w.wk = p[1], w.wv = p[2], w.wo = p[3], w.w1 = p[4], w.w2 = p[5], w.w3 = p[6];
		}
		// normalised x as [hi | lo] (2 dim per row): hi is the q columns' A operand, hi + lo
		// the k | v columns' (their cache rows then carry one f16 rounding, infer.cpp:299)
		unsigned *rg = b.range + (size_t)l * RG_N;
		const int he = hexp ? hexp[l] : 0;
		TRY(launch_rmsnorm(true, f, b.X, w.rms_att, c.dim, T, c.norm_eps, b.Xn, rg + RG_XATT, st));
		{
			pf::BSrc qkv{};
			qkv.p[0] = (const uint16_t *)w.wq;
			qkv.p[1] = (const uint16_t *)w.wk;
			qkv.p[2] = (const uint16_t *)w.wv;
			qkv.end[0] = q_dim;
			qkv.end[1] = q_dim + kv_dim;
			qkv.end[2] = q_dim + 2 * kv_dim;
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
			e.range = rg + RG_Q;
			// QKV + clip + RoPE as two GEMMs: q (K = dim over hi) and k | v from column
			// q_dim (K = 2 dim over hi | lo, the B rows wrapping at dim)
			if (small) {
				const pf::BRowsPlain bm{qkv};
				const int np = q_dim + 2 * kv_dim;
				TRY(launch_skinny(f, b.Xn, 2 * c.dim, T, c.dim, c.dim, bm, q_dim, ks_qkv, 0, np, b.skp, st));
				TRY(launch_skinny(f, b.Xn, 2 * c.dim, T, 2 * c.dim, c.dim, bm, 2 * kv_dim, 2 * ks_qkv, q_dim, np, b.skp,
				                  st));
				TRY(launch_skinny_reduce<false>(b.skp, ks_qkv, 2 * ks_qkv, q_dim, T, np, e, st));
			} else {
				if (split) { // q | k | v all over [hi | lo], Q stored [hi | lo]
					pf::E16QKVt<true> es;
					es.q = e.q, es.kc = e.kc, es.vc = e.vc, es.rope = e.rope, es.M = e.M, es.q_dim = e.q_dim;
					es.kv_dim = e.kv_dim, es.head_dim = e.head_dim, es.pos0 = e.pos0, es.clip = e.clip;
					es.range = e.range, es.q_lo = q_dim;
					TRY(launch_plain(f, bn_qkv_all, b.Xn, 2 * c.dim, T, 2 * c.dim, c.dim, qkv, q_dim + 2 * kv_dim, es, st));
				} else if (qkv1) { // one launch: the k | v tiles (K = 2 dim) first, then the q tiles (K = dim)
					TRY((launch_g8p<pf::E16QKV, pf::BRowsPlain, 2, 2>(f, b.Xn, 2 * c.dim, T, c.dim, c.dim,
					                                                   pf::BRowsPlain{qkv}, q_dim + 2 * kv_dim, e, st,
					                                                   0, q_dim, 2 * c.dim)));
				} else {
					TRY(launch_plain(f, bn_q, b.Xn, 2 * c.dim, T, c.dim, c.dim, qkv, q_dim, e, st));
					TRY(launch_plain(f, bn_kv, b.Xn, 2 * c.dim, T, 2 * c.dim, c.dim, qkv, 2 * kv_dim, e, st, q_dim));
				}
			}
		}
		TRY(launch_attn_prefill(b.Q, w.key_cache, w.value_cache, T, pos0, c.n_heads, c.n_kv_heads, c.head_dim, b.O,
								st, split));
		{
			pf::E16Residual e;
			e.x = b.X;
			e.ldx = c.dim;
			e.M = T;
			if (small) {
				TRY(launch_skinny(f, b.O, q_dim, T, q_dim, q_dim, pf::BRowsPlain{one(w.wo, c.dim)}, c.dim, ks_wo, 0, c.dim,
				                  b.skp, st));
				TRY(launch_skinny_reduce<false>(b.skp, ks_wo, ks_wo, c.dim, T, c.dim, e, st));
			} else {
				TRY(launch_plain(f, bn_wo, b.O, sp * q_dim, T, sp * q_dim, q_dim, one(w.wo, c.dim), c.dim, e, st));
			}
		}
		TRY(launch_rmsnorm(split, f, b.X, w.rms_ffn, c.dim, T, c.norm_eps, b.Xn, rg + RG_XFFN, st));
		const float hscale = ldexpf(1.0f, -he);
		if (small) {
			const pf::BRowsGlu<64> bm{(const uint16_t *)w.w1, (const uint16_t *)w.w3};
			TRY(launch_skinny(f, b.Xn, c.dim, T, c.dim, c.dim, bm, 2 * c.hidden_dim, ks_glu, 0, 2 * c.hidden_dim, b.skp,
			                  st));
			if (c.act == YALM_SILU) {
				pf::E16Glu<1> e;
				e.h = b.H, e.ldh = c.hidden_dim, e.M = T, e.hscale = hscale, e.range = rg + RG_H;
				TRY(launch_skinny_reduce<true>(b.skp, ks_glu, ks_glu, 2 * c.hidden_dim, T, 2 * c.hidden_dim, e, st));
			} else {
				pf::E16Glu<0> e;
				e.h = b.H, e.ldh = c.hidden_dim, e.M = T, e.hscale = hscale, e.range = rg + RG_H;
				TRY(launch_skinny_reduce<true>(b.skp, ks_glu, ks_glu, 2 * c.hidden_dim, T, 2 * c.hidden_dim, e, st));
			}
		} else {
			TRY(c.act == YALM_SILU ? enqueue_glu<1>(d, w, T, hscale, rg + RG_H)
								   : enqueue_glu<0>(d, w, T, hscale, rg + RG_H));
		}
		{
			pf::E16Residual e;
			e.x = b.X;
			e.ldx = c.dim;
			e.M = T;
			e.scale = ldexpf(1.0f, he);
			if (small) {
				TRY(launch_skinny(f, b.H, c.hidden_dim, T, c.hidden_dim, c.hidden_dim, pf::BRowsPlain{one(w.w2, c.dim)},
				                  c.dim, ks_w2, 0, c.dim, b.skp, st));
				TRY(launch_skinny_reduce<false>(b.skp, ks_w2, ks_w2, c.dim, T, c.dim, e, st));
			} else {
				TRY(launch_plain(f, bn_w2, b.H, sp * c.hidden_dim, T, sp * c.hidden_dim, c.hidden_dim, one(w.w2, c.dim),
								 c.dim, e, st));
			}
		}
	}
	if (!want_lp)
		return YALM_OK;
	TRY(launch_rmsnorm(split, f, b.X, d->rms_final, c.dim, T, c.norm_eps, b.Xn,
	                   b.range + (size_t)c.n_layers * RG_N + RG_XATT, st));
	const int cls_bn = pick_bn(f, PG_CLS, T, c.vocab_size, false);
	const int ntiles = cls_bn ? c.vocab_size / cls_bn : 1;
	pf::E16Logits e;
	e.pmax = b.pmax;
	e.psum = b.psum;
	e.tgt_logit = b.tgt_logit;
	e.targets = b.tgt;
	e.M = T;
	e.ntiles = ntiles;
	e.red = nullptr;
	const void *wcls = d->wcls;
	if (fp8) {
		const uint16_t *p[1];
		TRY(dequant(d, {{d->wcls, (size_t)c.vocab_size * c.dim}}, p, st));
		wcls = p[0];
	}
	TRY(launch_plain(f, cls_bn, b.Xn, sp * c.dim, T, sp * c.dim, c.dim, one(wcls, c.vocab_size), c.vocab_size, e, st));
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
	// The range guard (prefill.h range_note): a pass whose f16 operands all fit is the result.
	// Otherwise the FIRST slot out of range decides (everything after it saw inf / NaN): a GLU
	// output gets the exact power-of-two scale that brings its largest |h| under 2^14 and the
	// pass runs again (idempotent: the same cache rows and log-probs are rewritten); any
	// other operand out of range (the normalised x, Q, the final norm) is refused.
	const int L = c.n_layers;
	std::vector<int> hexp(L, 0);
	std::vector<unsigned> rg((size_t)(L + 1) * RG_N);
	b.last_passes = b.last_scaled = 0;
	for (int pass = 1;; ++pass) {
		HIPCHK(hipMemsetAsync(b.range, 0, rg.size() * 4, d->stream));
		TRY(enqueue_prefill(d, n, pos0, logprobs != nullptr, hexp.data()));
		HIPCHK(hipMemcpyAsync(rg.data(), b.range, rg.size() * 4, hipMemcpyDeviceToHost, d->stream));
		HIPCHK(hipStreamSynchronize(d->stream));
		b.last_passes = pass;
		int bad = -1;
		for (size_t i = 0; i < rg.size() && bad < 0; ++i)
			if (rg[i])
				bad = (int)i;
		if (bad < 0)
			break;
		const int l = bad / RG_N, kind = bad % RG_N;
		float mx;
		memcpy(&mx, &rg[bad], 4);
		static const char *what[RG_N] = {"the normalised x (attention input)", "Q", "the normalised x (FFN input)",
										 "the GLU output"};
		if (kind != RG_H || l >= L || !std::isfinite(mx) || pass > L + 1) {
			set_err(std::string("yalm_prefill: ") + (l >= L ? "the final norm's output" : what[kind]) + " of layer " +
					std::to_string(l) + " exceeds the f16 range of the MFMA operands (max |v| " +
					std::to_string(mx) + "); the decode path (yalm_forward) keeps it in f32");
			return YALM_ERR_UNSUPPORTED;
		}
		const int e = (int)std::ceil(std::log2(mx / 16384.0f));
		if (e <= hexp[l]) { // cannot happen for a finite max: a scale that did not help
			set_err("yalm_prefill: internal: the GLU output scale did not bring layer " + std::to_string(l) + " into range");
			return YALM_ERR_HIP;
		}
		hexp[l] = e;
	}
	for (int l = 0; l < L; ++l)
		b.last_scaled += hexp[l] > 0;
	if (logprobs)
		HIPCHK(hipMemcpy(logprobs, b.lp, sizeof(float) * n, hipMemcpyDeviceToHost));
	return YALM_OK;
}

extern "C" int yalm_prefill_info(yalm_decoder d, int *passes, int *scaled_layers) {
	ARGCHK(d, "null decoder");
	if (passes)
		*passes = d->pf.last_passes;
	if (scaled_layers)
		*scaled_layers = d->pf.last_scaled;
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
	const PfForms f = g_test_forms; // a test hook: the forms set by yalm_set_prefill_forms(NULL, ...)
	TRY(launch_plain(f, pick_bn(f, PG_TEST, M, N, false), (const uint16_t *)da.p, K, M, K, K, one(dw.p, N), N, e16,
	                 nullptr));
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
