// engine.hip — host side of the persistent per-token decode engine (engine.h):
// support check, per-decoder state, one launch per token (captured in the
// decoder's per-mode hipGraph like the launch path), error reporting.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "decoder.h"

#define ENG_C 4 // consumer waves per CU
#define ENG_L 4 // loader waves per CU

template <class WT>
static const void *engine_fn(int G) {
	if (G <= 1)
		return (const void *)engine_kernel<WT, ENG_C, ENG_L, 1>;
	if (G <= 2)
		return (const void *)engine_kernel<WT, ENG_C, ENG_L, 2>;
	return (const void *)engine_kernel<WT, ENG_C, ENG_L, 4>;
}

static const void *engine_fn_dt(int dtype, int G) {
	return dtype == YALM_F32 ? engine_fn<WF32>(G) : dtype == YALM_F16 ? engine_fn<WF16>(G) : engine_fn<WF8>(G);
}

// Can this decoder run as one persistent launch per token?
static bool engine_supported(const yalm_decoder_s *d, int nb, std::string *why) {
	const yalm_config &c = d->c;
	auto no = [&](const char *m) {
		if (why)
			*why = m;
		return false;
	};
	if (d->tp_size > 1 || d->comm || d->ipc)
		return no("tensor parallel decoder");
	if (c.head_dim != ENG_D)
		return no("head_dim != 128");
	const int G = c.n_heads / c.n_kv_heads;
	if (G < 1 || G > 4)
		return no("n_heads / n_kv_heads > 4");
	const int epl = c.weight_dtype == YALM_F32 ? 4 : c.weight_dtype == YALM_F16 ? 8 : 16;
	const int CH = 64 * epl;
	const int q_dim = c.n_heads * c.head_dim, kv_dim = c.n_kv_heads * c.head_dim;
	for (int n : {c.dim, q_dim, c.hidden_dim})
		if (n % CH != 0 || n > (64 / epl) * ENG_C * CH)
			return no("GEMV input length not a multiple of 64 * EPL, or longer than the register slice");
	auto rows = [&](int groups, int R) { return (groups + nb - 1) / nb * R; };
	constexpr int maxrows = ENG_MAXROWS - 4; // 4-row tiles may write up to 3 spare rows
	if (rows((q_dim + 2 * kv_dim) / 2, 2) > maxrows || rows(c.hidden_dim, 2) > maxrows || rows(c.dim, 1) > maxrows ||
	    rows(c.vocab_size, 1) > maxrows)
		return no("too many rows per CU");
	int occ = 0;
	const void *fn = engine_fn_dt(c.weight_dtype, G);
	if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)eng_lds_bytes<ENG_C>()) !=
	        hipSuccess ||
	    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 64 * (ENG_C + ENG_L), eng_lds_bytes<ENG_C>()) !=
	        hipSuccess ||
	    occ < 1)
		return no("engine kernel does not fit one workgroup per CU");
	return true;
}

int engine_init(yalm_decoder_s *d) {
	// opt-in until it beats the launch path on the bench workload
	const char *env = getenv("YALM_ENGINE");
	if (!env || atoi(env) == 0)
		return YALM_OK;
	const int nb = device_cu_count();
	if (!engine_supported(d, nb, nullptr))
		return YALM_OK;
	const yalm_config &c = d->c;
	std::vector<EngLayer> L(c.n_layers);
	for (int l = 0; l < c.n_layers; ++l) {
		const yalm_block_weights &w = d->b[l];
		L[l] = EngLayer{(const char *)w.wq, (const char *)w.wk, (const char *)w.wv, (const char *)w.wo,
		                (const char *)w.w1, (const char *)w.w2, (const char *)w.w3, w.rms_att,
		                w.rms_ffn,          w.key_cache,        w.value_cache};
	}
	const int nflags = (nb + 255) / 256 * 256;
	TRY(dalloc(d, (void **)&d->eng_layers, sizeof(EngLayer) * c.n_layers));
	TRY(dalloc(d, (void **)&d->eng_flags, sizeof(unsigned) * nflags));
	TRY(dalloc(d, (void **)&d->eng_gen, sizeof(unsigned) * 4));
	TRY(dalloc(d, (void **)&d->eng_err, sizeof(unsigned) * 4));
	TRY(dalloc(d, (void **)&d->eng_tickets, sizeof(unsigned) * c.n_kv_heads));
	TRY(dalloc(d, (void **)&d->eng_part, sizeof(float) * (size_t)c.n_heads * ENG_SMAX * (c.head_dim + 2)));
	TRY(dalloc(d, (void **)&d->eng_amax, sizeof(float) * 2 * nb));
	TRY(dalloc(d, (void **)&d->eng_args, sizeof(EngArgs) * N_GRAPHS));
	HIPCHK(hipMemcpy(d->eng_layers, L.data(), sizeof(EngLayer) * c.n_layers, hipMemcpyHostToDevice));
	const char *tenv = getenv("YALM_ENGINE_TRACE");
	if (tenv && atoi(tenv) != 0)
		TRY(dalloc(d, (void **)&d->eng_trace, sizeof(unsigned long long) * nb * (5 * c.n_layers + 2) * 8));
	const char *denv = getenv("YALM_ENGINE_DBG");
	const int dbg = denv ? atoi(denv) : 0;
	const char *depth_env = getenv("YALM_ENGINE_DEPTH");
	const int depth = depth_env ? std::max(1, std::min(7, atoi(depth_env))) : ENG_LD;
	const char *nt_env = getenv("YALM_ENGINE_NT");
	const int ld_nt = nt_env ? atoi(nt_env) != 0 : 1;
	const char *pf_env = getenv("YALM_ENGINE_PF"); // KB of prefetch run-ahead; > 0 turns the last loader wave into the prefetcher
	const int pf_kb = pf_env ? std::max(0, atoi(pf_env)) : 0;
	const char *lw_env = getenv("YALM_ENGINE_LOADERS");
	const int ld_max = pf_kb > 0 ? ENG_L - 1 : ENG_L;
	const int ld_waves = lw_env ? std::max(1, std::min(ld_max, atoi(lw_env))) : ld_max;
	const char *sl_env = getenv("YALM_ENGINE_SLEEP");
	const int poll_sleep = sl_env ? atoi(sl_env) : 1;

	EngArgs a[N_GRAPHS];
	for (int which = 0; which < N_GRAPHS; ++which) {
		EngArgs &e = a[which];
		e.layers = d->eng_layers;
		e.n_layers = c.n_layers;
		e.dim = c.dim;
		e.hidden = c.hidden_dim;
		e.q_dim = c.n_heads * c.head_dim;
		e.kv_dim = c.n_kv_heads * c.head_dim;
		e.n_heads = c.n_heads;
		e.n_kv = c.n_kv_heads;
		e.vocab = c.vocab_size;
		e.max_seq_len = c.max_seq_len;
		e.act = c.act == YALM_SILU ? 1 : 0;
		e.mode = which == GRAPH_HYDRATE ? EM_HYDRATE : which == GRAPH_LOGITS ? EM_LOGITS : EM_GREEDY;
		e.tokens_cap = d->tokens_cap;
		e.eps = c.norm_eps;
		e.qkv_clip = c.qkv_clip;
		e.inv_freq = d->inv_freq;
		e.emb = (const char *)d->emb;
		e.rms_final = d->rms_final;
		e.wcls = (const char *)d->wcls;
		e.step = d->step;
		e.x = d->x;
		e.q = d->q;
		e.xb2 = d->xb2;
		e.hb = d->hb;
		e.logits = d->logits;
		e.part = d->eng_part;
		e.amax = d->eng_amax;
		e.tickets = d->eng_tickets;
		e.flags = d->eng_flags;
		e.gen = d->eng_gen;
		e.err = d->eng_err;
		e.tokens = d->tokens;
		e.trace = d->eng_trace;
		e.dbg = dbg;
		e.ld_depth = depth;
		e.ld_nt = ld_nt;
		e.ld_waves = ld_waves;
		e.poll_sleep = poll_sleep;
		e.pf_ahead = pf_kb * 1024 / ENG_ITEM;
	}
	HIPCHK(hipMemcpy(d->eng_args, a, sizeof(a), hipMemcpyHostToDevice));
	d->eng_nb = nb;
	d->engine = true;
	return YALM_OK;
}

template <class WT>
static int launch_engine_t(yalm_decoder_s *d, int which) {
	const int G = d->c.n_heads / d->c.n_kv_heads;
	const size_t lds = eng_lds_bytes<ENG_C>();
	const dim3 grid(d->eng_nb), block(64 * (ENG_C + ENG_L));
	const EngArgs *a = d->eng_args + which;
	if (G <= 1)
		hipLaunchKernelGGL((engine_kernel<WT, ENG_C, ENG_L, 1>), grid, block, lds, d->stream, a);
	else if (G <= 2)
		hipLaunchKernelGGL((engine_kernel<WT, ENG_C, ENG_L, 2>), grid, block, lds, d->stream, a);
	else
		hipLaunchKernelGGL((engine_kernel<WT, ENG_C, ENG_L, 4>), grid, block, lds, d->stream, a);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

int engine_enqueue(yalm_decoder_s *d, int which) {
	switch (d->c.weight_dtype) {
	case YALM_F32:
		return launch_engine_t<WF32>(d, which);
	case YALM_F16:
		return launch_engine_t<WF16>(d, which);
	default:
		return launch_engine_t<WF8>(d, which);
	}
}

// After a stream sync: the engine's bounded spins report here instead of hanging.
int engine_check(yalm_decoder_s *d) {
	if (d->awo_err) { // the fused attention + Wo launch spins too (attn_wo.h)
		unsigned e = 0;
		HIPCHK(hipMemcpy(&e, d->awo_err, sizeof(e), hipMemcpyDeviceToHost));
		if (e) { // reported once: cleared so that later calls report only their own failures
			HIPCHK(hipMemset(d->awo_err, 0, sizeof(e)));
			set_err("fused attention + Wo launch gave up waiting for the attention heads (error bits " +
			        std::to_string(e) + "): grid not co-resident; YALM_ATTN_WO=0 selects separate launches");
			return YALM_ERR_HIP;
		}
	}
	if (d->ffn_err) { // and the fused feed-forward launch (ffn.h)
		unsigned e = 0;
		HIPCHK(hipMemcpy(&e, d->ffn_err, sizeof(e), hipMemcpyDeviceToHost));
		if (e) {
			HIPCHK(hipMemset(d->ffn_err, 0, sizeof(e)));
			set_err("fused feed-forward launch gave up waiting for the hb of every workgroup (error bits " +
			        std::to_string(e) + "): grid not co-resident; YALM_FFN=0 selects separate launches");
			return YALM_ERR_HIP;
		}
	}
	if (!d->engine)
		return YALM_OK;
	unsigned e = 0;
	HIPCHK(hipMemcpy(&e, d->eng_err, sizeof(e), hipMemcpyDeviceToHost));
	if (e) {
		HIPCHK(hipMemset(d->eng_err, 0, sizeof(e)));
		set_err("persistent decode engine gave up waiting (error bits " + std::to_string(e) +
		        "): grid not co-resident or a CU stalled; YALM_ENGINE=0 selects the launch path");
		return YALM_ERR_HIP;
	}
	return YALM_OK;
}

extern "C" int yalm_engine_trace(yalm_decoder d, unsigned long long *host, size_t count, int *workgroups) {
	ARGCHK(d && host, "null argument");
	ARGCHK(d->engine && d->eng_trace, "no engine trace (create the decoder with YALM_ENGINE_TRACE=1)");
	HIPCHK(hipStreamSynchronize(d->stream));
	const size_t total = (size_t)d->eng_nb * (5 * d->c.n_layers + 2) * 8;
	HIPCHK(hipMemcpy(host, d->eng_trace, sizeof(unsigned long long) * std::min(count, total), hipMemcpyDeviceToHost));
	if (workgroups)
		*workgroups = d->eng_nb;
	return YALM_OK;
}
