// awl.hip — the short-context fused attention + Wo kernel (attn_wo_local.h):
// its own translation unit (the decoder's main TU takes minutes to compile).
#include "attn_wo_local.h"
#include "decoder.h"

#include <algorithm>
#include <cstdlib>

template <class WT, int XS>
static const void *awl_fn_g(int G) {
	return G <= 1 ? (const void *)attn_wo_local_kernel<WT, 1, XS>
	       : G <= 2 ? (const void *)attn_wo_local_kernel<WT, 2, XS>
	       : G <= 4 ? (const void *)attn_wo_local_kernel<WT, 4, XS>
	                : (const void *)attn_wo_local_kernel<WT, 8, XS>;
}

static const void *attn_wo_local_pick(int dtype, int G, int XS) {
	if (dtype == YALM_F16)
		return XS == 1 ? awl_fn_g<WF16, 1>(G) : awl_fn_g<WF16, 2>(G);
	return XS == 1 ? awl_fn_g<WF8, 1>(G) : awl_fn_g<WF8, 2>(G);
}

int attn_wo_local_occupancy(int dtype, int G, int XS) {
	int occ = 0;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, attn_wo_local_pick(dtype, G, XS), AWL_THREADS, 0) !=
	    hipSuccess)
		return 0;
	return occ;
}

int launch_attn_wo_local(yalm_decoder_s *d, const yalm_block_weights &w) {
	const yalm_config &c = d->c;
	AttnWoLocalArgs p;
	p.n_heads = c.n_heads;
	p.n_kv = c.n_kv_heads;
	p.max_seq_len = c.max_seq_len;
	p.q_dim = c.n_heads * c.head_dim;
	p.dim = c.dim;
	p.wo = (const char *)w.wo;
	p.x = d->x;
	p.trace = d->awl_trace;
	p.kv_first = d->awl_kv_first;
	static const int ablate = getenv("YALM_AWL_ABLATE") ? atoi(getenv("YALM_AWL_ABLATE")) : 0;
	p.ablate = ablate;
	const int bytes = c.weight_dtype == YALM_F16 ? 2 : 1;
	const void *fn = attn_wo_local_pick(c.weight_dtype, c.n_heads / c.n_kv_heads, p.q_dim * bytes / 4096);
	const float *q = d->q;
	const uint16_t *kc = w.key_cache, *vc = w.value_cache;
	const StepState *st = d->step;
	void *args[] = {(void *)&q, (void *)&kc, (void *)&vc, (void *)&st, (void *)&p};
	HIPCHK(hipLaunchKernel(fn, dim3((c.dim + AWO_RPW - 1) / AWO_RPW), dim3(AWL_THREADS), args, 0, d->stream));
	return YALM_OK;
}

extern "C" int yalm_attn_wo_local_trace(yalm_decoder d, unsigned long long *host, size_t count, int *workgroups) {
	ARGCHK(d && host, "null argument");
	ARGCHK(d->awl_trace, "no local attn_wo trace (create the decoder with YALM_ATTN_WO_TRACE=1)");
	HIPCHK(hipStreamSynchronize(d->stream));
	const int nb = (d->c.dim + AWO_RPW - 1) / AWO_RPW;
	HIPCHK(hipMemcpy(host, d->awl_trace, sizeof(unsigned long long) * std::min(count, (size_t)4 * nb),
	                 hipMemcpyDeviceToHost));
	if (workgroups)
		*workgroups = nb;
	return YALM_OK;
}
