// dyn.hip — launch planning for the work-stealing row-block GEMV (gemv_dyn.h):
// per launch, the wave count (it must divide a group's items), the static
// prefix and the pooled tail. Own translation unit: the (weight type x policy x
// wave count) instantiations compile in parallel with yalm_hip.hip.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "decoder.h"
#include "gemv_dyn.h"

#define DYN_D 3 // dequeues in flight per workgroup (~1.1 us each under streaming, MI355X_MICROARCH.md row dequeue)

template <class WT, class P, bool NORM, int W, int IPW>
static int dyn_go(const P &p, const float *x, const float *normw, float eps, const DynArgs &dy, int nb, size_t lds,
                  hipStream_t st) {
	constexpr int GA = IPW == 1 ? 4 : 2; // groups in flight per wave: 4 (IPW 1) or 4 loads (IPW 2)
	auto kern = gemv_dyn_kernel<WT, P, IPW, GA, NORM, W, DYN_D>;
	static bool attr = false; // one-time attribute (kernel-wide, host-side cache)
	if (!attr) {
		// dynamic bytes on top of the static LDS queue (1 KB)
		HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
		attr = true;
	}
	hipLaunchKernelGGL(kern, dim3(nb), dim3((W + 1) * 64), lds, st, p, x, normw, eps, dy);
	HIPCHK(hipGetLastError());
	return YALM_OK;
}

// (streaming waves, items per wave per group) pairs compiled; the first with
// W * IPW == items per group is used (Mistral-7B: QKV, W1|W3, logits 8 x 2 (fp16) /
// 8 x 1 (fp8), W2 14 x 2 / 14 x 1; Llama-3.2-3B: 12 x 1, W2 8 x 2)
static const int DYN_SHAPES[][2] = {{8, 1}, {8, 2}, {12, 1}, {14, 1}, {14, 2}};

template <class WT, class P, bool NORM>
int launch_dyn(const P &p, const float *x, const float *normw, float eps, unsigned *ctr, int frac_pct, hipStream_t st) {
	constexpr int CH = YALM_WAVE * WT::EPL;
	if (p.n % CH != 0)
		return DYN_FALLBACK;
	const int ipg = P::R * (p.n / CH); // items per group
	int W = 0, IPW = 0;
	for (const auto &sh : DYN_SHAPES)
		if (sh[0] * sh[1] == ipg) {
			W = sh[0];
			IPW = sh[1];
			break;
		}
	if (!W)
		return DYN_FALLBACK;
	const int GA = IPW == 1 ? 4 : 2;
	const int nb = std::min(device_cu_count(), p.n_groups);
	const int per = p.n_groups / nb; // whole static rounds available
	int ks = frac_pct == 0 ? per : per - std::max(1, per * frac_pct / 100); // 0: static only (A/B)
	ks = std::max(ks, GA); // every wave's first GA groups static (issued before the x staging)
	if (ks > per)
		return DYN_FALLBACK; // too few groups to pool
	int pool = p.n_groups - nb * ks;
	while ((pool + DYN_SHARDS - 1) / DYN_SHARDS > DYN_QMAX - 8 && ks < per) { // LDS queue bound
		++ks;
		pool = p.n_groups - nb * ks;
	}
	if ((pool + DYN_SHARDS - 1) / DYN_SHARDS > DYN_QMAX - 8)
		return DYN_FALLBACK;
	const size_t lds = (W == 8 ? dyn_lds_floats<8>(p.n, ks, P::R)
	                    : W == 12 ? dyn_lds_floats<12>(p.n, ks, P::R)
	                              : dyn_lds_floats<14>(p.n, ks, P::R)) * sizeof(float);
	if (lds > 150 * 1024)
		return DYN_FALLBACK;
	DynArgs dy{ctr, ks, pool};
	if (W == 8 && IPW == 1)
		return dyn_go<WT, P, NORM, 8, 1>(p, x, normw, eps, dy, nb, lds, st);
	if (W == 8)
		return dyn_go<WT, P, NORM, 8, 2>(p, x, normw, eps, dy, nb, lds, st);
	if (W == 12)
		return dyn_go<WT, P, NORM, 12, 1>(p, x, normw, eps, dy, nb, lds, st);
	if (IPW == 1)
		return dyn_go<WT, P, NORM, 14, 1>(p, x, normw, eps, dy, nb, lds, st);
	return dyn_go<WT, P, NORM, 14, 2>(p, x, normw, eps, dy, nb, lds, st);
}

#define YALM_DYN_INST(WT)                                                                                              \
	template int launch_dyn<WT, PQKV<WT>, true>(const PQKV<WT> &, const float *, const float *, float, unsigned *, int, \
	                                            hipStream_t);                                                          \
	template int launch_dyn<WT, PGlu<WT, 1>, true>(const PGlu<WT, 1> &, const float *, const float *, float,            \
	                                               unsigned *, int, hipStream_t);                                      \
	template int launch_dyn<WT, PGlu<WT, 0>, true>(const PGlu<WT, 0> &, const float *, const float *, float,            \
	                                               unsigned *, int, hipStream_t);                                      \
	template int launch_dyn<WT, PResidual<WT, 1>, false>(const PResidual<WT, 1> &, const float *, const float *,        \
	                                                     float, unsigned *, int, hipStream_t);                         \
	template int launch_dyn<WT, PStore<WT, 2>, true>(const PStore<WT, 2> &, const float *, const float *, float,        \
	                                                 unsigned *, int, hipStream_t);                                    \
	template int launch_dyn<WT, PStore<WT, 1>, true>(const PStore<WT, 1> &, const float *, const float *, float,        \
	                                                 unsigned *, int, hipStream_t);

YALM_DYN_INST(WF16)
YALM_DYN_INST(WF8)
