// wg_timeline.hip — per-workgroup start/end timeline of the row-block GEMV
// (gemv_rb_kernel) at the Mistral-7B shapes: dispatch spread, per-CU duration
// and tail (time from the median workgroup's end to the last), to see where
// the per-kernel fixed cost of the decode GEMVs goes.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/wg_timeline tools/wg_timeline.hip
#define YALM_WG_TRACE
#include "../yalm_amd/csrc/gemv.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                                                         \
	do {                                                                                                               \
		hipError_t e_ = (x);                                                                                           \
		if (e_ != hipSuccess) {                                                                                        \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                  \
			exit(1);                                                                                                   \
		}                                                                                                              \
	} while (0)

template <class P, bool NORM>
static void run(const char *name, P p, const float *x, const float *nw, int nb, size_t wbytes, int layers,
                size_t layer_stride, unsigned long long *trace) {
	auto kern = gemv_rb_kernel<WF16, P, 4, NORM, 512>;
	const int ngl = (p.n_groups + nb - 1) / nb;
	const size_t lds = ((size_t)p.n + 64 + (size_t)ngl * P::R * 8) * 4;
	CHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
	hipEvent_t e0, e1;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	std::vector<unsigned long long> t(2 * nb);
	double span_sum = 0, disp_sum = 0, tail_sum = 0, med_sum = 0, ev_sum = 0;
	const int reps = 24;
	for (int r = 0; r < reps; ++r) {
		P q = p;
		const size_t off = (size_t)(r % layers) * layer_stride; // rotate: weights come from HBM
		q.w1 += off;
		q.w3 += off;
		CHK(hipEventRecord(e0, 0));
		hipLaunchKernelGGL(kern, dim3(nb), dim3(512), lds, 0, q, x, nw, 1e-5f);
		CHK(hipEventRecord(e1, 0));
		CHK(hipEventSynchronize(e1));
		float ms;
		CHK(hipEventElapsedTime(&ms, e0, e1));
		CHK(hipMemcpy(t.data(), trace, 16 * nb, hipMemcpyDeviceToHost));
		if (r < 4)
			continue;
		unsigned long long s0 = ~0ull, s1 = 0, e_max = 0;
		std::vector<double> ends(nb), durs(nb);
		for (int i = 0; i < nb; ++i) {
			s0 = std::min(s0, t[2 * i]);
			s1 = std::max(s1, t[2 * i]);
			e_max = std::max(e_max, t[2 * i + 1]);
		}
		for (int i = 0; i < nb; ++i)
			ends[i] = (t[2 * i + 1] - s0) * 0.01;
		std::sort(ends.begin(), ends.end());
		span_sum += (e_max - s0) * 0.01;
		disp_sum += (s1 - s0) * 0.01;
		med_sum += ends[nb / 2];
		tail_sum += (e_max - s0) * 0.01 - ends[nb / 2];
		ev_sum += ms * 1e3;
	}
	const int n = reps - 4;
	printf("%-6s %6.1f MB  event %6.2f us  WG span %6.2f us  dispatch spread %5.2f  median end %6.2f  tail (median->last) "
	       "%5.2f us  -> %5.2f TB/s over the span\n",
	       name, wbytes / 1e6, ev_sum / n, span_sum / n, disp_sum / n, med_sum / n, tail_sum / n,
	       wbytes / (span_sum / n * 1e-6) / 1e12);
}

int main() {
	int ncu = 0;
	CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	const int dim = 4096, hid = 14336, L = 8;
	const size_t glu_layer = 2ull * hid * dim * 2;
	char *w;
	CHK(hipMalloc(&w, glu_layer * L));
	CHK(hipMemset(w, 0, glu_layer * L));
	float *x, *nw, *out;
	CHK(hipMalloc(&x, hid * 4));
	CHK(hipMalloc(&nw, hid * 4));
	CHK(hipMalloc(&out, hid * 4));
	CHK(hipMemset(x, 0, hid * 4));
	CHK(hipMemset(nw, 0, hid * 4));
	unsigned long long *trace;
	CHK(hipMalloc(&trace, 16 * 4096));
	CHK(hipMemcpyToSymbol(HIP_SYMBOL(yalm_wg_trace), &trace, sizeof(trace)));
	for (int wpc : {1, 2}) {
		PGlu<WF16, 1> g;
		g.w1 = w;
		g.w3 = w + (size_t)hid * dim * 2;
		g.n = dim;
		g.out = out;
		g.n_groups = hid;
		char nm[32];
		snprintf(nm, sizeof nm, "glu/%d", wpc);
		run<PGlu<WF16, 1>, true>(nm, g, x, nw, ncu * wpc, glu_layer, L, glu_layer, trace);
	}
	return 0;
}
