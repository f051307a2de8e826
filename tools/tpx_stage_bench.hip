// tpx_stage_bench.hip — what a consumer GEMV's x staging from the IPC exchange costs
// (tp_exchange.h), against N source ranks: every one of 256 workgroups (512 threads) loads
// the N slots' {value, tag} granules of x (n 4096) and sums them, as gemv_rb_kernel<TIN>
// does, the tags already matching. Buffer uncached (hipDeviceMallocUncached, the product)
// or coarse-grained (hipMalloc), and against the alternatives: the plain x staging of
// one-GPU GEMVs (16 KB fp32 through L2) and a collect launch (few workgroups sum the slots
// into x once) followed by that plain staging. Also with a weight stream behind the staging
// (W bytes of nt loads spread over the grid), as in the real consumer.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/tpx_stage_bench tools/tpx_stage_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../yalm_amd/csrc/tp_exchange.h"

#define CK(x)                                                                                                          \
	do {                                                                                                               \
		hipError_t e_ = (x);                                                                                           \
		if (e_ != hipSuccess) {                                                                                        \
			printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                                           \
			return 1;                                                                                                  \
		}                                                                                                              \
	} while (0)

constexpr int THREADS = 512, N_X = 4096;

// stream `per_wg` bytes of weights per workgroup (nt 16-byte loads, U = 4 in flight), after
// the staging's loads are issued; returns a value so the loads stay
__device__ __forceinline__ float stream_w(const char *w, size_t per_wg) {
	const char *p = w + blockIdx.x * per_wg;
	float acc = 0.f;
	for (size_t o = threadIdx.x * 16; o < per_wg; o += THREADS * 16) {
		const u32x4_t v = load_nt16(p + o);
		acc += __uint_as_float(v[0] ^ v[3]);
	}
	return acc;
}

__global__ __launch_bounds__(THREADS) void stage_tin_k(TpX t, const float *normw, const char *w, size_t per_wg,
                                                       float *sink) {
	__shared__ __attribute__((aligned(16))) float xs[N_X + 64];
	const TpxView v = tpx_view(t, t.g());
	TpxPre<2> pre;
	tpx_prefetch<true, THREADS, 2>(pre, v, t, normw, N_X);
	const float a = per_wg ? stream_w(w, per_wg) : 0.f;
	tpx_stage_x<true, THREADS, 2>(xs, t, v, pre, normw, N_X, 1e-5f);
	if (xs[threadIdx.x] == 12345.f || a == 12345.f)
		sink[blockIdx.x] = a;
}

__global__ __launch_bounds__(THREADS) void stage_plain_k(const float *x, const float *normw, const char *w,
                                                         size_t per_wg, float *sink) {
	__shared__ __attribute__((aligned(16))) float xs[N_X + 64];
	float4_t r[2], nw[2];
	for (int k = 0; k < 2; ++k) {
		r[k] = *(const float4_t *)(x + (threadIdx.x + k * THREADS) * 4);
		nw[k] = *(const float4_t *)(normw + (threadIdx.x + k * THREADS) * 4);
	}
	const float a = per_wg ? stream_w(w, per_wg) : 0.f;
	float ss = 0.f;
	for (int k = 0; k < 2; ++k)
		ss = sumsq4(ss, r[k]);
	ss = wave_sum(ss);
	if ((threadIdx.x & 63) == 0)
		xs[N_X + (threadIdx.x >> 6)] = ss;
	__syncthreads();
	float tot = 0.f;
	for (int i = 0; i < THREADS / 64; ++i)
		tot += xs[N_X + i];
	const float sc = 1.f / sqrtf(tot / N_X + 1e-5f);
	for (int k = 0; k < 2; ++k) {
		float4_t q = r[k];
		for (int e = 0; e < 4; ++e)
			q[e] = q[e] * sc * nw[k][e];
		*(float4_t *)(xs + (threadIdx.x + k * THREADS) * 4) = q;
	}
	__syncthreads();
	if (xs[threadIdx.x] == 12345.f || a == 12345.f)
		sink[blockIdx.x] = a;
}

// collect: nwg workgroups, each sums its share of x from the N slots and writes x
__global__ __launch_bounds__(256) void collect_k(TpX t, float *x) {
	const unsigned g = t.g();
	const unsigned long long dl = __builtin_amdgcn_s_memrealtime() + TPX_TIMEOUT;
	for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N_X; i += gridDim.x * blockDim.x) {
		float s = tpx_get1(t, g, 0, i, dl);
		for (int p = 1; p < t.n; ++p)
			s += tpx_get1(t, g, p, i, dl);
		x[i] = s;
	}
}

__global__ void empty_k() {}

template <class F>
static float time_it(F launch, hipStream_t s, int reps = 200) {
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	for (int i = 0; i < 20; ++i)
		launch(s);
	(void)hipEventRecord(a, s);
	for (int i = 0; i < reps; ++i)
		launch(s);
	(void)hipEventRecord(b, s);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	return ms * 1e3f / reps;
}

int main() {
	hipStream_t s;
	CK(hipStreamCreate(&s));
	const int S = N_X;
	float *x, *normw, *sink;
	CK(hipMalloc(&x, N_X * 4));
	CK(hipMalloc(&normw, N_X * 4));
	CK(hipMalloc(&sink, 4096 * 4));
	CK(hipMemset(x, 0, N_X * 4));
	CK(hipMemset(normw, 0, N_X * 4));
	const size_t wbytes = 2ull << 30; // weight pool, rotated so the stream comes from HBM
	char *w;
	CK(hipMalloc(&w, wbytes));
	CK(hipMemset(w, 0, wbytes));
	StepState *st;
	CK(hipMalloc(&st, sizeof(StepState)));
	CK(hipMemset(st, 0, sizeof(StepState)));
	float none = 0.f;
	(void)none;
	printf("empty launch: %.2f us\n", time_it([&](hipStream_t q) { empty_k<<<1, 64, 0, q>>>(); }, s));
	for (size_t wb : {(size_t)0, (size_t)29 << 20, (size_t)235 << 20}) {
		const size_t per_wg = wb / 256 / 8192 * 8192;
		size_t off = 0;
		auto wnext = [&]() {
			const char *p = w + off;
			off += wb;
			if (off + wb > wbytes)
				off = 0;
			return p;
		};
		printf("--- weight stream %zu MB per launch\n", wb >> 20);
		printf("plain x staging (one GPU): %.2f us\n",
		       time_it([&](hipStream_t q) { stage_plain_k<<<256, THREADS, 0, q>>>(x, normw, wnext(), per_wg, sink); }, s));
		for (int uc = 1; uc >= 0; --uc)
			for (int n : {1, 2, 4, 8}) {
				const size_t bytes = 2ull * n * S * 8 + TPX_CTRL_WORDS * 4;
				void *buf;
				if (uc)
					CK(hipExtMallocWithFlags(&buf, bytes, hipDeviceMallocUncached));
				else
					CK(hipMalloc(&buf, bytes));
				std::vector<unsigned long long> h(2ull * n * S);
				for (size_t i = 0; i < h.size(); ++i) // exchange g = 0 (parity 0, tag 1) and g = 1 (tag 2)
					h[i] = (unsigned long long)__builtin_bit_cast(unsigned, 0.001f * (i % 97)) |
					       ((unsigned long long)(i < (size_t)n * S ? 1u : 2u) << 32);
				CK(hipMemset(buf, 0, bytes));
				CK(hipMemcpy(buf, h.data(), h.size() * 8, hipMemcpyHostToDevice));
				float **bufs;
				CK(hipMalloc(&bufs, sizeof(float *) * n));
				std::vector<float *> hb(n, (float *)buf);
				CK(hipMemcpy(bufs, hb.data(), sizeof(float *) * n, hipMemcpyHostToDevice));
				TpX t{};
				t.bufs = bufs;
				t.rank = 0;
				t.n = n;
				t.S = S;
				t.xw = x;
				t.step = st;
				t.ex = 0;
				const float us_tin = n > TPX_STAGE_MAX_RANKS ? 0.f : time_it(
				    [&](hipStream_t q) { stage_tin_k<<<256, THREADS, 0, q>>>(t, normw, wnext(), per_wg, sink); }, s);
				float us_col[3];
				const int nwg[3] = {1, 8, 32};
				for (int k = 0; k < 3; ++k)
					us_col[k] = time_it(
					    [&](hipStream_t q) {
						    collect_k<<<nwg[k], 256, 0, q>>>(t, x);
						    stage_plain_k<<<256, THREADS, 0, q>>>(x, normw, wnext(), per_wg, sink);
					    },
					    s);
				unsigned e = 0;
				CK(hipMemcpy(&e, (char *)buf + 2ull * n * S * 8, 4, hipMemcpyDeviceToHost));
				printf("%s N=%d: consumer staging %.2f us | collect(1 / 8 / 32 wg) + plain %.2f / %.2f / %.2f us%s\n",
				       uc ? "uncached" : "hipMalloc", n, us_tin, us_col[0], us_col[1], us_col[2],
				       e ? "  [TIMEOUT FLAG]" : "");
				CK(hipFree(bufs));
				CK(hipFree(buf));
			}
	}
	return 0;
}
