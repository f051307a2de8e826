// overlap_bench.hip — can a weight-streaming kernel hide its launch boundary by
// being dispatched in its predecessor's tail (second stream, no graph/stream
// edge to the predecessor) and waiting for the predecessor's per-workgroup
// flags on the device, with its first weight loads already in flight?
//
// A "layer" = 4 streaming phases of Mistral-7B fp16 sizes (QKV 50.3 MB, Wo
// 33.6 MB, W1|W3 235 MB, W2 117.4 MB), L layers back to back over distinct
// buffers (no cache reuse). Each phase: 256 workgroups (one per CU: dynamic LDS
// `lds` bytes keeps two phases' workgroups from sharing a CU when large),
// 8 streaming waves + 1 poll wave. Streaming wave: P 16-byte loads per lane issued
// at dispatch, then (after the poll wave saw every predecessor flag, and a
// 16 KB sc1 "activation" gather) the rest of its 1-KB items with U in flight.
// End: every wave drains, barrier, one sc1 flag store (launch epoch).
//
// Modes: serial (one stream, P = 0: the launch path today), overlap (phase k on
// stream k % 2, each stream waits only for its own previous phase), and both
// captured in a hipGraph. Prints us per layer and TB/s over the weight bytes.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/overlap_bench tools/overlap_bench.hip
#include <hip/hip_runtime.h>

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

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#define NW 8            // streaming waves
#define THREADS (NW * 64 + 64)
#define NB 256
#define TIMEOUT 200000000ull

__device__ __forceinline__ u32x4 ldnt(const char *p) { return __builtin_nontemporal_load((const u32x4 *)p); }

struct Args {
	const char *w;           // this phase's weights
	size_t bytes;
	const unsigned *prev;    // predecessor's flags [NB] (null: none)
	unsigned *mine;          // this phase's flags [NB]
	const float *act_in;     // 16 KB activation written by the predecessor (sc1)
	float *act_out;          // this phase's output slice (16 floats per workgroup)
	unsigned epoch;
	unsigned *err;
	unsigned long long *trace; // [NB][4]: dispatch, flags seen, stream end, or null
};

template <int U, int P>
__device__ __forceinline__ void phase_body(const Args &a, int b, float *xs) {
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
	const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
	// items: 1 KB, block j*NB + b (8 KB = one item per streaming wave)
	const int nblk = (int)(a.bytes / 8192);
	const int mine = wave < NW ? (nblk - b + NB - 1) / NB : 0;
	auto addr = [&](int j) { return a.w + ((size_t)(j * NB + b) * 8 + wave) * 1024 + lane * 16; };
	const char *dummy = (const char *)a.act_in + lane * 16;
	u32x4 buf[U + P];
	if (wave < NW) {
#pragma unroll
		for (int u = 0; u < U + P; ++u)
			buf[u] = ldnt(u < mine ? addr(u) : dummy);
	}
	if (wave == NW && a.prev) { // the poll wave: no loads of its own queued ahead (in-order vmcnt)
		const unsigned long long ts = __builtin_amdgcn_s_memrealtime();
		for (;;) {
			unsigned v[4];
#pragma unroll
			for (int k = 0; k < 4; ++k)
				v[k] = __hip_atomic_load(a.prev + lane + 64 * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			if (__all(v[0] == a.epoch && v[1] == a.epoch && v[2] == a.epoch && v[3] == a.epoch))
				break;
			__builtin_amdgcn_s_sleep(1);
			if (__builtin_amdgcn_s_memrealtime() - ts > TIMEOUT) {
				if (lane == 0)
					atomicOr(a.err, 1u);
				break;
			}
		}
	}
	__syncthreads();
	const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
	// 16 KB activation gather (sc1), as a GEMV stages x
	for (int i = tid * 4; i < 4096; i += THREADS * 4) {
		const unsigned long long *p = (const unsigned long long *)(a.act_in + i);
		const unsigned long long x0 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const unsigned long long x1 = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		xs[i] = __uint_as_float((unsigned)x0);
		xs[i + 1] = __uint_as_float((unsigned)(x0 >> 32));
		xs[i + 2] = __uint_as_float((unsigned)x1);
		xs[i + 3] = __uint_as_float((unsigned)(x1 >> 32));
	}
	__syncthreads();
	unsigned acc = 0;
	if (wave < NW) {
		for (int k = 0; k < mine; k += U + P) {
#pragma unroll
			for (int u = 0; u < U + P; ++u) {
				const int j = k + u;
				if (j < mine)
					acc ^= buf[u][0] ^ buf[u][1] ^ buf[u][2] ^ buf[u][3];
				buf[u] = ldnt(j + U + P < mine ? addr(j + U + P) : dummy);
			}
		}
	}
	acc += __float_as_uint(xs[(tid * 7) & 4095]);
	if (tid < 16)
		__hip_atomic_store(a.act_out + b * 16 + tid, (float)(acc & 0xff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
	if (tid == 0) {
		__hip_atomic_store(a.mine + b, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (a.trace) {
			a.trace[b * 4 + 0] = t0;
			a.trace[b * 4 + 1] = t1;
			a.trace[b * 4 + 2] = t2;
		}
	}
}
template <int U, int P>
__global__ __launch_bounds__(THREADS) void phase_kernel(Args a) {
	extern __shared__ __attribute__((aligned(16))) float xs[];
	phase_body<U, P>(a, blockIdx.x, xs);
}
// all phases of a layer as roles of ONE grid: workgroup b runs phase b / NB of
// the layer (blocks dispatch in index order, so a role's workgroups take the CUs
// its predecessor's workgroups free up, issue their first loads, then wait on the
// predecessor's flags; no role waits on a later one: no deadlock)
struct Args4 {
	Args a[4];
};
template <int U, int P>
__global__ __launch_bounds__(THREADS) void roles_kernel(Args4 r) {
	extern __shared__ __attribute__((aligned(16))) float xs[];
	const int role = blockIdx.x / NB;
	phase_body<U, P>(r.a[role], blockIdx.x - role * NB, xs);
}

typedef void (*KFn)(Args);

int main(int argc, char **argv) {
	setvbuf(stdout, NULL, _IONBF, 0);
	const int L = argc > 1 ? atoi(argv[1]) : 8;
	const int reps = 5;
	const size_t sz[4] = {50331648, 33554432, 234881024, 117440512};
	const int NPH = 4;
	size_t layer = 0;
	for (int p = 0; p < NPH; ++p)
		layer += sz[p];
	char *w;
	CHK(hipMalloc(&w, layer * L));
	CHK(hipMemset(w, 1, layer * L));
	float *act;
	CHK(hipMalloc(&act, 2 * 4096 * 4));
	CHK(hipMemset(act, 0, 2 * 4096 * 4));
	unsigned *flags, *err;
	CHK(hipMalloc(&flags, (size_t)NPH * L * NB * 4 + 4096));
	CHK(hipMemset(flags, 0, (size_t)NPH * L * NB * 4 + 4096));
	err = flags + (size_t)NPH * L * NB;
	unsigned long long *trace;
	CHK(hipMalloc(&trace, (size_t)NPH * L * NB * 4 * 8));
	hipStream_t s[2];
	CHK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
	CHK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
	hipEvent_t e0, e1, ej;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	CHK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
	unsigned epoch = 0;

	struct Cfg {
		const char *name;
		KFn fn;
		int lds;
		bool two;
		bool graph;
		void (*rfn)(Args4) = nullptr; // roles-in-one-grid kernel (one launch per layer)
		bool nopoll = false;          // serial launches without the flag poll (the launch path today)
	};
	std::vector<Cfg> cfgs = {
	    {"serial nopoll lds 96K", phase_kernel<4, 0>, 96 * 1024, false, false, nullptr, true},
	    {"serial nopoll graph  ", phase_kernel<4, 0>, 96 * 1024, false, true, nullptr, true},
	    {"serial   P=0  lds 96K", phase_kernel<4, 0>, 96 * 1024, false, false},
	    {"overlap  P=0  lds 96K", phase_kernel<4, 0>, 96 * 1024, true, false},
	    {"overlap  P=8  lds 96K", phase_kernel<4, 8>, 96 * 1024, true, false},
	    {"overlap  P=16 lds 96K", phase_kernel<4, 16>, 96 * 1024, true, false},
	    {"overlap  P=16 lds 20K", phase_kernel<4, 16>, 20 * 1024, true, false},
	    {"serial   P=0  graph  ", phase_kernel<4, 0>, 96 * 1024, false, true},
	    {"roles    P=0  lds 64K", nullptr, 64 * 1024, false, false, roles_kernel<4, 0>},
	    {"roles    P=8  lds 64K", nullptr, 64 * 1024, false, false, roles_kernel<4, 8>},
	    {"roles    P=16 lds 64K", nullptr, 64 * 1024, false, false, roles_kernel<4, 16>},
	    {"roles    P=16 lds 96K", nullptr, 96 * 1024, false, false, roles_kernel<4, 16>},
	    {"roles    P=8  lds 20K", nullptr, 20 * 1024, false, false, roles_kernel<4, 8>},
	    {"roles    P=16 graph  ", nullptr, 64 * 1024, false, true, roles_kernel<4, 16>},
	};
	for (auto &c : cfgs)
		CHK(hipFuncSetAttribute(c.rfn ? (const void *)c.rfn : (const void *)c.fn,
		                        hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));

	auto enqueue = [&](const Cfg &c, bool tr) {
		++epoch;
		// fork both streams from s[0]'s current point
		CHK(hipEventRecord(ej, s[0]));
		CHK(hipStreamWaitEvent(s[1], ej, 0));
		for (int l = 0; l < L; ++l) {
			Args4 r4;
			for (int p = 0; p < NPH; ++p) {
				const int k = l * NPH + p;
				Args a;
				size_t off = (size_t)l * layer;
				for (int q = 0; q < p; ++q)
					off += sz[q];
				a.w = w + off;
				a.bytes = sz[p];
				a.prev = k > 0 && !c.nopoll ? flags + (size_t)(k - 1) * NB : nullptr;
				a.mine = flags + (size_t)k * NB;
				a.act_in = act + (k & 1) * 4096;
				a.act_out = act + ((k + 1) & 1) * 4096;
				a.epoch = epoch;
				a.err = err;
				a.trace = tr ? trace + (size_t)k * NB * 4 : nullptr;
				hipStream_t st = c.two ? s[k & 1] : s[0];
				if (c.rfn)
					r4.a[p] = a;
				else
					hipLaunchKernelGGL(c.fn, dim3(NB), dim3(THREADS), c.lds, st, a);
			}
			if (c.rfn)
				hipLaunchKernelGGL(c.rfn, dim3(NB * NPH), dim3(THREADS), c.lds, s[0], r4);
		}
		CHK(hipEventRecord(ej, s[1]));
		CHK(hipStreamWaitEvent(s[0], ej, 0));
	};

	for (auto &c : cfgs) {
		float best = 1e9f;
		hipGraphExec_t ge = nullptr;
		if (c.graph) {
			// the graph bakes one epoch: reset flags before each replay
			hipGraph_t g;
			CHK(hipStreamBeginCapture(s[0], hipStreamCaptureModeRelaxed));
			CHK(hipMemsetAsync(flags, 0, (size_t)NPH * L * NB * 4, s[0]));
			enqueue(c, false);
			CHK(hipStreamEndCapture(s[0], &g));
			CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
		}
		for (int r = 0; r < reps; ++r) {
			CHK(hipEventRecord(e0, s[0]));
			if (c.graph)
				CHK(hipGraphLaunch(ge, s[0]));
			else
				enqueue(c, r == reps - 1);
			CHK(hipEventRecord(e1, s[0]));
			CHK(hipEventSynchronize(e1));
			float ms;
			CHK(hipEventElapsedTime(&ms, e0, e1));
			if (r > 0 && ms < best)
				best = ms;
		}
		unsigned e = 0;
		CHK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
		const double us_layer = best * 1e3 / L;
		printf("%s  %7.2f us/layer  %5.2f TB/s  err=%u\n", c.name, us_layer, layer / (us_layer * 1e-6) / 1e12, e);
		if (e)
			CHK(hipMemset(err, 0, 4));
		if (!c.graph && !c.rfn) {
			// timeline of the last replay: per phase, dispatch of its workgroups vs
			// the predecessor's last stream end
			std::vector<unsigned long long> h((size_t)NPH * L * NB * 4);
			CHK(hipMemcpy(h.data(), trace, h.size() * 8, hipMemcpyDeviceToHost));
			double sum_disp = 0, sum_seen = 0, sum_gap = 0;
			int n = 0;
			for (int k = 1; k < NPH * L; ++k) {
				unsigned long long pend = 0, dmin = ~0ull, dmax = 0, smax = 0, cend_min = ~0ull;
				for (int b = 0; b < NB; ++b) {
					pend = std::max(pend, h[((size_t)(k - 1) * NB + b) * 4 + 2]);
					dmin = std::min(dmin, h[((size_t)k * NB + b) * 4 + 0]);
					dmax = std::max(dmax, h[((size_t)k * NB + b) * 4 + 0]);
					smax = std::max(smax, h[((size_t)k * NB + b) * 4 + 1]);
				}
				(void)cend_min;
				sum_disp += ((double)dmax - (double)pend) / 100.0;
				sum_seen += ((double)smax - (double)pend) / 100.0;
				sum_gap += ((double)dmin - (double)pend) / 100.0;
				++n;
			}
			printf("    vs predecessor's last stream end: first dispatch %+6.2f us, last dispatch %+6.2f us, "
			       "last flags-seen %+6.2f us (mean over %d seams)\n",
			       sum_gap / n, sum_disp / n, sum_seen / n, n);
		}
		if (ge)
			CHK(hipGraphExecDestroy(ge));
	}
	return 0;
}
