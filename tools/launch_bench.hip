// launch_bench.hip — per-launch cost of trivial kernels on this system:
// eager back-to-back launches vs the same kernels as hipGraph nodes, for
// 1 and 512 workgroups, with and without one dependent global load.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/launch_bench tools/launch_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void empty_k() {}
__global__ void load_k(const int *p, int *o) {
	int v = p[blockIdx.x & 7];
	if (v == 12345)
		o[0] = v;
}

template <class F>
static float time_eager(F launch, int n, hipStream_t s) {
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int i = 0; i < 20; ++i)
		launch(s);
	hipEventRecord(a, s);
	for (int i = 0; i < n; ++i)
		launch(s);
	hipEventRecord(b, s);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	return ms * 1e3f / n;
}

template <class F>
static float time_graph(F launch, int nodes, int reps, hipStream_t s) {
	hipGraph_t g;
	hipGraphExec_t e;
	hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
	for (int i = 0; i < nodes; ++i)
		launch(s);
	hipStreamEndCapture(s, &g);
	hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
	hipGraphLaunch(e, s);
	hipStreamSynchronize(s);
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	hipEventRecord(a, s);
	for (int r = 0; r < reps; ++r)
		hipGraphLaunch(e, s);
	hipEventRecord(b, s);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	return ms * 1e3f / (nodes * reps);
}

int main() {
	hipStream_t s;
	hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
	int *p, *o;
	hipMalloc(&p, 4096);
	hipMalloc(&o, 4096);
	hipMemset(p, 0, 4096);
	auto e1 = [](hipStream_t st) { empty_k<<<1, 64, 0, st>>>(); };
	auto e512 = [](hipStream_t st) { empty_k<<<512, 256, 0, st>>>(); };
	auto l1 = [&](hipStream_t st) { load_k<<<1, 64, 0, st>>>(p, o); };
	auto l512 = [&](hipStream_t st) { load_k<<<512, 256, 0, st>>>(p, o); };
	printf("eager empty 1 WG      : %6.2f us/launch\n", time_eager(e1, 2000, s));
	printf("eager empty 512 WG    : %6.2f us/launch\n", time_eager(e512, 2000, s));
	printf("eager 1-load 1 WG     : %6.2f us/launch\n", time_eager(l1, 2000, s));
	printf("eager 1-load 512 WG   : %6.2f us/launch\n", time_eager(l512, 2000, s));
	printf("graph empty 1 WG      : %6.2f us/node\n", time_graph(e1, 200, 20, s));
	printf("graph empty 512 WG    : %6.2f us/node\n", time_graph(e512, 200, 20, s));
	printf("graph 1-load 1 WG     : %6.2f us/node\n", time_graph(l1, 200, 20, s));
	printf("graph 1-load 512 WG   : %6.2f us/node\n", time_graph(l512, 200, 20, s));
	return 0;
}
