// probe_engine.hip — unit probe of the engine's consumer primitives on the GPU:
// eng_dot16<WF16> (v_fma_mix_f32 asm) against cvt + fma, and eng_sum4_t (the
// transposed 4-row wave reduction) against a host sum. Prints max errors.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_engine tools/probe_engine.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../yalm_amd/csrc/engine.h"

__global__ void probe(const uint32_t *w, const float *x, const float *v4, float *dot_out, float *ref_out,
                      float *sum_out) {
	const int lane = threadIdx.x;
	u32x4_t wv = {w[lane * 4], w[lane * 4 + 1], w[lane * 4 + 2], w[lane * 4 + 3]};
	float xr[8];
	for (int e = 0; e < 8; ++e)
		xr[e] = x[lane * 8 + e];
	float a0 = 0.f, a1 = 0.f;
	eng_dot16<WF16>(a0, a1, wv, xr);
	dot_out[lane] = a0 + a1;
	float wf[8];
	WF16::unpack(wv, wf);
	float r0 = 0.f, r1 = 0.f;
	for (int e = 0; e < 8; e += 2) {
		r0 = fmaf(wf[e], xr[e], r0);
		r1 = fmaf(wf[e + 1], xr[e + 1], r1);
	}
	ref_out[lane] = r0 + r1;
	float v[4] = {v4[lane * 4], v4[lane * 4 + 1], v4[lane * 4 + 2], v4[lane * 4 + 3]};
	sum_out[lane] = eng_sum4_t(v);
}

int main() {
	std::vector<uint32_t> w(256);
	std::vector<float> x(512), v4(256);
	for (int i = 0; i < 256; ++i) {
		_Float16 lo = (_Float16)(0.01f * ((i * 37) % 101 - 50)), hi = (_Float16)(0.02f * ((i * 53) % 97 - 48));
		uint16_t l, h;
		__builtin_memcpy(&l, &lo, 2);
		__builtin_memcpy(&h, &hi, 2);
		w[i] = l | ((uint32_t)h << 16);
		v4[i] = (float)((i * 29) % 113) - 50.f;
	}
	for (int i = 0; i < 512; ++i)
		x[i] = 0.1f * ((i * 17) % 61 - 30);
	uint32_t *dw;
	float *dx, *dv, *d1, *d2, *d3;
	hipMalloc(&dw, 1024);
	hipMalloc(&dx, 2048);
	hipMalloc(&dv, 1024);
	hipMalloc(&d1, 256);
	hipMalloc(&d2, 256);
	hipMalloc(&d3, 256);
	hipMemcpy(dw, w.data(), 1024, hipMemcpyHostToDevice);
	hipMemcpy(dx, x.data(), 2048, hipMemcpyHostToDevice);
	hipMemcpy(dv, v4.data(), 1024, hipMemcpyHostToDevice);
	probe<<<1, 64>>>(dw, dx, dv, d1, d2, d3);
	std::vector<float> o1(64), o2(64), o3(64);
	hipMemcpy(o1.data(), d1, 256, hipMemcpyDeviceToHost);
	hipMemcpy(o2.data(), d2, 256, hipMemcpyDeviceToHost);
	hipMemcpy(o3.data(), d3, 256, hipMemcpyDeviceToHost);
	double e1 = 0;
	for (int i = 0; i < 64; ++i)
		e1 = fmax(e1, fabs(o1[i] - o2[i]));
	printf("fma_mix dot vs cvt+fma: max |diff| = %g (lane0 %g vs %g)\n", e1, o1[0], o2[0]);
	double e3 = 0;
	for (int l = 0; l < 64; ++l) {
		const int t = l / 16;
		double ref = 0;
		for (int j = 0; j < 64; ++j)
			ref += v4[j * 4 + t];
		e3 = fmax(e3, fabs(o3[l] - ref));
	}
	printf("sum4_t: max |diff| = %g (lane0 %g lane16 %g lane32 %g lane48 %g)\n", e3, o3[0], o3[16], o3[32], o3[48]);
	return 0;
}
