# Build: HIP decode engine (gfx950) + C++20 host + CPU oracle (test-only).
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall
CSRC = yalm_amd/csrc
HIP_SRCS = $(CSRC)/yalm_hip.hip $(CSRC)/prefill.hip
HIP_OBJS = $(patsubst $(CSRC)/%.hip,build/%.o,$(HIP_SRCS))
HIP_HDRS = $(wildcard $(CSRC)/*.h) include/yalm_hip.h

all: yalm_amd/libyalm_hip.so oracle host

yalm_amd/libyalm_hip.so: $(HIP_OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib


# prefill.hip: MFMA accumulators in arch VGPRs (no AGPR form): the attention kernel's O and
# S^T accumulators are touched by VALU (softmax, rescale), and the AGPR form copied all 64 O
# registers out and back on every key tile (260 registers -> 1 wave per SIMD; 175 without)
build/prefill.o: HIPFLAGS += -mllvm -amdgpu-mfma-vgpr-form

build/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

oracle:
	$(MAKE) -C oracle

host: yalm_amd/libyalm_hip.so
	$(MAKE) -C yalm_amd/host

# kernel resource usage (VGPR/SGPR/LDS/occupancy) report
resource-usage:
	for f in $(HIP_SRCS); do $(HIPCC) $(HIPFLAGS) -c -o /tmp/yalm_ru.o $$f -Rpass-analysis=kernel-resource-usage 2>&1; done | \
		grep -E "Function Name|VGPRs:|SGPRs|Occupancy|LDS Size" | paste - - - - - -

clean:
	rm -f yalm_amd/libyalm_hip.so $(HIP_OBJS)
	$(MAKE) -C oracle clean
	$(MAKE) -C yalm_amd/host clean

# microbenchmarks (tools/*.hip -> tools/<name>; git-ignored binaries)
TOOLS = stream_bench launch_bench persist_bench mall_bench concurrency_check wg_timeline
tools: $(addprefix tools/,$(TOOLS))
tools/%: tools/%.hip $(HIP_HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

.PHONY: all oracle host clean resource-usage tools
