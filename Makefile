# Build: HIP decode engine (gfx950) + C++20 host + CPU oracle (test-only).
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall
CSRC = yalm_amd/csrc
HIP_SRCS = $(CSRC)/yalm_hip.hip
HIP_HDRS = $(wildcard $(CSRC)/*.h) include/yalm_hip.h

all: yalm_amd/libyalm_hip.so oracle host

yalm_amd/libyalm_hip.so: $(HIP_SRCS) $(HIP_HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_SRCS)

oracle:
	$(MAKE) -C oracle

host: yalm_amd/libyalm_hip.so
	$(MAKE) -C yalm_amd/host

# kernel resource usage (VGPR/SGPR/LDS/occupancy) report
resource-usage:
	$(HIPCC) $(HIPFLAGS) -c -o /tmp/yalm_ru.o $(HIP_SRCS) -Rpass-analysis=kernel-resource-usage 2>&1 | \
		grep -E "Function Name|VGPRs:|SGPRs|Occupancy|LDS Size" | paste - - - - - -

clean:
	rm -f yalm_amd/libyalm_hip.so
	$(MAKE) -C oracle clean
	$(MAKE) -C yalm_amd/host clean

.PHONY: all oracle host clean resource-usage
