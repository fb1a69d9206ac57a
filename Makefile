# Makefile — builds the MI355X product (build/libsid.so, build/sid) and the
# test-only oracle (oracle/_build, oracle/_ref).  `make -j8`.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
BUILD ?= build
SRC := sid_amd/csrc
# -ffp-contract=off: device doubles round like the reference's x86-64 SSE2 build (no
# FMA contraction), and the double-double error-free transforms stay exact
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -Wall -Wno-unused-function -Iinclude
HOSTFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Iinclude
# EXTRA: A/B variants of the same sources (make BUILD=build_b EXTRA=-DNAME=VALUE)
HIPFLAGS += $(EXTRA)

KERNELS := local synth lynch textpath
HOSTSRC := capi lynch_host parse emit run
OBJS := $(KERNELS:%=$(BUILD)/%.o) $(HOSTSRC:%=$(BUILD)/%.o)
HDRS := include/sid.h $(wildcard $(SRC)/*.h)

all: $(BUILD)/libsid.so $(BUILD)/sid oracle

$(BUILD)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only translation units: compiled by hipcc as HIP (they include the HIP
# runtime headers); parse/emit use no HIP at all
$(BUILD)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/libsid.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) -lpthread

$(BUILD)/sid: $(SRC)/main.cpp $(BUILD)/libsid.so include/sid.h
	$(HIPCC) $(HOSTFLAGS) -o $@ $(SRC)/main.cpp -L$(BUILD) -lsid -Wl,-rpath,'$$ORIGIN' -lpthread

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

# measurement probes (tools/debug, not part of libsid; tools/gpu/probes.sh runs them)
probes: $(BUILD)/libsid.so
	$(HIPCC) -O3 -march=x86-64-v3 -o tools/debug/host_bw_probe tools/debug/host_bw_probe.cpp -lpthread
	$(HIPCC) -O3 -o tools/debug/pcie_probe tools/debug/pcie_probe.cpp -lpthread
	$(HIPCC) -O2 -Iinclude tools/debug/startup_probe.cpp -L$(BUILD) -lsid -Wl,-rpath,'$$ORIGIN' -o $(BUILD)/startup_probe
	$(HIPCC) -O2 -Iinclude tools/debug/exit_probe.cpp -L$(BUILD) -lsid -Wl,-rpath,'$$ORIGIN' -o $(BUILD)/exit_probe

.PHONY: probes
