# Top-level build: the gfx950 HIP library (the product), the drop-in CLI, and
# the CPU oracle (test infrastructure).  `python -c "import __graft_entry__ as g; g.build()"`
# runs the same targets.
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
JOBS ?= 8

# -ffp-contract=off: no FMA contraction, the sum/multiply sequence must stay
# the reference's.  Denormals are kept (no FTZ): diffusion fronts decay into
# the denormal range in long runs.  -fno-slp-vectorize: the SLP
# vectoriser pairs independent fp32 adds of different rows into v_pk_add_f32,
# and in the fp32 one-cell-per-lane box shapes of the pre-round-3 box order
# LLVM's GCN DPP Combine pass then miscompiles that code (DESIGN.md §9.2b:
# opt-bisect pins it to that pass; without SLP it is bitwise right); the
# kernels' own vector types still give packed math within a lane.  Measured
# equal or faster everywhere (fp32 box +6 %, profiles/r03/r03f_slp_ab.txt).
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
            -fno-gpu-flush-denormals-to-zero -Wall -Wno-pass-failed -Iinclude -Istencil_amd/csrc
CXXFLAGS ?= -O2 -std=c++17 -Wall -Wextra -ffp-contract=off -Iinclude

# The product library and its debug twin: the same kernel objects, linked
# with knobs.cpp built without / with -DSTENCIL_DEBUG_KNOBS (the debug library
# reads the experiment knobs -- workgroup shapes, forced z-chunks -- from the
# environment; the product runs AUTO's plan only).
LIB := stencil_amd/libstencil_hip.so
LIB_DBG := stencil_amd/libstencil_hip_debug.so
CLI := build/bin/stencil_main
SRCS := $(wildcard stencil_amd/csrc/*.hip)
OBJ ?= build/obj
# kernels_boxk_probe.hip (a code-generation probe) is built twice, with and without SLP
# vectorisation, and linked into the debug library only; the product links knobs.cpp's stubs instead
PROBE_OBJS := $(OBJ)/kernels_boxk_probe.o $(OBJ)/kernels_boxk_probe_noslp.o $(OBJ)/kernels_strip_probe.o
OBJS := $(filter-out $(PROBE_OBJS),$(patsubst stencil_amd/csrc/%.hip,$(OBJ)/%.o,$(SRCS)))
HOST_SRCS := $(wildcard stencil_amd/csrc/host/*.cpp)
HOST_HDRS := $(wildcard stencil_amd/csrc/host/*.hpp)

# test infrastructure: slab_core.hpp's round logic on a CPU fake device (sweeps by the oracle)
FAKE := tests/cpu_slab/libslab_fake.so

all: $(LIB) $(LIB_DBG) $(CLI) oracle $(FAKE)

$(OBJ)/%.o: stencil_amd/csrc/%.hip $(wildcard stencil_amd/csrc/*.hpp) include/stencil_hip.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/knobs.o: stencil_amd/csrc/knobs.cpp stencil_amd/csrc/common.hpp include/stencil_hip.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/knobs_debug.o: stencil_amd/csrc/knobs.cpp stencil_amd/csrc/common.hpp include/stencil_hip.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DSTENCIL_DEBUG_KNOBS -c $< -o $@

# the max-ILP copy of the strip kernel (kernels_strip_ilp.hip includes kernels_strip.hip); the scheduler
# flag goes to the device compilation only (the host x86 backend has no such scheduler)
$(OBJ)/kernels_strip_ilp.o: stencil_amd/csrc/kernels_strip.hip
$(OBJ)/kernels_strip_ilp.o: HIPFLAGS += -Xarch_device -mllvm=-misched=gcn-max-ilp
# the strip probe (debug library only): the max-ILP shapes again, as a compile-time variant
$(OBJ)/kernels_strip_probe.o: stencil_amd/csrc/kernels_strip.hip
$(OBJ)/kernels_strip_probe.o: HIPFLAGS += -Xarch_device -mllvm=-misched=gcn-max-ilp
# the 2D kernels (tb2ds / tb2d / tb2d1) under the same scheduler: C1 fp64 +1.4 %, fp32 +2.3 %, the rest within
# +-1.3 % (profiles/r03/r03am_*, r03an_*)
$(OBJ)/kernels_tb2d.o: HIPFLAGS += -Xarch_device -mllvm=-misched=gcn-max-ilp
# the box kernels without the scheduler's unclustered high-register-pressure stage: C5 (2048^3 fp64) +1.3 %,
# fp32 512^3 +1.8 %, other box shapes within 1 % (profiles/r03/r03ap_*, r03aq_*)
$(OBJ)/kernels_boxk.o: HIPFLAGS += -Xarch_device -mllvm=-amdgpu-disable-unclustered-high-rp-reschedule

$(OBJ)/kernels_boxk_probe_noslp.o: stencil_amd/csrc/kernels_boxk_probe.hip stencil_amd/csrc/kernels_boxk.hip $(wildcard stencil_amd/csrc/*.hpp) include/stencil_hip.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DPROBE_NOSLP -fno-slp-vectorize -c $< -o $@

$(OBJ)/kernels_boxk_probe.o: stencil_amd/csrc/kernels_boxk_probe.hip stencil_amd/csrc/kernels_boxk.hip $(wildcard stencil_amd/csrc/*.hpp) include/stencil_hip.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -fslp-vectorize -c $< -o $@

$(LIB): $(OBJS) $(OBJ)/knobs.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) $(OBJ)/knobs.o

$(LIB_DBG): $(OBJS) $(PROBE_OBJS) $(OBJ)/knobs_debug.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) $(PROBE_OBJS) $(OBJ)/knobs_debug.o

$(CLI): $(HOST_SRCS) $(HOST_HDRS) $(LIB) include/stencil_hip.h
	@mkdir -p build/bin
	$(CXX) $(CXXFLAGS) -o $@ $(HOST_SRCS) -Lstencil_amd -lstencil_hip -Wl,-rpath,'$$ORIGIN/../../stencil_amd'

oracle:
	$(MAKE) -C oracle
	bash oracle/ref/build.sh

oracle/liboracle.so: oracle/oracle.c oracle/oracle_impl.inc oracle/oracle.h
	$(MAKE) -C oracle

$(FAKE): tests/cpu_slab/fake_dev.cpp stencil_amd/csrc/slab_core.hpp stencil_amd/csrc/errors.hpp include/stencil_hip.h oracle/liboracle.so
	$(CXX) $(CXXFLAGS) -fPIC -shared -pthread -Istencil_amd/csrc -Ioracle -o $@ $< -Loracle -loracle \
	    -Wl,-rpath,'$$ORIGIN/../../oracle'

clean:
	rm -rf build $(LIB) $(LIB_DBG) $(FAKE)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
