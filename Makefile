# Top-level build: the gfx950 HIP library (the product), the drop-in CLI, and
# the CPU oracle (test infrastructure).  `python -c "import __graft_entry__ as g; g.build()"`
# runs the same targets.
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
JOBS ?= 8

# -ffp-contract=off: no FMA contraction, the sum/multiply sequence must stay
# the reference's.  Denormals are kept (no FTZ): diffusion fronts decay into
# the denormal range in long runs.
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fno-gpu-flush-denormals-to-zero -Wall -Wno-pass-failed -Iinclude -Istencil_amd/csrc
CXXFLAGS ?= -O2 -std=c++17 -Wall -Wextra -ffp-contract=off -Iinclude

LIB := stencil_amd/libstencil_hip.so
CLI := build/bin/stencil_main
SRCS := $(wildcard stencil_amd/csrc/*.hip)
OBJS := $(patsubst stencil_amd/csrc/%.hip,build/obj/%.o,$(SRCS))
HOST_SRCS := $(wildcard stencil_amd/csrc/host/*.cpp)
HOST_HDRS := $(wildcard stencil_amd/csrc/host/*.hpp)

all: $(LIB) $(CLI) oracle

build/obj/%.o: stencil_amd/csrc/%.hip $(wildcard stencil_amd/csrc/*.hpp) include/stencil_hip.h
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

$(CLI): $(HOST_SRCS) $(HOST_HDRS) $(LIB) include/stencil_hip.h
	@mkdir -p build/bin
	$(CXX) $(CXXFLAGS) -o $@ $(HOST_SRCS) -Lstencil_amd -lstencil_hip -Wl,-rpath,'$$ORIGIN/../../stencil_amd'

oracle:
	$(MAKE) -C oracle
	bash oracle/ref/build.sh

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
