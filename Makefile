# Build recipe for the MI355X engine (gfx950) and its CPU oracle.
#   make            -> lime_amd/liblime_amd.so, oracle/build/liblime_oracle.so, bin/lime-submit
# hipcc cross-compiles gfx950 without a GPU; outputs stay in-tree (git-ignored)
# so they travel to the GPU box with the gpurun snapshot.
HIPCC   ?= /opt/rocm/bin/hipcc
CXX     ?= g++
CC      ?= gcc
ARCH    ?= gfx950
HIPFLAGS = -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-value \
           -Wno-unused-variable -Wno-unused-result
CXXFLAGS = -O2 -std=c++17 -fPIC -Wall

SRC      = lime_amd/csrc
OBJDIR   = build/obj
HIP_SRCS = $(SRC)/capi.hip $(SRC)/scan.hip $(SRC)/sort.hip $(SRC)/merge.hip \
           $(SRC)/intersect.hip $(SRC)/subtract.hip $(SRC)/complement.hip \
           $(SRC)/bitset.hip $(SRC)/synth.hip $(SRC)/bedparse.hip \
           $(SRC)/bedwrite.hip $(SRC)/closest.hip $(SRC)/route.hip
HIP_OBJS = $(patsubst $(SRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS))
CPP_OBJS = $(OBJDIR)/bed.o
LIB      = lime_amd/liblime_amd.so
ORACLE   = oracle/build/liblime_oracle.so
CLI      = bin/lime-submit

all: $(LIB) $(ORACLE) $(CLI)

# measurement probes (tools/, not part of the product): make probes
probes: bin/bw_probe bin/alloc_probe bin/rocprim_sort_probe

bin/rocprim_sort_probe: tools/rocprim_sort_probe.hip
	@mkdir -p bin
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -Wno-unused-result -o $@ $<

bin/alloc_probe: tools/alloc_probe.hip
	@mkdir -p bin
	$(HIPCC) -O3 --offload-arch=$(ARCH) -Wno-unused-result -o $@ $<

bin/bw_probe: tools/bw_probe.hip
	@mkdir -p bin
	$(HIPCC) -O3 --offload-arch=$(ARCH) -Wno-unused-result -o $@ $<

$(OBJDIR)/%.o: $(SRC)/%.hip $(SRC)/common.hpp include/lime_amd.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/bed.o: $(SRC)/bed.cpp include/lime_amd.h
	@mkdir -p $(OBJDIR)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS) $(CPP_OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^

$(ORACLE): oracle/lime_oracle.c
	@mkdir -p oracle/build
	$(CC) -O2 -fPIC -shared -std=c99 -pthread -o $@ $<

$(CLI): lime_amd/cli/lime_submit.cpp include/lime_amd.hpp include/lime_amd.h $(LIB)
	@mkdir -p bin
	$(CXX) -O2 -std=c++17 -Iinclude -o $@ $< -Llime_amd -llime_amd -Wl,-rpath,'$$ORIGIN/../lime_amd'

clean:
	rm -rf build oracle/build $(LIB) bin

.PHONY: all clean probes

# tuning variant: 3 fill workgroups per CU (tools/ experiments only)
build/var3/liblime_amd.so: $(HIP_SRCS) $(SRC)/common.hpp include/lime_amd.h $(CPP_OBJS)
	@mkdir -p build/var3
	$(HIPCC) $(HIPFLAGS) -DLIME_FILL_WGS=3 -c $(SRC)/intersect.hip -o build/var3/intersect.o
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(filter-out $(OBJDIR)/intersect.o,$(HIP_OBJS)) build/var3/intersect.o $(CPP_OBJS)

# tuning variants of one translation unit (tools/gpu_ab.sh A/B only):
#   make build/var_<name>/liblime_amd.so VAR_SRC=merge VAR_DEFS="-DLIME_MS2_NT=256"
build/var_%/liblime_amd.so: $(HIP_SRCS) $(SRC)/common.hpp include/lime_amd.h $(CPP_OBJS) $(HIP_OBJS)
	@mkdir -p build/var_$*
	$(HIPCC) $(HIPFLAGS) $(VAR_DEFS) -c $(SRC)/$(VAR_SRC).hip -o build/var_$*/$(VAR_SRC).o
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(filter-out $(OBJDIR)/$(VAR_SRC).o,$(HIP_OBJS)) build/var_$*/$(VAR_SRC).o $(CPP_OBJS)
