# Builds every native artefact in-tree (the .so files travel to the GPU box).
#   orb_slam_fusion_amd/lib/liborbgpu.so   HIP kernels + C ABI (gfx950)
#   orb_slam_fusion_amd/lib/liborbsynth.so synthetic workloads (host)
#   oracle/_build/liborboracle.so          CPU oracle (test infrastructure)
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
CSRC     := orb_slam_fusion_amd/csrc
LIB      := orb_slam_fusion_amd/lib
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off -Wall
GPU_SRCS := $(CSRC)/orb_kernels.hip $(CSRC)/pose_kernels.hip $(CSRC)/lba_kernels.hip \
            $(CSRC)/stereo_kernels.hip $(CSRC)/match_kernels.hip $(CSRC)/bow_kernels.hip \
            $(CSRC)/inertial_kernels.hip $(CSRC)/inertial_api.cpp \
            $(CSRC)/orb_plan.cpp $(CSRC)/orb_api.cpp $(CSRC)/pose_api.cpp $(CSRC)/lba_api.cpp \
            $(CSRC)/match_api.cpp $(CSRC)/vocab_api.cpp
GPU_HDRS := $(wildcard $(CSRC)/*.h) $(wildcard $(CSRC)/*.inc) include/orbgpu.h

all: $(LIB)/liborbgpu.so $(LIB)/liborbgpu_checkuniform.so $(LIB)/liborbsynth.so build/valu_calib build/latency_inertial build/latency oracle

OBJDIR   := build/obj
GPU_OBJS := $(patsubst $(CSRC)/%,$(OBJDIR)/%.o,$(GPU_SRCS))

# one object per translation unit (parallel, incremental), then one link
$(OBJDIR)/%.o: $(CSRC)/% $(GPU_HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB)/liborbgpu.so: $(GPU_OBJS)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(GPU_OBJS)

# A/B variant of the library (tools/ab_fast.sh, tools/valu_ab.sh): FAST with
# the survivor list held whole instead of expanded per 64 group entries
VARB_DEF := -DORB_FAST_SV_FULL=1
$(OBJDIR)/varB/%.o: $(CSRC)/% $(GPU_HDRS)
	@mkdir -p $(OBJDIR)/varB
	$(HIPCC) $(HIPFLAGS) $(VARB_DEF) -c -o $@ $<

VARB_OBJS := $(OBJDIR)/varB/orb_kernels.hip.o $(OBJDIR)/varB/orb_plan.cpp.o \
             $(filter-out $(OBJDIR)/orb_kernels.hip.o $(OBJDIR)/orb_plan.cpp.o,$(GPU_OBJS))
$(LIB)/liborbgpu_varB.so: $(VARB_OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

varB: $(LIB)/liborbgpu_varB.so

# debug variant: every wave-uniform branch (uniform_dev.h) checks that all
# active lanes agree; orbgpu_debug_uniform_violations() reports the count
# (tests/conftest.py asserts zero after each test when this library is loaded:
# ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_checkuniform.so pytest -m gpu)
$(OBJDIR)/cu/%.o: $(CSRC)/% $(GPU_HDRS)
	@mkdir -p $(OBJDIR)/cu
	$(HIPCC) $(HIPFLAGS) -DORBGPU_CHECK_UNIFORM=1 -c -o $@ $<

CU_OBJS := $(patsubst $(CSRC)/%,$(OBJDIR)/cu/%.o,$(GPU_SRCS))
$(LIB)/liborbgpu_checkuniform.so: $(CU_OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

checkuniform: $(LIB)/liborbgpu_checkuniform.so

# ad-hoc A/B variant of the extractor (orb_kernels.hip and orb_plan.cpp
# compiled with DEFS, every other object shared): make var NAME=pf4 DEFS=-DORB_BLUR_PF=4
var: $(GPU_OBJS)
	@mkdir -p $(OBJDIR)/var_$(NAME)
	$(HIPCC) $(HIPFLAGS) $(DEFS) -c -o $(OBJDIR)/var_$(NAME)/orb_kernels.hip.o $(CSRC)/orb_kernels.hip
	$(HIPCC) $(HIPFLAGS) $(DEFS) -c -o $(OBJDIR)/var_$(NAME)/orb_plan.cpp.o $(CSRC)/orb_plan.cpp
	$(HIPCC) $(HIPFLAGS) -shared -o $(LIB)/liborbgpu_$(NAME).so $(OBJDIR)/var_$(NAME)/orb_kernels.hip.o \
	  $(OBJDIR)/var_$(NAME)/orb_plan.cpp.o $(filter-out $(OBJDIR)/orb_kernels.hip.o $(OBJDIR)/orb_plan.cpp.o,$(GPU_OBJS))

$(LIB)/liborbsynth.so: $(CSRC)/synth.cpp
	@mkdir -p $(LIB)
	$(CXX) -std=c++17 -O2 -fPIC -shared -o $@ $<

# VALU-issue calibration kernel for the SQ counters (tools/profile_round.sh)
build/valu_calib: tools/valu_calib.hip
	@mkdir -p build
	$(HIPCC) --offload-arch=$(ARCH) -O3 -fno-slp-vectorize -o $@ $<

# C++ caller of the C ABI for the per-frame stereo-inertial latency
# (tools/bench_latency_inertial.py runs it beside its Python leg)
build/latency_inertial: tools/latency_inertial.cc include/orbgpu.h $(LIB)/liborbgpu.so
	@mkdir -p build
	$(CXX) -std=c++17 -O2 -pthread -o $@ $< -L$(LIB) -lorbgpu -Wl,-rpath,'$$ORIGIN/../$(LIB)'

# C++ caller of the C ABI for the per-frame extract + PoseOptimization latency
# (tools/bench_latency.py runs it beside its Python leg); frames from liborbsynth
build/latency: tools/latency.cc include/orbgpu.h $(LIB)/liborbgpu.so $(LIB)/liborbsynth.so
	@mkdir -p build
	$(CXX) -std=c++17 -O2 -pthread -o $@ $< -L$(LIB) -lorbgpu -lorbsynth -Wl,-rpath,'$$ORIGIN/../$(LIB)'

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(LIB) oracle/_build build

# profiling variant: per-phase s_memtime totals (orbgpu_debug_stamps)
# STAMPS=1: k_fast_cells (+ pose kernel), STAMPS=2: k_octree
STAMPS ?= 1
STAMP_DEFS ?=
stamps:
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -DORB_STAMPS=$(STAMPS) $(STAMP_DEFS) -shared -o $(LIB)/liborbgpu_stamps.so $(GPU_SRCS)

.PHONY: varB var all oracle clean stamps checkuniform
