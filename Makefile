# Builds (all in-tree so the .so files travel to the GPU box with the snapshot):
#   intent-mpc_amd/lib/libimpc_qp.so      product: HIP kernels (gfx950) + C-ABI + host symbolic
#                                         analysis + MPC->QP builder
#   oracle/build/libosqp_oracle.so        test oracle: C restatement of OSQP 0.6.2 (gcc)
#   tests/native/build/libimpc_core_cpu.so test-only CPU build of admm_core.hpp (debug harness)
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
CC      ?= gcc
ROOT    := $(abspath $(dir $(lastword $(MAKEFILE_LIST))))
CSRC    := $(ROOT)/intent-mpc_amd/csrc
LIBDIR  := $(ROOT)/intent-mpc_amd/lib
ORADIR  := $(ROOT)/oracle/build
HARNDIR := $(ROOT)/tests/native/build

# -fno-unroll-loops: the structured kernel's runtime-bound loops (stage recursions, gathers,
# Cholesky) are unrolled by hand where it pays; compiler unrolling of the rest only raises
# register pressure past the 2-waves-per-SIMD budget (measured).
HIPFLAGS  := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -fno-unroll-loops
HOSTFLAGS := -O2 -std=c++17 -fPIC -ffp-contract=off -Wall
# RCCL (multi-GPU cost all-gather, include/impc_comm.h), from the same ROCm as the HIP runtime
LDLIBS    := -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# build identity baked into the library (impc_build_id): every source compiled into it + the flags
SRCS    := $(sort $(wildcard $(CSRC)/*.hip $(CSRC)/*.hpp $(CSRC)/*.cpp $(ROOT)/include/*.h))
BUILD_ID := src-$(shell cat $(SRCS) | { cat; echo '$(HIPFLAGS) $(HOSTFLAGS)'; } | sha256sum | cut -c1-16)
GIT_REV := $(shell git -C $(ROOT) rev-parse --short HEAD 2>/dev/null || echo unknown)
IDFLAGS  = -DIMPC_BUILD_ID='"$(BUILD_ID)$(1)"' -DIMPC_GIT_REV='"$(GIT_REV)"'

LIB     := $(LIBDIR)/libimpc_qp.so
PROFLIB := $(LIBDIR)/libimpc_qp_prof.so
ORACLE  := $(ORADIR)/libosqp_oracle.so
HARNESS := $(HARNDIR)/libimpc_core_cpu.so
EMU     := $(HARNDIR)/libwave_emu.so
EMU64   := $(HARNDIR)/libwave_emu64.so
SHIMT   := $(HARNDIR)/shim_test
REPLANX := $(HARNDIR)/replan_example

.PHONY: all lib oracle harness prof variant clean
all: lib oracle harness
lib: $(LIB)
oracle: $(ORACLE)
harness: $(HARNESS) $(EMU) $(EMU64) $(SHIMT) $(REPLANX)

$(LIBDIR)/impc_qp.o: $(CSRC)/impc_qp.hip $(CSRC)/admm_core.hpp $(CSRC)/symbolic.hpp $(CSRC)/mpc_wave.hpp \
		$(CSRC)/mpc_structure.hpp $(CSRC)/select.hpp $(CSRC)/mpc_build.hpp $(CSRC)/mpc_qp_internal.hpp \
		$(CSRC)/fanout.hpp $(CSRC)/predict.hpp $(CSRC)/comm.hpp $(CSRC)/reftraj.hpp $(ROOT)/include/impc_qp.h $(ROOT)/include/impc_select.h \
		$(ROOT)/include/impc_mpc.h $(ROOT)/include/impc_fanout.h $(ROOT)/include/impc_predict.h $(ROOT)/include/impc_comm.h \
		$(SRCS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(call IDFLAGS,) -c $< -o $@

# section-profiling variant of the library (tools/section_profile.py; never the product)
prof: $(PROFLIB)
$(LIBDIR)/impc_qp_prof.o: $(CSRC)/impc_qp.hip $(CSRC)/admm_core.hpp $(CSRC)/symbolic.hpp $(CSRC)/mpc_wave.hpp \
		$(CSRC)/mpc_structure.hpp $(CSRC)/select.hpp $(CSRC)/mpc_build.hpp $(CSRC)/mpc_qp_internal.hpp \
		$(CSRC)/fanout.hpp $(CSRC)/predict.hpp $(CSRC)/comm.hpp $(CSRC)/reftraj.hpp $(ROOT)/include/impc_qp.h $(ROOT)/include/impc_select.h $(ROOT)/include/impc_mpc.h \
		$(ROOT)/include/impc_fanout.h $(ROOT)/include/impc_predict.h
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(call IDFLAGS,-prof) -DIMPC_SECTION_PROF -c $< -o $@
$(PROFLIB): $(LIBDIR)/impc_qp_prof.o $(LIBDIR)/replan_run.o $(LIBDIR)/symbolic.o $(LIBDIR)/mpc_qp.o $(LIBDIR)/mpc_structure.o $(LIBDIR)/minsnap.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $^ -o $@ $(LDLIBS)

# the batched makePlanWithPred (include/impc_replan.h impc_replan_*): host orchestration + small
# kernels over the library's own entry points
$(LIBDIR)/replan_run.o: $(CSRC)/replan_run.hip $(CSRC)/lib_internal.hpp $(ROOT)/include/impc_replan.h \
		$(ROOT)/include/impc_qp.h $(ROOT)/include/impc_mpc.h $(ROOT)/include/impc_fanout.h $(ROOT)/include/impc_select.h
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/symbolic.o: $(CSRC)/symbolic.cpp $(CSRC)/symbolic.hpp
	@mkdir -p $(LIBDIR)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIBDIR)/minsnap.o: $(CSRC)/minsnap.cpp $(ROOT)/include/impc_minsnap.h $(ROOT)/include/impc_mpc.h
	@mkdir -p $(LIBDIR)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIBDIR)/mpc_qp.o: $(CSRC)/mpc_qp.cpp $(CSRC)/mpc_qp_internal.hpp $(ROOT)/include/impc_mpc.h
	@mkdir -p $(LIBDIR)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIBDIR)/mpc_structure.o: $(CSRC)/mpc_structure.cpp $(CSRC)/mpc_structure.hpp
	@mkdir -p $(LIBDIR)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIB): $(LIBDIR)/impc_qp.o $(LIBDIR)/replan_run.o $(LIBDIR)/symbolic.o $(LIBDIR)/mpc_qp.o $(LIBDIR)/mpc_structure.o $(LIBDIR)/minsnap.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $^ -o $@ $(LDLIBS)

$(ORACLE): $(ROOT)/oracle/osqp_oracle.c
	@mkdir -p $(ORADIR)
	$(CC) -O2 -fPIC -shared -std=c11 -ffp-contract=off -Wall -o $@ $< -lm -lpthread

$(HARNESS): $(ROOT)/tests/native/core_harness.cpp $(CSRC)/admm_core.hpp $(CSRC)/symbolic.cpp $(CSRC)/symbolic.hpp
	@mkdir -p $(HARNDIR)
	$(HIPCC) -x hip -O2 -std=c++17 -fPIC -shared --offload-arch=$(ARCH) -ffp-contract=off \
		$(ROOT)/tests/native/core_harness.cpp -x c++ $(CSRC)/symbolic.cpp -o $@

$(EMU): $(ROOT)/tests/native/wave_emu.cpp $(CSRC)/mpc_wave.hpp $(CSRC)/admm_core.hpp $(CSRC)/mpc_structure.cpp \
		$(CSRC)/mpc_structure.hpp
	@mkdir -p $(HARNDIR)
	$(HIPCC) -x hip --offload-host-only -std=c++20 -O2 -fPIC -shared -ffp-contract=off \
		$(ROOT)/tests/native/wave_emu.cpp -x c++ $(CSRC)/mpc_structure.cpp -o $@

# the one-QP-per-wavefront team shape (64 lanes, four variables per lane) in the same emulation
$(EMU64): $(ROOT)/tests/native/wave_emu.cpp $(CSRC)/mpc_wave.hpp $(CSRC)/admm_core.hpp $(CSRC)/mpc_structure.cpp \
		$(CSRC)/mpc_structure.hpp
	@mkdir -p $(HARNDIR)
	$(HIPCC) -x hip --offload-host-only -std=c++20 -O2 -fPIC -shared -ffp-contract=off -DEMU_NL=64 \
		$(ROOT)/tests/native/wave_emu.cpp -x c++ $(CSRC)/mpc_structure.cpp -o $@

# OsqpEigen shim driver (test-only Eigen stand-in; links the product library)
$(SHIMT): $(ROOT)/tests/native/shim_test.cpp $(ROOT)/include/OsqpEigen/OsqpEigen.h $(LIB)
	@mkdir -p $(HARNDIR)
	$(CXX) -O2 -std=c++17 -Wall -I$(ROOT)/tests/native/mock_eigen -I$(ROOT)/include $< -L$(LIBDIR) -limpc_qp \
		-Wl,-rpath,'$$ORIGIN/../../../intent-mpc_amd/lib' -o $@

# batched makePlanWithPred over the C-ABI only (C++ integration example, driven by the tests)
$(REPLANX): $(ROOT)/tests/native/replan_example.cpp $(ROOT)/include/impc_qp.h $(ROOT)/include/impc_mpc.h \
		$(ROOT)/include/impc_replan.h $(LIB)
	@mkdir -p $(HARNDIR)
	$(CXX) -O2 -std=c++17 -Wall -I$(ROOT)/include $< -L$(LIBDIR) -limpc_qp \
		-Wl,-rpath,'$$ORIGIN/../../../intent-mpc_amd/lib' -o $@

# kernel experiments (tools/ only): make variant V=name DEFS="-DX=1" -> lib/libimpc_qp_<name>.so,
# selected at run time with IMPC_LIB_VARIANT=<name>
variant: $(LIBDIR)/replan_run.o $(LIBDIR)/symbolic.o $(LIBDIR)/mpc_qp.o $(LIBDIR)/mpc_structure.o $(LIBDIR)/minsnap.o
	$(HIPCC) $(HIPFLAGS) $(call IDFLAGS,-$(V)) $(DEFS) -c $(CSRC)/impc_qp.hip -o $(LIBDIR)/impc_qp_$(V).o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(LIBDIR)/impc_qp_$(V).o $^ -o $(LIBDIR)/libimpc_qp_$(V).so $(LDLIBS)

clean:
	rm -rf $(LIBDIR) $(ORADIR) $(HARNDIR)
