# Build of the MI355X-native heat engine.
#   make            -> parallel_heat_amd/_lib/libheat.so  and  build/heat (CLI)
#   make asm        -> gfx950 ISA of the kernels in build/asm/ (inspection)
#   make resources  -> per-kernel VGPR/SGPR/LDS/occupancy report
# Everything targets gfx950 only (MI355X / CDNA4).
ROCM    ?= /opt/rocm
HIPCC   ?= $(ROCM)/bin/hipcc
ARCH    ?= gfx950
BUILD   ?= build
LIBDIR  := parallel_heat_amd/_lib
CXXSTD  := -std=c++17
# Host code: x86-64-v3 (FMA/AVX2) so the CPU oracle's fmaf is a single
# instruction; device code: gfx950.
COMMON  := $(CXXSTD) -O3 -fPIC -Wall -Wno-unused-result -Icsrc/include -mfma -mavx2 \
           -fopenmp
HIPFLAGS := $(COMMON) --offload-arch=$(ARCH) -munsafe-fp-atomics
LDFLAGS := -fopenmp -L$(ROCM)/lib -lrccl -ldl -Wl,-rpath,$(ROCM)/lib

SRCS_CPP := $(wildcard csrc/src/*.cpp)
# Experiment kernels (csrc/kernels/tb_exp.hpp): builds measured slower than
# the defaults, kept for A/Bs and their bitwise tests in their own library
# (`make exp` -> libheat_exp.so, loaded on demand), not in libheat.so.
EXP_HIP  := csrc/kernels/tb_packed.hip csrc/kernels/tb_narrow.hip csrc/kernels/tb_split_mixed.hip \
            csrc/kernels/tb_split_pk.hip csrc/kernels/tb_chain.hip csrc/kernels/exp_register.hip
SRCS_HIP := $(filter-out $(EXP_HIP),$(wildcard csrc/kernels/*.hip))
EXP_OBJS := $(patsubst csrc/kernels/%.hip,$(BUILD)/obj/%.o,$(EXP_HIP))
HDRS     := $(wildcard csrc/include/heat/*.hpp csrc/include/heat/*.h)
OBJS     := $(patsubst csrc/src/%.cpp,$(BUILD)/obj/%.o,$(SRCS_CPP)) \
            $(patsubst csrc/kernels/%.hip,$(BUILD)/obj/%.o,$(SRCS_HIP))

all: $(LIBDIR)/libheat.so $(BUILD)/heat

exp: $(LIBDIR)/libheat_exp.so

# Header dependencies come from the compiler (-MMD): a header edit rebuilds
# only the objects that include it (the TB kernel builds take minutes each).
DEPFLAGS = -MMD -MP
$(BUILD)/obj/%.o: csrc/src/%.cpp
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(DEPFLAGS) -x hip -c $< -o $@

KHDRS    := $(wildcard csrc/kernels/*.hpp csrc/kernels/*.inl)
$(BUILD)/obj/tb_scalar.o $(BUILD)/obj/tb_split.o $(BUILD)/obj/tb_tile.o $(BUILD)/obj/tb_resident.o \
  $(BUILD)/obj/tb_tile_xl0.o $(BUILD)/obj/tb_tile_xl1.o $(BUILD)/obj/tb_tile_xl2.o \
  $(BUILD)/obj/tb_resident_xl0.o $(BUILD)/obj/tb_resident_xl1.o $(BUILD)/obj/tb_resident_xl2.o \
  $(BUILD)/obj/tb_split_rla.o $(BUILD)/obj/tb_split_rlb.o $(BUILD)/obj/tb_split_rlc.o \
  $(BUILD)/obj/tb_split_mixed.o $(BUILD)/obj/tb_split_nt.o $(BUILD)/obj/tb_split_pk.o \
  $(BUILD)/obj/tb_chain.o: HIPFLAGS += -fno-slp-vectorize
# The streaming split build that runs the whole-GPU plates (8192^2 and up)
# takes LLVM's max-ILP machine scheduler: +1.5 % at 8192^2 in an interleaved
# same-box A/B; the resident tiles keep the default scheduler (no gain there).
# profiles/r6_sched.md
$(BUILD)/obj/tb_split_nt.o: HIPFLAGS += -mllvm -amdgpu-sched-strategy=max-ilp

$(BUILD)/obj/%.o: csrc/kernels/%.hip
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(DEPFLAGS) -c $< -o $@

-include $(OBJS:.o=.d) $(EXP_OBJS:.o=.d)
# An object without its .d file (built before -MMD, or never built) depends
# on every header: a shared-header edit can never link objects built against
# two layouts of one struct (TbArgs).
$(foreach o,$(OBJS) $(EXP_OBJS),$(if $(wildcard $(o:.o=.d)),,$(eval $(o): $(HDRS) $(KHDRS))))

# Linked under a temporary name and renamed: a copy of the tree taken while
# a build runs holds the old library or the new one, never a partial file.
$(LIBDIR)/libheat.so: $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@.tmp $(OBJS) $(LDFLAGS) && mv -f $@.tmp $@

# The experiment kernels link against the product library (the registry and
# every shared helper live there; rpath $ORIGIN: the copy next to it).
$(LIBDIR)/libheat_exp.so: $(EXP_OBJS) $(LIBDIR)/libheat.so
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@.tmp $(EXP_OBJS) -L$(LIBDIR) -l:libheat.so \
	  -Wl,-rpath,'$$ORIGIN' $(LDFLAGS) && mv -f $@.tmp $@

$(BUILD)/heat: csrc/apps/heat_main.cpp $(OBJS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -x hip csrc/apps/heat_main.cpp -x none $(OBJS) -o $@.tmp $(LDFLAGS) && mv -f $@.tmp $@

probe: $(BUILD)/overlap_probe
$(BUILD)/overlap_probe: tools/overlap_probe.cpp $(OBJS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -x hip tools/overlap_probe.cpp -x none $(OBJS) -o $@ $(LDFLAGS)

# One kernel source at a time (ASM=tb_split), with the same per-file flags as
# the object build: the TB builds take ~10 minutes each.
ASM ?= tb_split
asm:
	@mkdir -p $(BUILD)/asm
	cd $(BUILD)/asm && $(HIPCC) $(patsubst -Icsrc/include,-I../../csrc/include,$(HIPFLAGS)) \
	  $(if $(filter tb_scalar tb_split tb_tile,$(ASM)),-fno-slp-vectorize) --offload-device-only -S \
	  -o $(ASM).s ../../csrc/kernels/$(ASM).hip

# Every kernel of every unit, from the built library's code-object metadata
# (VGPR/AGPR/SGPR, scratch bytes per lane, spilled VGPRs, LDS);
# tests/test_kernel_resources.py holds the hot kernels to a scratch budget.
resources: $(LIBDIR)/libheat.so
	python3 tools/kernel_resources.py $(LIBDIR)/libheat.so

clean:
	rm -rf $(BUILD) $(LIBDIR)/libheat.so $(LIBDIR)/libheat_exp.so

.PHONY: all exp asm resources clean

# Host-only self-test of the CPU components, plain and under ASan/UBSan.
SELFTEST_SRCS := csrc/tests/selftest.cpp csrc/src/common.cpp csrc/src/topology.cpp \
                 csrc/src/io.cpp csrc/src/cpu_backend.cpp
$(BUILD)/selftest: $(SELFTEST_SRCS) $(HDRS)
	@mkdir -p $(BUILD)
	g++ -std=c++17 -O2 -g -Wall -Icsrc/include -mfma -mavx2 -fopenmp $(SELFTEST_SRCS) -o $@
$(BUILD)/selftest-asan: $(SELFTEST_SRCS) $(HDRS)
	@mkdir -p $(BUILD)
	g++ -std=c++17 -O1 -g -Wall -Icsrc/include -mfma -mavx2 -fopenmp \
	  -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=all \
	  $(SELFTEST_SRCS) -o $@
selftest: $(BUILD)/selftest
	$(BUILD)/selftest
selftest-asan: $(BUILD)/selftest-asan
	ASAN_OPTIONS=detect_leaks=1 $(BUILD)/selftest-asan
.PHONY: selftest selftest-asan

# Reference-compatible program names (mpi/Makefile:12-22, cuda/Makefile:13):
#   make ref-variants SIZE=900 STEPS=10000 STEP=20 THREADS=4
# writes build/ref/{heat_N,heat_omp_N,heat_con_N,heat_con_omp_N,cuda_heat}; run
# them as `NP=4 build/ref/heat_omp_900` (NP processes, like mpirun -np).
SIZE ?= 900
STEPS ?= 10000
STEP ?= 20
THREADS ?= 4
ref-variants: $(BUILD)/heat
	@mkdir -p $(BUILD)/ref
	@for v in "heat_$(SIZE):--threads 1" "heat_omp_$(SIZE):--threads $(THREADS)" \
	          "heat_con_$(SIZE):--threads 1 --converge --check-interval $(STEP)" \
	          "heat_con_omp_$(SIZE):--threads $(THREADS) --converge --check-interval $(STEP)"; do \
	  name=$${v%%:*}; args=$${v#*:}; \
	  printf '#!/bin/bash\n# %s: reference mpi/Makefile variant\nexec python3 -m torch.distributed.run --no-python --standalone --local-addr 127.0.0.1 --nproc-per-node $${NP:-1} %s --backend cpu --nx %s --ny %s --steps %s --naming mpi %s "$$@"\n' \
	    "$$name" "$(abspath $(BUILD)/heat)" $(SIZE) $(SIZE) $(STEPS) "$$args" > $(BUILD)/ref/$$name; \
	  chmod +x $(BUILD)/ref/$$name; done
	@printf '#!/bin/bash\n# cuda_heat: reference cuda/Makefile program\nexec %s --backend hip --nx %s --ny %s --steps %s --naming cuda "$$@"\n' \
	  "$(abspath $(BUILD)/heat)" $(SIZE) $(SIZE) $(STEPS) > $(BUILD)/ref/cuda_heat; chmod +x $(BUILD)/ref/cuda_heat
	@ls $(BUILD)/ref
.PHONY: ref-variants
