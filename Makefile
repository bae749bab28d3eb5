# Build of the MI355X renderer (gfx950) and its CLI. No cmake: hipcc only.
#   make            -> simpleraytracer_amd/lib/libModelRunner.so, bin/test_app
#   make oracle     -> oracle/build/libsrt_oracle.so (CPU checker; test infrastructure)
#   make ref        -> oracle/_ref/* (reference test_app built from /root/reference, if present)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
BUILD    := build/obj
LIBDIR   := simpleraytracer_amd/lib
LIB      := $(LIBDIR)/libModelRunner.so
CSRC     := simpleraytracer_amd/csrc

# -ffp-contract=off: every FMA in the canonical math is an explicit fmaf.
# -fno-slp-vectorize: keeps hipcc from pairing independent fp32 FMAs into v_pk_fma_f32 plus
#  register shuffles (packed f32 has no throughput advantage on gfx950).
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
            -fvisibility=hidden -DRADEONPROML_BUILD -Iinclude -Wall -Wno-unused-result
LDFLAGS  := -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined

OBJS := $(BUILD)/render.o $(BUILD)/spatial.o $(BUILD)/renderer.o $(BUILD)/engine.o $(BUILD)/comm.o $(BUILD)/cpu_render.o \
        $(BUILD)/scene.o $(BUILD)/image.o $(BUILD)/model.o $(BUILD)/context.o $(BUILD)/srt_api.o

HEADERS := $(wildcard $(CSRC)/*.h) include/model_runner.h include/srt_render.h

# Diagnostic build (per-block cull phase counters, srtDiagRead): never the product library.
DIAG_BUILD := build/diag
DIAG_LIB   := simpleraytracer_amd/lib_diag/libModelRunner.so
DIAG_OBJS  := $(patsubst $(BUILD)/%,$(DIAG_BUILD)/%,$(OBJS))

.PHONY: all oracle ref clean diag exp
all: $(LIB) bin/test_app

$(BUILD)/%.o: $(CSRC)/%.hip $(HEADERS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: $(CSRC)/%.cpp $(HEADERS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# The CPU backend: hardware fma (x86-64-v3) for its explicit fmaf; still no contraction.
$(BUILD)/cpu_render.o: $(CSRC)/cpu_render.cpp $(HEADERS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -mfma -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(OBJS) -o $@ $(LDFLAGS)

bin/test_app: tools/test_app.cpp $(LIB) include/model_runner.h include/srt_render.h
	@mkdir -p bin
	g++ -O2 -std=c++17 -Wall -Iinclude $< -o $@ -L$(LIBDIR) -lModelRunner -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)'

$(DIAG_BUILD)/%.o: $(CSRC)/%.hip $(HEADERS)
	@mkdir -p $(DIAG_BUILD)
	$(HIPCC) $(HIPFLAGS) -DSRT_DIAG -c $< -o $@

$(DIAG_BUILD)/%.o: $(CSRC)/%.cpp $(HEADERS)
	@mkdir -p $(DIAG_BUILD)
	$(HIPCC) $(HIPFLAGS) -DSRT_DIAG -c $< -o $@

$(DIAG_LIB): $(DIAG_OBJS)
	@mkdir -p $(dir $(DIAG_LIB))
	$(HIPCC) --offload-arch=$(ARCH) $(DIAG_OBJS) -o $@ $(LDFLAGS)

diag: $(DIAG_LIB)

# Experiment builds (measurement only): make exp EXP_NAME=x EXP_FLAGS="-DSRT_...=..." ->
# simpleraytracer_amd/lib_exp/x/libModelRunner.so (select with env SRT_LIB).
EXP_NAME  ?= default
EXP_FLAGS ?=
EXP_BUILD := build/exp/$(EXP_NAME)
EXP_LIB   := simpleraytracer_amd/lib_exp/$(EXP_NAME)/libModelRunner.so
exp:
	@mkdir -p $(EXP_BUILD) $(dir $(EXP_LIB))
	$(HIPCC) $(HIPFLAGS) $(EXP_FLAGS) -c $(CSRC)/render.hip -o $(EXP_BUILD)/render.o
	$(HIPCC) --offload-arch=$(ARCH) $(EXP_BUILD)/render.o $(filter-out $(BUILD)/render.o,$(OBJS)) -o $(EXP_LIB) $(LDFLAGS)

oracle:
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

clean:
	rm -rf build bin $(LIBDIR) $(dir $(DIAG_LIB)) simpleraytracer_amd/lib_exp
	$(MAKE) -C oracle clean

# A/B builds of the whole library (measurement only): make ab AB_NAME=x AB_FLAGS="-DSRT_...=..." ->
# simpleraytracer_amd/lib_ab/x/libModelRunner.so (every object compiled with the flags; SRT_LIB).
AB_NAME  ?= default
AB_FLAGS ?=
AB_BUILD := build/ab/$(AB_NAME)
AB_LIB   := simpleraytracer_amd/lib_ab/$(AB_NAME)/libModelRunner.so
AB_OBJS  := $(patsubst $(BUILD)/%,$(AB_BUILD)/%,$(OBJS))
$(AB_BUILD)/%.o: $(CSRC)/%.hip $(HEADERS)
	@mkdir -p $(AB_BUILD)
	$(HIPCC) $(HIPFLAGS) $(AB_FLAGS) -c $< -o $@
$(AB_BUILD)/cpu_render.o: $(CSRC)/cpu_render.cpp $(HEADERS)
	@mkdir -p $(AB_BUILD)
	$(HIPCC) $(HIPFLAGS) $(AB_FLAGS) -mfma -c $< -o $@
$(AB_BUILD)/%.o: $(CSRC)/%.cpp $(HEADERS)
	@mkdir -p $(AB_BUILD)
	$(HIPCC) $(HIPFLAGS) $(AB_FLAGS) -c $< -o $@
$(AB_LIB): $(AB_OBJS)
	@mkdir -p $(dir $(AB_LIB))
	$(HIPCC) --offload-arch=$(ARCH) $(AB_OBJS) -o $@ $(LDFLAGS)
.PHONY: ab
ab: $(AB_LIB)

# CPU sanitizer build (SURVEY.md section 5 "Build the CPU oracle with ASan/UBSan"): the library's host
# code (every hipcc line takes each -fsanitize= after -Xarch_host: the gfx950 code objects are built as
# usual) and the oracle under AddressSanitizer + UndefinedBehaviorSanitizer, for the CPU test suite on a
# host without a GPU (ML_VISIBLE_DEVICES=cpu backend, scene files, the ABI, the oracle):
#   make asan && tools/asan_tests.sh      (log: profiles/r04/asan/)
ASAN_BUILD  := build/asan
ASAN_LIB    := simpleraytracer_amd/lib_asan/libModelRunner.so
ASAN_ORACLE := oracle/build_asan/libsrt_oracle.so
ASAN_HOST   := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer \
               -Xarch_host -fno-sanitize-recover=undefined
ASAN_OBJS   := $(patsubst $(BUILD)/%,$(ASAN_BUILD)/%,$(OBJS))
LLVM_BIN    := /opt/rocm/lib/llvm/bin
$(ASAN_BUILD)/%.o: $(CSRC)/%.hip $(HEADERS)
	@mkdir -p $(ASAN_BUILD)
	$(HIPCC) $(HIPFLAGS) $(ASAN_HOST) -g -c $< -o $@
$(ASAN_BUILD)/cpu_render.o: $(CSRC)/cpu_render.cpp $(HEADERS)
	@mkdir -p $(ASAN_BUILD)
	$(HIPCC) $(HIPFLAGS) $(ASAN_HOST) -g -mfma -c $< -o $@
$(ASAN_BUILD)/%.o: $(CSRC)/%.cpp $(HEADERS)
	@mkdir -p $(ASAN_BUILD)
	$(HIPCC) $(HIPFLAGS) $(ASAN_HOST) -g -c $< -o $@
# No --no-undefined: the sanitizer runtime is preloaded into the test process (tools/asan_tests.sh).
$(ASAN_LIB): $(ASAN_OBJS)
	@mkdir -p $(dir $(ASAN_LIB))
	$(HIPCC) --offload-arch=$(ARCH) $(ASAN_HOST) $(ASAN_OBJS) -o $@ -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
$(ASAN_ORACLE): oracle/srt_oracle.c oracle/srt_oracle.h
	@mkdir -p $(dir $(ASAN_ORACLE))
	$(LLVM_BIN)/clang -O1 -g -std=c11 -fPIC -ffp-contract=off -mfma -fopenmp -Wall -Wextra \
	    -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined \
	    -shared oracle/srt_oracle.c -o $@ -lm -L/opt/rocm/lib/llvm/lib -Wl,-rpath,/opt/rocm/lib/llvm/lib
.PHONY: asan
asan: $(ASAN_LIB) $(ASAN_ORACLE)
