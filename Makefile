# Builds build/libbert.so — the drop-in for the reference's libbert.so
# (the path examples/sample_dylib.py:17 and benchmarks/run_mteb.py:47 dlopen).
#   make            -> build/libbert.so (HIP kernels for gfx950 + host runtime)
#   make oracle     -> oracle/_build/liboracle.so (CPU checker, tests only)
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
BUILD := build
SRC := embedding.cpp_amd/csrc
INC := -Iinclude -I$(SRC)
HOST_SRCS := gguf_io.cpp quantize.cpp quantize_model.cpp synth.cpp tokenizer.cpp runtime.cpp
HOST_OBJS := $(addprefix $(BUILD)/obj/,$(HOST_SRCS:.cpp=.o))
HIP_OBJS := $(BUILD)/obj/kernels.o $(BUILD)/obj/gemm_i8.o
# the library's sources, in the order bench.py's src_hash() reads them
SRC_HASH_FILES := $(sort $(wildcard $(SRC)/*.hip $(SRC)/*.cpp $(SRC)/*.h $(SRC)/*.inc include/*.h include/ggml/*.h)) Makefile
CXXFLAGS := -O2 -std=c++17 -fPIC -fvisibility=hidden -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-result \
            -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $(INC)
HIPFLAGS := -O3 -std=c++17 -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -Wno-unused-value -Wno-unused-result -fPIC -fvisibility=hidden -ffp-contract=off --offload-arch=$(ARCH) $(INC)

all: $(BUILD)/libbert.so $(BUILD)/div_check $(BUILD)/qkva_check $(BUILD)/mfma_bf16_split_probe $(BUILD)/tok_bench

$(BUILD)/obj/%.o: $(SRC)/%.cpp $(wildcard $(SRC)/*.h) include/bert.h include/bert_amd.h
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(BUILD)/obj/tokenizer.o: $(SRC)/unicode_tables.inc

$(BUILD)/obj/%.o: $(SRC)/%.hip $(SRC)/kernels.h $(SRC)/kernels_common.h $(SRC)/i8_core.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/libbert.so: $(HOST_OBJS) $(HIP_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread
	@# the commit this library was built from (bench.py / tools/pmc_traffic.py record it), and a
	@# hash of the sources it was built from (bench.py compares it with the tree it runs in, so a
	@# library built just before its sources were committed is still identified as their build)
	@{ git rev-parse HEAD 2>/dev/null || echo unknown; } | tr -d '\n' > $(BUILD)/BUILD_INFO
	@git diff --quiet HEAD -- embedding.cpp_amd include 2>/dev/null || printf ' +uncommitted' >> $(BUILD)/BUILD_INFO
	@printf ' src=%s' "$$(cat $(SRC_HASH_FILES) | sha256sum | cut -c1-16)" >> $(BUILD)/BUILD_INFO

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD)

.PHONY: all oracle clean

# development timing harness for the GEMM kernels (not shipped)
$(BUILD)/gemm_bench: tools/gemm_bench.hip embedding.cpp_amd/csrc/kernels.hip embedding.cpp_amd/csrc/kernels.h
	$(HIPCC) $(HIPFLAGS) $< -o $@

# device check that the short Q8 scale divisions equal IEEE division (tests/test_gpu_parity.py)
$(BUILD)/div_check: tools/div_check.hip
	@mkdir -p $(BUILD)
	$(HIPCC) -O3 --offload-arch=$(ARCH) -Wno-unused-value -Wno-unused-result $< -o $@

# device probe of the bf16 partial-product scale products (tests/test_gpu_parity.py)
$(BUILD)/mfma_bf16_split_probe: tools/mfma_bf16_split_probe.hip
	@mkdir -p $(BUILD)
	$(HIPCC) -O3 --offload-arch=$(ARCH) $< -o $@

# host-only tokenizer timing (development; DESIGN.md §6 consumer line)
$(BUILD)/tok_bench: tools/tok_bench.cpp $(BUILD)/obj/gguf_io.o $(BUILD)/obj/tokenizer.o
	@mkdir -p $(BUILD)
	$(CXX) -O2 -std=c++17 -I$(SRC) $^ -o $@ -lpthread

# development timing harness for the int8-MFMA GEMMs (not shipped)

$(BUILD)/i8_bench$(I8_SUFFIX): tools/i8_bench.hip $(SRC)/gemm_i8.hip $(SRC)/kernels.h $(SRC)/kernels_common.h $(SRC)/i8_core.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $< -o $@

# development check of the fused kernel's head-pair grouping, F16 (tools/qkva_check.hip)
$(BUILD)/qkva_check: tools/qkva_check.hip $(SRC)/kernels.hip $(SRC)/kernels.h $(SRC)/kernels_common.h $(SRC)/i8_core.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $< -o $@

# host code (GGUF reader/writer, tokenizer, quantiser) under ASan + UBSan, CPU only (tests/test_sanitizers.py)
SAN_SRCS := $(SRC)/gguf_io.cpp $(SRC)/tokenizer.cpp $(SRC)/quantize.cpp $(SRC)/quantize_model.cpp $(SRC)/synth.cpp tools/host_sanitize.cpp
$(BUILD)/host_sanitize: $(SAN_SRCS) $(wildcard $(SRC)/*.h) $(SRC)/unicode_tables.inc
	@mkdir -p $(BUILD)
	$(CXX) -O1 -g -std=c++17 -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer \
	    -Iinclude -I$(SRC) $(SAN_SRCS) -o $@ -lpthread

# The reference's own consumer programs (examples/server.cpp, main.cpp), compiled unchanged
# against include/ and linked with build/libbert.so — only where the reference checkout is
# present (this container); the binaries travel to the GPU box with the tree
# (tests/test_gpu_parity.py::test_reference_server_drop_in runs the server there).
REF ?= /root/reference
$(BUILD)/ref_%: $(REF)/examples/%.cpp $(BUILD)/libbert.so include/bert.h include/ggml.h
	$(CXX) -std=c++17 -O2 -Iinclude $< -o $@ -L$(BUILD) -lbert -Wl,-rpath,'$$ORIGIN'

# models/quantize.cpp (reference) includes "ggml/ggml.h": include/ggml/ggml.h is the same shim
$(BUILD)/ref_quantize: $(REF)/models/quantize.cpp $(BUILD)/libbert.so include/bert.h include/ggml/ggml.h
	$(CXX) -std=c++17 -O2 -Iinclude $< -o $@ -L$(BUILD) -lbert -Wl,-rpath,'$$ORIGIN'

ref_consumers: $(BUILD)/ref_server $(BUILD)/ref_main $(BUILD)/ref_quantize
.PHONY: ref_consumers

# development timing of the fused kernel's phases (tools/qkva_time.hip)
$(BUILD)/qkva_time: tools/qkva_time.hip $(SRC)/kernels.hip $(SRC)/kernels.h $(SRC)/kernels_common.h $(SRC)/i8_core.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $< -o $@

# FETCH_SIZE / WRITE_SIZE calibration per access width (tools/pmc_calib.hip)
$(BUILD)/pmc_calib: tools/pmc_calib.hip
	@mkdir -p $(BUILD)
	$(HIPCC) -O3 --offload-arch=gfx950 $< -o $@

# development per-phase stamps of the persistent int8 GEMMs (tools/phase_stamps.hip)
$(BUILD)/phase_stamps: tools/phase_stamps.hip $(SRC)/gemm_i8.hip $(SRC)/kernels.h $(SRC)/kernels_common.h $(SRC)/i8_core.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $< -o $@

# the fused kernel's phase stamps (tools/qkva_time.hip -DPHASE_STAMPS)
$(BUILD)/qkva_stamps: tools/qkva_time.hip tools/stamps.h $(SRC)/kernels.hip $(SRC)/kernels.h $(SRC)/kernels_common.h $(SRC)/i8_core.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DPHASE_STAMPS=1 $< -o $@

# the long-sentence attention's timing and per-stage stamps (tools/attn_long_time.hip)
$(BUILD)/attn_long_time: tools/attn_long_time.hip $(SRC)/kernels.hip $(SRC)/kernels.h $(SRC)/kernels_common.h $(SRC)/i8_core.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $< -o $@
$(BUILD)/attn_long_stamps: tools/attn_long_time.hip tools/stamps.h $(SRC)/kernels.hip $(SRC)/kernels.h $(SRC)/kernels_common.h $(SRC)/i8_core.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DPHASE_STAMPS=1 $< -o $@
