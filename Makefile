# Builds libsvc_hip.so (gfx950) in-tree. Usage: make -j8
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC_DIR := svc_inference_pipeline_amd/csrc
SRCS := $(wildcard $(SRC_DIR)/*.hip)
OBJS := $(patsubst $(SRC_DIR)/%.hip,build/%.o,$(SRCS))
LIB := svc_inference_pipeline_amd/libsvc_hip.so
CXXFLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-function -Wno-unused-variable \
            -Iinclude -I$(SRC_DIR)

all: $(LIB)

build/%.o: $(SRC_DIR)/%.hip $(wildcard $(SRC_DIR)/*.h) include/svc_hip.h
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

# attention's softmax maxima: no NaN reaches them (masked keys are -inf), so the compiler need not canonicalise every
# MFMA result before v_max_f32 (16 of 24 v_max per key tile were those copies)
build/attention.o: CXXFLAGS += -fno-honor-nans

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

clean:
	rm -rf build $(LIB)

.PHONY: all clean
