# Build of the gfx950 engine (C-ABI shared library) and the CPU oracle pieces.
HIPCC ?= /opt/rocm/bin/hipcc
PKG := attack-pretrain-models-of-code_amd
CSRC := $(PKG)/csrc
LIB := $(PKG)/lib/libalert_engine.so
SRCS := $(CSRC)/engine.hip $(CSRC)/gemm_f32.hip $(CSRC)/attention_f32.hip $(CSRC)/rowops.hip $(CSRC)/splice_topk.hip
HDRS := $(CSRC)/common.h include/alert_engine.h
HIPFLAGS := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -Wall -Wno-unused-result

all: $(LIB)

$(LIB): $(SRCS) $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -o $@ $(SRCS)

clean:
	rm -f $(LIB)

.PHONY: all clean
