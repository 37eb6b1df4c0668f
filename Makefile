# Build of the gfx950 engine (C-ABI shared library) and the CPU oracle pieces.
# Every .hip is compiled to its own object (in parallel under make -j), then linked.
HIPCC ?= /opt/rocm/bin/hipcc
PKG := attack-pretrain-models-of-code_amd
CSRC := $(PKG)/csrc
OBJDIR := $(PKG)/build
LIB := $(PKG)/lib/libalert_engine.so
SRCS := $(CSRC)/engine.hip $(CSRC)/gemm_f32.hip $(CSRC)/gemm_x3.hip $(CSRC)/gemm_planes.hip $(CSRC)/attention_f32.hip $(CSRC)/attention_x3.hip $(CSRC)/attention_pp.hip $(CSRC)/rowops.hip $(CSRC)/splice_topk.hip $(CSRC)/cls_attention.hip
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS))
# the hash of the sources each library is built from, embedded at link time (buildinfo.py:
# the loaders refuse a library built from other sources)
BUILDINFO := python3 $(PKG)/buildinfo.py
HDRS := $(CSRC)/common.h include/alert_engine.h
HIPFLAGS := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-result

HOSTLIB := $(PKG)/lib/libalert_host.so
HOSTSRCS := $(CSRC)/host/bpe.cpp $(CSRC)/host/lexer.cpp $(CSRC)/host/mutate.cpp $(CSRC)/host/dfg.cpp $(CSRC)/host/dfg_java.cpp $(CSRC)/host/dfg_python.cpp $(CSRC)/host/gcb.cpp $(CSRC)/host/capi.cpp
HOSTHDRS := $(CSRC)/host/host.h $(CSRC)/host/dfg_util.h $(CSRC)/host/unicode_tables.h include/alert_host.h
CXX ?= g++
HOSTFLAGS := -O2 -std=c++17 -fPIC -shared -pthread -Wall -Wextra -Wno-unused-parameter -Iinclude

all: $(LIB) $(HOSTLIB)

$(HOSTLIB): $(HOSTSRCS) $(HOSTHDRS) $(PKG)/buildinfo.py
	@mkdir -p $(dir $@) $(OBJDIR)
	printf 'extern "C" const char* ah_source_hash(void) { return "%s"; }\n' "$$($(BUILDINFO) host)" > $(OBJDIR)/host_hash.cpp
	$(CXX) $(HOSTFLAGS) -o $@ $(HOSTSRCS) $(OBJDIR)/host_hash.cpp

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJS) $(wildcard $(CSRC)/*.hip $(CSRC)/*.h) $(PKG)/buildinfo.py
	@mkdir -p $(dir $@)
	printf 'extern "C" const char* ae_source_hash(void) { return "%s"; }\n' "$$($(BUILDINFO) engine)" > $(OBJDIR)/engine_hash.cpp
	$(CXX) -O2 -fPIC -c -o $(OBJDIR)/engine_hash.o $(OBJDIR)/engine_hash.cpp
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(OBJS) $(OBJDIR)/engine_hash.o

clean:
	rm -f $(LIB) $(HOSTLIB) $(OBJS)

.PHONY: all clean
