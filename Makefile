# Build of the gfx950 engine (C-ABI shared library), its tools twin and the host featurisation
# library.  Every .hip is compiled to its own object (in parallel under make -j), then linked.
#   lib/libalert_engine.so        the product: exactly the entry points the engine runs
#   lib/libalert_engine_tools.so  the same sources with -DAE_TOOLS: + the timing / A-B entry
#                                 points (ae_bench_*, kernel variants, DIAG timing builds whose
#                                 results are WRONG on purpose) and the engine's AE_* knobs, for
#                                 tools/*.py and the alternative-form parity tests
HIPCC ?= /opt/rocm/bin/hipcc
PKG := attack-pretrain-models-of-code_amd
CSRC := $(PKG)/csrc
OBJDIR := $(PKG)/build
LIB := $(PKG)/lib/libalert_engine.so
SRCS := $(CSRC)/engine.hip $(CSRC)/gemm_f32.hip $(CSRC)/gemm_x3.hip $(CSRC)/gemm_planes.hip $(CSRC)/attention_f32.hip $(CSRC)/attention_pp.hip $(CSRC)/rowops.hip $(CSRC)/splice_topk.hip $(CSRC)/cls_attention.hip
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS))
TOOLSLIB := $(PKG)/lib/libalert_engine_tools.so
TOOLSSRCS := $(SRCS) $(CSRC)/attention_x3.hip
TOOLSOBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/tools/%.o,$(TOOLSSRCS))
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

all: $(LIB) $(TOOLSLIB) $(HOSTLIB)

$(HOSTLIB): $(HOSTSRCS) $(HOSTHDRS) $(PKG)/buildinfo.py
	@mkdir -p $(dir $@) $(OBJDIR)
	printf 'extern "C" const char* ah_source_hash(void) { return "%s"; }\n' "$$($(BUILDINFO) host)" > $(OBJDIR)/host_hash.cpp
	$(CXX) $(HOSTFLAGS) -o $@ $(HOSTSRCS) $(OBJDIR)/host_hash.cpp

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJDIR)/tools/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DAE_TOOLS -c -o $@ $<

$(TOOLSLIB): $(TOOLSOBJS) $(wildcard $(CSRC)/*.hip $(CSRC)/*.h) $(PKG)/buildinfo.py
	@mkdir -p $(dir $@) $(OBJDIR)/tools
	printf 'extern "C" const char* ae_source_hash(void) { return "%s"; }\n' "$$($(BUILDINFO) engine)" > $(OBJDIR)/tools/engine_hash.cpp
	$(CXX) -O2 -fPIC -c -o $(OBJDIR)/tools/engine_hash.o $(OBJDIR)/tools/engine_hash.cpp
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(TOOLSOBJS) $(OBJDIR)/tools/engine_hash.o

$(LIB): $(OBJS) $(wildcard $(CSRC)/*.hip $(CSRC)/*.h) $(PKG)/buildinfo.py
	@mkdir -p $(dir $@)
	printf 'extern "C" const char* ae_source_hash(void) { return "%s"; }\n' "$$($(BUILDINFO) engine)" > $(OBJDIR)/engine_hash.cpp
	$(CXX) -O2 -fPIC -c -o $(OBJDIR)/engine_hash.o $(OBJDIR)/engine_hash.cpp
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(OBJS) $(OBJDIR)/engine_hash.o

clean:
	rm -f $(LIB) $(TOOLSLIB) $(HOSTLIB) $(OBJS) $(TOOLSOBJS)

.PHONY: all clean
