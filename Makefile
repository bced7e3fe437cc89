# Build of the MI355X-native SCCG hot path (gfx950).  `make` builds everything that ships:
#   sccg-genome-compression_amd/lib/libsccg.so     C ABI (include/sccg.h) + HIP kernels
#   sccg-genome-compression_amd/bin/compression    reference-compatible CLIs over the C ABI
#   sccg-genome-compression_amd/bin/decompression
#   sccg-genome-compression_amd/tools/libsccg_synth.so, sccg_synth   synthetic pairs
# and the test-only oracle (oracle/, plus oracle/_ref when /root/reference exists).
PKG      := sccg-genome-compression_amd
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
SRCS     := $(PKG)/csrc/scan.hip $(PKG)/csrc/ingest.hip $(PKG)/csrc/local.hip $(PKG)/csrc/walk.hip \
            $(PKG)/csrc/decomp.hip $(PKG)/csrc/delta.hip $(PKG)/csrc/sccg_api.cpp $(PKG)/csrc/prof.cpp
HDRS     := $(wildcard $(PKG)/csrc/*.h) include/sccg.h
OBJDIR   := $(PKG)/build
OBJS     := $(patsubst $(PKG)/csrc/%,$(OBJDIR)/%.o,$(SRCS))
LIB      := $(PKG)/lib/libsccg.so
JOBS     ?= 8

all: lib cli tools oracle

lib: $(LIB)

$(OBJDIR)/%.hip.o: $(PKG)/csrc/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.cpp.o: $(PKG)/csrc/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(PKG)/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS)

cli: $(PKG)/bin/compression $(PKG)/bin/decompression

$(PKG)/bin/%: $(PKG)/cli/%.cpp $(LIB) include/sccg.h $(PKG)/cli/cli_common.h
	@mkdir -p $(PKG)/bin
	g++ -O2 -std=c++17 -Iinclude -o $@ $< -L$(PKG)/lib -lsccg -Wl,-rpath,'$$ORIGIN/../lib'

tools: $(PKG)/tools/libsccg_synth.so $(PKG)/tools/sccg_synth

$(PKG)/tools/libsccg_synth.so: $(PKG)/tools/synth.c $(PKG)/tools/synth.h
	gcc -O2 -Wall -shared -fPIC -o $@ $<

$(PKG)/tools/sccg_synth: $(PKG)/tools/synth.c $(PKG)/tools/synth_cli.c $(PKG)/tools/synth.h
	gcc -O2 -Wall -o $@ $(PKG)/tools/synth.c $(PKG)/tools/synth_cli.c

oracle:
	$(MAKE) -C oracle
	@if [ -f /root/reference/compression.cpp ]; then $(MAKE) -C oracle ref; fi

clean:
	rm -rf $(OBJDIR) $(PKG)/lib $(PKG)/bin $(PKG)/tools/*.so $(PKG)/tools/sccg_synth
	$(MAKE) -C oracle clean

.PHONY: all lib cli tools oracle clean
