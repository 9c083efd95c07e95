# Build: HIP kernels (gfx950) + C ABI -> libfattn.so, the kernel_test harness,
# and the test-only CPU oracle (oracle/Makefile).  No cmake/ninja needed.
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
PKG     := ggml-cuda-experiments_amd
LIBDIR  := $(PKG)/lib
BINDIR  := $(PKG)/bin
LIB     := $(LIBDIR)/libfattn.so
HARNESS := $(BINDIR)/kernel_test

HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
            -munsafe-fp-atomics -Iinclude
CSRC := $(wildcard $(PKG)/csrc/*.hip)
CHDR := $(wildcard $(PKG)/csrc/*.h) include/fattn.h include/fattn_debug.h

.PHONY: all lib harness oracle clean asm stamps tests-hip probe isa variant

all: lib harness oracle tests-hip probe isa

lib: $(LIB)

# one object per translation unit (make -j builds the head dims in parallel)
OBJDIR := build/obj
OBJS := $(patsubst $(PKG)/csrc/%.hip,$(OBJDIR)/%.o,$(CSRC))

$(OBJDIR)/%.o: $(PKG)/csrc/%.hip $(CHDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared $(OBJS) -o $@

# diagnostic library (tools/stamps.py): per-wave phase stamps; never loaded by the product path
STAMP_OBJS := $(patsubst $(PKG)/csrc/%.hip,$(OBJDIR)/stamps_%.o,$(CSRC))
$(OBJDIR)/stamps_%.o: $(PKG)/csrc/%.hip $(CHDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_STAMPS -c $< -o $@
stamps: $(LIBDIR)/libfattn_stamps.so
$(LIBDIR)/libfattn_stamps.so: $(STAMP_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared $(STAMP_OBJS) -o $@

# diagnostic / A-B variant of the library (never the product):
#   make variant VAR=nr3 VFLAGS=-DFATTN_BDP_MAX_RAW=3  ->  lib/libfattn_nr3.so
VAR ?= var
VFLAGS ?=
VAR_OBJS := $(patsubst $(PKG)/csrc/%.hip,$(OBJDIR)/$(VAR)_%.o,$(CSRC))
$(OBJDIR)/$(VAR)_%.o: $(PKG)/csrc/%.hip $(CHDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c $< -o $@
variant: $(VAR_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared $(VAR_OBJS) -o $(LIBDIR)/libfattn_$(VAR).so

harness: $(HARNESS)

$(HARNESS): $(PKG)/host/kernel_test.cpp $(LIB) include/fattn.h
	@mkdir -p $(BINDIR)
	$(HIPCC) -O2 -std=c++17 -ffp-contract=off -Iinclude $(PKG)/host/kernel_test.cpp -L$(LIBDIR) -lfattn -lrccl -pthread \
	    -Wl,-rpath,'$$ORIGIN/../lib' -o $@

oracle:
	$(MAKE) -C oracle

# measurement probe for bench.py's roofline (dwordx4 copy / read ceilings); not part of libfattn
PROBE := $(LIBDIR)/libhbmcopy.so
probe: $(PROBE)
$(PROBE): tools/hbm_copy.hip
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared $< -o $@

# The -save-temps ISA of every translation unit of libfattn.so, same flags as
# the library (tools/isa_hazard_check.py audits it and checks that it equals
# the shipped code objects; tests/test_isa_hazards.py)
ISADIR := build/isa
ISAS := $(patsubst $(PKG)/csrc/%.hip,$(ISADIR)/%.s,$(CSRC))
isa: $(ISAS)
$(ISADIR)/%.s: $(PKG)/csrc/%.hip $(CHDR)
	@mkdir -p $(ISADIR)/$*.tmp
	cd $(ISADIR)/$*.tmp && $(HIPCC) $(subst -Iinclude,-I$(CURDIR)/include,$(HIPFLAGS)) -c $(CURDIR)/$< -save-temps -o $*.o
	mv $(ISADIR)/$*.tmp/$*-hip-amdgcn-amd-amdhsa-$(ARCH).s $@
	rm -rf $(ISADIR)/$*.tmp

# ISA dump for inspection (not part of the build): make asm ASMSRC=fattn_launch_d128
ASMSRC ?= fattn_launch_d128
asm:
	@mkdir -p build/asm
	cd build/asm && $(HIPCC) $(HIPFLAGS) -I../../include -c ../../$(PKG)/csrc/$(ASMSRC).hip -save-temps -o $(ASMSRC).o

clean:
	rm -rf $(LIBDIR) $(BINDIR) build
	$(MAKE) -C oracle clean

# test-only HIP probes (tests/hip) -> tests/_build/libprims.so
tests-hip: tests/_build/libprims.so

tests/_build/libprims.so: tests/hip/prims.hip $(CHDR)
	@mkdir -p tests/_build
	$(HIPCC) $(HIPFLAGS) -shared tests/hip/prims.hip -o $@
