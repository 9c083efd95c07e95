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
CHDR := $(wildcard $(PKG)/csrc/*.h) include/fattn.h

.PHONY: all lib harness oracle clean asm stamps tests-hip

all: lib harness oracle tests-hip

lib: $(LIB)

$(LIB): $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared $(CSRC) -o $@

# diagnostic libraries (tools/stamps.py, tools/variants.py); never loaded by the product path
stamps: $(LIBDIR)/libfattn_stamps.so $(LIBDIR)/libfattn_nocompute.so $(LIBDIR)/libfattn_nc.so \
        $(LIBDIR)/libfattn_nctail.so $(LIBDIR)/libfattn_notail.so $(LIBDIR)/libfattn_nopub.so \
        $(LIBDIR)/libfattn_noatomic.so $(LIBDIR)/libfattn_nomem.so $(LIBDIR)/libfattn_nomem_notail.so \
        $(LIBDIR)/libfattn_nomem_nopub.so $(LIBDIR)/libfattn_stamps_nomem.so

$(LIBDIR)/libfattn_nt.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DMA_NO_NT -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_nt_stamps.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DMA_NO_NT -DFATTN_STAMPS -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_pf4nosgb.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_PF4_NO_SGB -shared $(CSRC) -o $@

ntdiag: $(LIBDIR)/libfattn_nt.so $(LIBDIR)/libfattn_nt_stamps.so

mqdiag: $(LIBDIR)/libfattn_mq_nomem.so $(LIBDIR)/libfattn_mq_nodeq.so $(LIBDIR)/libfattn_mq_nocomp.so \
        $(LIBDIR)/libfattn_pf_nosm.so

$(LIBDIR)/libfattn_pf_nosm.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_PF_NOSOFTMAX -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_mq_nomem.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_MQ_NOMEM -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_mq_nodeq.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_MQ_NODEQ -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_mq_nocomp.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_MQ_NOCOMPUTE -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_nomem_notail.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DIAG_NOMEM -DFATTN_DIAG_NOTAIL -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_nomem_nopub.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DIAG_NOMEM -DFATTN_DIAG_NOPUBLISH -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_stamps_nomem.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_STAMPS -DFATTN_DIAG_NOMEM -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_nomem.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DIAG_NOMEM -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_nopub.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DIAG_NOPUBLISH -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_noatomic.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DIAG_NOATOMIC -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_nc.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DIAG_NOCOMPUTE -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_nctail.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DIAG_NOCOMPUTE -DFATTN_DIAG_NOTAIL -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_notail.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_DIAG_NOTAIL -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_nocompute.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_STAMPS -DFATTN_DIAG_NOCOMPUTE -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_stamps.so: $(CSRC) $(CHDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_STAMPS -shared $(CSRC) -o $@

harness: $(HARNESS)

$(HARNESS): $(PKG)/host/kernel_test.cpp $(LIB) include/fattn.h
	@mkdir -p $(BINDIR)
	$(HIPCC) -O2 -std=c++17 -ffp-contract=off -Iinclude $(PKG)/host/kernel_test.cpp -L$(LIBDIR) -lfattn \
	    -Wl,-rpath,'$$ORIGIN/../lib' -o $@

oracle:
	$(MAKE) -C oracle

# ISA dump for inspection (not part of the build)
asm:
	@mkdir -p build/asm
	cd build/asm && $(HIPCC) $(HIPFLAGS) -c ../../$(PKG)/csrc/fattn_api.hip -save-temps -o fattn_api.o

clean:
	rm -rf $(LIBDIR) $(BINDIR) build
	$(MAKE) -C oracle clean

# test-only HIP probes (tests/hip) -> tests/_build/libprims.so
tests-hip: tests/_build/libprims.so

tests/_build/libprims.so: tests/hip/prims.hip $(CHDR)
	@mkdir -p tests/_build
	$(HIPCC) $(HIPFLAGS) -shared tests/hip/prims.hip -o $@

# pipelined prefill schedule variants (tools/gpu_pfp.sh); diagnostic only
pfpvar: $(LIBDIR)/libfattn_pfp_nosgb.so $(LIBDIR)/libfattn_pfp_a4b3.so $(LIBDIR)/libfattn_pfp_a9b6.so \
        $(LIBDIR)/libfattn_pfp_r4r8.so $(LIBDIR)/libfattn_pfp_r8r16.so

$(LIBDIR)/libfattn_pfp_nosgb.so: $(CSRC) $(CHDR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_PFP_NO_SGB -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_pfp_a4b3.so: $(CSRC) $(CHDR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_PFP_FILL_A=4 -DFATTN_PFP_FILL_B=3 -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_pfp_a9b6.so: $(CSRC) $(CHDR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_PFP_FILL_A=9 -DFATTN_PFP_FILL_B=6 -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_pfp_r4r8.so: $(CSRC) $(CHDR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_PFP_AHEAD_A=4 -DFATTN_PFP_AHEAD_B=8 -shared $(CSRC) -o $@

$(LIBDIR)/libfattn_pfp_r8r16.so: $(CSRC) $(CHDR)
	$(HIPCC) $(HIPFLAGS) -DFATTN_PFP_AHEAD_A=8 -DFATTN_PFP_AHEAD_B=16 -shared $(CSRC) -o $@
