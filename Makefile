# Top-level build.  Product: fabric_amd/libfgv.so (HIP for gfx950 + C++ host, C ABI in
# include/fgv.h).  Test infrastructure: oracle/liboracle.so.  Workload generator:
# fabric_amd/synth/libfgv_synth.so.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result
# header dependencies per object (build/*.d, written by the compiler)
DEPFLAGS := -MMD -MP
CSRC := fabric_amd/csrc
OBJDIR := build
KOBJS := $(OBJDIR)/sha256.o $(OBJDIR)/p256_kernels.o $(OBJDIR)/der_kernel.o $(OBJDIR)/fgv_host.o $(OBJDIR)/fgv_block.o $(OBJDIR)/mvcc.o $(OBJDIR)/fgv_mvcc.o \
	$(OBJDIR)/finalize.o $(OBJDIR)/fgv_integrity.o $(OBJDIR)/blockdev.o $(OBJDIR)/blockdev_lds.o $(OBJDIR)/blockdev_sha.o $(OBJDIR)/blockdev_fold.o $(OBJDIR)/fgv_commit.o $(OBJDIR)/fgv_channel.o \
	$(OBJDIR)/fgv_group.o $(OBJDIR)/fgv_msp.o $(OBJDIR)/fgv_x509.o $(OBJDIR)/p384.o $(OBJDIR)/mvcc_ub.o

all: fabric_amd/libfgv.so oracle/liboracle.so fabric_amd/synth/libfgv_synth.so tests/gpu_helpers/libhexcheck.so

$(OBJDIR):
	mkdir -p $(OBJDIR)

$(OBJDIR)/%.o: $(CSRC)/%.hip | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(DEPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(DEPFLAGS) -c $< -o $@

fabric_amd/libfgv.so: $(KOBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(KOBJS) -lpthread

oracle/liboracle.so: oracle/fgv_oracle.c oracle/fgv_oracle.h
	$(MAKE) -C oracle

fabric_amd/synth/libfgv_synth.so: fabric_amd/synth/fgv_synth.c
	gcc -O2 -fPIC -shared -Wall -o $@ $< -lcrypto -lpthread

# test helper (not part of the product): the device txid decoder on chosen offsets
tests/gpu_helpers/libhexcheck.so: tests/gpu_helpers/hexcheck.hip $(CSRC)/fin_dev.h
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

-include $(wildcard $(OBJDIR)/*.d)

clean:
	rm -rf $(OBJDIR) fabric_amd/libfgv.so oracle/liboracle.so fabric_amd/synth/libfgv_synth.so tests/gpu_helpers/libhexcheck.so

.PHONY: all clean
