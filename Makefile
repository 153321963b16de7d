# Top-level build.  Product: fabric_amd/libfgv.so (HIP for gfx950 + C++ host, C ABI in
# include/fgv.h).  Test infrastructure: oracle/liboracle.so.  Workload generator:
# fabric_amd/synth/libfgv_synth.so.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result
CSRC := fabric_amd/csrc
OBJDIR := build
KOBJS := $(OBJDIR)/sha256.o $(OBJDIR)/p256_kernels.o $(OBJDIR)/der_kernel.o $(OBJDIR)/fgv_host.o $(OBJDIR)/fgv_block.o $(OBJDIR)/mvcc.o $(OBJDIR)/fgv_mvcc.o \
	$(OBJDIR)/finalize.o $(OBJDIR)/fgv_integrity.o $(OBJDIR)/blockdev.o $(OBJDIR)/fgv_commit.o $(OBJDIR)/fgv_channel.o \
	$(OBJDIR)/fgv_group.o $(OBJDIR)/fgv_msp.o $(OBJDIR)/fgv_x509.o
HDRS := $(CSRC)/p256_field.h $(CSRC)/p256_fe28.h $(CSRC)/p256_modinv.h $(CSRC)/sha256_dev.h $(CSRC)/fgv_kernels.h $(CSRC)/fgv_der.h $(CSRC)/fgv_internal.h include/fgv.h $(CSRC)/blockdev.h $(CSRC)/pbwire_dev.h $(CSRC)/fin_dev.h

all: fabric_amd/libfgv.so oracle/liboracle.so fabric_amd/synth/libfgv_synth.so tests/gpu_helpers/libhexcheck.so

$(OBJDIR):
	mkdir -p $(OBJDIR)

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/fgv_host.o: $(CSRC)/fgv_host.cpp $(HDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/fgv_block.o: $(CSRC)/fgv_block.cpp $(HDRS) $(CSRC)/pbwire.h $(CSRC)/fgv_visitors.h $(CSRC)/fgv_channel.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/fgv_mvcc.o: $(CSRC)/fgv_mvcc.cpp $(HDRS) $(CSRC)/pbwire.h $(CSRC)/fgv_visitors.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/fgv_integrity.o: $(CSRC)/fgv_integrity.cpp $(HDRS) $(CSRC)/pbwire.h $(CSRC)/fgv_visitors.h $(CSRC)/sha256_host.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/fgv_channel.o: $(CSRC)/fgv_channel.cpp $(CSRC)/fgv_channel.h $(HDRS) $(CSRC)/pbwire.h $(CSRC)/fgv_visitors.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/fgv_group.o: $(CSRC)/fgv_group.cpp $(HDRS) $(CSRC)/thread_pool.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/fgv_msp.o: $(CSRC)/fgv_msp.cpp $(HDRS) $(CSRC)/fgv_channel.h $(CSRC)/fgv_x509.h $(CSRC)/pbwire.h $(CSRC)/fgv_visitors.h $(CSRC)/sha256_host.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/fgv_x509.o: $(CSRC)/fgv_x509.cpp $(CSRC)/fgv_x509.h $(CSRC)/pbwire.h $(CSRC)/sha256_host.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/fgv_commit.o: $(CSRC)/fgv_commit.cpp $(HDRS) $(CSRC)/pbwire.h $(CSRC)/fgv_visitors.h $(CSRC)/sha256_host.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

fabric_amd/libfgv.so: $(KOBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(KOBJS) -lpthread

oracle/liboracle.so: oracle/fgv_oracle.c oracle/fgv_oracle.h
	$(MAKE) -C oracle

fabric_amd/synth/libfgv_synth.so: fabric_amd/synth/fgv_synth.c
	gcc -O2 -fPIC -shared -Wall -o $@ $< -lcrypto -lpthread

# test helper (not part of the product): the device txid decoder on chosen offsets
tests/gpu_helpers/libhexcheck.so: tests/gpu_helpers/hexcheck.hip $(CSRC)/fin_dev.h
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

clean:
	rm -rf $(OBJDIR) fabric_amd/libfgv.so oracle/liboracle.so fabric_amd/synth/libfgv_synth.so tests/gpu_helpers/libhexcheck.so

.PHONY: all clean
