# Top-level build: the HIP engine (product), the plain-C host CLI, the oracle.
#   make            -> linearprogramming_amd/liblpg.so, host/lpgcli, oracle/liblpo.so
#   make ref        -> oracle/_ref/lp (reference CLI; needs /root/reference)
HIPCC    ?= /opt/rocm/bin/hipcc
CC       ?= gcc
ARCH     ?= gfx950
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result
CSRC      = linearprogramming_amd/csrc
LIB       = linearprogramming_amd/liblpg.so

all: $(LIB) host/lpgcli oracle

$(LIB): $(CSRC)/lpg_kernels.hip $(CSRC)/lpg_block.hip $(CSRC)/lpg_dual.hip $(CSRC)/lpg_ctx.hip $(CSRC)/lpg_internal.h $(CSRC)/lpg_device.h include/lpg.h
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(CSRC)/lpg_kernels.hip $(CSRC)/lpg_block.hip $(CSRC)/lpg_dual.hip $(CSRC)/lpg_ctx.hip -ldl

host/lpgcli: host/lpgcli.c host/lpfront.c host/lpfront.h include/lpg.h $(LIB)
	$(CC) -O2 -std=c11 -Wall -Wextra -Iinclude -o $@ host/lpgcli.c host/lpfront.c -L$(dir $(LIB)) -llpg -Wl,-rpath,'$$ORIGIN/../linearprogramming_amd' -lm

oracle:
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

# phase-stamped build for tools/phase_probe.py and tools/block_probe.py (diagnostics only)
phases: tools/liblpg_phases.so
tools/liblpg_phases.so: $(CSRC)/lpg_kernels.hip $(CSRC)/lpg_block.hip $(CSRC)/lpg_dual.hip $(CSRC)/lpg_ctx.hip $(CSRC)/lpg_internal.h $(CSRC)/lpg_device.h
	$(HIPCC) $(HIPFLAGS) -DLPG_PHASES -shared -o $@ $(CSRC)/lpg_kernels.hip $(CSRC)/lpg_block.hip $(CSRC)/lpg_dual.hip $(CSRC)/lpg_ctx.hip -ldl

asm: $(CSRC)/lpg_kernels.hip
	$(HIPCC) $(HIPFLAGS) -c --save-temps -o /tmp/lpg_kernels.o $(CSRC)/lpg_kernels.hip

clean:
	rm -f $(LIB) host/lpgcli
	$(MAKE) -C oracle clean

.PHONY: all oracle ref asm clean phases
