# Top-level build: the HIP engine (product), the plain-C host CLI, the oracle.
#   make            -> linearprogramming_amd/liblpg.so (+ liblpg_testhooks.so, tests only), host/lpgcli,
#                      oracle/liblpo.so
#   make ref        -> oracle/_ref/lp (reference CLI; needs /root/reference)
HIPCC    ?= /opt/rocm/bin/hipcc
CC       ?= gcc
ARCH     ?= gfx950
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result
CSRC      = linearprogramming_amd/csrc
LIB       = linearprogramming_amd/liblpg.so


OBJDIR    = build/obj
KOBJS     = $(OBJDIR)/lpg_kernels.o $(OBJDIR)/lpg_block.o $(OBJDIR)/lpg_dual.o $(OBJDIR)/lpg_stamp.o
HDRS      = $(CSRC)/lpg_internal.h $(CSRC)/lpg_device.h include/lpg.h
HOOKLIB   = linearprogramming_amd/liblpg_testhooks.so
# the source stamp compiled into the library (lpg_build_stamp; _lib.load()
# refuses a library whose stamp is not the sources')
STAMP    := $(shell python3 linearprogramming_amd/_stamp.py)

all: $(LIB) $(HOOKLIB) host/lpgcli oracle

$(OBJDIR)/lpg_stamp.o: $(wildcard $(CSRC)/*.hip) $(HDRS) linearprogramming_amd/_stamp.py
	@mkdir -p $(OBJDIR)
	printf '#include "lpg.h"\nconst char *lpg_build_stamp(void) { return "%s"; }\n' '$(STAMP)' > $(OBJDIR)/lpg_stamp.c
	$(CC) -O2 -fPIC -Iinclude -c -o $@ $(OBJDIR)/lpg_stamp.c

# one object per translation unit (no cross-TU device code: every kernel is
# launched from the file that defines it), so the product library and the
# test-hook variant share the kernel objects
$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJDIR)/lpg_ctx_testhooks.o: $(CSRC)/lpg_ctx.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DLPG_TEST_HOOKS -c -o $@ $<

$(LIB): $(KOBJS) $(OBJDIR)/lpg_ctx.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^ -ldl

# the same engine with the test-only fault hooks compiled in (LPG_TEST_HOOKS:
# env LPG_TEST_PENDING_FAULT); -Bsymbolic so that, loaded RTLD_LOCAL next to
# liblpg.so in one test process, it binds to its own definitions. Only tests
# load it (tests/test_gpu_block.py); the product library has no hook.
$(HOOKLIB): $(KOBJS) $(OBJDIR)/lpg_ctx_testhooks.o
	$(HIPCC) $(HIPFLAGS) -shared -Wl,-Bsymbolic -o $@ $^ -ldl

host/lpgcli: host/lpgcli.c host/lpfront.c host/lpfront.h include/lpg.h $(LIB)
	$(CC) -O2 -std=c11 -Wall -Wextra -Iinclude -o $@ host/lpgcli.c host/lpfront.c -L$(dir $(LIB)) -llpg -Wl,-rpath,'$$ORIGIN/../linearprogramming_amd' -lm

oracle:
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

# phase-stamped build for tools/phase_probe.py and tools/block_probe.py
# (diagnostics only; tools/probe/ travels to the GPU box, delete it when done)
phases: tools/probe/liblpg_phases.so
tools/probe/liblpg_phases.so: $(CSRC)/lpg_kernels.hip $(CSRC)/lpg_block.hip $(CSRC)/lpg_dual.hip $(CSRC)/lpg_ctx.hip $(CSRC)/lpg_internal.h $(CSRC)/lpg_device.h $(OBJDIR)/lpg_stamp.o
	@mkdir -p tools/probe
	$(HIPCC) $(HIPFLAGS) -DLPG_PHASES -shared -o $@ $(OBJDIR)/lpg_stamp.o $(CSRC)/lpg_kernels.hip $(CSRC)/lpg_block.hip $(CSRC)/lpg_dual.hip $(CSRC)/lpg_ctx.hip -ldl

# publish / decision-seen stamps of every workgroup only (tools/block_probe.py PHASES_LIB=liblpg_pub.so)
pub: tools/probe/liblpg_pub.so
tools/probe/liblpg_pub.so: $(CSRC)/lpg_kernels.hip $(CSRC)/lpg_block.hip $(CSRC)/lpg_dual.hip $(CSRC)/lpg_ctx.hip $(CSRC)/lpg_internal.h $(CSRC)/lpg_device.h $(OBJDIR)/lpg_stamp.o
	@mkdir -p tools/probe
	$(HIPCC) $(HIPFLAGS) -DLPG_PHASES -DLPG_PHASES_PUBONLY -shared -o $@ $(OBJDIR)/lpg_stamp.o $(CSRC)/lpg_kernels.hip $(CSRC)/lpg_block.hip $(CSRC)/lpg_dual.hip $(CSRC)/lpg_ctx.hip -ldl

asm: $(CSRC)/lpg_kernels.hip
	$(HIPCC) $(HIPFLAGS) -c --save-temps -o /tmp/lpg_kernels.o $(CSRC)/lpg_kernels.hip

clean:
	rm -f $(LIB) $(HOOKLIB) host/lpgcli
	rm -rf $(OBJDIR)
	$(MAKE) -C oracle clean

.PHONY: all oracle ref asm clean phases pub
