# Builds the gfx950 checksum engine and the (test-only) CPU oracle.
#   tcp_amd/libtcpcsum.so      product: HIP kernels + C ABI (include/tcpcsum.h)
#   oracle/build/liboracle.so  test infrastructure: C restatement, -O2 -g
#   oracle/build/liboracle_O0.so  same at -O0 -g (the reference Makefile's flags)
#   tests/c/abi_smoke          C program that links the ABI (C-callable proof)
#   tools/mmsg_bench           sendmmsg-seam latency on the reference's buffer layout
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
CC ?= gcc
ARCH ?= gfx950
# Product build only: the tuning / knock-out knobs of tcp_amd/csrc/tcpcsum_internal.h
# are refused here (#error); measurement builds compile their own objects (tools/*_ab.py).
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-parameter -Wno-unused-value -Wno-unused-result
CFLAGS_LIB ?= -O2 -fPIC -Wall -Wextra

LIB := tcp_amd/libtcpcsum.so
HIP_SRCS := tcp_amd/csrc/tcpcsum_kernels.hip tcp_amd/csrc/tcpcsum_api.hip tcp_amd/csrc/tcpcsum_host.hip
HDRS := include/tcpcsum.h tcp_amd/csrc/tcpcsum_internal.h tcp_amd/csrc/host_registry.h tcp_amd/csrc/copy_pool.h
OBJDIR := build/obj
# Build provenance (tcpcsum_build_info): sha256 over these files, in this order —
# tcp_amd/provenance.py computes the same over the tree it runs in.
HASH_SRCS := include/tcpcsum.h tcp_amd/csrc/tcpcsum_internal.h tcp_amd/csrc/host_registry.h tcp_amd/csrc/copy_pool.h \
	tcp_amd/csrc/tcpcsum_kernels.hip tcp_amd/csrc/tcpcsum_api.hip tcp_amd/csrc/tcpcsum_host.hip \
	tcp_amd/csrc/scalar_dropin.c Makefile
SRC_HASH := $(shell cat $(HASH_SRCS) | sha256sum | cut -c1-64)

PRELOAD := tcp_amd/libtcpcsum_preload.so

all: $(LIB) $(PRELOAD) $(WRAP) oracle tests/c/abi_smoke tests/c/mmsg_loop tests/c/mmsg_loop_wrap \
	tests/c/mmsg_loop_wrap_nopool tests/c/raw_echo tools/mmsg_bench

$(OBJDIR)/%.o: tcp_amd/csrc/%.hip $(HDRS) Makefile
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -Iinclude -c $< -o $@

# the one object that carries the source hash: rebuilt whenever any hashed file changes
$(OBJDIR)/tcpcsum_api.o: tcp_amd/csrc/tcpcsum_api.hip $(HASH_SRCS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -Iinclude '-DTCPCSUM_SRC_HASH="$(SRC_HASH)"' -c $< -o $@

$(OBJDIR)/scalar_dropin.o: tcp_amd/csrc/scalar_dropin.c include/tcpcsum.h
	@mkdir -p $(OBJDIR)
	$(CC) $(CFLAGS_LIB) -Iinclude -c $< -o $@

$(LIB): $(OBJDIR)/tcpcsum_kernels.o $(OBJDIR)/tcpcsum_api.o $(OBJDIR)/tcpcsum_host.o $(OBJDIR)/scalar_dropin.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@.tmp $^ -Wl,-soname,libtcpcsum.so -lpthread
	mv $@.tmp $@

# LD_PRELOAD seam library (sendmmsg / recvmmsg interposer) over the C ABI
$(PRELOAD): tcp_amd/csrc/preload_mmsg.c tcp_amd/csrc/preload_arena.h tcp_amd/csrc/rx_compact.h include/tcpcsum.h $(LIB)
	$(CC) -O2 -fPIC -shared -Wall -Wextra -Iinclude -o $@ $< -Ltcp_amd -ltcpcsum -ldl -lpthread -Wl,-rpath,'$$ORIGIN'

# the same seam as a static archive for the link-time form (-Wl,--wrap=sendmmsg,...): two
# members, the seams and the arena's allocation wraps (pulled in only by --wrap=malloc ...)
WRAP := tcp_amd/libtcpcsum_wrap.a
$(WRAP): tcp_amd/csrc/preload_mmsg.c tcp_amd/csrc/preload_arena.h tcp_amd/csrc/rx_compact.h include/tcpcsum.h
	@mkdir -p $(OBJDIR)
	$(CC) -O2 -fPIC -Wall -Wextra -Iinclude -DTCPCSUM_WRAP -DTCPCSUM_WRAP_PART=1 -c $< -o $(OBJDIR)/wrap_mmsg.o
	$(CC) -O2 -fPIC -Wall -Wextra -Iinclude -DTCPCSUM_WRAP -DTCPCSUM_WRAP_PART=2 -c $< -o $(OBJDIR)/wrap_alloc.o
	rm -f $@
	ar rcs $@ $(OBJDIR)/wrap_mmsg.o $(OBJDIR)/wrap_alloc.o

WRAP_MMSG := -Wl,--wrap=sendmmsg,--wrap=recvmmsg
WRAP_LDFLAGS := $(WRAP_MMSG),--wrap=malloc,--wrap=calloc,--wrap=free,--wrap=realloc

# tests/c/mmsg_loop linked with the seam at build time instead of LD_PRELOAD
tests/c/mmsg_loop_wrap: tests/c/mmsg_loop.c include/tcpcsum.h $(LIB) $(WRAP)
	$(CC) -O2 -Wall -Wextra -Iinclude -o $@ $< $(WRAP_LDFLAGS) $(WRAP) -Ltcp_amd -ltcpcsum -ldl -lpthread \
		-Wl,-rpath,'$$ORIGIN/../../tcp_amd'

# the same with the two mmsg wraps only (no pool): the allocation member stays out of the link
tests/c/mmsg_loop_wrap_nopool: tests/c/mmsg_loop.c include/tcpcsum.h $(LIB) $(WRAP)
	$(CC) -O2 -Wall -Wextra -Iinclude -o $@ $< $(WRAP_MMSG) $(WRAP) -Ltcp_amd -ltcpcsum -ldl -lpthread \
		-Wl,-rpath,'$$ORIGIN/../../tcp_amd'

oracle: oracle/build/liboracle.so oracle/build/liboracle_O0.so

oracle/build/liboracle.so: oracle/csum_oracle.c oracle/oracle.h oracle/cpu_bench.inc.c
	@mkdir -p oracle/build
	$(CC) -O2 -g -fPIC -shared -pthread -Wall -Wextra -o $@ $<

oracle/build/liboracle_O0.so: oracle/csum_oracle.c oracle/oracle.h oracle/cpu_bench.inc.c
	@mkdir -p oracle/build
	$(CC) -O0 -g -fPIC -shared -pthread -Wall -Wextra -o $@ $<

tests/c/abi_smoke: tests/c/abi_smoke.c include/tcpcsum.h $(LIB)
	$(CC) -O2 -Wall -Wextra -Iinclude -o $@ $< -Ltcp_amd -ltcpcsum -Wl,-rpath,'$$ORIGIN/../../tcp_amd'

tests/c/mmsg_loop: tests/c/mmsg_loop.c include/tcpcsum.h $(LIB)
	$(CC) -O2 -Wall -Wextra -Iinclude -o $@ $< -Ltcp_amd -ltcpcsum -Wl,-rpath,'$$ORIGIN/../../tcp_amd'

tests/c/raw_echo: tests/c/raw_echo.c include/tcpcsum.h $(LIB)
	$(CC) -O2 -Wall -Wextra -Iinclude -o $@ $< -Ltcp_amd -ltcpcsum -Wl,-rpath,'$$ORIGIN/../../tcp_amd'

tools/mmsg_bench: tools/mmsg_bench.c include/tcpcsum.h $(LIB)
	$(CC) -O2 -Wall -Wextra -Iinclude -o $@ $< -Ltcp_amd -ltcpcsum -Wl,-rpath,'$$ORIGIN/../tcp_amd'

clean:
	rm -rf build oracle/build $(LIB) $(PRELOAD) $(WRAP) tests/c/abi_smoke tests/c/mmsg_loop tests/c/mmsg_loop_wrap \
		tests/c/mmsg_loop_wrap_nopool \
		tests/c/raw_echo tools/mmsg_bench

.PHONY: all oracle clean
