# Build of the MI355X word-count engine (gfx950).  In-tree outputs so that the
# built .so files travel with the repo snapshot to the GPU box.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-result
# kernels: the scheduler that groups memory instructions into clauses measured
# ~1.5-2 % faster on the C2 bench (k_map 1.16 -> 1.14 ms)
KERNEL_FLAGS ?= -mllvm -amdgpu-sched-strategy=max-memory-clause
PKG := map-oxidize_amd
CSRC := $(PKG)/csrc
OUT := $(PKG)/mox

all: $(OUT)/libmox.so $(OUT)/libmox_corpus.so $(OUT)/meduce-gpu $(OUT)/libmox_check.so $(OUT)/libmox_hc.so oracle

$(OUT)/mox_kernels.o: $(CSRC)/mox_kernels.hip $(CSRC)/mox_internal.h Makefile
	$(HIPCC) $(HIPFLAGS) $(KERNEL_FLAGS) -c $< -o $@

HOST_DEPS := $(CSRC)/mox_host.h $(CSRC)/mox_internal.h $(CSRC)/mox_table.h include/mox.h
$(OUT)/mox_engine.o: $(CSRC)/mox_engine.hip $(HOST_DEPS) $(CSRC)/mox_unicode_tables.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT)/mox_multi.o: $(CSRC)/mox_multi.hip $(HOST_DEPS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT)/mox_bsort.o: $(CSRC)/mox_bsort.hip $(HOST_DEPS)
	$(HIPCC) $(HIPFLAGS) $(KERNEL_FLAGS) -c $< -o $@

$(OUT)/mox_table.o: $(CSRC)/mox_table.cpp $(CSRC)/mox_table.h
	g++ -O3 -std=c++17 -fPIC -Wall -Wextra -c $< -o $@

$(OUT)/libmox.so: $(OUT)/mox_kernels.o $(OUT)/mox_engine.o $(OUT)/mox_multi.o $(OUT)/mox_bsort.o $(OUT)/mox_table.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# check build: device bounds checks on every derived index (MOX_CHK, mox_internal.h);
# tests load it with MOX_LIB=.../libmox_check.so
$(OUT)/mox_kernels_check.o: $(CSRC)/mox_kernels.hip $(CSRC)/mox_internal.h Makefile
	$(HIPCC) $(HIPFLAGS) $(KERNEL_FLAGS) -DMOX_CHECK -c $< -o $@

$(OUT)/mox_engine_check.o: $(CSRC)/mox_engine.hip $(HOST_DEPS) $(CSRC)/mox_unicode_tables.h
	$(HIPCC) $(HIPFLAGS) -DMOX_CHECK -c $< -o $@

$(OUT)/libmox_check.so: $(OUT)/mox_kernels_check.o $(OUT)/mox_engine_check.o $(OUT)/mox_multi.o $(OUT)/mox_bsort.o $(OUT)/mox_table.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

check: $(OUT)/libmox_check.so

# forced-collision check build: key hashes truncated to a few bits so that every
# exactness fallback (byte compares behind a hash match) runs, with path hit
# counters and the bounds checks (mox_internal.h, MOX_HASH_COLLIDE); tests load it
# with mox.Engine(lib_path=...) (tests/test_gpu_collide.py)
HC_FLAGS := -DMOX_HASH_COLLIDE -DMOX_CHECK
$(OUT)/mox_kernels_hc.o: $(CSRC)/mox_kernels.hip $(CSRC)/mox_internal.h Makefile
	$(HIPCC) $(HIPFLAGS) $(KERNEL_FLAGS) $(HC_FLAGS) -c $< -o $@

$(OUT)/mox_engine_hc.o: $(CSRC)/mox_engine.hip $(HOST_DEPS) $(CSRC)/mox_unicode_tables.h
	$(HIPCC) $(HIPFLAGS) $(HC_FLAGS) -c $< -o $@

$(OUT)/mox_multi_hc.o: $(CSRC)/mox_multi.hip $(HOST_DEPS)
	$(HIPCC) $(HIPFLAGS) $(HC_FLAGS) -c $< -o $@

$(OUT)/libmox_hc.so: $(OUT)/mox_kernels_hc.o $(OUT)/mox_engine_hc.o $(OUT)/mox_multi_hc.o $(OUT)/mox_bsort.o $(OUT)/mox_table.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

hc: $(OUT)/libmox_hc.so

$(OUT)/libmox_corpus.so: $(CSRC)/mox_corpus.c
	gcc -O3 -fPIC -shared -Wall -Wextra -o $@ $< -lpthread -lm

$(OUT)/meduce-gpu: $(CSRC)/meduce_gpu.cpp include/mox.h $(OUT)/libmox.so
	g++ -O2 -std=c++17 -Wall -o $@ $< -Iinclude -L$(OUT) -lmox -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(OUT)/*.o $(OUT)/*.so $(OUT)/meduce-gpu
	$(MAKE) -C oracle clean

.PHONY: all clean oracle check hc
