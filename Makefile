# Top-level build. `python -c "import __graft_entry__ as g; g.build()"` runs
# the same steps. Everything is built in-tree so the .so files travel to the
# GPU box with the snapshot.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wextra \
           -Wno-unused-parameter -munsafe-fp-atomics

LIB = tulips_amd/libtulips_csum.so
SRCS = tulips_amd/csrc/csum_kernels.hip tulips_amd/csrc/csum_capi.hip \
       tulips_amd/csrc/csum_host.hip tulips_amd/csrc/rss_toeplitz.hip \
       tulips_amd/csrc/frames.hip tulips_amd/csrc/segment.hip \
       tulips_amd/csrc/stream_state.hip tulips_amd/csrc/csum_multi.hip \
       tulips_amd/csrc/rss_route.hip
HDRS = tulips_amd/csrc/csum_common.h tulips_amd/csrc/csum_launch.h \
       tulips_amd/csrc/csum_device.h tulips_amd/csrc/zc_mailbox.h \
       tulips_amd/csrc/span_kernel.h tulips_amd/csrc/rss_common.h tulips_amd/csrc/rss_route.h \
       tulips_amd/csrc/frame_common.h tulips_amd/csrc/seg_device.h tulips_amd/csrc/stream_state.h \
       include/tulips_csum.h
OBJS = $(patsubst tulips_amd/csrc/%.hip,build/%.o,$(SRCS))

.PHONY: all lib benchlib oracle clean asm variants native

all: lib benchlib oracle native

lib: $(LIB)

build/%.o: tulips_amd/csrc/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS) tulips_amd/csrc/libtulips_csum.map
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) \
	    -Wl,--version-script=tulips_amd/csrc/libtulips_csum.map

# benchlib/libtulips_csum_bench.so: measurement ceilings, the device data
# fill and C-timed latency loops (include/tulips_csum_bench.h), loaded by
# bench.py / tools / tests beside the product; links the product for the
# entry points it times.
BENCHLIB = benchlib/libtulips_csum_bench.so
benchlib: $(BENCHLIB)

build/bench_kernels.o: benchlib/csrc/bench_kernels.hip include/tulips_csum_bench.h $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/bench_host.o: benchlib/csrc/bench_host.cpp include/tulips_csum_bench.h include/tulips_csum.h
	@mkdir -p build
	g++ -O2 -std=c++17 -fPIC -Wall -Wextra -c $< -o $@

$(BENCHLIB): build/bench_kernels.o build/bench_host.o $(LIB) benchlib/csrc/libtulips_csum_bench.map
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ build/bench_kernels.o build/bench_host.o \
	    -Ltulips_amd -ltulips_csum -Wl,-rpath,'$$ORIGIN/../tulips_amd' \
	    -Wl,--version-script=benchlib/csrc/libtulips_csum_bench.map

oracle:
	$(MAKE) -C oracle

# tests/native/runtime_check: the library driven through its C ABI from a
# plain C++ process on the ROCm runtime an integrator links (no torch).
# Built in-tree (tests/native/_build is git-ignored but travels to the box).
NATIVE = tests/native/_build/runtime_check
native: $(NATIVE)

$(NATIVE): tests/native/runtime_check.cpp include/tulips_csum.h $(LIB)
	@mkdir -p tests/native/_build
	g++ -O2 -std=c++17 -Wall -Wextra -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o $@ $< \
	    -Ltulips_amd -ltulips_csum -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../../tulips_amd' -Wl,-rpath,/opt/rocm/lib -ldl

# Measured variants of rounds 1-2 (hybrid, lane-parallel cursors,
# workgroup-balanced, halo / boundary-slot / staged span forms, per-wave
# stamps): tools/sessions/variants/, built apart and never loaded by the product.
variants:
	$(MAKE) -C tools/sessions/variants

# Device assembly + resource usage of the kernels (for inspection).
asm:
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/asm/csum_kernels.s \
	    tulips_amd/csrc/csum_kernels.hip -Rpass-analysis=kernel-resource-usage 2> build/asm/resource.txt

clean:
	rm -rf build $(LIB) $(BENCHLIB) tests/native/_build
	$(MAKE) -C oracle clean
