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
       tulips_amd/csrc/frame_common.h tulips_amd/csrc/stream_state.h \
       include/tulips_csum.h include/tulips_csum_util.h
OBJS = $(patsubst tulips_amd/csrc/%.hip,build/%.o,$(SRCS))

.PHONY: all lib oracle clean asm variants

all: lib oracle

lib: $(LIB)

build/%.o: tulips_amd/csrc/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

# Measured variants of rounds 1-2 (hybrid, lane-parallel cursors,
# workgroup-balanced, halo / boundary-slot / staged span forms, per-wave
# stamps): tools/variants/, built apart and never loaded by the product.
variants:
	$(MAKE) -C tools/variants

# Device assembly + resource usage of the kernels (for inspection).
asm:
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/asm/csum_kernels.s \
	    tulips_amd/csrc/csum_kernels.hip -Rpass-analysis=kernel-resource-usage 2> build/asm/resource.txt

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean
