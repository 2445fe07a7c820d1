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
       tulips_amd/csrc/stream_state.hip tulips_amd/csrc/csum_multi.hip
HDRS = tulips_amd/csrc/csum_common.h tulips_amd/csrc/csum_launch.h \
       tulips_amd/csrc/frame_common.h tulips_amd/csrc/stream_state.h \
       include/tulips_csum.h include/tulips_csum_util.h
OBJS = $(patsubst tulips_amd/csrc/%.hip,build/%.o,$(SRCS))

.PHONY: all lib oracle clean asm stamps xcd_ab spandiag genstore s3ab

all: lib oracle

lib: $(LIB)

build/%.o: tulips_amd/csrc/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

# Diagnostic build: per-wave realtime stamps (tools/probe_stamps.py). Never
# loaded by the product.
stamps: tools/libcsum_stamps.so

tools/libcsum_stamps.so: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DTULIPS_CSUM_STAMPS -shared -o $@ $(SRCS)

# Diagnostic A/B builds of the XCD cluster size (tools/ab_xcd.sh). Never
# loaded by the product.
XCD_AB = 1 2 4 8 32 1024
xcd_ab: $(foreach c,$(XCD_AB),tools/libcsum_xcd$(c).so)

tools/libcsum_xcd%.so: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DTULIPS_XCD_CLUSTER=$* -shared -o $@ $(SRCS)

# Diagnostic builds of the arena-span kernel that stop after staging the
# chunks (1: without, 2: with the offsets window), once [lo, hi) is known (3),
# before the segment pass (4), without result stores (5), or with each
# workgroup's results stored to its own 256-byte block (6)
# (tools/probe_spandiag.py).
# Never loaded by the product.
spandiag: $(foreach d,1 2 3 4 5 6,tools/libcsum_spandiag$(d).so)

tools/libcsum_spandiag%.so: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DTULIPS_SPAN_DIAG=$* -shared -o $@ $(SRCS)

# Diagnostic builds of frame generation's field stores (1: whole 16-byte
# chunks, 2: the frame's whole first 64-byte line, 3: 2-byte stores with the
# header chunks loaded temporal, 4: nt 2-byte stores; tools/probe_genstore.py).
# Never loaded by the product.
genstore: $(foreach d,1 2 3 4,tools/libcsum_genstore$(d).so)

tools/libcsum_genstore%.so: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DTULIPS_GEN_STORE=$* -shared -o $@ $(SRCS)

# Diagnostic A/B builds of the split-form span words' stride (words per
# range: 1 = packed, 16 = one 128-byte line each; tools/ab_probe.sh).
# Never loaded by the product.
# Cluster (consecutive ranges per XCD run) and offsets-window A/B builds:
# tools/ab_s3c<C>w<NWIN>.so.
s3ab: tools/ab_s3s1.so tools/ab_s3s16.so tools/ab_s3c8w1024.so tools/ab_s3c32w1024.so \
      tools/ab_s3c8w512.so tools/ab_s3c32w512.so

tools/ab_s3s%.so: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DTULIPS_SPAN3_STRIDE=$* -shared -o $@ $(SRCS)

tools/ab_s3c8w1024.so tools/ab_s3c32w1024.so tools/ab_s3c8w512.so tools/ab_s3c32w512.so: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DTULIPS_SPAN3_CLUSTER=$(word 1,$(subst w, ,$(patsubst tools/ab_s3c%.so,%,$@))) \
	    -DTULIPS_SPAN3_NWIN=$(word 2,$(subst w, ,$(patsubst tools/ab_s3c%.so,%,$@))) -shared -o $@ $(SRCS)

# Device assembly + resource usage of the kernels (for inspection).
asm:
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/asm/csum_kernels.s \
	    tulips_amd/csrc/csum_kernels.hip -Rpass-analysis=kernel-resource-usage 2> build/asm/resource.txt

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean
