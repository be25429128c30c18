# Build of libqlx.so (HIP for gfx950 + C++ host) and the CPU oracle (test infrastructure).
#   make            -> q-learning_amd/lib/libqlx.so + oracle/liboracle.so + oracle/cpu_baseline
#   make lib        -> product only
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := q-learning_amd
SRC := $(PKG)/csrc
OUT := $(PKG)/lib
JOBS ?= 8

HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-result \
            -I include -I $(SRC) -munsafe-fp-atomics
# physics/raster must round every a*b+c twice like the reference (Rust never fuses)
STRICT := -ffp-contract=off
LDFLAGS := -shared -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib

OBJS := $(OUT)/obj/common.o $(OUT)/obj/env_breakout.o $(OUT)/obj/replay.o $(OUT)/obj/qnet.o $(OUT)/obj/qnet32.o $(OUT)/obj/learner.o \
        $(OUT)/obj/ballgame.o $(OUT)/obj/tf_bundle.o $(OUT)/obj/per.o $(OUT)/obj/stats.o

HDRS := include/qlx.h $(wildcard $(SRC)/*.h)

all: lib oracle

lib: $(OUT)/libqlx.so

$(OUT)/obj:
	mkdir -p $@

$(OUT)/obj/common.o: $(SRC)/common.cpp $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT)/obj/env_breakout.o: $(SRC)/env_breakout.hip $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) $(STRICT) -c $< -o $@

$(OUT)/obj/replay.o: $(SRC)/replay.hip $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# (bf16 Q-net on the default scheduler since round 5: 789K -> 797K env-steps/s against max-ILP, the slab reduction
# 11.4 -> 10.0 us)
$(OUT)/obj/qnet.o: $(SRC)/qnet.hip $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# fp32 Q-net: bit-exact against the oracle, so no contraction anywhere (every fma is an explicit fmaf / MFMA)
# Q-net objects: the backend's max-ILP scheduling strategy (measured at C3: fp32 195.5K -> 196.2K env-steps/s, every GEMM
# layer equal or faster; max-memory-clause 191.0K, iterative-ilp 196.6K; bf16 745.7K -> 749.3K)
Q32SCHED := -mllvm --amdgpu-sched-strategy=max-ilp
# fp32 Q-net: MFMA accumulators in VGPRs (the AGPR form rotated the pair GEMMs' accumulators through v_accvgpr moves every
# slab - VALU time the fp32 MFMAs cannot overlap; measured: conv2 / conv3 pairs 96.4 / 72.1 -> 95.9 / 71.2 us)
Q32VFORM := -mllvm -amdgpu-mfma-vgpr-form=1

$(OUT)/obj/qnet32.o: $(SRC)/qnet32.hip $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) $(STRICT) $(Q32SCHED) $(Q32VFORM) -c $< -o $@

$(OUT)/obj/learner.o: $(SRC)/learner.hip $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) $(STRICT) -c $< -o $@

$(OUT)/obj/tf_bundle.o: $(SRC)/tf_bundle.cpp $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# BallGame env step is restated like the reference's f32 rewards (no FMA-sensitive math); the net is fp32 SIMT
$(OUT)/obj/ballgame.o: $(SRC)/ballgame.hip $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# sum-tree descent and IS weights are compared bit-for-bit with the oracle: no contraction
$(OUT)/obj/per.o: $(SRC)/per.hip $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) $(STRICT) -c $< -o $@

$(OUT)/obj/stats.o: $(SRC)/stats.hip $(HDRS) | $(OUT)/obj
	$(HIPCC) $(HIPFLAGS) $(STRICT) -c $< -o $@

$(OUT)/libqlx.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) $(OBJS) $(LDFLAGS) -o $@

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(OUT) && $(MAKE) -C oracle clean

.PHONY: all lib oracle clean
