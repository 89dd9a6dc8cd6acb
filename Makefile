# Builds libmiclip.so (HIP/CDNA4, gfx950) in-tree so it travels to the GPU box.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := aihab-clip_amd
SRC_DIR  := $(PKG)/csrc
OBJ_DIR  := build/obj
LIB      := $(PKG)/miclip/libmiclip.so
SRCS     := $(wildcard $(SRC_DIR)/*.hip)
OBJS     := $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(SRCS))
HDRS     := $(wildcard $(SRC_DIR)/*.h) include/miclip.h
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function \
            -Wno-unused-variable -Iinclude

all: $(LIB)

# attention: no NaN inputs by construction (masked scores are -inf), so fmaxf
# needs no per-operand canonicalising v_max (20 -> 7 v_max per key tile)
$(OBJ_DIR)/attention.o: HIPFLAGS += -fno-honor-nans -fno-slp-vectorize

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJS) -o $@

asm: $(SRCS)
	@mkdir -p build/asm
	for f in $(SRCS); do $(HIPCC) $(HIPFLAGS) --cuda-device-only -S $$f -o build/asm/$$(basename $$f .hip).s; done

# diagnostic libraries with in-kernel cycle stamps (scripts/stamps/run.py)
stamps: $(OBJS)
	@mkdir -p build/stamps
	$(HIPCC) $(HIPFLAGS) -c scripts/stamps/stamp_gemm.hip -o build/stamps/stamp_gemm.o
	$(HIPCC) $(HIPFLAGS) -fno-honor-nans -fno-slp-vectorize -c scripts/stamps/stamp_attn.hip -o build/stamps/stamp_attn.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) build/stamps/stamp_gemm.o $(filter-out $(OBJ_DIR)/gemm.o,$(OBJS)) -o build/stamps/libstamp_gemm.so
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) build/stamps/stamp_attn.o $(filter-out $(OBJ_DIR)/attention.o,$(OBJS)) -o build/stamps/libstamp_attn.so
	$(HIPCC) $(HIPFLAGS) -c scripts/stamps/stamp_gemm_kloop.hip -o build/stamps/stamp_gemm_kloop.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) build/stamps/stamp_gemm_kloop.o $(filter-out $(OBJ_DIR)/gemm.o,$(OBJS)) -o build/stamps/libstamp_gemm_kloop.so
	$(HIPCC) $(HIPFLAGS) -c scripts/stamps/stamp_gemm_kphase.hip -o build/stamps/stamp_gemm_kphase.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) build/stamps/stamp_gemm_kphase.o $(filter-out $(OBJ_DIR)/gemm.o,$(OBJS)) -o build/stamps/libstamp_gemm_kphase.so

# timing diagnostics (outputs meaningless): the library without the vision-tower
# attention / without the large ln_stats launches, to price what each costs inside
# the two-stream step (bench.py with MICLIP_LIB=build/diag/libmiclip_<x>.so). The
# product sources carry no diagnostic code: the entry point is renamed at compile
# time and wrapped by scripts/diag/skip.hip.
DIAG_DIR := build/diag
diag: $(OBJS)
	@mkdir -p $(DIAG_DIR)
	$(HIPCC) $(HIPFLAGS) -fno-honor-nans -fno-slp-vectorize -Dattention=attention_product -c $(SRC_DIR)/attention.hip -o $(DIAG_DIR)/attention_renamed.o
	$(HIPCC) $(HIPFLAGS) -DSKIP_ATTN -c scripts/diag/skip.hip -o $(DIAG_DIR)/skip_attn.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(DIAG_DIR)/attention_renamed.o $(DIAG_DIR)/skip_attn.o $(filter-out $(OBJ_DIR)/attention.o,$(OBJS)) -o $(DIAG_DIR)/libmiclip_noattn.so
	$(HIPCC) $(HIPFLAGS) -Dln_stats=ln_stats_product -c $(SRC_DIR)/norm.hip -o $(DIAG_DIR)/norm_renamed.o
	$(HIPCC) $(HIPFLAGS) -DSKIP_LNSTATS -c scripts/diag/skip.hip -o $(DIAG_DIR)/skip_lns.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(DIAG_DIR)/norm_renamed.o $(DIAG_DIR)/skip_lns.o $(filter-out $(OBJ_DIR)/norm.o,$(OBJS)) -o $(DIAG_DIR)/libmiclip_nolns.so

clean:
	rm -rf build $(LIB)

.PHONY: all clean asm stamps diag
