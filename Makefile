# Build of the MI355X AMG solve-phase engine (no cmake; plain make).
#
#   make            -> amg_amd/lib/libsss_amg.so  (host C + gfx950 HIP kernels, one C-ABI library)
#                      amg_amd/bin/amg            (the reference-compatible CLI)
#   make oracle     -> oracle/liboracle.so (+ oracle/_ref/libsss_ref.so when /root/reference exists)
#   make clean
#
# Host C is compiled with gcc exactly like the reference (x86-64 baseline, no FMA contraction);
# HIP with -ffp-contract=off so the parity kernels match the host arithmetic bit for bit.

ROCM    ?= /opt/rocm
HIPCC   ?= $(ROCM)/bin/hipcc
ARCH    ?= gfx950
CC      ?= gcc
JOBS    ?= 8

BUILD   ?= build
LIBDIR  ?= amg_amd/lib
EXTRA   ?=
BINDIR  := amg_amd/bin

CFLAGS   := -O3 -fPIC -ffp-contract=off -fopenmp -std=gnu11 -Wall -Wno-unused-result -I$(ROCM)/include
HIPFLAGS := -O3 -fPIC -std=c++17 --offload-arch=$(ARCH) -ffp-contract=off -Wall -Wno-unused-result $(EXTRA)
           

HOST_SRC := $(wildcard amg_amd/host/sss_*.c)
HOST_LIB_SRC := $(filter-out amg_amd/host/sss_main.c,$(HOST_SRC))
HIP_SRC  := $(wildcard amg_amd/csrc/*.hip)
HOST_OBJ := $(patsubst amg_amd/host/%.c,$(BUILD)/host/%.o,$(HOST_LIB_SRC))
HIP_OBJ  := $(patsubst amg_amd/csrc/%.hip,$(BUILD)/hip/%.o,$(HIP_SRC))
HEADERS  := $(wildcard include/*.h amg_amd/host/*.h amg_amd/csrc/*.hpp)

LIB := $(LIBDIR)/libsss_amg.so
BIN := $(BINDIR)/amg

.PHONY: all oracle clean
all: $(LIB) $(BIN)

$(BUILD)/host/%.o: amg_amd/host/%.c $(HEADERS)
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(BUILD)/hip/%.o: amg_amd/csrc/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(HOST_OBJ) $(HIP_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared -fPIC -o $@ $^ -Wl,-Bsymbolic-functions -lgomp -L$(ROCM)/lib -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,$(ROCM)/lib

$(BIN): amg_amd/host/sss_main.c $(LIB) $(HEADERS)
	@mkdir -p $(BINDIR)
	$(CC) $(CFLAGS) -o $@ amg_amd/host/sss_main.c -L$(LIBDIR) -lsss_amg -Wl,-rpath,'$$ORIGIN/../lib' -lm

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIBDIR) $(BINDIR)
	$(MAKE) -C oracle clean
