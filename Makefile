# Build: the HIP product library (gfx950) and the CPU oracle (test infrastructure).
#   make            -> both
#   make product    -> crdt-enc_amd/libcrdtenc.so
#   make oracle     -> oracle/libce_oracle.so
#   make prof       -> crdt-enc_amd/libcrdtenc_prof.so (CE_PROF / CE_ABLATE diagnostics; load it
#                      with CRDTENC_LIB=crdt-enc_amd/libcrdtenc_prof.so)
HIPCC      ?= /opt/rocm/bin/hipcc
ARCH       ?= gfx950
PKG        := crdt-enc_amd
CSRC       := $(PKG)/csrc
PRODUCT    := $(PKG)/libcrdtenc.so
ORACLE     := oracle/libce_oracle.so

HIP_SRCS   := $(wildcard $(CSRC)/*.hip)
CPP_SRCS   := $(wildcard $(CSRC)/*.cpp)
HDRS       := $(wildcard $(CSRC)/*.h) $(wildcard include/*.h)
HIP_OBJS   := $(patsubst $(CSRC)/%.hip,$(PKG)/build/%.o,$(HIP_SRCS))
CPP_OBJS   := $(patsubst $(CSRC)/%.cpp,$(PKG)/build/%.o,$(CPP_SRCS))
PROF_LIB   := $(PKG)/libcrdtenc_prof.so
PROF_OBJS  := $(patsubst $(CSRC)/%.hip,$(PKG)/build_prof/%.o,$(HIP_SRCS)) \
              $(patsubst $(CSRC)/%.cpp,$(PKG)/build_prof/%.o,$(CPP_SRCS))

HIPFLAGS   := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -mllvm -pragma-unroll-threshold=1000000 -Iinclude -I$(CSRC) -Wall -Wno-unused-function
CXXFLAGS   := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Xarch_host -march=x86-64-v3 -Iinclude -I$(CSRC) -Wall -Wno-unused-function

all: product oracle

product: $(PRODUCT)
oracle: $(ORACLE)

$(PKG)/build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(PKG)/build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/build/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(PKG)/build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(PKG)/build_prof/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(PKG)/build_prof
	$(HIPCC) $(HIPFLAGS) -DCE_FUSED_DIAG=1 -c $< -o $@

$(PKG)/build_prof/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(PKG)/build_prof
	$(HIPCC) $(CXXFLAGS) -DCE_FUSED_DIAG=1 -c $< -o $@

prof: $(PROF_LIB)

$(PROF_LIB): $(PROF_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread -lhsa-runtime64

$(PRODUCT): $(HIP_OBJS) $(CPP_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread -lhsa-runtime64

$(ORACLE): oracle/ce_oracle.c oracle/ce_oracle.h
	gcc -O3 -march=x86-64-v3 -fPIC -shared -Wall -Wextra -o $@ oracle/ce_oracle.c -lpthread

clean:
	rm -rf $(PKG)/build $(PKG)/build_prof $(PRODUCT) $(PROF_LIB) $(ORACLE)

.PHONY: all product oracle prof clean
