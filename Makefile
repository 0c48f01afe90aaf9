# Build of the MI355X (gfx950) solve loop.  Driven by __graft_entry__.build()
# (`make -j8 all`); everything lands in-tree so it travels to the GPU box.
#   libfrecsys_hip.so  -- HIP kernels + C-ABI (include/frecsys_hip.h)
#   libfrecsys_model.so -- C-ABI of the model classes (include/frecsys_model.h)
#   run_model          -- reference-compatible CLI (C++ host over the C-ABI)
#   liboracle.so       -- CPU restatement, TEST INFRASTRUCTURE ONLY
PKG      := safer2-recommender_amd
CSRC     := $(PKG)/csrc
OBJ      := $(PKG)/build
LIB      := $(PKG)/frecsys_hip/libfrecsys_hip.so
ORACLE   := oracle/liboracle.so
RUNMODEL := $(PKG)/bin/run_model
MODELDUMP := $(PKG)/bin/model_dump
MODELLIB := $(PKG)/frecsys_hip/libfrecsys_model.so
ARCH     ?= gfx950
HIPCC    ?= /opt/rocm/bin/hipcc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
CXXFLAGS := -O3 -std=c++17 -Wall -I include -I $(PKG)/include -pthread

HIP_SRCS := $(CSRC)/solve.hip $(CSRC)/dual.hip $(CSRC)/spectral.hip $(CSRC)/gramian.hip \
            $(CSRC)/loss.hip $(CSRC)/wide.hip $(CSRC)/wide_syrk.hip $(CSRC)/topk.hip $(CSRC)/pp.hip \
            $(CSRC)/capi.hip
HIP_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJ)/%.o,$(HIP_SRCS))
HDRS     := $(CSRC)/kernels.h $(CSRC)/common.h $(CSRC)/chol.h $(CSRC)/wide.h include/frecsys_hip.h

.PHONY: all lib oracle run_model model_dump model_lib clean ablation
all: lib oracle run_model model_dump model_lib
model_lib: $(MODELLIB)
lib: $(LIB)
oracle: $(ORACLE)
run_model: $(RUNMODEL)
model_dump: $(MODELDUMP)

# the wide SYRK: no SLP pairing of its scalar f32 subtractions (v_pk_add_f32
# beside MFMAs costs issue cycles)
$(OBJ)/wide_syrk.o ab/obj/wide_syrk.o: HIPFLAGS += -fno-slp-vectorize
$(OBJ)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIP_OBJS) -lrccl

$(ORACLE): oracle/frecsys_oracle.c oracle/frecsys_oracle.h oracle/cpu_baseline.c
	gcc -O3 -march=native -std=c11 -fPIC -shared -Wall -o $@ oracle/frecsys_oracle.c oracle/cpu_baseline.c -lpthread -lm

FRECSYS_HDRS := $(wildcard $(PKG)/include/frecsys/*.h)
$(RUNMODEL): $(PKG)/tools/run_model.cc $(FRECSYS_HDRS) include/frecsys_hip.h $(LIB)
	@mkdir -p $(PKG)/bin
	g++ $(CXXFLAGS) -o $@ $(PKG)/tools/run_model.cc -L$(PKG)/frecsys_hip -lfrecsys_hip \
	    -Wl,-rpath,'$$ORIGIN/../frecsys_hip'

$(MODELLIB): $(PKG)/tools/model_capi.cc $(FRECSYS_HDRS) include/frecsys_hip.h include/frecsys_model.h $(LIB)
	g++ $(CXXFLAGS) -fPIC -shared -o $@ $(PKG)/tools/model_capi.cc -L$(PKG)/frecsys_hip -lfrecsys_hip \
	    -Wl,-rpath,'$$ORIGIN'

clean:
	rm -rf $(OBJ) $(LIB) $(MODELLIB) $(ORACLE) $(PKG)/bin

$(MODELDUMP): tests/cpp/model_dump.cc $(FRECSYS_HDRS) include/frecsys_hip.h $(LIB)
	@mkdir -p $(PKG)/bin
	g++ $(CXXFLAGS) -o $@ tests/cpp/model_dump.cc -L$(PKG)/frecsys_hip -lfrecsys_hip \
	    -Wl,-rpath,'$$ORIGIN/../frecsys_hip'

# Profiling-only build with the FRECSYS_DEBUG_SKIP ablation masks compiled in
# (the shipped library refuses the variable); LD_LIBRARY_PATH / a copy over
# frecsys_hip/libfrecsys_hip.so swaps it in for an ablation run.
ABL_LIB := ab/libfrecsys_hip_ablation.so
ABL_OBJS := $(patsubst $(CSRC)/%.hip,ab/obj/%.o,$(HIP_SRCS))
ablation: $(ABL_LIB)
ab/obj/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p ab/obj
	$(HIPCC) $(HIPFLAGS) -DFRECSYS_ABLATION -c $< -o $@
$(ABL_LIB): $(ABL_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(ABL_OBJS) -lrccl

# A/B build of the library with extra defines, for a timed comparison on the
# GPU box (a copy over frecsys_hip/libfrecsys_hip.so swaps it in there), e.g.
#   make abvar ABDEF=-DFRECSYS_CHOL_X6=1 ABNAME=x6  ->  ab/libfrecsys_hip_x6.so
ABNAME ?= var
.PHONY: abvar
abvar: $(HIP_SRCS) $(HDRS)
	@mkdir -p ab/obj/$(ABNAME)
	for f in $(HIP_SRCS); do $(HIPCC) $(HIPFLAGS) $(ABDEF) -c $$f -o ab/obj/$(ABNAME)/$$(basename $$f .hip).o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o ab/libfrecsys_hip_$(ABNAME).so ab/obj/$(ABNAME)/*.o -lrccl
