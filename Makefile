# Top-level build: product libraries (HIP for gfx950 + host C++) and the
# oracle (test infrastructure).  No cmake/ninja needed.
#
#   make            -> dealii-ns-gls_amd/lib/libglsmesh.so, libglsamd.so, oracle/liboracle.so
#   make mesh|amd|oracle
#   make clean

PKG      := dealii-ns-gls_amd
LIBDIR   := $(PKG)/lib
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950

CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -munsafe-fp-atomics \
            -Wall -Wno-unused-parameter -Wno-unused-function

# rocsolver/rocblas: dense LU of the coarse multigrid level only; rccl: ghost exchange
# rocprofiler-sdk-roctx: the timer sections' roctx ranges (trace.cc)
AMD_LIBS := -L/opt/rocm/lib -lrocsolver -lrocblas -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib

MESH_SRC := $(PKG)/host/mesh.cc
AMD_SRC  := $(wildcard $(PKG)/csrc/*.hip) $(wildcard $(PKG)/csrc/*.cc)
AMD_HDR  := $(wildcard $(PKG)/csrc/*.h) $(wildcard $(PKG)/csrc/*.inc) $(wildcard $(PKG)/csrc/*.cuh) include/gls_op.h

all: mesh amd oracle cpptest tools

tools: $(LIBDIR)/libglsamd.so $(LIBDIR)/libglsmesh.so
	$(MAKE) -C tools all

mesh: $(LIBDIR)/libglsmesh.so
amd: $(LIBDIR)/libglsamd.so
oracle:
	$(MAKE) -C oracle

$(LIBDIR)/libglsmesh.so: $(MESH_SRC) include/gls_mesh.h
	@mkdir -p $(LIBDIR)
	$(CXX) $(CXXFLAGS) -shared -o $@ $(MESH_SRC)

# one object per source (make -j builds them in parallel), then one link
OBJDIR   := $(PKG)/build
AMD_OBJ  := $(patsubst $(PKG)/csrc/%,$(OBJDIR)/%.o,$(AMD_SRC))

$(OBJDIR)/%.o: $(PKG)/csrc/% $(AMD_HDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/libglsamd.so: $(AMD_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(AMD_OBJ) $(AMD_LIBS)

# C++ facade parity program (test infrastructure: links the oracle)
CPPTEST := tests/cpp/build/test_operator
cpptest: $(CPPTEST)
$(CPPTEST): tests/cpp/test_operator.cc include/gls_operator.hpp include/gls_op.h include/gls_mesh.h \
            $(LIBDIR)/libglsamd.so $(LIBDIR)/libglsmesh.so oracle
	@mkdir -p tests/cpp/build
	$(CXX) -O2 -std=c++17 -Wall -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include -o $@ $< \
	  -L$(LIBDIR) -lglsamd -lglsmesh -Loracle -loracle -L/opt/rocm/lib -lamdhip64 \
	  -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)' -Wl,-rpath,'$$ORIGIN/../../../oracle' \
	  -Wl,-rpath,/opt/rocm/lib

clean:
	rm -f $(LIBDIR)/*.so $(CPPTEST)
	rm -rf $(OBJDIR)
	$(MAKE) -C oracle clean

.PHONY: all mesh amd oracle cpptest tools clean

