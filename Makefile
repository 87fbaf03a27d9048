# Build recipe (also driven by __graft_entry__.build()).
#   libmantis_amd.so  : product — HIP kernels (gfx950) + C++ host orchestration + RCCL
#   hostcheck / synth : CPU test helpers (device-logic headers built for the host; scene renderer)
#   oracle            : CPU restatement of the reference (test infrastructure)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS = -O3 -std=c++17 --offload-arch=$(ARCH) -ffp-contract=off -fPIC -Wall -Wno-unused-function -Wno-unused-variable
CSRC = mantis_amd/csrc

.PHONY: all product oracle ref tools clean
all: product tools oracle

product: mantis_amd/libmantis_amd.so
mantis_amd/libmantis_amd.so: $(CSRC)/api.hip $(CSRC)/kernels.hip $(CSRC)/gn_impl.hip $(CSRC)/dense_impl.hip $(wildcard $(CSRC)/*.h) include/mantis.h include/mantis_ros.h
	$(HIPCC) $(HIPFLAGS) -shared -pthread -o $@ $(CSRC)/api.hip -lrccl

tools: build/libmantis_hostcheck.so tools/libmantis_synth.so
build/libmantis_hostcheck.so: $(CSRC)/hostcheck.cpp $(wildcard $(CSRC)/mk_*.h)
	mkdir -p build
	g++ -O2 -std=c++17 -fPIC -ffp-contract=off -shared -o $@ $(CSRC)/hostcheck.cpp
tools/libmantis_synth.so: tools/synth_host.cpp $(CSRC)/synth.h
	g++ -O2 -std=c++17 -fPIC -shared -o $@ tools/synth_host.cpp

oracle:
	$(MAKE) -C oracle all
ref:
	$(MAKE) -C oracle ref

clean:
	rm -f mantis_amd/libmantis_amd.so build/libmantis_hostcheck.so tools/libmantis_synth.so
	$(MAKE) -C oracle clean
