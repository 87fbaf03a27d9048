# Build recipe (also driven by __graft_entry__.build()).
#   libmantis_amd.so  : product — HIP kernels (gfx950) + C++ host orchestration + RCCL
#   hostcheck / synth : CPU test helpers (device-logic headers built for the host; scene renderer)
#   oracle            : CPU restatement of the reference (test infrastructure)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# -fno-slp-vectorize: the SLP vectorizer packs the FP32 screen of the scorers
# into v_pk_* pairs whose scalar operands need SGPR pairs, and the spills that
# follow cost more than the packing saves (score stage 12.5 -> 11.0 ms per 4096
# frames, 17.1k -> 18.1k rig poses/s, A/B on one box)
HIPFLAGS = -O3 -std=c++17 --offload-arch=$(ARCH) -ffp-contract=off -fno-slp-vectorize -fPIC -Wall -Wno-unused-function -Wno-unused-variable
CSRC = mantis_amd/csrc

.PHONY: all product oracle ref tools clean sanitize
all: product tools oracle

product: mantis_amd/libmantis_amd.so
mantis_amd/libmantis_amd.so: $(CSRC)/api.hip $(CSRC)/kernels.hip $(CSRC)/gn_impl.hip $(CSRC)/dense_impl.hip $(wildcard $(CSRC)/*.h) $(CSRC)/mk_rpp_np.inc $(CSRC)/markov_impl.hip include/mantis.h include/mantis_ros.h
	$(HIPCC) $(HIPFLAGS) -shared -pthread -o $@ $(CSRC)/api.hip -lrccl

tools: build/libmantis_hostcheck.so tools/libmantis_synth.so
build/libmantis_hostcheck.so: $(CSRC)/hostcheck.cpp $(wildcard $(CSRC)/mk_*.h) $(CSRC)/mk_rpp_np.inc
	mkdir -p build
	g++ -O2 -std=c++17 -fPIC -ffp-contract=off -shared -o $@ $(CSRC)/hostcheck.cpp
tools/libmantis_synth.so: tools/synth_host.cpp $(CSRC)/synth.h
	g++ -O2 -std=c++17 -fPIC -shared -o $@ tools/synth_host.cpp

oracle:
	$(MAKE) -C oracle all
ref:
	$(MAKE) -C oracle ref

# CPU sanitizers: the oracle and the host build of the device-logic
# headers with AddressSanitizer + UndefinedBehaviorSanitizer, then the CPU test
# suite against them (python is not instrumented: libasan is preloaded, leak
# checking off). Targets the reference's defined out-of-buffer reads (SURVEY
# Q10, HypothesisEvaluation.h:246-261) that the restatement turns into bounds.
SANFLAGS = -O1 -g -std=c++17 -fPIC -ffp-contract=off -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined
SAN_ORACLE_SRC = oracle/o_imgproc.cpp oracle/o_rpp.cpp oracle/o_mantis3.cpp oracle/o_markov.cpp
build/san/liboracle.so: $(SAN_ORACLE_SRC) $(wildcard oracle/*.hpp) oracle/oracle.h
	mkdir -p build/san
	g++ $(SANFLAGS) -shared -o $@ $(SAN_ORACLE_SRC)
build/san/libmantis_hostcheck.so: $(CSRC)/hostcheck.cpp $(wildcard $(CSRC)/mk_*.h) $(CSRC)/mk_rpp_np.inc
	mkdir -p build/san
	g++ $(SANFLAGS) -shared -o $@ $(CSRC)/hostcheck.cpp
sanitize: build/san/liboracle.so build/san/libmantis_hostcheck.so tools/libmantis_synth.so product
	MANTIS_SANITIZE=1 MANTIS_ORACLE_SO=$(CURDIR)/build/san/liboracle.so MANTIS_HOSTCHECK_SO=$(CURDIR)/build/san/libmantis_hostcheck.so \
	LD_PRELOAD="$$(g++ -print-file-name=libasan.so) $$(g++ -print-file-name=libubsan.so) $$LD_PRELOAD" \
	ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
	python3 -m pytest tests -x -q -m "not gpu" -p no:cacheprovider $(SAN_PYTEST)

clean:
	rm -f mantis_amd/libmantis_amd.so build/libmantis_hostcheck.so tools/libmantis_synth.so
	rm -rf build/san
	$(MAKE) -C oracle clean
