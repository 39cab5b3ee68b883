# Host sanitizer build ("Host ASan/UBSan in CPU tests"): the host
# code of libgol.so (engine.cpp, plan.cpp, stripes.cpp: planner, schedule, partition
# and config logic)
# under AddressSanitizer + UndefinedBehaviorSanitizer, linked with the regular
# gfx950 kernel objects (device code is never sanitized: GPU ASan does not exist
# on this pool).  CPU only -- tools/asan_cpu_suite.sh runs the CPU test suite
# against it with the clang runtime preloaded.  Not part of the shipped build.
#   make -f asan.mk        -> build/asan/libgol_asan.so
include Makefile
LLVM ?= $(ROCM)/lib/llvm/bin
ASAN_HOST = -O1 -g -fno-omit-frame-pointer -Xarch_host -fsanitize=address \
	-Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined
ASAN_OBJ = $(filter-out $(foreach u,$(HOST),build/$(u).o),$(OBJ)) $(foreach u,$(HOST),build/asan/$(u).o)

asan: build/asan/libgol_asan.so

build/asan/%.o: csrc/%.cpp $(HDR)
	@mkdir -p build/asan
	$(HIPCC) -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter $(ASAN_HOST) -c -o $@ $<

build/asan/libgol_asan.so: $(ASAN_OBJ)
	$(LLVM)/clang++ -shared -shared-libasan -fno-gpu-sanitize -fsanitize=address,undefined \
		-o $@ $(ASAN_OBJ) -L$(ROCM)/lib -lamdhip64 -lrccl -Wl,-rpath,$(ROCM)/lib

.DEFAULT_GOAL := asan
.PHONY: asan
