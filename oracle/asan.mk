# The oracle under AddressSanitizer + UndefinedBehaviorSanitizer, built with the
# same clang as libgol_asan.so so one sanitizer runtime serves both
# (tools/asan_cpu_suite.sh).  Test infrastructure only.
LLVM ?= /opt/rocm/lib/llvm/bin
asan: liboracle_asan.so
liboracle_asan.so: gol_oracle.c
	$(LLVM)/clang -O1 -g -fno-omit-frame-pointer -fPIC -Wall -Wextra -std=c11 -D_GNU_SOURCE \
		-fsanitize=address,undefined -fno-sanitize-recover=undefined -shared-libasan \
		-shared -o $@ $< -lpthread
.PHONY: asan
