# Top-level build helpers.  The product library is built by
# `python -c "import __graft_entry__ as g; g.build()"` (hipcc, gfx950); this
# Makefile adds the CPU sanitizer runs of SURVEY §5 on libfdcn's host code.
#
#   make lib        the in-tree libfdcn.so (same as __graft_entry__.build_lib)
#   make sanitize   asan + tsan below (CPU only, no GPU needed)
#   make asan       fdcn_host.hip + fdcn_plan.hip (every host entry point that
#                   runs without a device: plan checks, plan builders, log
#                   grid, tau sequence, dividend jump, vmath) compiled for the
#                   host with AddressSanitizer + UndefinedBehaviorSanitizer
#                   (-fno-sanitize-recover: the first report aborts), linked
#                   with the regular device objects into build/asan/libfdcn.so;
#                   the bitwise plan tests then run against it
#                   then tools/sanitize/session_book_driver.cpp: the device
#                   sessions' host-only bookkeeping (csrc/fdcn_session_book.h:
#                   pinned staging arena, slot and event tables) under the same
#                   two sanitizers, malloc standing in for hipHostMalloc
#   make tsan       the same two units under ThreadSanitizer with
#                   tools/sanitize/plan_driver.cpp: the plan builders' worker
#                   threads, two callers at once
# Sanitizers instrument host code only (-Xarch_host on every hipcc line).
HIPCC ?= /opt/rocm/bin/hipcc
PY ?= python3
ASAN_RT := $(firstword $(wildcard /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so))
HOSTONLY := --offload-arch=gfx950 --offload-host-only -std=c++17 -fPIC -g -O1 -Wall
ASAN := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
        -Xarch_host -fno-sanitize-recover=all -Xarch_host -fno-omit-frame-pointer
TSAN := -Xarch_host -fsanitize=thread
CSRC := finite_difference_amd/csrc
HOST_SRCS := $(CSRC)/fdcn_host.hip $(CSRC)/fdcn_plan.hip
HDRS := include/fdcn.h include/fdcn_diag.h $(CSRC)/fdcn_shared.h $(CSRC)/fdcn_session_book.h
DEV_OBJS := build/obj/fdcn_kernels.o build/obj/fdcn_analytic.o build/obj/fdcn_session.o \
            build/obj/fdcn_vc.o
SAN_TESTS := tests/test_tau_sequence.py tests/test_capi_symbols.py tests/test_scenario_batch.py \
             tests/test_american_batch.py tests/test_barrier_host.py tests/test_american_host.py

.PHONY: lib sanitize asan tsan clean-sanitize

lib:
	$(PY) -c "import __graft_entry__ as g; g.build_lib()"

$(DEV_OBJS): lib

build/asan/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build/asan
	$(HIPCC) $(HOSTONLY) $(ASAN) -c -o $@ $<

build/asan/libfdcn.so: build/asan/fdcn_host.o build/asan/fdcn_plan.o $(DEV_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -shared-libsan $(ASAN) -o $@ $^

build/asan/session_book_driver: tools/sanitize/session_book_driver.cpp $(CSRC)/fdcn_session_book.h
	@mkdir -p build/asan
	$(CXX) -std=c++17 -g -O1 -Wall -fsanitize=address,undefined -fno-sanitize-recover=all \
	    -fno-omit-frame-pointer -o $@ $<

asan: build/asan/libfdcn.so build/asan/session_book_driver
	ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
	    ./build/asan/session_book_driver
	LD_PRELOAD=$(ASAN_RT) ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:abort_on_error=1 \
	UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
	$(PY) -m pytest $(SAN_TESTS) -q -x -p no:cacheprovider --fdcn-lib build/asan/libfdcn.so

build/tsan/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build/tsan
	$(HIPCC) $(HOSTONLY) $(TSAN) -c -o $@ $<

build/tsan/plan_driver.o: tools/sanitize/plan_driver.cpp include/fdcn.h
	@mkdir -p build/tsan
	$(HIPCC) -std=c++17 -g -O1 -Wall $(TSAN) -c -o $@ $<

build/tsan/plan_driver: build/tsan/plan_driver.o build/tsan/fdcn_host.o build/tsan/fdcn_plan.o
	$(HIPCC) --offload-arch=gfx950 --offload-host-only $(TSAN) -o $@ $^ -lpthread

tsan: build/tsan/plan_driver
	TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 ./build/tsan/plan_driver

sanitize: asan tsan

clean-sanitize:
	rm -rf build/asan build/tsan
