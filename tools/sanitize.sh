#!/bin/bash
# Host AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU path
# (SURVEY.md section 5): the product library's HOST code (the host executor's
# thread pool and systems, the C ABI, the host policy) and the oracle, built
# with ASan + UBSan, under the CPU test suite (pytest -m "not gpu").  Device
# code is compiled as usual (no GPU sanitizer: -fsanitize applies to the host
# side only, -Xarch_host).  Runs in the build container, no GPU.
#
#   bash tools/sanitize.sh [pytest args...]     log: profiles/<round>/sanitize_*.log
set -eu
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
LLVM=/opt/rocm/lib/llvm
RT=$(ls "$LLVM"/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n 1)
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"

# 1. the product library, host side sanitized (variant build under _variants/san)
python3 -m madrona_basketball_amd.build --variant san \
    --flag=-Xarch_host --flag=-fsanitize=address --flag=-Xarch_host --flag=-fsanitize=undefined \
    --flag=-Xarch_host --flag=-fno-sanitize-recover=undefined --flag=-Xarch_host --flag=-fno-omit-frame-pointer
LIB=$R/madrona_basketball_amd/_variants/san/libmadrona_basketball_amd.so

# 2. the oracle (same source and flags as oracle/Makefile, clang + sanitizers)
mkdir -p "$R/oracle/_san"
"$LLVM/bin/clang" -O1 -std=c11 -fPIC -ffp-contract=off -fno-fast-math $SAN -shared \
    -o "$R/oracle/_san/liboracle_bb.so" "$R/oracle/bb_oracle.c" -lm

# 3. the CPU suite with the ASan runtime preloaded (python itself is not
# instrumented; its own allocations are not leak-checked)
cd "$R"
export MADRONA_BB_LIB=$LIB MADRONA_BB_ORACLE_LIB=$R/oracle/_san/liboracle_bb.so
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
LD_PRELOAD=$RT python3 -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
# the runtime was live in those processes (the instrumented libraries resolve
# their __asan / __ubsan hooks against it)
LD_PRELOAD=$RT python3 -c "import ctypes; L = ctypes.CDLL('$LIB'); ctypes.CDLL(None).__asan_init; \
print('asan runtime live; instrumented:', len([1 for n in ('__asan_report_load4', '__ubsan_handle_add_overflow') \
if hasattr(ctypes.CDLL(None), n)]), 'hooks resolved')"
