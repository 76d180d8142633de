#!/bin/bash
# Host-side sanitizers: ASan + UBSan builds of libfmpnp.so's host code (the C ABI's
# validation, the planner, workspace sizing, launch glue; device code is not instrumented) and of
# the C oracle, then the CPU test suite with both loaded (clang's ASan runtime preloaded into
# python; FMPNP_PLAN_CUS lets the planner run without a GPU).  The log goes to $1
# (default profiles/r04_sanitize_cpu.log).
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LOG=${1:-$ROOT/profiles/r04_sanitize_cpu.log}
make -s -C "$ROOT/featuremetric-pnp_amd" -j8 sanitize || exit 1
make -s -C "$ROOT/oracle" sanitize || exit 1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
{
  echo "# tools/sanitize.sh: $(date -u +%FT%TZ), git $(git -C "$ROOT" rev-parse --short HEAD 2>/dev/null)"
  echo "# libfmpnp: featuremetric-pnp_amd/fmpnp/lib_san/libfmpnp.so (host: -fsanitize=address,undefined)"
  echo "# oracle:   oracle/build_san/liborc_fmpnp.so (-fsanitize=address,undefined)"
  echo "# runtime:  $RT"
  cd "$ROOT" && LD_PRELOAD="$RT" \
    ASAN_OPTIONS=detect_leaks=0:alloc_dealloc_mismatch=0:halt_on_error=1:abort_on_error=1 \
    UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    FMPNP_LIB_PATH="$ROOT/featuremetric-pnp_amd/fmpnp/lib_san/libfmpnp.so" \
    ORC_LIB_PATH="$ROOT/oracle/build_san/liborc_fmpnp.so" FMPNP_PLAN_CUS=256 \
    python -m pytest tests -m "not gpu" -q -p no:cacheprovider 2>&1
  # canary: the same environment must catch an out-of-bounds read (orc_sobel told C=2 on a 1-plane
  # buffer) -- proves the instrumentation is live, not just linked
  cd "$ROOT" && LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0 ORC_LIB_PATH="$ROOT/oracle/build_san/liborc_fmpnp.so" \
    python -c "
import ctypes, numpy as np, oracle.oracle as o
x = np.zeros((1, 8, 8)); g = np.zeros((2, 8, 8))
o.lib().orc_sobel(o._ptr(x), 2, 8, 8, o._ptr(g), o._ptr(g.copy()))
" > /tmp/san_canary.txt 2>&1
  if grep -q "ERROR: AddressSanitizer: heap-buffer-overflow" /tmp/san_canary.txt; then
    echo "canary: out-of-bounds read caught by AddressSanitizer (instrumentation live)"
  else
    echo "canary: NOT caught"; cat /tmp/san_canary.txt; exit 1
  fi
} | tee "$LOG"
