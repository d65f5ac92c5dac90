#!/bin/bash
# Host AddressSanitizer + UndefinedBehaviorSanitizer run of the composite C-ABI on the GPU box (no host ASan
# build).  Build beforehand on the CPU: make -C fft-isdf-scratch_amd/csrc asan (the library's host
# code and the driver instrumented; the device code is built as usual).
# Usage (repo root, GPU box): bash tools/asan_check.sh [OUTDIR] [CASE...]
set -o pipefail
OUT=${1:-gpurun_out/asan}
shift
CASES=${*:-toy222 toy333_fr toy666}
mkdir -p $OUT
# leak reports would list the HIP runtime's own process-lifetime allocations; the harness
# preloads a library of its own, so the sanitizer runtime is not first in the link order
export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:abort_on_error=0:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
for c in $CASES; do
  timeout -k 10 120 python -u tools/asan/check.py make $c $OUT/$c || exit 1
  timeout -k 10 120 ./tools/asan/capi_asan $OUT/$c/case.bin $OUT/$c/out.bin > $OUT/$c/run.log 2>&1
  rc=$?
  cat $OUT/$c/run.log
  [ $rc -eq 0 ] || { echo "capi_asan $c exited $rc"; exit 1; }
  timeout -k 10 120 python -u tools/asan/check.py verify $c $OUT/$c || exit 1
  rm -f $OUT/$c/case.bin $OUT/$c/out.bin
done
echo "host ASan: all cases clean"
