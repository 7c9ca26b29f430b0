#!/bin/bash
# CPU sanitizer run: AddressSanitizer + UBSan on the C oracle, the host
# side of libmpcekf.so (ROM validation, argument checks, mpcekf_cl_eig; its kernels are
# not run: no GPU here) and the MEX gateway with its test shim, then the CPU test files
# that drive them.  One sanitizer runtime (clang's) is preloaded into Python.
#   bash tools/sanitize.sh [LOG]      (default profiles/r06_sanitizers.log)
set -o pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r06_sanitizers.log}
CL=/opt/rocm/lib/llvm/bin/clang
SAN="-O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined"
B=mpc-ekf4fastcharge_amd/_build
S=$B/san
mkdir -p $S
make -s -C oracle asan || exit 1
python3 -c "import sys; sys.path.insert(0, '.'); import importlib; importlib.import_module('mpc-ekf4fastcharge_amd.build').build()" || exit 1
SRC_HASH=$(python3 -c "import sys; sys.path.insert(0, '.'); import importlib; print(importlib.import_module('mpc-ekf4fastcharge_amd.build').source_hash())")
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -DMPCEKF_SRC_HASH=\"$SRC_HASH\" \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
  -c mpc-ekf4fastcharge_amd/csrc/mpcekf_host.cpp -o $S/mpcekf_host.o || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $S/libmpcekf.so $B/mpcekf_kernels.o $B/mpcekf_wide.o $B/mpcekf_io.o \
  $S/mpcekf_host.o || exit 1
$CL $SAN -fPIC -std=c11 -Wall -Wno-unused-parameter -Itests/mex -Iinclude -shared -o $S/libmpcekf_mexshim.so \
  tests/mex/mexshim.c matlab/mpcekf_mex.c -L$S -lmpcekf -Wl,-rpath,"$(pwd)/$S" || exit 1
RT=$($CL -print-file-name=libclang_rt.asan-x86_64.so)
export LD_LIBRARY_PATH=/opt/rocm/lib/llvm/lib:$LD_LIBRARY_PATH
{
  echo "# $(date -u +%FT%TZ)  build $SRC_HASH  clang ASan+UBSan (halt on error), runtime $RT"
  echo "# oracle/_build/liboracle_asan.so, $S/libmpcekf.so (host TU instrumented), $S/libmpcekf_mexshim.so"
  LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
  UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  MPCEKF_LIB=$S/libmpcekf.so ORACLE_LIB=oracle/_build/liboracle_asan.so MEXSHIM_LIB=$S/libmpcekf_mexshim.so \
    python3 -m pytest tests/test_oracle.py tests/test_oracle_mb.py tests/test_diag.py tests/test_abi.py \
      tests/test_rom.py tests/test_mex_gateway.py tests/test_handles.py tests/test_tab_handles.py \
      -m "not gpu" -q -p no:cacheprovider 2>&1
  echo "# exit status $?"
  for f in oracle/_build/liboracle_asan.so $S/libmpcekf.so $S/libmpcekf_mexshim.so; do
    echo "# $f: $(nm -D $f | grep -c '__asan_report\|__ubsan_handle') sanitizer entry points referenced"
  done
} | tee $LOG
