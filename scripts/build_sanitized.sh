#!/bin/bash
# scripts/build_sanitized.sh -- host-sanitizer builds of the runtime for the
# race/memory stress test (tests/cpp/race_stress.cpp).  SURVEY.md §5 asks for
# the C-ABI to be checked under -fsanitize=thread; GPU-side sanitizers are not
# available on the pool, so only HOST code is instrumented: every
# -fsanitize= on a hipcc line sits behind -Xarch_host, and the gfx950 kernels
# are the product's own object.
#   qsfs-fuse_amd/lib/san/race_stress_tsan   runtime + test under ThreadSanitizer
#   qsfs-fuse_amd/lib/san/race_stress_asan   runtime + test under AddressSanitizer + UBSan
#   qsfs-fuse_amd/lib/san/nested_read_{tsan,asan}  tests/cpp/nested_read.cpp over the same runtime
# Builds in this container (hipcc cross-compiles); runs on the GPU box
# (tests/test_gpu_sanitizers.py).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
CXX=${CXX_SAN:-/opt/rocm/llvm/bin/clang++}
CC=${CC_SAN:-/opt/rocm/llvm/bin/clang}
OUT=$R/qsfs-fuse_amd/lib/san
mkdir -p "$OUT"
make -s -C "$R/qsfs-fuse_amd" lib/md5_kernels.o
for v in tsan asan; do
  case $v in
    tsan) SAN="-fsanitize=thread" ;;
    asan) SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer" ;;
  esac
  HOSTSAN=""
  for f in $SAN; do HOSTSAN="$HOSTSAN -Xarch_host $f"; done
  RT_OBJS=""
  for u in qsmd5_runtime qsmd5_rt_device qsmd5_rt_staging qsmd5_rt_route qsmd5_rt_read; do
    $HIPCC -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $HOSTSAN \
      -x hip -c "$R/qsfs-fuse_amd/csrc/$u.cpp" -o "$OUT/${u}_$v.o"
    RT_OBJS="$RT_OBJS $OUT/${u}_$v.o"
  done
  $CXX -O1 -g -std=c++17 -fPIC $SAN -c "$R/qsfs-fuse_amd/csrc/md5_cpu.cpp" -o "$OUT/md5_cpu_$v.o"
  $CXX -O1 -g -std=c++17 -fPIC $SAN -c "$R/qsfs-fuse_amd/csrc/md5_cpu_mb.cpp" -o "$OUT/md5_cpu_mb_$v.o"
  $CXX -O1 -g -std=c++17 $SAN -c "$R/tests/cpp/race_stress.cpp" -o "$OUT/race_stress_$v.o"
  $CC -O1 -g -std=c11 $SAN -c "$R/oracle/md5_oracle.c" -o "$OUT/md5_oracle_$v.o"
  $CXX $SAN -o "$OUT/race_stress_$v" "$OUT/race_stress_$v.o" $RT_OBJS "$OUT/md5_cpu_$v.o" "$OUT/md5_cpu_mb_$v.o" \
    "$R/qsfs-fuse_amd/lib/md5_kernels.o" "$OUT/md5_oracle_$v.o" \
    -L/opt/rocm/lib -lamdhip64 -lpthread -Wl,-rpath,/opt/rocm/lib
  # read callbacks calling back into the library (round 6):
  # reader crews, nested calls, a shutdown pending meanwhile
  $CXX -O1 -g -std=c++17 $SAN -c "$R/tests/cpp/nested_read.cpp" -o "$OUT/nested_read_$v.o"
  $CXX $SAN -o "$OUT/nested_read_$v" "$OUT/nested_read_$v.o" $RT_OBJS "$OUT/md5_cpu_$v.o" "$OUT/md5_cpu_mb_$v.o" \
    "$R/qsfs-fuse_amd/lib/md5_kernels.o" -L/opt/rocm/lib -lamdhip64 -lpthread -Wl,-rpath,/opt/rocm/lib
done
echo "sanitized builds: $OUT/race_stress_tsan $OUT/race_stress_asan $OUT/nested_read_tsan $OUT/nested_read_asan"
