#!/usr/bin/env bash
# oracle/build_ref.sh -- build the REFERENCE's own MD5 (test infrastructure).
#
# Compiles /root/reference/src/base/MD5.cpp where it lies (never copied into
# this repo) together with oracle/ref/ref_md5_capi.cpp into
#   oracle/_ref/libref_md5.so      (-O2, the CPU baseline and golden source)
#   oracle/_ref/libref_md5_O0.so   (-O0, "as shipped": cmake with no build type)
# Only boost/shared_ptr.hpp from the reference's vendored boost 1.49 headers is
# needed.  oracle/_ref/ is git-ignored.  Absent /root/reference (e.g. on the GPU
# box) this is a no-op and previously built files are used as they are.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REF="${QSFS_REFERENCE:-/root/reference}"
OUT="$HERE/_ref"
if [[ ! -f "$REF/src/base/MD5.cpp" ]]; then
  echo "build_ref: $REF not present; keeping existing $OUT" >&2
  exit 0
fi
mkdir -p "$OUT"
INC=(-I"$REF/src/base" -I"$REF/third_party/boost_1_49_0")
for opt in O2 O0; do
  suffix=""
  [[ "$opt" == "O0" ]] && suffix="_O0"
  g++ -std=c++11 -"$opt" -fPIC -shared -w "${INC[@]}" \
      "$HERE/ref/ref_md5_capi.cpp" "$REF/src/base/MD5.cpp" \
      -o "$OUT/libref_md5${suffix}.so" -lpthread
done
echo "build_ref: built $OUT/libref_md5.so $OUT/libref_md5_O0.so"
