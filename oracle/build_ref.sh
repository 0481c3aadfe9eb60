#!/bin/sh
# Builds oracle/_ref/libref_headers.so: oracle/ref_headers.cpp over the
# reference's own, unmodified headers, straight from /root/reference.
# TEST INFRASTRUCTURE ONLY (fixture generation in this container; the GPU box
# has no /root/reference and never runs this).  Output goes to oracle/_ref/
# only (git-ignored).  No reference file is copied, patched or shimmed.
#
# Flags: -DWIN32 selects SePreDefine.h's __declspec(align) branch (the one the
# reference's own build takes); -fms-extensions -fdeclspec accept
# __declspec / __forceinline; -fdelayed-template-parsing lets MSVC-style
# templates in SeMatrix.h parse.  -ffp-contract=off: no fused multiply-adds
# the reference's MSVC build would not make.
set -eu
HERE=$(cd "$(dirname "$0")" && pwd)
REF=${REF:-/root/reference}
CXX=${CXX:-/opt/rocm/llvm/bin/clang++}
if [ ! -f "$REF/SeMorton.h" ]; then
    echo "build_ref.sh: $REF not present (fixtures are generated in the build container only)" >&2
    exit 2
fi
mkdir -p "$HERE/_ref"
"$CXX" -std=c++17 -O2 -fPIC -shared -ffp-contract=off \
    -DWIN32 -fms-extensions -fdeclspec -fdelayed-template-parsing \
    -Wno-explicit-specialization-storage-class \
    -I"$REF" "$HERE/ref_headers.cpp" -o "$HERE/_ref/libref_headers.so"
echo "$HERE/_ref/libref_headers.so"
