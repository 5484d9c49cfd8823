#!/bin/bash
# Diagnostics: libscvx_hip.so with csrc/scp_ipm.hip (or another source given as SRC=) rebuilt with extra -D
# flags, every other object taken from the in-tree build/ -> variants/<name>/libscvx_hip.so (SCVX_HIP_LIB=...).
# usage: [SRC=path.hip] tools/build_scp_variant.sh <name> [-DFLAG ...]
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/dynamic-programming-multiagent-trajectory-optimiziation_amd
SRC=${SRC:-$PKG/csrc/scp_ipm.hip}
OUT=$ROOT/variants/$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$ROOT/include -I$PKG/build -I$PKG/csrc -Wno-pass-failed "$@" -c $SRC -o $OUT/scp_ipm.o
objs=$(ls $PKG/build/*.o | grep -v '/scp_ipm.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libscvx_hip.so $objs $OUT/scp_ipm.o -L/opt/rocm/lib -lhiprtc -Wl,-rpath,/opt/rocm/lib
rm -f $OUT/scp_ipm.o
echo $OUT/libscvx_hip.so
