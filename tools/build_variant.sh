#!/bin/bash
# Diagnostics: build libscvx_hip.so with extra -D flags into variants/<name>/ (load it with SCVX_HIP_LIB=...).
# usage: tools/build_variant.sh <name> [-DFLAG ...]
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/dynamic-programming-multiagent-trajectory-optimiziation_amd
OUT=$ROOT/variants/$NAME
mkdir -p $OUT
make -s -C $PKG build/foh_body.inc build/qp_ipm.inc build/scp_kernel.inc build/wave_ops.inc build/scvx_hip_h.inc build/intersample_body.inc   # the hipRTC header texts (embedded in the library)
# QUAD_FLAGS: extra flags for the n = 12 translation unit only (qp_inst_quad.hip), as the Makefile's per-file flags
ls $PKG/csrc/*.hip | xargs -P 8 -I{} sh -c "case {} in *qp_inst_quad.hip) X='$QUAD_FLAGS';; *) X='';; esac; /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$ROOT/include -I$PKG/build -Wno-pass-failed $* \$X -c {} -o $OUT/\$(basename {} .hip).o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libscvx_hip.so $OUT/*.o -L/opt/rocm/lib -lhiprtc -Wl,-rpath,/opt/rocm/lib
rm -f $OUT/*.o
echo $OUT/libscvx_hip.so
