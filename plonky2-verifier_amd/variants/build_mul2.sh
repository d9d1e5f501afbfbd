#!/bin/bash
# Fault-isolation build: libp2v with the branch form of the general multiply
# (gl::mul_nc_dev_v<2>) instead of the branch-free one.  Loaded through P2V_LIB.
set -e
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -DP2V_GENERAL_MUL=2"
mkdir -p variants/build_mul2
for t in kernels vanish json_pack; do /opt/rocm/bin/hipcc $F -c -o variants/build_mul2/$t.o csrc/$t.hip & done
/opt/rocm/bin/hipcc $F -x hip -c -o variants/build_mul2/api.o csrc/api.cpp &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libp2v_mul2.so variants/build_mul2/*.o build/circuit.o
