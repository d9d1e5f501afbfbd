#!/bin/bash
# Measurement / isolation builds of libp2v with extra compile flags, loaded through P2V_LIB:
#   variants/build.sh <name> "<flags>"   ->   variants/libp2v_<name>.so
#   pm:    -DP2V_PROOF_MAJOR=1   (kernels read the proof-major batch in place, no k_transpose)
set -e
cd "$(dirname "$0")/.."
NAME=$1; EXTRA=$2
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Werror=inline-asm $EXTRA"
mkdir -p variants/build_$NAME
for t in kernels vanish vanish_poseidon json_pack util; do /opt/rocm/bin/hipcc $F -c -o variants/build_$NAME/$t.o csrc/$t.hip & done
/opt/rocm/bin/hipcc $F -x hip -c -o variants/build_$NAME/api.o csrc/api.cpp &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libp2v_$NAME.so variants/build_$NAME/*.o build/circuit.o build/version.o
