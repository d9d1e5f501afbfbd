#!/bin/bash
# AddressSanitizer + UBSan over libp2v's host readers (tools/asan/host_fuzz.cpp); CPU only.
set -e
cd "$(dirname "$0")"
OUT=${OUT:-/tmp/p2v_asan}
mkdir -p $OUT
g++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined \
    -o $OUT/host_fuzz host_fuzz.cpp ../../plonky2-verifier_amd/csrc/circuit.cpp
python3 - "$OUT" <<'PY'
import sys, os
sys.path.insert(0, os.path.abspath("../../tests")); sys.path.insert(0, os.path.abspath("../../plonky2-verifier_amd"))
from support import gen_circuit, proof_bytes
import p2v
out = sys.argv[1]
gc = gen_circuit(6, 4, 1, 1, 28, 8)
pr = gc.proof(1, 1)
for name, data in (("common.json", gc.common), ("vkey.json", gc.vkey), ("proof.json", pr), ("proof.bin", proof_bytes(pr)),
                   ("circuit.words", p2v.circuit_words(gc.common, gc.vkey).tobytes()), ("proof.words", p2v.proof_words(pr).tobytes())):
    open(os.path.join(out, name), "wb").write(data)
PY
ASAN_OPTIONS=detect_leaks=1 $OUT/host_fuzz $OUT/common.json $OUT/vkey.json $OUT/proof.json $OUT/proof.bin $OUT/circuit.words $OUT/proof.words ${ITERS:-1500}
