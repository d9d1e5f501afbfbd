#!/bin/bash
# from-host verification (p2v_verify_batch_devices, pinned and pageable input) by chunk size, at
# 16 384 and 65 536 proofs per call: does a smaller chunk than auto (about n/8) shorten the
# pipeline's fill and drain
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zg
mkdir -p $O
P2V_PROBE_CHUNKS=0,512,1024,2048,4096 timeout -k 10 300 python3 tools/host_batch_probe.py 16384 > $O/n16k.txt 2>&1 || { tail -5 $O/n16k.txt; exit 1; }
cat $O/n16k.txt
P2V_PROBE_CHUNKS=0,1024,2048,4096 timeout -k 10 300 python3 tools/host_batch_probe.py 65536 > $O/n64k.txt 2>&1 || { tail -5 $O/n64k.txt; exit 1; }
cat $O/n64k.txt
echo done
