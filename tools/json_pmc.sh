#!/bin/bash
# PMC passes over tools/json_ingest_probe.py (k_json_pack): instruction mix, occupancy, HBM bytes
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/jpmc
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-include-regex k_json_pack --output-format csv -d $OUT/sq -o run -- python3 tools/json_ingest_probe.py 4096 > $OUT/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_json_pack --output-format csv -d $OUT/fetch -o run -- python3 tools/json_ingest_probe.py 4096 > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-include-regex k_json_pack --output-format csv -d $OUT/write -o run -- python3 tools/json_ingest_probe.py 4096 > $OUT/write.log 2>&1
echo done
