#!/bin/bash
# round 6: the row form's merged partial blocks with their chain rows on the idle lanes 12-14
# (lposeidon.h pblock_par, P2V_ROW_PAR=1) with the split uniform S-box (P2V_ROW_SBOX2=1) against =0: KAT, host
# mismatches and dependent-chain latency (tools/microbench/perm_bench.hip mode 10), alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06u
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    for a in "1 2000" "64 500" "1024 200"; do
      echo "ROW_SBOX2=$v rows/perms $a" >> $O/row_par.txt
      timeout -k 10 60 tools/microbench/bin/perm_bench_ls$v $a 10 >> $O/row_par.txt || { cat $O/row_par.txt; exit 1; }
    done
  done
done
cat $O/row_par.txt
echo done
