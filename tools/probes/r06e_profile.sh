#!/bin/bash
# round 6 final-code profiles (tools/profile_round.sh r06e: kernel stats default + serial, FETCH /
# WRITE / VALU PMC passes, the same for the C3 circuit), then smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 bash tools/profile_round.sh r06e > gpurun_out/r06e_profile.log 2>&1 || { tail -20 gpurun_out/r06e_profile.log; exit 1; }
tail -2 gpurun_out/r06e_profile.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/prof_r06e/smoke.log 2>&1 || { tail -20 gpurun_out/prof_r06e/smoke.log; exit 1; }
tail -1 gpurun_out/prof_r06e/smoke.log
echo done
