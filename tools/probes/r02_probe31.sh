#!/bin/bash
# two checks in one box: the N>1 launcher path (probe 29), then k_merkle at 6 waves (probe 30)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
bash tools/r02_probe29.sh
bash tools/r02_probe30.sh
echo done
