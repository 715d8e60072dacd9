#!/bin/bash
# A GPU-box pytest pass over a selection: gpurun --timeout 900 -- bash tools/gpu_tests.sh TAG 'pytest -k expr' [files...]
set -eo pipefail
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 840 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
grep -E "PASSED|FAILED|SKIPPED|ERROR" "$OUT/pytest.log" | tail -60
tail -2 "$OUT/pytest.log"
