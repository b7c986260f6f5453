#!/bin/bash
# TBE kernel probe on the GPU box: TBE parity tests, then tools/tbe_bwd_bench.py under a
# rocprofv3 kernel trace.  Usage: bash tools/tbe_probe.sh <tag>
set -o pipefail
TAG=${1:-tbe}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -k tbe -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o kt \
  -- python3 "$ROOT/tools/tbe_bwd_bench.py" > "$OUT/out.txt" 2> "$OUT/prof.err" || exit $?
grep "^T=" "$OUT/out.txt"
