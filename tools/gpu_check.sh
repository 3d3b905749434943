#!/bin/bash
# GPU box: the round-end checks in one call -- GPU test suite, smoke(), bench line, rocprofv3 kernel
# stats of the bench.  Usage: tools/gpu_check.sh <outdir under gpurun_out> [pytest args...]
set -o pipefail
OUT=gpurun_out/${1:-check}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -5 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-block --no-seal > "$OUT/stats.log" 2>&1 || { echo "rocprof failed"; tail -5 "$OUT/stats.log"; exit 1; }
echo done
