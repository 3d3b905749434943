#!/bin/bash
# GPU box: GPU test suite (optional), then bench variants for an A/B (no CPU baseline, SEAL or block
# legs).  Usage: tools/gpu_ab.sh OUTDIR [--tests] "name ENV=v ..." ...  Each variant writes
# OUTDIR/<name>.json (the bench line); stops at the first failure.
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$1" = "--tests" ]; then
    shift
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -15 "$OUT/pytest.log"; exit 1; }
    tail -1 "$OUT/pytest.log"
fi
for spec in "$@"; do
    name=${spec%% *}
    envs=${spec#"$name"}
    env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-block --no-seal > "$OUT/$name.log" 2>&1 || { echo "variant $name failed"; tail -5 "$OUT/$name.log"; exit 1; }
    tail -1 "$OUT/$name.log" > "$OUT/$name.json"
    python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['median_ms_per_step'], d['parity'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
done
