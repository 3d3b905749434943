#!/bin/bash
# GPU box: rehearse the driver's N > 1 bench runs with 2 ranks sharing one GPU (gloo, host-staged
# exchange; timings meaningless): the default matvec line and its block leg.
set -o pipefail
OUT=gpurun_out/${1:-rehearsal}
mkdir -p "$OUT"
export TMPDIR=/tmp FHESPEAR_DIST_BACKEND=gloo FHESPEAR_DEVICE=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 > "$OUT/bench_n2.log" 2>&1 || { echo "n2 failed"; tail -20 "$OUT/bench_n2.log"; exit 1; }
grep '^{' "$OUT/bench_n2.log" | tail -1 > "$OUT/bench_n2.json"
python3 -c "import json; d=json.load(open('$OUT/bench_n2.json')); print(d['n_gpus'], d['value'], d['unit'], d['rwkv_block'].get('sec_per_block'), d['rwkv_block'].get('max_abs_err_vs_plaintext_block'), d['config']['parallelism'])"
