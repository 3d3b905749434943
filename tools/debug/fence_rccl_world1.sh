#!/bin/bash
# The failure fence over RCCL (round 6): bench.py under torch.distributed.run at world 1 with the multi-rank step
# (FHESPEAR_BENCH_DIST=1, backend nccl = RCCL), a failure injected on rank 0 (a) in the block leg at stage 1 and
# (b) in the matvec leg's timed steps, where RCCL gathers are in flight on torch's stream.  Each case must abort
# the RCCL process group, re-create it, run the later legs on it and print the line; the process must exit 0.
#   tools/debug/fence_rccl_world1.sh OUT      (OUT under gpurun_out/)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
ARGS="--gpus 1 --steps 5 --warmup 1 --no-cpu-baseline --no-seal --sustain-s 0 --block-steps 1 --cfg5-blocks 2"
port=29541
for inj in "block/stage1@0" "matvec/step2@0"; do
    name=$(echo "$inj" | tr '/@' '__')
    env FHESPEAR_BENCH_DIST=1 FHESPEAR_BENCH_INJECT="$inj" timeout -k 10 400 python -m torch.distributed.run --nnodes 1 \
        --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py $ARGS > "$OUT/fence_$name.log" 2>&1
    rc=$?
    grep '^{' "$OUT/fence_$name.log" | tail -1 > "$OUT/fence_$name.json"
    echo "inject $inj: exit $rc"
    python3 -c "
import json, sys
d = json.load(open('$OUT/fence_$name.json'))
print(json.dumps({'value': d.get('value'), 'leg_faults': d.get('leg_faults'), 'block': (d.get('summary') or {}).get('rwkv_block'),
                  'cfg5': (d.get('summary') or {}).get('cfg5_chain')})[:1500])" || exit 1
    [ "$rc" = 0 ] || exit "$rc"
    port=$((port + 1))
done
echo "done $OUT"
