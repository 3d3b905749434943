#!/bin/bash
# A/B of the compact-diagonal Hadamard variants (round 6): each library variant under
# fhe-spear_amd/lib/variants/ first passes the compact-vs-dense limb test, then the bench's block and cfg5 legs
# run for every variant in turn, twice, interleaved (placement and clocks drift between processes).
#   tools/debug/ab_compact.sh OUT VARIANT [VARIANT ...]      (OUT under gpurun_out/)
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
lib() { echo "$PWD/fhe-spear_amd/lib/variants/libfhespear_hip_$1.so"; }
for v in "$@"; do
    FHESPEAR_LIB=$(lib "$v") timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
        --timeout-method thread -k "compact or periodic" > "$OUT/test_$v.log" 2>&1 || { tail -30 "$OUT/test_$v.log"; exit 1; }
    echo "$v: $(tail -1 "$OUT/test_$v.log")"
done
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-seal --sustain-s 0"
for rep in 1 2; do
    for v in "$@"; do
        FHESPEAR_LIB=$(lib "$v") timeout -k 10 300 python bench.py $ARGS > "$OUT/bench_${v}_$rep.log" 2>&1 || { tail -30 "$OUT/bench_${v}_$rep.log"; exit 1; }
        grep '^{' "$OUT/bench_${v}_$rep.log" | tail -1 > "$OUT/bench_${v}_$rep.json"
        python3 -c "
import json; d = json.load(open('$OUT/bench_${v}_$rep.json'))
b, c = d.get('rwkv_block') or {}, d.get('cfg5_chain') or {}
print('$v rep $rep: block', b.get('sec_per_block'), 'server_ms', b.get('server_ms'), '| cfg5', c.get('total_seconds'),
      c.get('sec_per_block'), 'digest', (c.get('parity') or {}).get('matches_one_rank'), '| matvec', d.get('value'))" || exit 1
    done
done
echo "done $OUT"
