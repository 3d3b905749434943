#!/bin/bash
# GPU box: end-of-session confirmation -- GPU suite and smoke, then the profile round (bench line,
# rocprofv3 stats, FETCH/WRITE and VALU PMC passes for the hash-matched traffic record).
set -o pipefail
OUT=gpurun_out/${1:-r03s2_end}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -5 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
bash tools/profile_round.sh || { echo "profile failed"; tail -5 gpurun_out/prof/*.log; exit 1; }
mv gpurun_out/prof "$OUT/prof"
python3 -c "import json; d=json.loads(open('$OUT/prof/bench.json').read()); print(d['value'], d['parity']['cfg2_sha256_match'], d['roofline']['traffic'], d['rwkv_block'].get('sec_per_block'), d['rwkv_block'].get('parity',{}).get('r_projection_limbs_match_cpu_port'))"
