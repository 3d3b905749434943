set -o pipefail
bash tools/profile_round.sh || { echo "profile failed"; tail -5 gpurun_out/prof/*.log; exit 1; }
rm -rf gpurun_out/r03s2q && mkdir -p gpurun_out/r03s2q && mv gpurun_out/prof gpurun_out/r03s2q/prof
python3 -c "import json; d=json.loads(open('gpurun_out/r03s2q/prof/bench.json').read()); print(d['value'], d['parity']['cfg2_sha256_match'], d['roofline']['traffic'], d['rwkv_block'].get('sec_per_block'), d['rwkv_block'].get('parity',{}).get('r_projection_limbs_match_cpu_port'))"
