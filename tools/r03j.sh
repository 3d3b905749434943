set -o pipefail
mkdir -p gpurun_out/r03j
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bench_legs.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r03j/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03j/pytest.log; exit 1; }
tail -2 gpurun_out/r03j/pytest.log
timeout -k 10 500 python bench.py > gpurun_out/r03j/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r03j/bench.log; exit 1; }
tail -1 gpurun_out/r03j/bench.log > gpurun_out/r03j/bench.json
python -c "import json; d=json.loads(open('gpurun_out/r03j/bench.json').read()); print(d['value'], d['parity']['cfg2_sha256_match'], json.dumps(d['rwkv_block'])[:600])"
