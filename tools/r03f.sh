set -o pipefail
mkdir -p gpurun_out/r03f
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_giant_shard.py tests/test_rwkv_block.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03f/pytest_shard.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/r03f/pytest_shard.log; exit 1; }
tail -2 gpurun_out/r03f/pytest_shard.log
timeout -k 10 300 python -u tools/giant_shard.py --D 2048 --mode baby --simulate-world 2 4 8 --reps 5 > gpurun_out/r03f/baby_sim.log 2>&1 || { echo "baby sim failed"; tail -20 gpurun_out/r03f/baby_sim.log; exit 1; }
tail -12 gpurun_out/r03f/baby_sim.log
timeout -k 10 300 python -u tools/giant_shard.py --D 2048 --mode giant --simulate-world 2 4 8 --reps 5 > gpurun_out/r03f/giant_sim.log 2>&1 || { echo "giant sim failed"; tail -20 gpurun_out/r03f/giant_sim.log; exit 1; }
tail -12 gpurun_out/r03f/giant_sim.log
bash tools/profile_round.sh && mv gpurun_out/prof gpurun_out/r03f/prof && cat gpurun_out/r03f/prof/bench.json | cut -c1-600
