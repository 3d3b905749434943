set -o pipefail
mkdir -p gpurun_out/r03g
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_golden_replay.py tests/test_giant_shard.py tests/test_rwkv_block.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03g/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03g/pytest.log; exit 1; }
tail -2 gpurun_out/r03g/pytest.log
TR="python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 $TR --master-port 29611 tools/giant_shard.py --D 2048 --mode baby --simulate-world 2 4 8 --reps 5 > gpurun_out/r03g/baby_sim.log 2>&1 || { echo "baby sim failed"; tail -20 gpurun_out/r03g/baby_sim.log; exit 1; }
grep -E "sharded|per-rank" gpurun_out/r03g/baby_sim.log
