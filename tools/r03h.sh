set -o pipefail
mkdir -p gpurun_out/r03h
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_giant_shard.py tests/test_rwkv_block.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03h/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03h/pytest.log; exit 1; }
tail -2 gpurun_out/r03h/pytest.log
TR="python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 400 $TR --master-port 29611 tools/giant_shard.py --D 2048 --mode giant --reps 5 --simulate-grid 1x1 1x2 2x1 1x4 2x2 4x1 1x8 2x4 4x2 8x1 1x3 3x1 > gpurun_out/r03h/grid_sim.log 2>&1 || { echo "grid sim failed"; tail -20 gpurun_out/r03h/grid_sim.log; exit 1; }
grep -E "sharded|grid" gpurun_out/r03h/grid_sim.log
