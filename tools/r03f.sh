set -o pipefail
mkdir -p gpurun_out/r03f
export TMPDIR=/tmp
TR="python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 $TR --master-port 29611 tools/giant_shard.py --D 2048 --mode baby --simulate-world 2 4 8 --reps 5 > gpurun_out/r03f/baby_sim.log 2>&1 || { echo "baby sim failed"; tail -20 gpurun_out/r03f/baby_sim.log; exit 1; }
tail -12 gpurun_out/r03f/baby_sim.log
timeout -k 10 300 $TR --master-port 29613 tools/giant_shard.py --D 2048 --mode giant --simulate-world 2 4 8 --reps 5 > gpurun_out/r03f/giant_sim.log 2>&1 || { echo "giant sim failed"; tail -20 gpurun_out/r03f/giant_sim.log; exit 1; }
tail -12 gpurun_out/r03f/giant_sim.log
bash tools/profile_round.sh && rm -rf gpurun_out/r03f/prof && mv gpurun_out/prof gpurun_out/r03f/prof && cut -c1-600 gpurun_out/r03f/prof/bench.json
