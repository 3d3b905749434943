set -o pipefail
export FHESPEAR_PARITY_RNG=1   # deterministic encryption randomness: the digests are comparable across runs
mkdir -p gpurun_out/r04y
A="--N 32768 --L0 36 --P 3 --D 2048 --F 4096 --blocks 2"
FFN_DIGEST=1 timeout -k 10 300 python tools/ffn_block.py $A > gpurun_out/r04y/ffn_world1.log 2>&1 &&
FHESPEAR_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/ffn_block.py $A --dist --backend gloo --shard giant > gpurun_out/r04y/ffn_world2_giant.log 2>&1 &&
FHESPEAR_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29562 tools/ffn_block.py $A --dist --backend gloo --shard grid --rb 2 > gpurun_out/r04y/ffn_world4_grid.log 2>&1
rc=$?
grep -h "ct_sha256" gpurun_out/r04y/*.log
exit $rc
