# cfg5 chain with a bootstrap over ranks at full ring size (gloo, ranks sharing one GPU): the one-rank
# chain and the 2-rank chain (giant groups of the FFN matvecs and of the bootstrap's linear transforms
# sharded) must end on the same ciphertext digest.  Timings meaningless (shared GPU, host-staged exchange).
set -o pipefail
export FHESPEAR_PARITY_RNG=1
mkdir -p gpurun_out/r04boot
A="--N 32768 --L0 36 --P 3 --D 2048 --F 4096 --blocks 12 --bootstrap"
FFN_DIGEST=1 timeout -k 10 500 python tools/ffn_block.py $A > gpurun_out/r04boot/ffn_boot_world1.log 2>&1 &&
FHESPEAR_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29563 tools/ffn_block.py $A --dist --backend gloo --shard giant > gpurun_out/r04boot/ffn_boot_world2_giant.log 2>&1
rc=$?
grep -h "ct_sha256" gpurun_out/r04boot/*.log
exit $rc
