set -o pipefail
mkdir -p gpurun_out/r04seal
V=fhe-spear_amd/lib/variants/libfhespear_hip_prev.so
B="--config cfg2seal --steps 10 --warmup 2 --no-cpu-baseline --no-block --no-seal"
timeout -k 10 300 python3 bench.py $B > gpurun_out/r04seal/new.log 2>&1 &&
FHESPEAR_LIB=$V timeout -k 10 300 python3 bench.py $B > gpurun_out/r04seal/prev.log 2>&1 &&
timeout -k 10 300 python3 bench.py $B > gpurun_out/r04seal/new2.log 2>&1 &&
FHESPEAR_LIB=$V timeout -k 10 300 python3 bench.py $B > gpurun_out/r04seal/prev2.log 2>&1 &&
for f in new prev new2 prev2; do grep '^{' gpurun_out/r04seal/$f.log | tail -1 > gpurun_out/r04seal/$f.json; python3 tools/show_bench.py gpurun_out/r04seal/$f.json $f; done
