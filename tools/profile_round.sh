#!/bin/bash
# GPU box: full bench line + rocprofv3 kernel stats + FETCH/WRITE PMC passes for the cfg2 bench.
# Writes gpurun_out/prof/{bench.json,stats/,fetch/,write/,traffic.json}.
set -e
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py > gpurun_out/prof/bench.log 2>&1
tail -n 1 gpurun_out/prof/bench.log > gpurun_out/prof/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-block --no-seal > gpurun_out/prof/stats.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-include-regex "k_modup|k_ks_ip|k_bsgs_inner|k_moddown|k_ks_intt|k_giant_sum" --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-block --no-seal > gpurun_out/prof/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-include-regex "k_modup|k_ks_ip|k_bsgs_inner|k_moddown|k_ks_intt|k_giant_sum" --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-block --no-seal > gpurun_out/prof/write.log 2>&1
python3 tools/pmc_traffic.py gpurun_out/prof/fetch/run_counter_collection.csv gpurun_out/prof/write/run_counter_collection.csv 7 gpurun_out/prof/traffic.json
timeout -k 10 300 rocprofv3 --kernel-include-regex "k_modup|k_ks_ip|k_bsgs_inner|k_moddown|k_ks_intt|k_giant_sum" --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/prof/valu -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-block --no-seal > gpurun_out/prof/valu.log 2>&1
python3 tools/pmc_valu.py gpurun_out/prof/valu/run_counter_collection.csv 7 gpurun_out/prof/valu.json
