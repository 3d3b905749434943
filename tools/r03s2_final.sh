#!/bin/bash
# GPU box: round-3 session-2 confirmation -- GPU suite, smoke, bench line, rocprofv3 stats
# (tools/gpu_check.sh), then the block leg's client-side costs (tools/debug/block_overhead.py).
set -o pipefail
bash tools/gpu_check.sh ${1:-r03s2_final} || exit 1
timeout -k 10 300 python tools/debug/block_overhead.py > gpurun_out/${1:-r03s2_final}/block_overhead.log 2>&1 || { echo "block_overhead failed"; tail -5 gpurun_out/${1:-r03s2_final}/block_overhead.log; exit 1; }
tail -1 gpurun_out/${1:-r03s2_final}/block_overhead.log
