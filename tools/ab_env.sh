#!/bin/bash
# A/B one environment variable on the cfg2 bench (GPU box): tools/ab_env.sh VAR v1 v2 ...
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  env $var=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abenv_$v.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/abenv_$v.log').read().strip().splitlines()[-1]); print('$var=$v', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
done
