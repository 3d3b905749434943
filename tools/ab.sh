#!/bin/bash
# A/B the default library against lib/variants/*.so on the cfg2 bench (GPU box).
mkdir -p gpurun_out
for v in default "$@"; do
  if [ "$v" = default ]; then L=; else L=fhe-spear_amd/lib/variants/libfhespear_hip_$v.so; fi
  FHESPEAR_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-block > gpurun_out/ab_$v.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
done
