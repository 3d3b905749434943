#!/bin/bash
# Run bench for a list of "LIB|ENV1=v ENV2=w" configurations (GPU box).
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  lib=${cfg%%|*}; envs=${cfg#*|}
  if [ "$lib" = default ]; then L=; else L=fhe-spear_amd/lib/variants/libfhespear_hip_$lib.so; fi
  env FHESPEAR_LIB=$L $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abm_$i.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/abm_$i.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
  i=$((i+1))
done
