#!/bin/bash
# GPU box: A/B of ModUp's 4 x 2 XCD map (lib variant m42) -- bench legs, then a FETCH_SIZE pass of k_modup
# for each library.
set -o pipefail
OUT=gpurun_out/r03s2_m42
V=fhe-spear_amd/lib/variants/libfhespear_hip_m42.so
bash tools/gpu_ab.sh r03s2_m42 "m42 FHESPEAR_LIB=$V" "base FHESPEAR_LIB=" "m42b FHESPEAR_LIB=$V" "baseb FHESPEAR_LIB=" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in m42 base; do
  if [ $v = m42 ]; then export FHESPEAR_LIB=$V; else unset FHESPEAR_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-include-regex "k_modup" --pmc FETCH_SIZE -d $OUT/fetch_$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-block --no-seal > $OUT/fetch_$v.log 2>&1 || { echo "fetch $v failed"; exit 1; }
  python3 -c "
import csv
r=[x for x in csv.DictReader(open('$OUT/fetch_$v/run_counter_collection.csv')) if 'k_modup' in x['Kernel_Name']]
tot=sum(float(x['Counter_Value']) for x in r)
print('$v', 'k_modup FETCH_SIZE x2 per step (7 steps):', round(tot*2*1024/7/1e9,3), 'GB over', len(r), 'dispatches')"
done
