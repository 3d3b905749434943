set -o pipefail
V="FHESPEAR_LIB=$GRAFT_REPO_ROOT/fhe-spear_amd/lib/variants/libfhespear_hip_modupnt.so"
bash tools/gpu_ab.sh r03l "base1" "nt1 $V" "base2" "nt2 $V" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in base nt; do
  if [ $n = nt ]; then export FHESPEAR_LIB=$GRAFT_REPO_ROOT/fhe-spear_amd/lib/variants/libfhespear_hip_modupnt.so; fi
  timeout -k 10 300 rocprofv3 --kernel-include-regex "k_modup" --pmc FETCH_SIZE -d gpurun_out/r03l/f_$n -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-block --no-seal > gpurun_out/r03l/f_$n.log 2>&1 || exit 1
  python3 -c "
import csv; t=sum(float(r['Counter_Value']) for r in csv.DictReader(open('gpurun_out/r03l/f_$n/run_counter_collection.csv')) if r['Counter_Name']=='FETCH_SIZE')
print('$n k_modup FETCH x2 GB/step', 2*t*1024/7/1e9)"
done
