#!/bin/bash
# GPU box: one parametrised script for every gpurun call (replaces the per-round one-offs).
#   tools/gpu.sh OUT STEP [STEP ...]      (OUT is a directory under gpurun_out/)
# Steps, run in order, each under its own time limit; the script stops at the first failure:
#   tests[=pytest args]     GPU suite (default: all of tests/ -m gpu; args may quote, e.g. -k 'a or b')
#   smoke                   __graft_entry__.smoke()                              -> OUT/smoke.log
#   bench[=bench args]      one bench line (default: the driver's default line)  -> OUT/bench.json
#   ab=NAME[:ENV=v,ENV=v]   cfg2 matvec-only bench under extra environment (AB_ARGS: more bench args) -> OUT/ab_NAME.json
#   abx=NAME[:ENV=v,ENV=v]  bench with AB_ARGS only (no matvec-only flags)           -> OUT/ab_NAME.json
#   trace[=bench args]      rocprofv3 --kernel-trace --stats of a matvec-only bench -> OUT/trace_<config>/,
#                           OUT/rocprof_summary_<config>.json (tools/rocprof_summary.py: per-dispatch
#                           steady state of the timed steps)
#   pmc[=config]            FETCH_SIZE, WRITE_SIZE and VALU counter passes (one rocprofv3 run each)
#                           -> OUT/pmc_traffic_<config>.json, OUT/pmc_valu_<config>.json
#   stall[=config]          wave-cycle attribution passes (SQ_WAIT_*, LDS, instruction mix) -> OUT/pmc_stall_<config>.json
#   rehearse=N[:bench args] N ranks sharing this one GPU (gloo, host-staged exchange, 2 GiB allocation cache per rank; timings
#                           meaningless): bench.py --gpus N self-launches them -> OUT/rehearse_nN.json
#   dist1[=NAME[:ENV=v,..]] matvec bench at world 1 under torchrun with the RCCL gather step -> OUT/NAME.json
#   py=SCRIPT[:args]        python SCRIPT args                                  -> OUT/py_<name>.log
#   exe=BINARY              a prebuilt microbenchmark                          -> OUT/exe_<name>.log
#   pstall=SCRIPT[:args]    the stall passes over a script's kernels (KREGEX)       -> OUT/pmc_stall_<name>.json
#   ptrace=SCRIPT[:args]    the same under rocprofv3 --kernel-trace --stats      -> OUT/ptrace_<name>/
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
MV="--no-cpu-baseline --no-block --no-seal --no-cfg5"
PMV="$MV --sustain-s 0"   # counter passes: the timed steps only (no sustained run under the profiler)
fail() { echo "step $1 failed"; tail -20 "$2"; exit 1; }
for step in "$@"; do
    name=${step%%=*}
    arg=""
    [ "$name" != "$step" ] && arg=${step#*=}
    case "$name" in
    tests)
        # eval: quotes inside the step's argument group (e.g. -k 'a or b')
        eval "timeout -k 10 1500 python -u -m pytest -m gpu -x -v --durations=25 --timeout 300 --timeout-method thread ${arg:-tests}" \
            > "$OUT/pytest.log" 2>&1 || fail tests "$OUT/pytest.log"
        tail -1 "$OUT/pytest.log" ;;
    smoke)
        timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail smoke "$OUT/smoke.log"
        tail -1 "$OUT/smoke.log" ;;
    bench)
        timeout -k 10 600 python bench.py $arg > "$OUT/bench.log" 2>&1 || fail bench "$OUT/bench.log"
        grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
        python3 tools/show_bench.py "$OUT/bench.json" ;;
    ab)
        v=${arg%%:*}
        envs=""
        [ "$v" != "$arg" ] && envs=$(echo "${arg#*:}" | tr ',' ' ')
        env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 $MV $AB_ARGS > "$OUT/ab_$v.log" 2>&1 || fail "ab $v" "$OUT/ab_$v.log"
        grep '^{' "$OUT/ab_$v.log" | tail -1 > "$OUT/ab_$v.json"
        python3 tools/show_bench.py "$OUT/ab_$v.json" "$v" ;;
    abx)
        # as ab, but the bench arguments are AB_ARGS alone (no matvec-only flags): e.g. the cfg5 leg
        v=${arg%%:*}
        envs=""
        [ "$v" != "$arg" ] && envs=$(echo "${arg#*:}" | tr ',' ' ')
        env $envs timeout -k 10 600 python3 bench.py $AB_ARGS > "$OUT/ab_$v.log" 2>&1 || fail "abx $v" "$OUT/ab_$v.log"
        grep '^{' "$OUT/ab_$v.log" | tail -1 > "$OUT/ab_$v.json"
        python3 tools/show_bench.py "$OUT/ab_$v.json" "$v" ;;
    trace)
        cfg=$(echo "$arg" | sed -n 's/.*--config \([a-z0-9_]*\).*/\1/p')
        cfg=${cfg:-cfg2}
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$cfg" -o run --output-format csv \
            -- python3 bench.py --steps 20 --warmup 3 $MV $arg > "$OUT/trace_$cfg.log" 2>&1 || fail trace "$OUT/trace_$cfg.log"
        grep '^{' "$OUT/trace_$cfg.log" | tail -1 > "$OUT/trace_bench_$cfg.json"
        python3 tools/rocprof_summary.py "$OUT/trace_$cfg" "$OUT/trace_bench_$cfg.json" "$OUT/rocprof_summary_$cfg.json" || exit 1
        # keep rocprofv3's --stats summary, drop the per-dispatch trace (the sustained run makes it large)
        find "$OUT/trace_$cfg" -name '*kernel_trace.csv' -delete ;;
    pmc)
        cfg=${arg:-cfg2}
        K="k_modup|k_ks_ip|k_bsgs_inner|k_moddown|k_ks_intt|k_giant_sum|k_centered"
        for c in "fetch FETCH_SIZE" "write WRITE_SIZE" "valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
            d=${c%% *}
            timeout -s KILL 240 rocprofv3 --kernel-include-regex "$K" --pmc ${c#* } -d "$OUT/pmc_$d" -o run \
                --output-format csv -- python3 bench.py --config "$cfg" --steps 3 --warmup 1 $PMV > "$OUT/pmc_$d.log" 2>&1 \
                || fail "pmc $d" "$OUT/pmc_$d.log"
        done
        python3 tools/pmc_traffic.py "$OUT/pmc_fetch/run_counter_collection.csv" \
            "$OUT/pmc_write/run_counter_collection.csv" 7 "$OUT/pmc_traffic_$cfg.json" || exit 1
        python3 tools/pmc_valu.py "$OUT/pmc_valu/run_counter_collection.csv" 7 "$OUT/pmc_valu_$cfg.json" || exit 1
        rm -rf "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_valu" ;;
    stall)
        # where k_modup_h's / k_bsgs_inner's wave cycles go (tools/pmc_stall.py): the counter list, then two SQ
        # passes of 8 counters (+ GRBM) each, one rocprofv3 run per pass
        cfg=${arg:-cfg2}
        timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || fail "counter list" "$OUT/counters_list.txt"
        K="k_modup|k_bsgs_inner|k_ks_ip"
        i=0
        for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
                 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
            i=$((i + 1))
            timeout -s KILL 240 rocprofv3 --kernel-include-regex "$K" --pmc $c -d "$OUT/stall_$i" -o run \
                --output-format csv -- python3 bench.py --config "$cfg" --steps 3 --warmup 1 $PMV > "$OUT/stall_$i.log" 2>&1 \
                || fail "stall pass $i" "$OUT/stall_$i.log"
        done
        python3 tools/pmc_stall.py "$OUT/pmc_stall_$cfg.json" 7 "$OUT/stall_1/run_counter_collection.csv" \
            "$OUT/stall_2/run_counter_collection.csv" || exit 1
        rm -rf "$OUT/stall_1" "$OUT/stall_2" ;;   # raw counter dumps: gpurun copies back at most 64 MiB
    pstall)
        # the same two SQ passes over a script's kernels (KREGEX: which kernels) -> OUT/pmc_stall_<script>.json
        s=${arg%%:*}
        a=""
        [ "$s" != "$arg" ] && a=${arg#*:}
        b=$(basename "$s" .py)
        K=${KREGEX:-k_ntt_fwd_from_dbl|k_modup_h}
        i=0
        for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
                 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
            i=$((i + 1))
            timeout -s KILL 400 rocprofv3 --kernel-include-regex "$K" --pmc $c -d "$OUT/pstall_$i" -o run \
                --output-format csv -- python3 -u "$s" $a > "$OUT/pstall_$i.log" 2>&1 || fail "pstall pass $i" "$OUT/pstall_$i.log"
        done
        python3 tools/pmc_stall.py "$OUT/pmc_stall_$b.json" 1 "$OUT/pstall_1/run_counter_collection.csv" \
            "$OUT/pstall_2/run_counter_collection.csv" || exit 1 ;;
    dist1)
        # the multi-rank step (RCCL gather, device-side stream ordering) at world 1 on this one GPU
        v=${arg%%:*}
        v=${v:-dist1}
        envs=""
        [ "$v" != "$arg" ] && [ -n "$arg" ] && envs=$(echo "${arg#*:}" | tr ',' ' ')
        env FHESPEAR_BENCH_DIST=1 $envs timeout -k 10 400 python -m torch.distributed.run --nnodes 1 \
            --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 3 $MV \
            > "$OUT/$v.log" 2>&1 || fail dist1 "$OUT/$v.log"
        grep '^{' "$OUT/$v.log" | tail -1 > "$OUT/$v.json"
        python3 tools/show_bench.py "$OUT/$v.json" "$v" ;;
    rehearse)
        n=${arg%%:*}
        a=""
        [ "$n" != "$arg" ] && a=${arg#*:}
        FHESPEAR_DIST_BACKEND=gloo FHESPEAR_DEVICE=0 FHESPEAR_CACHE_BYTES=${FHESPEAR_CACHE_BYTES:-2147483648} timeout -k 10 1100 python bench.py --gpus "$n" $a \
            > "$OUT/rehearse_n$n.log" 2>&1 || fail "rehearse $n" "$OUT/rehearse_n$n.log"
        grep '^{' "$OUT/rehearse_n$n.log" | tail -1 > "$OUT/rehearse_n$n.json"
        python3 tools/show_bench.py "$OUT/rehearse_n$n.json" ;;
    ptrace)
        s=${arg%%:*}
        a=""
        [ "$s" != "$arg" ] && a=${arg#*:}
        b=$(basename "$s" .py)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/ptrace_$b" -o run --output-format csv \
            -- python3 -u "$s" $a > "$OUT/ptrace_$b.log" 2>&1 || fail "ptrace $s" "$OUT/ptrace_$b.log" ;;
    exe)
        # a prebuilt microbenchmark binary (tools/microbench/*, built here with hipcc)
        b=$(basename "$arg")
        timeout -k 10 180 "$arg" > "$OUT/exe_$b.log" 2>&1 || fail "exe $arg" "$OUT/exe_$b.log"
        tail -4 "$OUT/exe_$b.log" ;;
    py)
        s=${arg%%:*}
        a=""
        [ "$s" != "$arg" ] && a=${arg#*:}
        b=$(basename "$s" .py)
        timeout -k 10 900 python -u "$s" $a > "$OUT/py_$b.log" 2>&1 || fail "py $s" "$OUT/py_$b.log"
        tail -3 "$OUT/py_$b.log" ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
echo "done $OUT"
