#!/bin/bash
# A/B of runtime knobs on the cfg2 bench: tools/ab_env.sh OUT "name VAR=v VAR=v" "name2 ..." ...
# Each variant is one bench.py run (no CPU baseline) under its own time limit; one JSON summary line
# per variant is appended to OUT.  Stops at the first failing run.
out=$1
shift
cfg=${AB_CONFIG:-cfg2}
steps=${AB_STEPS:-10}
for spec in "$@"; do
    name=${spec%% *}
    envs=${spec#"$name"}
    line=$(env $envs timeout -k 10 300 python3 bench.py --config "$cfg" --steps "$steps" --warmup 3 --no-cpu-baseline --no-block) || {
        echo "variant $name failed (rc $?)" >> "$out"
        exit 1
    }
    python3 - "$name" "$envs" "$line" >> "$out" <<'EOF'
import json, sys
name, envs, line = sys.argv[1], sys.argv[2].strip(), sys.argv[3]
d = json.loads(line.strip().splitlines()[-1])
k = {n: v["ms_per_step"] for n, v in d.get("kernels", {}).items()}
print(json.dumps({"variant": name, "env": envs, "value": d["value"], "ms_per_step": d["ms_per_step"], "kernels_ms": k}))
EOF
    tail -1 "$out"
done
