#!/bin/bash
# Local helper (this container, not the GPU box): run one gpurun call, and when the pool had no free box
# (status "transient": nothing ran, nothing charged) try again after a pause, at most 12 times.  A call
# that ran -- passed, failed or timed out -- is never repeated.
#   tools/gpurun_wait.sh LOG TIMEOUT 'command'
log=$1
lim=$2
case "$log" in -*) echo "gpurun_wait.sh: LOG must come first (got '$log')" >&2; exit 2;; esac
case "$lim" in ''|*[!0-9]*) echo "gpurun_wait.sh: TIMEOUT must be a number of seconds (got '$lim')" >&2; exit 2;; esac
shift 2
for i in $(seq 1 12); do
    /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$log" 2>&1
    rc=$?
    if grep -q "status=transient" "$log" && ! grep -q "run [1-9][0-9.]*s of limit" "$log"; then
        echo "attempt $i: no box, waiting" >> "$log.attempts"
        sleep 150
        continue
    fi
    exit $rc
done
exit 3
