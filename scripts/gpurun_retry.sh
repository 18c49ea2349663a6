#!/bin/bash
# gpurun with a bounded wait for a free box: re-submits ONLY when the call never ran (status
# "transient": no box / slot free, nothing charged); any call that ran -- passed or failed -- is
# final. Usage: scripts/gpurun_retry.sh TIMEOUT 'command'   (output: the gpurun client's)
T=$1; shift
for attempt in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(d.get('status'), d.get('rc'))" 2>/dev/null)
  case "$st" in
    "transient None") echo "[retry] no box (attempt $attempt), waiting 150 s"; sleep 150 ;;
    *) exit $rc ;;
  esac
done
exit 3
