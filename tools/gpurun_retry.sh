#!/bin/bash
# Submit one gpurun call; resubmit only when the infrastructure reports a transient failure
# (the box was lost while being prepared / no slot: nothing of the command ran). A command that
# ran and failed is never resubmitted.
# usage: tools/gpurun_retry.sh <limit-seconds> <command...>
lim=$1; shift
case "$lim" in ""|*[!0-9]*) echo "usage: $0 <limit-seconds> <command...>"; exit 2 ;; esac
for i in 1 2 3 4 5 6 7 8; do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$rc" = 3 ] || [ "$st" = "transient" ]; then echo "[retry] transient ($rc/$st), attempt $i"; sleep 60; continue; fi
  exit $rc
done
exit 3
