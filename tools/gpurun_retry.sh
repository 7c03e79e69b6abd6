#!/bin/bash
# Run a gpurun call; retry ONLY when the infrastructure reports a transient
# failure before anything ran (box not prepared / no slot). GPU-step failures
# are never retried.
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" = "transient" ] || [ $rc -eq 3 ]; then
    echo "[gpurun_retry] transient ($st rc=$rc); waiting before attempt $((attempt+1))"
    sleep $((20 * attempt))
    continue
  fi
  exit $rc
done
exit $rc
