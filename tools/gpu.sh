#!/bin/bash
# Submit one gpurun call. If the pool reports an infrastructure-side "transient"
# failure (the box never ran the command, nothing charged), wait and resubmit,
# at most 3 times. A command that actually ran is never resubmitted.
cd "$(dirname "$0")/.."
for attempt in 1 2 3; do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  echo "[gpu.sh] infrastructure transient (attempt $attempt), waiting 60 s" >&2
  sleep 60
done
exit $rc
