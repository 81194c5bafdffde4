#!/bin/bash
# Submit one gpurun call; resubmit ONLY when gpurun reports that the box was
# never prepared (status "transient": nothing ran, nothing charged).  A call
# that ran — whatever its exit status — is never repeated.
# usage: tools/gpurun_retry.sh <timeout_s> '<command>'
cd "$(dirname "$0")/.." || exit 2
t=$1; shift
for attempt in 1 2 3 4 5 6 7 8 9 10 11 12; do
    rm -f gpurun_out/*.log gpurun_out/session.log
    /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
    rc=$?
    st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
    if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
    echo "[retry] attempt $attempt: status=$st rc=$rc; waiting 120 s" >&2
    sleep 120
done
exit $rc
