#!/bin/bash
# gpurun a command, trying again only while the pool has no free slot or box (status "transient": nothing ran,
# nothing was charged); any other outcome -- success, failure, timeout -- ends it.  OUT=<log> TIMEOUT=<s>.
#   OUT=/tmp/x.out TIMEOUT=1200 bash tools/gpurun_wait.sh '<command>'
for try in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout ${TIMEOUT:-1200} -- "$1" > $OUT 2>&1
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  [ "$st" != "transient" ] && exit 0
  echo "[gpurun_wait] try $try: no slot, waiting" >> $OUT.tries
  sleep 150
done
