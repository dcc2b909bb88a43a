#!/bin/bash
# round 6 (t): one replay of the captured C2 step in launch order (start offsets, durations)
# — where the replay's wall time beyond its kernel sum goes — at K = 2500 and K = 10
set -o pipefail
O=gpurun_out/${TAG:-r06t}
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for spec in "2500 auto" "10 provable"; do
  set -- $spec
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sq$1 -o sq -- python3 $R/tools/probe_replay.py $1 20 $2 > $R/$O/replay$1.json 2> $R/$O/replay$1.err || { echo "trace $1 failed"; tail -20 $R/$O/replay$1.err; exit 1; }
  cat $R/$O/replay$1.json
  DB=$(ls /tmp/sq$1/*.db /tmp/sq$1/*/*.db 2>/dev/null | head -1)
  python3 $R/tools/rocpd_sequence.py $DB 160 > $R/$O/seq$1.txt && tail -1 $R/$O/seq$1.txt
  python3 $R/tools/rocpd_timeline.py $DB > $R/$O/timeline$1.json && cat $R/$O/timeline$1.json
done
