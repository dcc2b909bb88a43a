#!/bin/bash
# round 4 final tree (z2b): the C4 rocprof record (kernel trace + PMC passes)
set -o pipefail
timeout -k 10 1100 bash tools/profile_round.sh r04z_c4 || exit 1
