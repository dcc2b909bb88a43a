#!/bin/bash
# round 6 final tree (c): the C4 bench under rocprofv3 (kernel trace + PMC passes, so the
# bench line's roofline.traffic resolves) and the minibatch kernels' trace + PMC passes
set -o pipefail
timeout -k 10 1000 bash tools/profile_round.sh ${TAG:-r06fin}_c4 || { echo "profile_round failed"; exit 1; }
O=gpurun_out/${TAG:-r06fin}_mb bash tools/gpu/r06fin_mb_pmc.sh || { echo "mb pmc failed"; exit 1; }
