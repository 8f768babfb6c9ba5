#!/bin/bash
# round 4 call 11 = call 10 (4-wave pgemm) then call 9 (EP8 Mixtral shapes, mixed-step A/B)
set -o pipefail
bash scripts/r4_gpu_10.sh || exit $?
bash scripts/r4_gpu_9.sh
