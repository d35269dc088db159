#!/bin/bash
# round 3 (final evidence after the halo swizzle): traffic records of the full model and configs
# 2 / 3, kernel trace, PMC, bench lines
set -o pipefail
bash tools/run_r03_evidence.sh r03x || exit 1
bash tools/run_r03r.sh || exit 2
