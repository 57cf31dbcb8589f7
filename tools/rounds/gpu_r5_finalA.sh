#!/bin/bash
# Round 5 closing pass A: every GPU test + smoke(), then every profile shape of this build (gpu_r5_profiles.sh ->
# gpurun_out/r5prof/, committed as profiles/r05_pmc/).
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_tests.sh
bash tools/gpu_r5_profiles.sh
