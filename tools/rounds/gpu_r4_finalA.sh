#!/bin/bash
# Round 4 closing pass A: every GPU test + smoke(), then every profile shape (kernel stats + traces, FETCH_SIZE
# and WRITE_SIZE passes; gpu_r4_profiles.sh -> gpurun_out/r4prof/).
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_tests.sh
bash tools/gpu_r4_profiles.sh
