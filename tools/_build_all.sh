# rebuild libmgx + the two phase-stamp diagnostic variants
set -e
make -s -C minigrid-rl_amd
make -s -C minigrid-rl_amd EXTRA=-DMGX_STAMPS=1 OUT=mgx/libmgx_stamps.so -B
make -s -C minigrid-rl_amd EXTRA=-DMGX_STAMPS=2 OUT=mgx/libmgx_stamps2.so -B
make -s -C minigrid-rl_amd EXTRA=-DMGX_STAMPS=3 OUT=mgx/libmgx_stamps3.so -B
