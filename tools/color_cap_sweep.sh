#!/bin/bash
# Colour-pass grid cap sweep (GSR_COLOR_BLOCKS; 0 = uncapped): C3 bench line per value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cb in ${CAPS:-512 0 1024 2048}; do
  GSR_COLOR_BLOCKS=$cb timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/cap_$cb.log 2>&1 || { echo "cap $cb failed"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cap', sys.argv[2], d['value'], d['serial_ms_per_frame'], d['stage_ms'])" gpurun_out/cap_$cb.log $cb
done
