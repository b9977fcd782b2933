#!/bin/bash
# Every BASELINE.json config that fits one GPU, one JSON line each, into gpurun_out/configs/:
# C2 (100k SH0), C3 (1M SH3, the headline), C5 (1M, 1000-frame orbit camera), c3r (the clustered
# scene), a C3 1/8 strip, C4's full frame on one
# GPU (N=1), and C4's per-rank work (6M Gaussians at 3840x2160, one of 8 strips, --sim-strip) for every strip.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/configs
run() {  # name args...
    local name=$1; shift
    timeout -k 10 300 python bench.py "$@" > gpurun_out/configs/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/configs/$name.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['serial_ms_per_frame'], d['frame_stats'])" gpurun_out/configs/$name.log $name
}
run c2 --config c2 --steps 500 --warmup 50 --no-cpu-baseline
run c3 --config c3 --steps 200 --warmup 20 --no-cpu-baseline
run c5 --config c5 --steps 1000 --warmup 50 --no-cpu-baseline
run c3r --config c3r --steps 200 --warmup 20 --no-cpu-baseline
run c3_strip3of8 --config c3 --sim-strip 3/8 --steps 500 --warmup 50 --no-cpu-baseline
run c3_strip0of8 --config c3 --sim-strip 0/8 --steps 500 --warmup 50 --no-cpu-baseline
run c4_full --config c4 --steps 50 --warmup 5 --no-cpu-baseline
for r in 0 1 2 3 4 5 6 7; do
  run c4_strip${r}of8 --config c4 --sim-strip $r/8 --steps 100 --warmup 10 --no-cpu-baseline
done
