cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --sim-strip $r/8 > gpurun_out/sim_$r.log 2>&1 || { echo FAIL $r; tail -3 gpurun_out/sim_$r.log; exit 1; }
  echo "strip $r/8: $(grep -o '"value": [0-9.]*' gpurun_out/sim_$r.log) $(grep -o '"stage_ms": {[^}]*}' gpurun_out/sim_$r.log)"
done
