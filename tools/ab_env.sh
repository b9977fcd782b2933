# A/B bench runs over environment settings: each line of $ENVS is "VAR=val VAR2=val" ("-" = none).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
i=0
while IFS= read -r v; do
  [ -z "$v" ] && continue
  e=$v; [ "$v" = "-" ] && e=""
  env $e timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abe_$i.log 2>&1 || { echo "FAILED: $v"; tail -5 gpurun_out/abe_$i.log; exit 1; }
  echo "[$v] $(grep -o '"value": [0-9.]*' gpurun_out/abe_$i.log) $(grep -o '"stage_ms": {[^}]*}' gpurun_out/abe_$i.log)"
  i=$((i+1))
done <<< "$ENVS"
