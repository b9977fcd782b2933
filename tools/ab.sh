# A/B bench runs: each line of $VARIANTS is a set of bench.py flags ("-" = defaults).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
i=0
while IFS= read -r v; do
  [ -z "$v" ] && continue
  f=$v; [ "$v" = "-" ] && f=""
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline $f > gpurun_out/ab_$i.log 2>&1 || { echo "FAILED: $v"; tail -5 gpurun_out/ab_$i.log; exit 1; }
  echo "[$v] $(grep -o '"value": [0-9.]*' gpurun_out/ab_$i.log) $(grep -o '"stage_ms": {[^}]*}' gpurun_out/ab_$i.log)"
  i=$((i+1))
done <<< "$VARIANTS"
