cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for mode in fast packed exact; do for bb in x; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --blend $mode > gpurun_out/bv_${mode}_$bb.log 2>&1 || exit 1
  echo "$mode $bb: $(grep -o '"value": [0-9.]*\|"blend": [0-9.]*' gpurun_out/bv_${mode}_$bb.log | tr '\n' ' ')"
done; done
