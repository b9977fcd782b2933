cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for sh in 0 1 2 3 4; do timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --sort-shape $sh > gpurun_out/var_$sh.log 2>&1 || exit 1; echo "shape $sh: $(grep -o '"value": [0-9.]*\|"tile_sort": [0-9.]*' gpurun_out/var_$sh.log | tr '\n' ' ')"; done
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --onesweep > gpurun_out/var_os.log 2>&1 || exit 1; echo "onesweep: $(grep -o '"value": [0-9.]*\|"tile_sort": [0-9.]*\|"depth_sort": [0-9.]*' gpurun_out/var_os.log | tr '\n' ' ')"
