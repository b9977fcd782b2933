set -u
cd $GRAFT_REPO_ROOT
T=r03b ERR_STATS=0 bash tools/gpu_evidence.sh || exit 1
for c in c3 c3r; do
  timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --cpu-seconds 8 > gpurun_out/r03b_bench_$c.json 2> gpurun_out/r03b_bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/r03b_bench_$c.err; exit 1; }
  tail -c 600 gpurun_out/r03b_bench_$c.json; echo
done
CONFIG=c3 TAG=r03b bash tools/profile_config.sh || exit 1
