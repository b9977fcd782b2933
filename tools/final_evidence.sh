#!/bin/bash
# End-of-round evidence for the in-tree library, tag T (GPU box): smoke + the GPU suite
# (tools/gpu_evidence.sh), the serial C3 rocprofv3 profile (tools/profile_config.sh), its
# summaries written into profiles/ on the box (so the bench finds the profile of this build) and
# copied to gpurun_out/, then the default bench line.  The first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${T:?set T}
export T ERR_STATS=${ERR_STATS:-0}
bash tools/gpu_evidence.sh || exit 1
TAG=$T CONFIG=c3 bash tools/profile_config.sh || exit 1
python tools/prof_summary.py gpurun_out/prof_${T}_c3 --json profiles/${T}_c3_kernels.json \
    > gpurun_out/${T}_c3_summary.md || exit 1
python tools/sq_summary.py gpurun_out/prof_${T}_c3 k_blend_q --json profiles/${T}_c3_blend_sq.json \
    > gpurun_out/${T}_c3_blend_sq.txt || exit 1
cp profiles/${T}_c3_kernels.json profiles/${T}_c3_blend_sq.json gpurun_out/
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err || exit 1
tail -c 600 gpurun_out/${T}_bench_default.json
