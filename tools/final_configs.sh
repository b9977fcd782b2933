#!/bin/bash
# End-of-round profiles of the other configs for the in-tree library, tag T (GPU box): for each
# config, the serial rocprofv3 trace + FETCH / WRITE + the blend's SQ counters
# (tools/profile_config.sh), summarised into profiles/ on the box (so the bench finds this
# build's profile) and copied to gpurun_out/; then every config's bench line
# (tools/configs_bench.sh).  The first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${T:?set T}
for spec in ${CONFIGS:-c2 c3r c5 c4 c4:3/8 c3:3/8}; do
    cfg=${spec%%:*}; strip=""; key=$cfg
    if [ "$spec" != "$cfg" ]; then strip=${spec#*:}; key="$cfg-strip${strip/\//}"; fi
    extra=""; [ -n "$strip" ] && extra="--sim-strip $strip"
    steps=30; [ "$cfg" = c4 ] && [ -z "$strip" ] && steps=10
    tag=$T; [ -n "$strip" ] && tag="${T}s${strip/\//}"  # (its own output directory)
    TAG=$tag CONFIG=$cfg EXTRA="$extra" STEPS=$steps bash tools/profile_config.sh || exit 1
    src=gpurun_out/prof_${tag}_${cfg}
    if [ -n "$strip" ]; then
        rm -rf "gpurun_out/prof_${T}_${key}"
        mv "$src" "gpurun_out/prof_${T}_${key}"
        src=gpurun_out/prof_${T}_${key}
    fi
    python tools/prof_summary.py "$src" --json profiles/${T}_${key}_kernels.json \
        > gpurun_out/${T}_${key}_summary.md || exit 1
    python tools/sq_summary.py "$src" k_blend_q --json profiles/${T}_${key}_blend_sq.json \
        > gpurun_out/${T}_${key}_blend_sq.txt || exit 1
    cp profiles/${T}_${key}_kernels.json profiles/${T}_${key}_blend_sq.json gpurun_out/
    # the raw traces stay on the box (gpurun copies back at most 64 MiB); the summaries travel
    [ "${KEEP_RAW:-0}" = "1" ] || rm -rf "$src"
done
[ "${BENCH:-1}" = "1" ] && { bash tools/configs_bench.sh > gpurun_out/${T}_configs_bench.txt 2>&1 || exit 1; }
exit 0
