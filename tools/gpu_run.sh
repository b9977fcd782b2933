#!/bin/bash
# Local guard before a gpurun call: rebuild libgsr.so and refuse to ship a stale library.
# Usage: tools/gpu_run.sh '<command for the GPU box>' [timeout_s]
set -e
cd "$(dirname "$0")/.."
make -C gaussiansplattingviewer_amd/csrc -j8 >/tmp/gsr_build.log 2>&1 || { grep -E "error" -A3 /tmp/gsr_build.log | head -30; echo "BUILD FAILED"; exit 1; }
make -C gaussiansplattingviewer_amd/csrc -q || { echo "library not up to date"; exit 1; }
exec /usr/local/graft/bin/gpurun --timeout "${2:-900}" -- "$1"
