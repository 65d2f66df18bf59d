#!/bin/bash
# on-the-fly correlation: kernel tests + bench + profile; then the fp32 step's op table
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-of}
bash scripts/gpu_otf.sh ${TAG} || exit 1
cat gpurun_out/${TAG}_categories.txt
bash scripts/gpu_fp32_prof.sh || exit 1
