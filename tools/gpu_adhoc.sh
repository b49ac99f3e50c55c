#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WL=products_bsr16_f16 VARS="4099 4107" bash tools/bsr_variants.sh || exit 1
WL=products_bsr16_f16 EXTRA="--dtype fp32" VARS="4100 4108" bash tools/bsr_variants.sh || exit 1
