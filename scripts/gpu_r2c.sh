#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
TAG=${TAG:-c} TLIM=900 bash scripts/gpu_test.sh || exit 1
TAG=${TAG:-c} bash scripts/gpu_bench2.sh
