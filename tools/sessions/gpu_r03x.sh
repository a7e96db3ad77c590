#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
bash tools/sessions/gpu_r03w.sh || exit $?
bash tools/sessions/gpu_r03v.sh || exit $?
