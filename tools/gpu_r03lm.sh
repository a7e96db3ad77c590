set -u
bash tools/gpu_r03m.sh || exit $?
bash tools/gpu_r03l.sh || exit $?
