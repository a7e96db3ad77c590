set -u
bash tools/sessions/gpu_r03m.sh || exit $?
bash tools/sessions/gpu_r03l.sh || exit $?
