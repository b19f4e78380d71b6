# final-tree check: smoke, whole GPU suite, bench, kernel profile
set -o pipefail
mkdir -p gpurun_out
PYTEST_X= TAG=${TAG:-r3fin} bash tools/gpu_run.sh smoke tests bench prof
