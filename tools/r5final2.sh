set -o pipefail
export PTAG=r5final2
BENCH=0 LEGS="ast ast-fp8" bash tools/gpu_profile.sh
