set -o pipefail
export PTAG=r5final5
LEGS="envnet" bash tools/gpu_profile.sh
