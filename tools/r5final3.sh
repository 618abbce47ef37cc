set -o pipefail
export PTAG=r5final3
LEGS="envnet" bash tools/gpu_profile.sh
