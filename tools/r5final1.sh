set -o pipefail
export PTAG=r5final
LEGS="envnet" bash tools/gpu_profile.sh
