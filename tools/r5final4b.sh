set -o pipefail
export PTAG=r5final4
LEGS="envnet" bash tools/gpu_profile.sh
