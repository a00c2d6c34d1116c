set -e -o pipefail
bash tools_dev/gpu_round.sh r04final
