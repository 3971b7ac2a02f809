set -o pipefail
bash tools/gpu_split.sh && bash tools/gpu_split_prof.sh
