set -o pipefail
bash tools/gpu_parse_ab.sh && bash tools/gpu_prof_parse.sh
