# One measurement call for a profile directory: gpu_round.sh (GPU tests, smoke, R18 bench,
# rocprofv3 stats, PMC passes) followed by gpu_models.sh (DLA34 / YOLACT lines + stats).
set -e
TAG=${1:-r2i}
bash tools/gpu_round.sh $TAG
bash tools/gpu_models.sh ${TAG}_models
