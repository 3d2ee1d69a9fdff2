# the head: GPU test suite, profiles (scripts/prof_r04.sh) and the whole-step
# traffic (scripts/step_traffic.sh) of one build.  usage: TAG=r04ab bash scripts/gpu_r04ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04ab}
TAG=$TAG bash scripts/gpu_r04u.sh && TAG=$TAG bash scripts/step_traffic.sh
