#!/bin/bash
# Round evidence in one GPU call: the GPU test suite + smoke (tools/gpu_check.sh) and the round
# profile with HBM traffic passes (tools/prof_round.sh).  Usage: bash tools/round_check.sh TAG
set -o pipefail
TAG=${1:-round}
bash tools/gpu_check.sh $TAG && bash tools/prof_round.sh ${TAG}_prof
