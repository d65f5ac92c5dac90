# kernel trace of one emulated rank (rank 4 of 8): the factor chain's kernels against the y build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04_t17 -o emu -- python3 bench.py --emulate-ranks 8 --emulate-only 4 --steps 3 --warmup 1 > gpurun_out/r04_t17.json 2> gpurun_out/r04_t17.err
ls gpurun_out/r04_t17/ | head
exit 0
