#!/bin/bash
# The exact LRU on the gpurun box: tools/profile_lru.sh [tag]
# 1 M config-4 events over an LRU of 2048 (two batches), the perf line, then the kernel-trace
# summary of one batch.  Everything lands in gpurun_out/proflru_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
B=$(python3 -c "import sys; sys.path.insert(0, 'ebpf-discovery_amd'); import ebd; print(ebd.build_id())") || exit 1
T=${1:-$B}
O=gpurun_out/proflru_$T
mkdir -p "$O"
tools/gpu_steps.sh \
	"lru1m:200:python3 tools/perf_walk.py --events 1000000 --lru 2048 --reps 2 > $O/exact_lru_1M.json" \
	"lrukst:300:rocprofv3 --kernel-trace --stats -d $O/kst -o k --output-format csv -- python3 tools/perf_walk.py --events 1000000 --lru 2048 --reps 1" || exit $?
echo "build $B -> $O"
