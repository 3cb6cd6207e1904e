#!/bin/bash
# Config 4 (fragmented keep-alive sessions) on the gpurun box:
#   tools/profile_config4.sh [tag]
# the kernel-trace --stats summary of a short config-4 bench, then the bench line itself
# (with its CPU baseline).  Everything lands in gpurun_out/prof4_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
B=$(python3 -c "import sys; sys.path.insert(0, 'ebpf-discovery_amd'); import ebd; print(ebd.build_id())") || exit 1
T=${1:-$B}
O=gpurun_out/prof4_$T
mkdir -p "$O"
tools/gpu_steps.sh \
	"kstats4:300:rocprofv3 --kernel-trace --stats -d $O/kst -o k --output-format csv -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline" \
	"bench4:400:python3 bench.py --config 4 > $O/bench.json" || exit $?
echo "build $B -> $O"
