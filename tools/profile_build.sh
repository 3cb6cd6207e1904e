#!/bin/bash
# Measurement set for the current build, run on the gpurun box:
#   tools/profile_build.sh [tag]
# 1. FETCH_SIZE and WRITE_SIZE passes (one rocprofv3 --pmc run each) over bench.py,
# 2. the kernel-trace --stats summary of the same command,
# 3. the PMC summary bench.py matches by build id (gpurun_out/prof_<tag>/pmc_fetch_config3.json),
# 4. the bench line itself, reading that summary.
# Everything lands in gpurun_out/prof_<tag>/; copy what is judged into profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
B=$(python3 -c "import sys; sys.path.insert(0, 'ebpf-discovery_amd'); import ebd; print(ebd.build_id())") || exit 1
T=${1:-$B}
O=gpurun_out/prof_$T
mkdir -p "$O"
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config4"
tools/gpu_steps.sh \
	"pmc_fetch:240:rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o p --output-format csv -- $CMD" \
	"pmc_write:240:rocprofv3 --pmc WRITE_SIZE -d $O/write -o p --output-format csv -- $CMD" \
	"kstats:240:rocprofv3 --kernel-trace --stats -d $O/kst -o k --output-format csv -- $CMD" \
	"pmcjson:60:python3 tools/pmc_fetch_json.py --fetch $O/fetch --write $O/write --events 100000000 --config 3 --build-id $B --out $O/pmc_fetch_config3.json" \
	"bench:400:python3 bench.py --pmc $O/pmc_fetch_config3.json > $O/bench.json" || exit $?
echo "build $B -> $O"
