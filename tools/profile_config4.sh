#!/bin/bash
# Config 4 (fragmented keep-alive sessions) on the gpurun box:
#   tools/profile_config4.sh [tag]
# 1. FETCH_SIZE and WRITE_SIZE passes (one rocprofv3 --pmc run each) over a config-4 bench,
#    summarised for k_walk and k_emit per step (gpurun_out/prof4_<tag>/pmc_fetch_config4.json,
#    which bench.py matches by build id for the config-4 roofline's traffic),
# 2. the kernel-trace --stats summary of the same command,
# 3. the bench line itself (with its CPU baseline), reading that summary.
# Everything lands in gpurun_out/prof4_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
B=$(python3 -c "import sys; sys.path.insert(0, 'ebpf-discovery_amd'); import ebd; print(ebd.build_id())") || exit 1
T=${1:-$B}
O=gpurun_out/prof4_$T
mkdir -p "$O"
CMD="python3 bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline"
# events per step and poll cycles per step of the config-4 bench (one launch of each kernel per cycle)
EV=$(timeout -k 10 400 python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['config']['events_per_gpu'], d['config']['poll_cycles_per_step'])") || exit 1
set -- $EV
tools/gpu_steps.sh \
	"pmc4_fetch:300:rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o p --output-format csv -- $CMD" \
	"pmc4_write:300:rocprofv3 --pmc WRITE_SIZE -d $O/write -o p --output-format csv -- $CMD" \
	"pmc4json:60:python3 tools/pmc_fetch_json.py --fetch $O/fetch --write $O/write --events $1 --config 4 --kernel k_walk,k_emit --launches-per-step $2 --build-id $B --out $O/pmc_fetch_config4.json" \
	"kstats4:300:rocprofv3 --kernel-trace --stats -d $O/kst -o k --output-format csv -- $CMD" \
	"bench4:400:python3 bench.py --config 4 --pmc4 $O/pmc_fetch_config4.json > $O/bench.json" || exit $?
echo "build $B -> $O"
