#!/bin/bash
# tools/pmc_lds.sh <out_dir> <variant or default>...: LDS / issue counter pass over perf_fresh
# (20 M config-3 events) for each library, one rocprofv3 --pmc run each.
out=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for v in "$@"; do
	if [ "$v" = default ]; then unset EBD_LIB; else export EBD_LIB=$PWD/ebpf-discovery_amd/build/variants/libebd_amd_$v.so; fi
	timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES \
		-d "$out/$v" -o p --output-format csv -- python3 tools/perf_fresh.py --reps 1 > /dev/null || exit $?
	echo "== $v"
	python3 tools/pmc_summary.py "$out/$v" k_fresh
done
