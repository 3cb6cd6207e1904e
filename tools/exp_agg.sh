#!/bin/bash
# k_agg_fast experiment builds side by side, warm and cold (20 M config-3 events):
#   tools/exp_agg.sh <variant>...   (variant "default" = the in-tree library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for v in "$@"; do
	if [ "$v" = default ]; then unset EBD_LIB; else export EBD_LIB=$PWD/ebpf-discovery_amd/build/variants/libebd_amd_$v.so; fi
	for mode in "" "--cold"; do
		echo "=== $v $mode"
		timeout -k 10 ${EXP_TIMEOUT:-90} python tools/perf_fresh.py --events 20000000 --reps 3 $mode | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps({'step_ms': round(d['step_ms'], 3), **{k: round(v, 3) for k, v in d['kernel_ms'].items()}}))" || exit $?
	done
done
