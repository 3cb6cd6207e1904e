#!/bin/bash
# k_fresh experiment builds side by side (one perf_fresh run each, 20 M config-3 events):
#   tools/exp_fresh.sh <variant>...   (variant "default" = the in-tree library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
	if [ "$v" = default ]; then unset EBD_LIB; else export EBD_LIB=$PWD/ebpf-discovery_amd/build/variants/libebd_amd_$v.so; fi
	echo "=== $v"
	timeout -k 10 ${EXP_TIMEOUT:-90} python tools/perf_fresh.py --events 20000000 --reps 3 || exit $?
done
