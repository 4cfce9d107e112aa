cd "${GRAFT_REPO_ROOT:-/root/repo}"
RANKS=8 VARIANTS=14,16,17,18,21 timeout -k 10 200 python tools/perf_sweep.py 2>&1 | grep -v amdgpu.ids || exit 1
RANKS=2 VARIANTS=14,16,17,18 timeout -k 10 200 python tools/perf_sweep.py 2>&1 | grep -v amdgpu.ids || exit 1
