cd ${GRAFT_REPO_ROOT:-/root/repo}
for ranks in 8 1; do for lib in se0 se1 ts5; do
  MOBILERT_LIB=ab/$lib.so RANKS=$ranks ROUNDS=3 VARIANTS="24=0,24=1" timeout -k 10 200 python tools/tune_ab.py 2>&1 | grep setting | grep -v identical | sed "s|^|N=$ranks $lib |"
done; done
