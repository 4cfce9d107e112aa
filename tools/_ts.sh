cd ${GRAFT_REPO_ROOT:-/root/repo}
for ranks in 1 8; do for lib in ts6 ts5; do
  MOBILERT_LIB=ab/$lib.so RANKS=$ranks ROUNDS=3 VARIANTS="24=0,24=1,24=1+25=0" timeout -k 10 200 python tools/tune_ab.py 2>&1 | grep setting | sed "s|^|N=$ranks $lib |"
done; done
