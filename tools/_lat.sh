cd ${GRAFT_REPO_ROOT:-/root/repo}; R=$(pwd)
for ranks in 8 1; do for lib in sf0 sf1 sf0 sf1; do
  MOBILERT_LIB=ab/$lib.so RANKS=$ranks ROUNDS=2 VARIANTS="" timeout -k 10 200 python tools/tune_ab.py 2>&1 | grep setting | sed "s|^|N=$ranks $lib |"
done; done
