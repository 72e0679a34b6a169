cd ${GRAFT_REPO_ROOT:-.}
for f in 0 1 2 3; do echo "flags=$f"; timeout -k 10 120 python tools/diag_stamps.py 2 200 $f k_solve | tail -1 || exit 1; done
