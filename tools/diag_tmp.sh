cd $GRAFT_REPO_ROOT
for d in 0 1 2 3; do echo "VR_DIAG=$d"; VR_DIAG=$d python tools/sweep.py --rounds 3 --configs c3,c3exact,c2 2>&1 | grep -E "median"; done
