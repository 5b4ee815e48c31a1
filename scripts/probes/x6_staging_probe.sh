cd $GRAFT_REPO_ROOT
for v in full noB noA none; do VARIANT=$v HG_LIB=$GRAFT_REPO_ROOT/build/x6p/$v/libhgsim.so timeout -k 10 120 python scripts/probes/x6_staging_probe.py 2>/dev/null || exit 1; done
