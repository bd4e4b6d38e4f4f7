cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
timeout -k 10 200 python tools/stamps.py > $O/stamps_warm.txt 2>&1 || { tail -20 $O/stamps_warm.txt; exit 1; }
timeout -k 10 200 python tools/stamps.py --cold > $O/stamps_cold.txt 2>&1 || { tail -20 $O/stamps_cold.txt; exit 1; }
cat $O/stamps_warm.txt
