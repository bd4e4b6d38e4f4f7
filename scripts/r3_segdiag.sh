cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3; mkdir -p $O
timeout -k 10 200 python tools/seg_windows.py > $O/seg_windows.txt 2>&1; rc=$?; cat $O/seg_windows.txt | tail -25; exit $rc
