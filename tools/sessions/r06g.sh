# round 6, call g: C3 chain placement — chain workgroups padded to one a CU (RP_HL_LDS_PAD), with
# groups of 128 and 256
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06g}; mkdir -p $O
timeout -k 10 500 python3 -u tools/c3_ab.py --batches 1024 --rounds 2 --variants side,pad,side-g256,pad-g256 > $O/c3ab.log 2>&1 || { echo "c3ab failed"; tail -20 $O/c3ab.log; exit 1; }
grep -v "^{" $O/c3ab.log
