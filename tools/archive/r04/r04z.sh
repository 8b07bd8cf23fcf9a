# round 4, call z: wire wave phase cycles of the current kernels (-DRP_WIRE_PROF)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04z; mkdir -p $O
RP_AMD_LIB=$PWD/ringpop-node_amd/ab/librpamd_wprof.so timeout -k 10 200 python -u bench.py --no-cpu --no-api --sim-n 0 --sim5-n 0 --no-merge --steps 2 --warmup 1 --batch-log2 20 > $O/wprof.json 2> $O/wprof.err || { echo bench wprof failed; tail -20 $O/wprof.err; exit 1; }
grep "wire wave cycles" $O/wprof.err | tail -1
