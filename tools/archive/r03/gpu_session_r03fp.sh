cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03fp
L="--no-merge --sim-n 0 --sim5-n 0 --no-wire --no-api --no-cpu --steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03fp/new -o run -- python3 -u bench.py $L > gpurun_out/r03fp/new.json 2> gpurun_out/r03fp/new.err || { echo prof failed; tail gpurun_out/r03fp/new.err; exit 1; }
RP_AMD_LIB=$PWD/tools/ablib/librpamd_base.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03fp/base -o run -- python3 -u bench.py $L > gpurun_out/r03fp/base.json 2> gpurun_out/r03fp/base.err || { echo prof failed; tail gpurun_out/r03fp/base.err; exit 1; }
echo done
