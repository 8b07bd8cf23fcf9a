# D1 sender chains: k_ck_pair 8 vs 4 views per workgroup; sim goldens + digests with 4, first 12 C5 rounds traced each way
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03aa
RP_SIM_D1_VPG=4 timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_sim_gpu.py tests/test_sim_digests_gpu.py > gpurun_out/r03aa/tests4.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r03aa/tests4.log; exit 1; }
tail -1 gpurun_out/r03aa/tests4.log
for v in 8 4; do
RP_SIM_D1_VPG=$v timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r03aa/p$v -o run -- python3 -u tools/sim_c5_probe.py 100000 14 > gpurun_out/r03aa/p$v.log 2>&1 || { echo prof failed; tail -5 gpurun_out/r03aa/p$v.log; exit 1; }
done
echo done
