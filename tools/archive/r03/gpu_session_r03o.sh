# k_ck_lanes timing ablations at C5 (results wrong under ablation; times only): fixups, word production
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03o
for v in 0 1 2; do
RP_SIM_CK_ABLATE=$v timeout -k 10 200 rocprofv3 --kernel-trace --kernel-include-regex k_ck_lanes -d gpurun_out/r03o/p$v -o run -- python3 -u tools/sim_c5_probe.py 100000 12 > gpurun_out/r03o/p$v.log 2>&1 || { echo prof failed; tail -5 gpurun_out/r03o/p$v.log; exit 1; }
db=$(find gpurun_out/r03o/p$v -name '*.db' | head -1)
echo "ablate $v"; python3 tools/prof_db.py $db | cut -c1-20,100-200
done
