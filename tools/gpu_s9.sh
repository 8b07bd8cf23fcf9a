set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s9
for n in 10000 25000 50000; do
  for m in pc lanes; do
    RP_SIM_CK=$m timeout -k 10 200 python -u tools/sim_probe.py $n 1 300 > gpurun_out/s9/sim_${n}_$m.log 2>&1 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s9/prof10k -o run -- python -u tools/sim_probe.py 10000 1 300 > gpurun_out/s9/prof10k.log 2>&1
RP_SIM_CK=lanes timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s9/prof10k_lanes -o run -- python -u tools/sim_probe.py 10000 1 300 > gpurun_out/s9/prof10k_lanes.log 2>&1
