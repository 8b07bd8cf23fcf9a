# round 5, call r: SQ counters of the C5 refresh kernels (12 rounds), k_ck_lanes against k_ck_tab
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05r; mkdir -p $O
for v in base tab; do
  if [ $v = tab ]; then export RP_SIM_TAB=1; else unset RP_SIM_TAB; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $O/$v -o run -- python3 -u tools/sim_c5_probe.py 100000 12 > $O/$v.log 2>&1 || { echo "$v failed"; tail -20 $O/$v.log; exit 1; }
done
echo done
