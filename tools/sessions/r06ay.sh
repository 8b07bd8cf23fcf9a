# round 6, call ay: PMC passes over the lean kernel, the wave-specialised kernel (4:12) and its two
# ablations (key stream alone, trips alone): L2 busy and tag stalls, L1->L2 requests and their
# latency, TA / TD busy, L1 stalls. One counter group a pass, each its own run.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06ay}; mkdir -p $O
V=default/lookupN3,ws412/lookupN3,ws412-abl1/lookupN3,ws412-abl2/lookupN3
for grp in "TCC_BUSY_avr TCC_TAG_STALL_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" "TA_BUSY_avr TD_BUSY_sum GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/$tag -o run -- python3 tools/ab_lookup.py --rounds 2 --only $V > $O/$tag.log 2>&1 || { echo "pmc $grp failed"; tail -5 $O/$tag.log; exit 1; }
  echo "pmc $grp ok"
done
python3 tools/pmc_ws_summary.py $O > $O/summary.json && cat $O/summary.json
