# round 5, call ay: PMC passes of the C2 lookupN(3) kernel at the end of the round (ablation branches compiled out), with the
# hash-only calibration kernel, summarised into profiles/pmc_traffic.json form
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ay; mkdir -p $O
timeout -k 10 900 bash tools/pmc_lookup.sh $O/pmc "default/lookupN3,probe/ablate-hash-only" > $O/pmc.log 2>&1 || { echo pmc failed; tail -20 $O/pmc.log; exit 1; }
cat $O/pmc.log
PMC_MEASURED_ON="round 5 end (k_lookupn_lean<8,3,4>, hinted index, no ablation branches), tools/sessions/r05ay.sh" python3 tools/pmc_summary.py $O/pmc > $O/pmc_traffic.json || exit 1
python3 -c "import json;d=json.load(open('$O/pmc_traffic.json'));print({k:d[k] for k in ('lookupn_hbm_bytes_per_launch','l2_hit_rate','l1_to_l2_read_requests_per_key')})"
rm -rf $O/pmc/*/run_kernel_trace.csv
