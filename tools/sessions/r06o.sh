# round 6, call o: how much of a service call is the table read's latency — the same A/B with 8,192
# distinct keys (cold table lines) against 16 (lines hot in the service CU's L2), one and eight
# pollers, with the device phase stamps (RP_SVC_PROF) in a separate pass
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06o}; mkdir -p $O
for rep in 1 2 3; do
  for v in 1:8192 8:8192 1:16 8:16; do
    w=${v%:*}; k=${v#*:}
    RP_SVC_WAVES=$w timeout -k 10 120 node tools/svc_latency.js 10000 4000 $k > $O/lat_${w}_${k}_$rep.json 2> $O/lat_${w}_${k}_$rep.err || { echo "latency run failed $v"; cat $O/lat_${w}_${k}_$rep.err; exit 1; }
    echo "w=$w keys=$k rep=$rep $(python3 -c "import json,sys;d=json.load(open('$O/lat_${w}_${k}_$rep.json'));print(d['lookup_service']['median_us'],d['lookup_service']['p10_us'],d['lookup_service']['p90_us'],d['lookupN3_service']['median_us'],d['lookupN3_service']['p90_us'])")"
  done
done
for v in 1:8192 1:16 8:8192 8:16; do
  w=${v%:*}; k=${v#*:}
  RP_SVC_PROF=1 RP_SVC_WAVES=$w timeout -k 10 120 node tools/svc_latency.js 10000 4000 $k > $O/prof_${w}_${k}.json 2> $O/prof_${w}_${k}.err || { echo "prof run failed $v"; cat $O/prof_${w}_${k}.err; exit 1; }
  echo "prof w=$w keys=$k"; cat $O/prof_${w}_${k}.err
done
