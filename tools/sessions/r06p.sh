# round 6, call p: the service's record answered without LDS (dt_answer_fast) and the header read
# from registers, against the round-5 answer (RP_SVC_ANS=0): parity, then latency (cold / hot keys)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${O:-$PWD/gpurun_out/r06p}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ring_gpu.py -k "service" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  for v in 1:8192 0:8192 1:16 0:16; do
    a=${v%:*}; k=${v#*:}
    RP_SVC_ANS=$a timeout -k 10 120 node tools/svc_latency.js 10000 4000 $k > $O/lat_${a}_${k}_$rep.json 2> $O/lat_${a}_${k}_$rep.err || { echo "latency run failed $v"; cat $O/lat_${a}_${k}_$rep.err; exit 1; }
    echo "ans=$a keys=$k rep=$rep $(python3 -c "import json,sys;d=json.load(open('$O/lat_${a}_${k}_$rep.json'));print(d['lookup_service']['median_us'],d['lookup_service']['p10_us'],d['lookup_service']['p90_us'],d['lookupN3_service']['median_us'],d['lookupN3_service']['p90_us'])")"
  done
done
for v in 1:8192 0:8192 1:16 0:16; do
  a=${v%:*}; k=${v#*:}
  RP_SVC_PROF=1 RP_SVC_WAVES=1 RP_SVC_ANS=$a timeout -k 10 120 node tools/svc_latency.js 10000 4000 $k > $O/prof_${a}_${k}.json 2> $O/prof_${a}_${k}.err || { echo "prof run failed $v"; cat $O/prof_${a}_${k}.err; exit 1; }
  echo "prof ans=$a keys=$k (one wave)"; cat $O/prof_${a}_${k}.err
done
